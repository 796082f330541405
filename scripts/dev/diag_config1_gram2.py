"""configs[1]: the device Gram matrix L^T L (any summation order of the device GEMMs) gives a
one-step Woodbury panel that takes ~570 iterations; host BLAS Grams of the same device L (any
order) ~366.  Which part of the difference D = G_dev - G_host matters?

    python scripts/dev/diag_config1_gram2.py       (GPU box)

Panels from G_host + t D (t = 0.1, 0.3, 1), from D's diagonal / off-diagonal part only, from a
symmetric random perturbation of the same Frobenius norm, and from G_dev rounded to fewer bits,
each applied on the host in the scipy-1.7.3 recurrence with the device operator.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd"), str(REPO / "scripts" / "dev")]

import sgdml_amd  # noqa: E402
from diag_config1_gram import LAM, N_ATOMS, SIG, TOL, dev_gram, panel  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.sgdml import descriptors  # noqa: E402


def main():
    g = REPO / "tests" / "golden"
    f = np.load(g / "nanotube_n15540.npz", allow_pickle=False)
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    n, k = y.size, 2701
    out = {}
    with sgdml_amd.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(N_ATOMS)[None, :], SIG)
        s.set_operator(-1.0, LAM)
        s.precon_pivchol(k, build_woodbury=False)
        Lt = np.ascontiguousarray(s.precon_panel())
        Gh = Lt @ Lt.T
        Gd = dev_gram(s, Lt, 8)
        Gd = np.tril(Gd) + np.tril(Gd, -1).T
        D = Gd - Gh
        out["D_fro_rel"] = float(np.linalg.norm(D) / np.linalg.norm(Gh))
        out["D_diag_rel_max"] = float(np.max(np.abs(np.diag(D)) / np.diag(Gh)))
        ev = np.linalg.eigvalsh(Gh)
        out["G_eig_min_max"] = [float(ev[0]), float(ev[-1])]
        U = np.linalg.eigh(Gh)[1]
        Dp = U.T @ D @ U
        out["D_in_eigbasis_smallest_block"] = float(np.abs(Dp[:50, :50]).max())
        rng = np.random.default_rng(7)
        Rn = rng.standard_normal((k, k))
        Rn = (Rn + Rn.T) / 2
        Rn *= np.linalg.norm(D) / np.linalg.norm(Rn)
        grams = {"host": Gh, "dev": Gd, "t0.1": Gh + 0.1 * D, "t0.3": Gh + 0.3 * D,
                 "diagD": Gh + np.diag(np.diag(D)), "offdiagD": Gh + D - np.diag(np.diag(D)),
                 "randsym": Gh + Rn, "host_rel_noise": Gh * (1 + 4e-16 * (Rn / np.abs(Rn).max()))}
        for name, G in grams.items():
            T = panel(G, Lt)
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=2000,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            out[name] = int(it)
            print(json.dumps({name: int(it)}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
