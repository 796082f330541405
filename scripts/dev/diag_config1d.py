"""configs[1] full size: one CholeskyQR2-style refinement of the Woodbury panel.

    python scripts/dev/diag_config1d.py        (GPU box; tests/golden/nanotube_n15540.npz)

T = L2^-1 L^T is the top block (transposed) of Q1 = A R1^-1, A = [L; sqrt(lam) I], R1^T R1 =
A^T A = lam I + L^T L (one CholeskyQR step).  diag_config1c.py: a Householder QR of A gives
362 iterations, LAPACK's Cholesky + triangular solve 364, the device build 571, an explicit
inverse 577.  A second CholeskyQR step re-orthogonalises Q1 (Q1 bottom = sqrt(lam) L2^-T):
G2 = Q1^T Q1 = T T^T + lam L2^-1 L2^-T (= I exactly), C C^T = G2, T2 = C^-1 T.  Here it is applied on the host to each panel (device-built, inverse,
perturbed, LAPACK) and every T2 is solved by the host-driven scipy-1.7.3 recurrence with the
device operator.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import scipy.linalg

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

import sgdml_amd  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.sgdml import descriptors  # noqa: E402

N_ATOMS, SIG, LAM, TOL = 370, 10.0, 1e-10, 1e-6


def refine(T, B):
    G2 = T @ T.T + LAM * B
    C = scipy.linalg.cholesky(G2, lower=True)
    return scipy.linalg.solve_triangular(C, T, lower=True)


def main():
    g = REPO / "tests" / "golden"
    f = np.load(g / "nanotube_n15540.npz", allow_pickle=False)
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    n, k = y.size, int(f["index_columns"].size)
    out = {"n": n, "k": k, "oracle_iters": int(f["iters"])}
    with sgdml_amd.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(N_ATOMS)[None, :], SIG)
        s.set_operator(-1.0, LAM)
        s.precon_pivchol(k, build_woodbury=False)
        Lt = s.precon_panel()
        G1 = LAM * np.eye(k) + Lt @ Lt.T
        L2 = scipy.linalg.cholesky(G1, lower=True)
        L2inv = scipy.linalg.solve_triangular(L2, np.eye(k), lower=True)
        Binv = L2inv @ L2inv.T  # L2^-1 L2^-T
        T0 = scipy.linalg.solve_triangular(L2, Lt, lower=True)
        rng = np.random.default_rng(11)
        s.precon_lowrank(Lt)
        base = {"lapack": T0, "device": s.precon_panel(), "inverse": np.tril(L2inv) @ Lt,
                "noise2e-15": T0 * (1.0 + 2e-15 * rng.standard_normal(T0.shape))}
        panels = {}
        for name, T in base.items():
            panels[name] = T
            panels[name + "+refined"] = refine(T, Binv)
        # the device's own refined build (MLFF_WB_REFINE=1, woodbury_inplace) and its PCG
        import os

        os.environ["MLFF_WB_REFINE"] = "1"
        with sgdml_amd.KernelSolver(n) as s2:
            s2.sgdml_operator(Rd, Rdd, np.arange(N_ATOMS)[None, :], SIG)
            s2.set_operator(-1.0, LAM)
            piv2, sec = s2.precon_pivchol(k)
            panels["device_refined_build"] = s2.precon_panel()
            res = s2.pcg(y, tol=TOL, maxiter=5 * n)
            out["device_refined_pcg"] = {"iters": int(res.iters), "info": int(res.info),
                                         "build_s": sec,
                                         "rel_dalpha": float(np.linalg.norm(-res.x - f["alphas"]) /
                                                             np.linalg.norm(f["alphas"]))}
            print(json.dumps({"device_refined_pcg": out["device_refined_pcg"]}), flush=True)
        del os.environ["MLFF_WB_REFINE"]
        res = s.pcg(y, tol=TOL, maxiter=5 * n)
        out["device_pcg"] = {"iters": int(res.iters)}
        for name, T in panels.items():
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=5 * n,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            out[name] = {"iters": int(it), "info": int(info),
                         "panel_rel_diff": float(np.linalg.norm(T - T0) / np.linalg.norm(T0)),
                         "rel_dalpha": float(np.linalg.norm(-x - f["alphas"]) /
                                             np.linalg.norm(f["alphas"]))}
            print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
