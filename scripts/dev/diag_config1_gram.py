"""configs[1] (nanotube N = 15540, k = 2701): which step of the device's one-step Woodbury panel
moves the count from the oracle's 367 to ~570 (the two-step panel takes 366).

    python scripts/dev/diag_config1_gram.py        (GPU box; tests/golden/nanotube_n15540.npz)

From the device factor L (pivoted Cholesky without Woodbury): the Gram matrix L^T L by host BLAS
and by the device fp64 GEMM (matrix cores, one pass and split-K slabs), each factored and solved
on the host (LAPACK); the device's own one-step panel; every panel applied on the host in the
scipy-1.7.3 recurrence with the device operator.
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np
import scipy.linalg

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

import sgdml_amd  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.sgdml import descriptors  # noqa: E402
from sgdml_amd import _native as nat  # noqa: E402

N_ATOMS, SIG, LAM, TOL = 370, 10.0, 1e-10, 1e-6


def dev_gram(s, Lt, splits):
    k, n = Lt.shape
    G = np.zeros((k, k))
    nat.check(nat.load_library().mlff_test_gemm(s._ctx, 0, 1, k, k, n, 1.0, nat.dptr(Lt), n,
                                                nat.dptr(Lt), n, 1.0 if splits > 1 else 0.0,
                                                nat.dptr(G), k, splits), s._ctx, "mlff_test_gemm")
    return -G if splits > 1 else G  # split-K path returns C - alpha A B^T with C = 0


def panel(Gm, Lt):
    k = Gm.shape[0]
    L2 = scipy.linalg.cholesky(LAM * np.eye(k) + Gm, lower=True)
    return scipy.linalg.solve_triangular(L2, Lt, lower=True)


def main():
    g = REPO / "tests" / "golden"
    f = np.load(g / "nanotube_n15540.npz", allow_pickle=False)
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    n, k = y.size, 2701
    out = {}
    os.environ["MLFF_WB_REFINE"] = "0"
    with sgdml_amd.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(N_ATOMS)[None, :], SIG)
        s.set_operator(-1.0, LAM)
        s.precon_pivchol(k, build_woodbury=False)
        Lt = np.ascontiguousarray(s.precon_panel())
        Gh = Lt @ Lt.T
        panels = {"host_gram": panel(Gh, Lt)}
        for sp in (1, 8):
            Gd = dev_gram(s, Lt, sp)
            out[f"gram_dev_s{sp}_rel_diff"] = float(np.linalg.norm(Gd - Gh) / np.linalg.norm(Gh))
            out[f"gram_dev_s{sp}_asym"] = float(np.abs(Gd - Gd.T).max())
            panels[f"dev_gram_s{sp}"] = panel(np.tril(Gd) + np.tril(Gd, -1).T, Lt)
        s.precon_lowrank(Lt)
        panels["device_onestep"] = s.precon_panel()
        out["device_onestep_device_pcg"] = int(s.pcg(y, tol=TOL, maxiter=5 * n).iters)
        ref = panels["host_gram"]
        for name, T in panels.items():
            out[name + "_rel_diff"] = float(np.linalg.norm(T - ref) / np.linalg.norm(ref))
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=2000,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            out[name + "_host_apply"] = int(it)
            print(json.dumps({name: int(it), "rel_diff": out[name + "_rel_diff"]}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
