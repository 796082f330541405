"""Where the configs[1] full-size GPU solve (570 iterations) parts from the oracle's (367):
the pivoted-Cholesky factor L, the Woodbury panel T built from it, or the PCG around them.

    python scripts/dev/diag_config1.py        (GPU box; tests/golden/nanotube_n15540.npz)

1. GPU pivoted Cholesky (rank 2701, no Woodbury): pivots and pivot values against the
   fixture's (the oracle's L[m_pi, m]^2), L^T fetched from the panel.
2. Woodbury panel of that L on the host (oracle.precon.woodbury_panel, LAPACK) and on the GPU
   (mlff_precon_lowrank = woodbury_inplace): difference of the panels and of one apply.
3. The scipy-1.7.3 CG recurrence (oracle.pcg.cg_legacy) driven from the host with the GPU
   operator (mlff_matvec) and either panel applied on the host, next to the GPU PCG with the
   GPU panel: which piece moves the count from 367.
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

import sgdml_amd  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.precon import woodbury_panel  # noqa: E402
from oracle.sgdml import descriptors  # noqa: E402

N_ATOMS, SIG, LAM, TOL = 370, 10.0, 1e-10, 1e-6


def main():
    g = REPO / "tests" / "golden"
    f = np.load(g / "nanotube_n15540.npz", allow_pickle=False)
    band = json.loads((g / "nanotube_n15540_band.json").read_text())
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    n, k = y.size, int(band["k"])
    out = {"n": n, "k": k, "oracle_iters": int(f["iters"])}
    with sgdml_amd.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(N_ATOMS)[None, :], SIG)
        s.set_operator(-1.0, LAM)
        t0 = time.time()
        piv, _ = s.precon_pivchol(k, build_woodbury=False)
        Lt = s.precon_panel()  # L^T, k x n
        out["pivchol_s"] = time.time() - t0
        out["pivots_equal"] = bool(np.array_equal(piv[:k], f["index_columns"]))
        pv = Lt[np.arange(k), piv[:k]] ** 2
        rel = np.abs(pv - f["pivot_values"]) / np.abs(f["pivot_values"])
        out["pivot_value_rel_err_max"] = float(rel.max())
        out["pivot_value_rel_err_at"] = {int(m): float(rel[m]) for m in (0, 100, 1000, 2000, k - 1)}
        out["pivot_values_oracle_first_last"] = [float(f["pivot_values"][0]),
                                                 float(f["pivot_values"][-1])]
        t0 = time.time()
        Th, _ = woodbury_panel(np.ascontiguousarray(Lt.T), LAM)
        out["host_woodbury_s"] = time.time() - t0
        s.precon_lowrank(Lt)
        Tg = s.precon_panel()
        out["panel_rel_diff"] = float(np.linalg.norm(Tg - Th) / np.linalg.norm(Th))
        r = np.random.default_rng(0).standard_normal(n)
        zh = (r - Th.T @ (Th @ r)) / LAM
        zg = (r - Tg.T @ (Tg @ r)) / LAM
        zd = s.precon_apply(r)
        out["apply_rel_diff_host_vs_gpu_panel"] = float(np.linalg.norm(zg - zh) / np.linalg.norm(zh))
        out["apply_rel_diff_device_vs_host"] = float(np.linalg.norm(zd - zh) / np.linalg.norm(zh))
        # GPU PCG with the GPU Woodbury panel of the GPU L
        res = s.pcg(y, tol=TOL, maxiter=5 * n)
        out["gpu_pcg_iters"] = int(res.iters)
        # the host panel in two more summation orders of its Gram matrix L^T L (the oracle's
        # band varied the operator and the apply, not the panel's construction)
        import scipy.linalg

        def panel_from_gram(Gm):
            L2 = scipy.linalg.cholesky(LAM * np.eye(k) + Gm, lower=True)
            return scipy.linalg.solve_triangular(L2, Lt, lower=True)

        Lr = np.ascontiguousarray(Lt[:, ::-1])
        T_rev = panel_from_gram(Lr @ Lr.T)
        blocks = np.array_split(np.arange(n), 8)
        T_blk = panel_from_gram(sum(Lt[:, b] @ Lt[:, b].T for b in blocks))
        out["panel_rel_diff_rev"] = float(np.linalg.norm(T_rev - Th) / np.linalg.norm(Th))
        out["panel_rel_diff_blk8"] = float(np.linalg.norm(T_blk - Th) / np.linalg.norm(Th))
        # host-driven recurrence, GPU operator, each panel applied on the host
        for name, T in (("host_panel", Th), ("gpu_panel", Tg), ("host_panel_gram_rev", T_rev),
                        ("host_panel_gram_blk8", T_blk)):
            t0 = time.time()
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=5 * n,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            out[f"host_cg_{name}_iters"] = int(it)
            out[f"host_cg_{name}_s"] = time.time() - t0
            out[f"host_cg_{name}_rel_dalpha"] = float(
                np.linalg.norm(-x - f["alphas"]) / np.linalg.norm(f["alphas"]))
            print(json.dumps({name: int(it)}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
