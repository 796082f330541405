"""The Woodbury panel's second CholeskyQR step on the many-point ethanol system (N = 15741,
rank 1264 pivoted Cholesky): bench lines at HEAD found the device solve to 1e-6 converging in
1749 iterations with the one-step panel and not at all (78705) with the refined one.

    python scripts/dev/diag_ethanol_refine.py       (GPU box)

From the device L: the condition of A = [L; sqrt(lam) I] (singular values of L), and the count of
the host-driven scipy-1.7.3 recurrence (device operator) with the LAPACK one-step panel, the
LAPACK panel refined on the host, a Householder-QR panel, the device one-step panel and the
device refined panel.
"""
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
from sgdml_amd import synthetic  # noqa: E402
from sgdml_amd.rule_of_thumb import get_params, rule_of_thumb  # noqa: E402

LAM, TOL = 1e-10, 1e-6


def main(M=583):
    ds = synthetic.ethanol_like(M, seed=0)
    y, _ = synthetic.labels(ds["F"])
    n = y.size
    m, kmin, _ = get_params("ethanol")
    k = int(rule_of_thumb(n=n, k_min=kmin, m=m))
    Rd, Rdd = sgdml_amd.sgdml_descriptors(ds["R"])
    out = {"n": n, "k": k}
    panels = {}
    for refine in ("0", "1"):
        os.environ["MLFF_WB_REFINE"] = refine
        with sgdml_amd.KernelSolver(n) as s:
            s.sgdml_operator(Rd, Rdd, np.arange(9)[None, :], 10.0)
            s.set_operator(-1.0, LAM)
            s.precon_pivchol(k)
            panels["device_" + ("refined" if refine == "1" else "onestep")] = s.precon_panel()
            r = s.pcg(y, tol=TOL, maxiter=20000)
            out["device_pcg_" + refine] = [int(r.iters), float(r.resid / np.linalg.norm(y))]
    os.environ["MLFF_WB_REFINE"] = "0"
    with sgdml_amd.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(9)[None, :], 10.0)
        s.set_operator(-1.0, LAM)
        s.precon_pivchol(k, build_woodbury=False)
        Lt = s.precon_panel()
        sv = np.linalg.svd(Lt, compute_uv=False)
        out["sigma2_max"], out["sigma2_min"] = float(sv[0] ** 2), float(sv[-1] ** 2)
        out["cond_A"] = float(np.sqrt((sv[0] ** 2 + LAM) / (sv[-1] ** 2 + LAM)))
        G = LAM * np.eye(k) + Lt @ Lt.T
        L2 = scipy.linalg.cholesky(G, lower=True)
        T0 = scipy.linalg.solve_triangular(L2, Lt, lower=True)
        Li = scipy.linalg.solve_triangular(L2, np.eye(k), lower=True)
        G2 = T0 @ T0.T + LAM * (Li @ Li.T)
        out["G2_minus_I_max"] = float(np.abs(G2 - np.eye(k)).max())
        C = scipy.linalg.cholesky(G2, lower=True)
        panels["lapack"] = T0
        panels["lapack_refined"] = scipy.linalg.solve_triangular(C, T0, lower=True)
        Q = np.linalg.qr(np.vstack([Lt.T, np.sqrt(LAM) * np.eye(k)]), mode="reduced")[0]
        panels["qr"] = np.ascontiguousarray(Q[:n].T)
        for name, T in panels.items():
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=4000,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            out[name] = [int(it), int(info)]
            print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
