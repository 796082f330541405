"""Where the device's Woodbury-panel solve parts from the oracle on the energy-consistent ethanol
system (N = 15741, M = 583, k = 1264; tests/golden/make_ethanol_full.py): the CPU oracle takes
~1350 iterations to 1e-6 with the reference's one-step LAPACK panel and ~770 with accurately
evaluated panels (Householder QR / two CholeskyQR steps), the device 1343 (one-step panel) and
878 (refined panel, its default).  Panel or apply?

    python scripts/dev/diag_ethanol_harmonic.py       (GPU box)

Host-driven scipy-1.7.3 recurrence with the DEVICE operator (s.matvec) and a HOST apply
(T^T (T r) by BLAS) of: the device one-step / refined panels, the LAPACK one-step / refined
panels and a Householder-QR panel of the device L; plus the device solves (device apply) and the
error of one device apply against the same panel's apply in extended precision.
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
from oracle.sgdml import descriptors  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402

LAM, TOL = 1e-10, 1e-6


def ld_apply(T, r):
    Tl = T.astype(np.longdouble)
    rl = r.astype(np.longdouble)
    return ((rl - Tl.T @ (Tl @ rl)) / LAM).astype(np.float64)


def gemm_bias():
    """Signed rounding error of the device fp64 GEMM (MFMA path and VALU path) against the exact
    product (np.longdouble, then fp64): a round-to-nearest sum has mean signed error ~0 ulp; a
    truncating or otherwise biased accumulation does not."""
    import ctypes

    from sgdml_amd import _native as nat

    rng = np.random.default_rng(5)
    res = {}
    for name, (M_, N_, K_) in {"mfma": (256, 256, 512), "valu": (32, 64, 16)}.items():
        A = rng.uniform(0.5, 1.0, (M_, K_))
        B = rng.uniform(0.5, 1.0, (K_, N_))
        C = np.zeros((M_, N_))
        with sgdml_amd.KernelSolver(64) as s:
            nat.check(nat.load_library().mlff_test_gemm(
                s._ctx, 0, 0, M_, N_, K_, 1.0, nat.dptr(A), K_, nat.dptr(B), N_, 0.0, nat.dptr(C),
                N_, 1), s._ctx, "mlff_test_gemm")
        ex = (A.astype(np.longdouble) @ B.astype(np.longdouble))
        err = ((C - ex) / np.spacing(ex.astype(np.float64))).astype(np.float64)
        host = ((A @ B - ex) / np.spacing(ex.astype(np.float64))).astype(np.float64)
        res[name] = {"mean_ulp": float(err.mean()), "rms_ulp": float(np.sqrt((err ** 2).mean())),
                     "host_blas_mean_ulp": float(host.mean()),
                     "host_blas_rms_ulp": float(np.sqrt((host ** 2).mean()))}
    return res


def main(M=583, k=int(os.environ.get("DIAG_K", "1264"))):
    ds = synthetic.ethanol_harmonic(M, seed=0)
    y, _ = synthetic.labels(ds["F"])
    n = y.size
    Rd, Rdd = descriptors(ds["R"])
    out = {"n": n, "k": k}
    try:
        out["gemm_bias"] = gemm_bias()
        print(json.dumps(out["gemm_bias"]), flush=True)
    except Exception as e:  # noqa: BLE001
        print("gemm_bias failed:", repr(e), flush=True)
    panels = {}
    rng = np.random.default_rng(3)
    rtest = rng.standard_normal(n)
    for refine in ("0", "1", "2"):
        os.environ["MLFF_WB_REFINE"] = refine
        with sgdml_amd.KernelSolver(n) as s:
            s.sgdml_operator(Rd, Rdd, np.arange(9)[None, :], 10.0)
            s.set_operator(-1.0, LAM)
            s.precon_pivchol(k)
            name = "device_" + {"0": "onestep", "1": "refined", "2": "refined2"}[refine]
            T = s.precon_panel()
            panels[name] = T
            zd = s.precon_apply(rtest)
            zl = ld_apply(T, rtest)
            zh = (rtest - T.T @ (T @ rtest)) / LAM
            out[name + "_apply_err"] = {"device": float(np.linalg.norm(zd - zl) / np.linalg.norm(zl)),
                                        "host_blas": float(np.linalg.norm(zh - zl) / np.linalg.norm(zl))}
            r = s.pcg(y, tol=TOL, maxiter=20000)
            out[name + "_device_pcg"] = int(r.iters)
            print(json.dumps({k_: out[k_] for k_ in out if k_.startswith(name)}), flush=True)
    os.environ["MLFF_WB_REFINE"] = "0"
    with sgdml_amd.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(9)[None, :], 10.0)
        s.set_operator(-1.0, LAM)
        s.precon_pivchol(k, build_woodbury=False)
        Lt = s.precon_panel()
        G = LAM * np.eye(k) + Lt @ Lt.T
        L2 = scipy.linalg.cholesky(G, lower=True)
        T0 = scipy.linalg.solve_triangular(L2, Lt, lower=True)
        Li = scipy.linalg.solve_triangular(L2, np.eye(k), lower=True)
        C = scipy.linalg.cholesky(T0 @ T0.T + LAM * (Li @ Li.T), lower=True)
        panels["lapack"] = T0
        panels["lapack_refined"] = scipy.linalg.solve_triangular(C, T0, lower=True)
        Q = np.linalg.qr(np.vstack([Lt.T, np.sqrt(LAM) * np.eye(k)]), mode="reduced")[0]
        panels["qr"] = np.ascontiguousarray(Q[:n].T)
        ref = panels["qr"]
        for name, T in panels.items():
            # distance of the projector T^T T from the QR one on a random vector
            out[name + "_proj_dist"] = float(np.linalg.norm(T.T @ (T @ rtest) - ref.T @ (ref @ rtest))
                                             / np.linalg.norm(rtest))
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=4000,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            out[name + "_host_apply"] = [int(it), int(info)]
            print(json.dumps({name: out[name + "_host_apply"], "proj_dist": out[name + "_proj_dist"]}),
                  flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
