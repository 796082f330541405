"""configs[1] full size, continued (diag_config1b.py: LAPACK-built Woodbury panels of the device
L give 364-366 iterations, the same panels with independent per-entry relative noise of 2e-15
give 555-577, the device-built panel 571).  Which rounding pattern keeps the count at 365?

    python scripts/dev/diag_config1c.py        (GPU box; tests/golden/nanotube_n15540.npz)

Panels T = L2^-1 L^T (L2 = chol(lam I + L^T L)) from the device L, each solved by the host-driven
scipy-1.7.3 recurrence with the device operator:
* rowspace noise s: T_lapack + s (E T_lapack), E a k x k Gaussian matrix: the error stays in the
  row space of L^T (a k x k mixing, as a perturbed L2 gives);
* colwise noise s: T_lapack + s |T| G, G an N x k ... per-entry Gaussian (diag_config1b: 555);
* inverse: T = inv(L2) @ L^T (explicit triangular inverse, one GEMM: rounding of the k x k inverse
  then a GEMM);
* fsub_div / fsub_mul: blocked forward substitution (64-row bands, GEMM band updates), the rows of a
  band solved one at a time dividing by the diagonal / multiplying by its reciprocal;
* potrf_div: the device's potrf_lower schedule (64-column blocks, divisions) with LAPACK's TRSM.
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np
import scipy.linalg

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

import sgdml_amd  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.sgdml import descriptors  # noqa: E402

N_ATOMS, SIG, LAM, TOL = 370, 10.0, 1e-10, 1e-6
QR_ONLY = "--qr" in sys.argv


def fsub(L2, W, nb, mode):
    W = np.array(W, copy=True)
    k = L2.shape[0]
    for i0 in range(0, k, nb):
        i1 = min(i0 + nb, k)
        if i0 > 0:
            W[i0:i1] -= L2[i0:i1, :i0] @ W[:i0]
        for r in range(i0, i1):
            v = W[r] - L2[r, i0:r] @ W[i0:r] if r > i0 else W[r]
            W[r] = v / L2[r, r] if mode == "div" else v * (1.0 / L2[r, r])
    return W


def potrf_div(A, nb=64):
    """potrf_lower's schedule: unblocked column Cholesky of each 64-block dividing by the
    pivot, panel solve by division, GEMM trailing update."""
    A = np.array(A, copy=True)
    k = A.shape[0]
    for j0 in range(0, k, nb):
        j1 = min(j0 + nb, k)
        B = A[j0:j1, j0:j1]
        for c in range(j1 - j0):
            B[c, c] = np.sqrt(B[c, c])
            B[c + 1:, c] = B[c + 1:, c] / B[c, c]
            B[c + 1:, c + 1:] -= np.outer(B[c + 1:, c], B[c + 1:, c])
        if j1 < k:
            P = A[j1:, j0:j1]
            Ld = np.tril(B)
            for c in range(j1 - j0):
                P[:, c] = (P[:, c] - P[:, :c] @ Ld[c, :c]) / Ld[c, c]
            A[j1:, j1:] -= P @ P.T
    return np.tril(A)


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
        G = LAM * np.eye(k) + Lt @ Lt.T
        L2 = scipy.linalg.cholesky(G, lower=True)
        T0 = scipy.linalg.solve_triangular(L2, Lt, lower=True)
        rng = np.random.default_rng(11)
        panels = {"lapack": T0}
        for sc in (2e-15, 1e-14):
            E = rng.standard_normal((k, k)) / np.sqrt(k)
            panels[f"rowspace_noise{sc:g}"] = T0 + sc * (E @ T0)
        panels["colwise_noise2e-15"] = T0 * (1.0 + 2e-15 * rng.standard_normal(T0.shape))
        if QR_ONLY:
            panels = {"lapack": T0}
        # T without the Gram matrix: [L; sqrt(lam) I] = Q R gives R^T R = lam I + L^T L, so
        # T = R^-T L^T = Q[:n]^T (Householder QR: no squared condition number)
        Q = np.linalg.qr(np.vstack([Lt.T, np.sqrt(LAM) * np.eye(k)]), mode="reduced")[0]
        panels["qr"] = np.ascontiguousarray(Q[:n].T)
        del Q
        Linv = scipy.linalg.solve_triangular(L2, np.eye(k), lower=True)
        panels["inverse"] = np.tril(Linv) @ Lt
        t0 = time.time()
        if QR_ONLY:
            panels = {k_: v_ for k_, v_ in panels.items() if k_ in ("lapack", "qr", "inverse")}
            s.precon_lowrank(Lt)
            panels["device"] = s.precon_panel()
            return solve_all(s, panels, y, f, Lt, T0, out, n)
        panels["fsub_div"] = fsub(L2, Lt, 64, "div")
        panels["fsub_mul"] = fsub(L2, Lt, 64, "mul")
        out["fsub_s"] = time.time() - t0
        t0 = time.time()
        L2d = potrf_div(G)
        out["potrf_div_s"] = time.time() - t0
        out["potrf_div_rel_diff"] = float(np.linalg.norm(L2d - L2) / np.linalg.norm(L2))
        panels["potrf_div"] = scipy.linalg.solve_triangular(L2d, Lt, lower=True)
        panels["potrf_div+fsub_div"] = fsub(L2d, Lt, 64, "div")
        s.precon_lowrank(Lt)
        panels["device"] = s.precon_panel()
        return solve_all(s, panels, y, f, Lt, T0, out, n)


def solve_all(s, panels, y, f, Lt, T0, out, n):
    if True:
        for name, T in panels.items():
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=5 * n,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            # the part of T outside the row space of L^T (least squares T ~ C L^T)
            out[name] = {"iters": int(it), "info": int(info),
                         "panel_rel_diff": float(np.linalg.norm(T - T0) / np.linalg.norm(T0)),
                         "rel_dalpha": float(np.linalg.norm(-x - f["alphas"]) /
                                             np.linalg.norm(f["alphas"]))}
            print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
