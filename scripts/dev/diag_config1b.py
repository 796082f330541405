"""configs[1] full size: is the PCG count's dependence on the Woodbury panel a property of the
reference's formula (chaos under rounding) or of the device's build?

    python scripts/dev/diag_config1b.py        (GPU box; tests/golden/nanotube_n15540.npz)

diag_config1.py found: the device L (pivot values within 3e-13 of the oracle's), its panel
T = chol(lam I + L^T L)^-1 L^T built on the host with LAPACK -> 364-365 iterations of the host-
driven scipy-1.7.3 recurrence (GPU operator), built on the device -> 571, although the two panels
differ by 5e-15 relative.  Here, from the same device L, host-built panels that follow the
device's algorithm and other rounding patterns:
* blocked: right-looking blocked Cholesky (64-column blocks: LAPACK on the diagonal block,
  triangular panel solve, GEMM trailing update) and blocked forward substitution (64-row bands,
  GEMM band update) -- the device's potrf_lower / trsm_lower_wide schedule, BLAS sums inside;
* blocked32 / blocked128: the same with 32 / 128-wide blocks;
* noise s: the LAPACK panel with independent Gaussian relative perturbations of size s per entry.
Every panel: the count of the host-driven recurrence, ||T - T_lapack|| / ||T_lapack||, and the
smallest eigenvalue of the preconditioned operator's Woodbury factor I - T^T T restricted to
range(L) relative to its exact value lam / (sigma^2 + lam) (from the SVD of L).
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


def blocked_cholesky(A, nb):
    A = np.array(A, copy=True)
    k = A.shape[0]
    for j0 in range(0, k, nb):
        j1 = min(j0 + nb, k)
        A[j0:j1, j0:j1] = scipy.linalg.cholesky(A[j0:j1, j0:j1], lower=True)
        if j1 < k:
            Ld = A[j0:j1, j0:j1]
            A[j1:, j0:j1] = scipy.linalg.solve_triangular(Ld, A[j1:, j0:j1].T, lower=True).T
            P = A[j1:, j0:j1]
            A[j1:, j1:] -= P @ P.T
    return np.tril(A)


def blocked_trsm(L, W, nb):
    W = np.array(W, copy=True)
    k = L.shape[0]
    for i0 in range(0, k, nb):
        i1 = min(i0 + nb, k)
        if i0 > 0:
            W[i0:i1] -= L[i0:i1, :i0] @ W[:i0]
        W[i0:i1] = scipy.linalg.solve_triangular(L[i0:i1, i0:i1], W[i0:i1], lower=True)
    return W


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
        # singular values of L: the directions where r - T^T T r cancels to lam / (sigma^2 + lam)
        sig2 = np.linalg.eigvalsh(G - LAM * np.eye(k))
        out["sigma2_max"] = float(sig2[-1])
        out["sigma2_min"] = float(sig2[0])
        out["sigma2_above_1e2"] = int((sig2 > 1e2).sum())
        out["sigma2_above_1e4"] = int((sig2 > 1e4).sum())
        L2 = scipy.linalg.cholesky(G, lower=True)
        T0 = scipy.linalg.solve_triangular(L2, Lt, lower=True)
        U, sv, _ = np.linalg.svd(Lt.T, full_matrices=False)  # n x k, range(L)
        panels = {"lapack": T0}
        for nb in (64, 32, 128):
            Lb = blocked_cholesky(G, nb)
            panels[f"blocked{nb}"] = blocked_trsm(Lb, Lt, nb)
        rng = np.random.default_rng(7)
        for sc in (2e-15, 5e-15, 2e-14):
            panels[f"noise{sc:g}"] = T0 * (1.0 + sc * rng.standard_normal(T0.shape))
        s.precon_lowrank(Lt)
        panels["device"] = s.precon_panel()
        for name, T in panels.items():
            t0 = time.time()
            x, info, tr, it = cg_legacy(s.matvec, y, tol=TOL, maxiter=5 * n,
                                        psolve=lambda v, T=T: (v - T.T @ (T @ v)) / LAM)
            TU = T @ U
            ev = np.linalg.eigvalsh(np.eye(k) - TU.T @ TU)  # I - T^T T on range(L), basis U
            exact = LAM / (sv ** 2 + LAM)
            out[name] = {"iters": int(it), "info": int(info),
                         "panel_rel_diff": float(np.linalg.norm(T - T0) / np.linalg.norm(T0)),
                         "woodbury_eig_min": float(ev[0]), "exact_eig_min": float(exact.min()),
                         "woodbury_eigs_negative": int((ev < 0).sum()),
                         "rel_dalpha": float(np.linalg.norm(-x - f["alphas"]) /
                                             np.linalg.norm(f["alphas"])),
                         "s": time.time() - t0}
            print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
