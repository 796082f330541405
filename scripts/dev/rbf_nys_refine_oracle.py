"""configs[2] at N = 8192 on the CPU oracle: does re-orthogonalising the Nystrom panel (the second
CholeskyQR step the device applies to the Woodbury panel) move the oracle's count?
The GPU takes 2863 iterations with or without it (profiles/r04/nys_refine_ab/); the oracle's BLAS
order 2963.  Prints the oracle's counts with the plain and the refined panel (BLAS order).

    python scripts/dev/rbf_nys_refine_oracle.py      (CPU, ~10 min)
"""
import json
import sys
from pathlib import Path

import numpy as np
import scipy.linalg

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd"), str(REPO / "tests" / "golden")]

from make_rbf_band import ELL, K_RANK, LAM, TOL, problem  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.precon import cho_factor_stable  # noqa: E402
from oracle.rbf import rbf_kernel  # noqa: E402


def main(n=8192):
    X, b, idx = problem(n)
    K = rbf_kernel(X, ELL)
    S_nm = K[:, idx]
    U, lower = cho_factor_stable(S_nm[idx, :])
    C = scipy.linalg.solve_triangular(U, S_nm.T, lower=lower, trans="T").T
    inner = C.T @ C
    inner[np.diag_indices_from(inner)] += LAM
    lo = scipy.linalg.eigh(inner, eigvals_only=True, subset_by_index=[0, 0])[0]
    lam_eff = LAM + (1e-15 if lo <= 0 else -1e-15)
    V, lower = cho_factor_stable(inner)
    B = scipy.linalg.solve_triangular(V, C.T, lower=lower, trans="T")
    Vu = np.triu(V) if not lower else np.tril(V).T  # upper factor: V^T V = inner + shift
    Vi = scipy.linalg.solve_triangular(Vu, np.eye(K_RANK), lower=False)  # V^-1
    G2 = B @ B.T + lam_eff * (Vi.T @ Vi)  # Q1^T Q1, Q1 bottom = sqrt(lam') V^-1
    C2 = scipy.linalg.cholesky(G2, lower=True)
    B2 = scipy.linalg.solve_triangular(C2, B, lower=True)
    out = {"n": n, "G2_dev_from_I": float(np.abs(G2 - np.eye(K_RANK)).max())}
    for name, T in (("plain", B), ("refined", B2)):
        x, info, tr, it = cg_legacy(lambda v: K @ v + LAM * v, b, tol=TOL, maxiter=5 * n,
                                    psolve=lambda r, T=T: -((T.T @ (T @ r) - r) / LAM))
        out[name] = int(it)
        print(json.dumps({name: int(it)}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
