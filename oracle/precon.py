"""Low-rank preconditioners of the reference, restated in NumPy/SciPy.

TEST INFRASTRUCTURE (see oracle/__init__.py).

All functions work on S = sigma_K * K, the PSD matrix whose columns the
reference's pivoted Cholesky fetches (get_col of -K_op, iterative_cholesky.py:152-156)
and whose K_mm block it factors (`_cho_factor_stable(-K_mm)`, iterative_solver.py:218).
Preconditioner panels are returned "wide" (k x N) together with the sign
sigma_p of the apply z = sigma_p * lam^-1 * (r - T^T T r).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg


def pivoted_cholesky(get_col, diagonal, max_rank):
    """incomplete_cholesky.py:24-93.  Returns (L (N x k), index_columns (N,))."""
    diag = np.array(diagonal, dtype=np.float64, copy=True)
    n = diag.size
    index_columns = np.arange(n)
    L = np.zeros((n, max_rank))
    for m in range(max_rank):
        i_argmax = int(np.argmax(diag[index_columns][m:]) + m)           # :53
        index_columns[m], index_columns[i_argmax] = index_columns[i_argmax], index_columns[m]
        m_pi = index_columns[m]
        i_pi = index_columns[m + 1:]
        pivot_element = diag[m_pi]
        assert pivot_element > 0, "given matrix is not PSD"              # :62
        L[m_pi, m] = np.sqrt(pivot_element)
        k = get_col(m_pi)
        schur = 0
        if m > 0:
            schur = np.einsum("c, rc->r", L[m_pi, :m], L[i_pi, :m])      # :72
        L[i_pi, m] = (k[i_pi] - schur) / L[m_pi, m]                       # :75
        diag[i_pi] -= L[i_pi, m] ** 2                                     # :78
    return L, index_columns


def woodbury_panel(L, lam):
    """iterative_cholesky.py:141-148: T = chol(lam I + L^T L)^-1 L^T, apply (r - T^T T r)/lam."""
    k = L.shape[1]
    kernel = lam * np.eye(k) + (L.T @ L)
    L2 = scipy.linalg.cholesky(kernel, lower=True)
    T = scipy.linalg.solve_triangular(L2, L.T, lower=True)
    return T, 1.0


def cho_factor_stable(M):
    """iterative_solver.py:576-583 (the code after :583 is unreachable)."""
    M = np.array(M, dtype=np.float64, copy=True)
    lo_eig = scipy.linalg.eigh(M, eigvals_only=True, subset_by_index=[0, 0])
    sgn = 1 if lo_eig <= 0 else -1
    M[np.diag_indices_from(M)] += sgn * 1.0e-15
    return scipy.linalg.cho_factor(M, overwrite_a=False, check_finite=False)


def nystrom_panel(S_nm, idx, lam, variant=0):
    """Nystrom preconditioner panel from the column panel S[:, idx] (N x k).

    variant 0: Iterative._init_precon_operator (iterative_solver.py:112-322):
      U = chol_stable(S_mm); C = S_nm U^-1; V = chol_stable(C^T C + lam I);
      B = V^-T C^T; apply (B^T B v - v)/lam  -> sigma_p = -1.
    variant 1: _init_precon_operator_sb (iterative_solver.py:343-381):
      L_m = chol(S_mm + 1e-16 I); Kb = S_nm L_m^-T; L_in = chol(lam I + Kb^T Kb);
      P = L_in^-1 Kb^T; apply -(v - P^T P v)/lam -> sigma_p = -1.
    """
    S_nm = np.array(S_nm, dtype=np.float64, copy=True)
    k = S_nm.shape[1]
    S_mm = S_nm[idx, :]
    if variant == 0:
        U, lower = cho_factor_stable(S_mm)
        C = scipy.linalg.solve_triangular(U, S_nm.T, lower=lower, trans="T").T
        inner = C.T.dot(C)
        inner[np.diag_indices_from(inner)] += lam
        V, lower = cho_factor_stable(inner)
        B = scipy.linalg.solve_triangular(V, C.T, lower=lower, trans="T")
        return B, -1.0
    L_m = scipy.linalg.cholesky(S_mm + 1e-16 * np.eye(k), lower=True)
    Kbar = scipy.linalg.solve_triangular(L_m, S_nm.T, lower=True).T
    inner = lam * np.eye(k) + Kbar.T @ Kbar
    L_in = scipy.linalg.cholesky(inner, lower=True)
    P = scipy.linalg.solve_triangular(L_in, Kbar.T, lower=True)
    return P, -1.0


def apply_panel(T, sigma_p, lam, r):
    """z = sigma_p * lam^-1 * (r - T^T (T r))."""
    lam_inv = 1.0 / lam
    return sigma_p * (lam_inv * (r - T.T @ (T @ r)))


def lev_scores(S_nm, idx, lam):
    """Numeric part of _lev_scores (iterative_solver.py:489-552)."""
    S_nm = np.array(S_nm, dtype=np.float64, copy=True)
    S_mm = S_nm[idx, :]
    L, lower = cho_factor_stable(S_mm)
    B = scipy.linalg.solve_triangular(L, S_nm.T, lower=lower, trans="T")
    B_BT_lam = B.dot(B.T)
    B_BT_lam[np.diag_indices_from(B_BT_lam)] += lam
    C, C_lower = cho_factor_stable(B_BT_lam)
    C_B = scipy.linalg.solve_triangular(C, B, lower=C_lower, trans="T")
    return np.einsum("i...,i...->...", C_B, C_B)


def svd_panel(S, k, lam):
    """svd_preconditioner (iterative_solver.py:1297-1329): L = U sqrt(s)[:, :k], Woodbury."""
    U, s, _ = scipy.linalg.svd(S)
    L = (U * np.sqrt(s))[:, :k]
    return woodbury_panel(L, lam)


def rank_k_lev_scores(S, k):
    """_rank_k_leverage_scores (iterative_solver.py:1110-1175): ||U_k row|| (not squared)."""
    U, _, _ = scipy.linalg.svd(S)
    return np.linalg.norm(U[:, :k], axis=1)
