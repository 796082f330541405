"""sGDML descriptors and dense Matern-5/2 Hessian kernel, restated in NumPy.

TEST INFRASTRUCTURE (see oracle/__init__.py).
"""
from __future__ import annotations

import numpy as np


def descriptors(R):
    """Desc.from_R without cutoff / PBC (desc.py:80-234, 292-358).
    R: M x n x 3  ->  R_desc (M x D) = 1/r_ab, R_d_desc (M x D x 3) = (r_a - r_b)/r_ab^3,
    pairs (a, b) in np.tril_indices(n, -1) order."""
    R = np.asarray(R, dtype=np.float64)
    M, n, _ = R.shape
    a, b = np.tril_indices(n, k=-1)
    pdiff = R[:, a, :] - R[:, b, :]
    pdist = np.sqrt(np.sum(pdiff ** 2, axis=2))
    return 1.0 / pdist, pdiff / (pdist ** 3)[:, :, None]


def desc_perm(perm):
    """Desc.perm (desc.py:360-389): atom permutation -> descriptor permutation."""
    n = len(perm)
    rest = np.zeros((n, n))
    rest[np.tril_indices(n, -1)] = list(range((n ** 2 - n) // 2))
    rest = rest + rest.T
    rest = rest[perm, :]
    rest = rest[:, perm]
    return rest[np.tril_indices(n, -1)].astype(int)


def tril_perms_lin(perms):
    """train.py:783-790."""
    perms = np.atleast_2d(perms)
    n_perms, n = perms.shape
    D = n * (n - 1) // 2
    tril_perms = np.array([desc_perm(p) for p in perms])
    perm_offsets = np.arange(n_perms)[:, None] * D
    return (tril_perms + perm_offsets).flatten("F")


def d_desc_from_comp(R_d_desc, n):
    """desc.py:444-462: compact (D x 3) Jacobian -> full (D x 3n)."""
    D = R_d_desc.shape[0]
    i, j = np.tril_indices(n, k=-1)
    out = np.zeros((D, n, 3))
    out[np.arange(D), j, :] = R_d_desc
    out[np.arange(D), i, :] = -R_d_desc
    return out.reshape(D, 3 * n)


def assemble_kernel(R_desc, R_d_desc, tril_perms_lin_, sig, use_E_cstr=False):
    """GDMLTrain._assemble_kernel_mat with col_idxs = all (train.py:81-236, 1121-1308).
    use_E_cstr: M energy rows / columns appended (train.py:212-236, 1205-1208), filled by
    column worker j for every row point i in increasing j (the order a one-process Pool
    runs the workers in, so for a non-group permutation set the E-E entry (a, b) holds
    the value of worker max(a, b))."""
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    dim_i = 3 * n
    n_perms = int(len(tril_perms_lin_) / D)
    nE = M if use_E_cstr else 0
    K = np.empty((M * dim_i + nE, M * dim_i + nE))
    mat52_base_div = 3 * sig ** 4
    sqrt5 = np.sqrt(5.0)
    sig_pow2 = sig ** 2
    J = [d_desc_from_comp(R_d_desc[m], n) for m in range(M)]
    for j in range(M):
        rj_desc_perms = np.reshape(np.tile(R_desc[j, :], n_perms)[tril_perms_lin_],
                                   (n_perms, -1), order="F")
        rj_d_desc_perms = np.reshape(np.tile(J[j].T, n_perms)[:, tril_perms_lin_],
                                     (-1, D, n_perms))
        for i in range(j, M):
            diff = R_desc[i, :] - rj_desc_perms
            norm = sqrt5 * np.linalg.norm(diff, axis=1)
            mat52 = np.exp(-norm / sig) / mat52_base_div * 5
            O = np.einsum("ki,kj->ij", diff * mat52[:, None] * 5,
                          np.einsum("ki,jik -> kj", diff, rj_d_desc_perms))
            O -= np.einsum("ikj,j->ki", rj_d_desc_perms, (sig_pow2 + sig * norm) * mat52)
            blk = J[i].T.dot(O)
            K[i * dim_i:(i + 1) * dim_i, j * dim_i:(j + 1) * dim_i] = blk
            K[j * dim_i:(j + 1) * dim_i, i * dim_i:(i + 1) * dim_i] = blk.T
        if use_E_cstr:
            e0 = M * dim_i
            for i in range(M):
                diff = R_desc[i, :] - rj_desc_perms
                norm = sqrt5 * np.linalg.norm(diff, axis=1)
                kfe = 5 * diff / (3 * sig ** 3) * (norm[:, None] + sig) * np.exp(-norm / sig)[:, None]
                kfe = -np.einsum("ik,jki -> j", kfe, rj_d_desc_perms)
                K[j * dim_i:(j + 1) * dim_i, e0 + i] = kfe
                K[e0 + i, j * dim_i:(j + 1) * dim_i] = kfe
                K[e0 + i, e0 + j] = K[e0 + j, e0 + i] = -(
                    1 + (norm / sig) * (1 + norm / (3 * sig))).dot(np.exp(-norm / sig))
    return K


def kernel_matvec_matrix_free(R_desc, R_d_desc, perms, sig, x, use_E_cstr=False):
    """K x without forming K, as the reference's CG operator evaluates it: the
    force prediction of GDMLPredict with alphas = x (predict.py:72-234, set_alphas
    :400-445, Desc.d_desc_dot_vec / vec_dot_d_desc desc.py:464-508) for every
    training point i as the query:
        z_j      = J_j x_j                              (D)
        diff_ijp = Rd_i - Rd_j[P_p]                     (D), norm = sqrt5 |diff|
        F_i      = sum_jp 5 m (diff . z_j[P_p]) diff - w z_j[P_p]
        y_i      = J_i^T F_i
    with m = exp(-norm/sig) 5/(3 sig^4), w = (sig^2 + sig norm) m.  For a
    permutation group this equals the assembled K @ x; for other permutation sets
    it is the reference's K_op (not its mirrored assembly).
    use_E_cstr: x = [x_F (3 n M); x_E (M)] (iterative_solver.py:423-440, predict.py:206-218):
        F_i     += sum_jp x_E[j] w diff
        out_E_i  = -(sum_jp a_ijp w + sum_jp K_ee x_E[j]),
        K_ee     = (1 + norm/sig (1 + norm/(3 sig))) exp(-norm/sig)."""
    R_desc = np.asarray(R_desc, dtype=np.float64)
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    perms = np.atleast_2d(perms)
    P = np.array([desc_perm(p) for p in perms])  # n_perms x D descriptor maps
    s_at, t_at = np.tril_indices(n, k=-1)          # pair d = (s, t), s > t
    x = np.asarray(x, dtype=np.float64)
    xE = x[3 * n * M:] if use_E_cstr else None
    X = x[:3 * n * M].reshape(M, n, 3)
    outE = np.empty(M)
    z = np.einsum("mdc,mdc->md", R_d_desc, X[:, t_at, :] - X[:, s_at, :])
    Rt = R_desc[:, P]                               # M x n_perms x D: Rd_j[P_p d]
    Zt = z[:, P]
    sqrt5 = np.sqrt(5.0)
    y = np.empty((M, n, 3))
    for i in range(M):
        diff = R_desc[i][None, None, :] - Rt        # M x n_perms x D
        norm = sqrt5 * np.linalg.norm(diff, axis=2)
        m = np.exp(-norm / sig) * 5.0 / (3.0 * sig ** 4)
        w = (sig ** 2 + sig * norm) * m
        a = np.einsum("jpd,jpd->jp", diff, Zt)
        F = np.einsum("jp,jpd->d", 5.0 * m * a, diff) - np.einsum("jp,jpd->d", w, Zt)
        if use_E_cstr:
            F = F + np.einsum("jp,jpd->d", xE[:, None] * w, diff)
            kee = (1 + (norm / sig) * (1 + norm / (3 * sig))) * np.exp(-norm / sig)
            outE[i] = -(np.sum(a * w) + np.sum(kee * xE[:, None]))
        # y_i = J_i^T F: atom t gets +Rdd F, atom s gets -Rdd F
        contrib = R_d_desc[i] * F[:, None]
        yi = np.zeros((n, 3))
        np.add.at(yi, t_at, contrib)
        np.add.at(yi, s_at, -contrib)
        y[i] = yi
    return np.concatenate([y.reshape(-1), outE]) if use_E_cstr else y.reshape(-1)


def kernel_column_matrix_free(R_desc, R_d_desc, perms, sig, g):
    """K e_g of kernel_matvec_matrix_free (the reference's get_col through K_op,
    iterative_cholesky.py:152-156 with predict.py:72-234) from the one training point it touches:
    e_g (g = j 3n + 3a + c) makes z_j = J_j e_(a,c) the only non-zero z, so
        F_i = sum_p 5 m_ijp (diff_ijp . z_j[P_p]) diff_ijp - w_ijp z_j[P_p],   y_i = J_i^T F_i
    -- O(M n_perms D) instead of a full operator application (O(M^2 n_perms D)); the same products,
    the zero terms of the other training points left out, so the column equals K_op e_g to the
    rounding of its sums (<= 3e-16 of its largest entry,
    tests/test_oracle_golden.py::test_column_restatement_matches_operator)."""
    R_desc = np.asarray(R_desc, dtype=np.float64)
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    perms = np.atleast_2d(perms)
    P = np.array([desc_perm(p) for p in perms])
    s_at, t_at = np.tril_indices(n, k=-1)
    j, a, c = g // (3 * n), (g % (3 * n)) // 3, g % 3
    X = np.zeros((n, 3))
    X[a, c] = 1.0
    z = np.einsum("dc,dc->d", R_d_desc[j], X[t_at, :] - X[s_at, :])   # J_j e_(a,c)
    Rt = R_desc[j][P][None]                         # 1 x n_perms x D
    Zt = z[P][None]
    sqrt5 = np.sqrt(5.0)
    y = np.empty((M, n, 3))
    for i in range(M):
        diff = R_desc[i][None, None, :] - Rt
        norm = sqrt5 * np.linalg.norm(diff, axis=2)
        m = np.exp(-norm / sig) * 5.0 / (3.0 * sig ** 4)
        w = (sig ** 2 + sig * norm) * m
        aa = np.einsum("jpd,jpd->jp", diff, Zt)
        F = np.einsum("jp,jpd->d", 5.0 * m * aa, diff) - np.einsum("jp,jpd->d", w, Zt)
        contrib = R_d_desc[i] * F[:, None]
        yi = np.zeros((n, 3))
        np.add.at(yi, t_at, contrib)
        np.add.at(yi, s_at, -contrib)
        y[i] = yi
    return y.reshape(-1)


def pair_records(R_desc, R_d_desc, perms, sig):
    """The x-independent per-(i, j, p) quantities of the operator above, as the GPU keeps
    them (kernels_gen.hip k_sgdml_uv, mirror = 0): u = J_i^T diff (query point side),
    v = J_j^T P_p^T diff (training point side, 3n each), 5 m and w.
    Returns U, V (M x M x n_perms x 3n), m5, w (M x M x n_perms)."""
    R_desc = np.asarray(R_desc, dtype=np.float64)
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    P = np.array([desc_perm(p) for p in np.atleast_2d(perms)])
    npm = P.shape[0]
    J = [d_desc_from_comp(R_d_desc[m], n) for m in range(M)]  # D x 3n
    sqrt5 = np.sqrt(5.0)
    U = np.empty((M, M, npm, 3 * n))
    V = np.empty((M, M, npm, 3 * n))
    m5 = np.empty((M, M, npm))
    w = np.empty((M, M, npm))
    for i in range(M):
        for j in range(M):
            for p in range(npm):
                diff = R_desc[i] - R_desc[j][P[p]]
                norm = sqrt5 * np.linalg.norm(diff)
                m = np.exp(-norm / sig) * 5.0 / (3.0 * sig ** 4)
                m5[i, j, p], w[i, j, p] = 5.0 * m, (sig ** 2 + sig * norm) * m
                U[i, j, p] = J[i].T @ diff
                dp = np.empty(D)
                dp[P[p]] = diff               # P_p^T diff
                V[i, j, p] = J[j].T @ dp
    return U, V, m5, w


def kernel_matvec_factored(R_desc, R_d_desc, perms, sig, x, records=None):
    """The operator above regrouped as the GPU's record-factored form evaluates it
    (kernels_mf.hip k_rec_g / k_rec_fin):
        c_ijp = 5 m (v_ijp . x_j)          (= 5 m (diff . z_j[P_p]))
        G_i   = sum_jp w_ijp z_j[P_p]
        y_i   = sum_jp c_ijp u_ijp - J_i^T G_i      (= J_i^T F_i)
    Same products as kernel_matvec_matrix_free, other grouping."""
    R_desc = np.asarray(R_desc, dtype=np.float64)
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    P = np.array([desc_perm(p) for p in np.atleast_2d(perms)])
    U, V, m5, w = records if records is not None else pair_records(R_desc, R_d_desc, perms, sig)
    s_at, t_at = np.tril_indices(n, k=-1)
    X = np.asarray(x, dtype=np.float64).reshape(M, n, 3)
    z = np.einsum("mdc,mdc->md", R_d_desc, X[:, t_at, :] - X[:, s_at, :])
    Zt = z[:, P]                                    # M x n_perms x D
    y = np.empty((M, 3 * n))
    for i in range(M):
        c = m5[i] * np.einsum("jpa,ja->jp", V[i], X.reshape(M, 3 * n))
        G = np.einsum("jp,jpd->d", w[i], Zt)
        contrib = R_d_desc[i] * G[:, None]
        jtg = np.zeros((n, 3))
        np.add.at(jtg, t_at, contrib)
        np.add.at(jtg, s_at, -contrib)
        y[i] = np.einsum("jp,jpa->a", c, U[i]) - jtg.reshape(-1)
    return y.reshape(-1)


def kernel_diag(R_desc, R_d_desc, perms, sig, use_E_cstr=False):
    """diag(K) of the assembled sGDML kernel, one diagonal block K[i, i] per training point
    (IterativeCholesky._assemble_kernel_mat_diag, iterative_cholesky.py:241-373, which
    returns -diag for the PSD operator -K).  The block is
        K_ii = J_i^T (5 sum_p m_p diff_p (diff_p . J_i[P_p]) - sum_p w_p J_i[P_p]),
    diff_p = Rd_i - Rd_i[P_p].  For a single identity permutation diff = 0 and
    diag_(a,c) = -(5 / (3 sig^2)) sum_{b != a} Rdd_i[pair(a, b), c]^2, evaluated without
    forming the D x 3n Jacobian (the nanotube's is 68265 x 1110).
    use_E_cstr: the M energy entries K[E_i, E_i] = -sum_p K_ee(|Rd_i - Rd_i[P_p]|) of
    train.py:232-234 appended."""
    R_desc = np.asarray(R_desc, dtype=np.float64)
    R_d_desc = np.asarray(R_d_desc, dtype=np.float64)
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    perms = np.atleast_2d(perms)
    if use_E_cstr:
        P = np.array([desc_perm(p) for p in perms])
        norm = np.sqrt(5.0) * np.linalg.norm(R_desc[:, None, :] - R_desc[:, P], axis=2)  # M x n_perms
        kee = ((1 + (norm / sig) * (1 + norm / (3 * sig))) * np.exp(-norm / sig)).sum(axis=1)
        return np.concatenate([kernel_diag(R_desc, R_d_desc, perms, sig), -kee])
    s_at, t_at = np.tril_indices(n, k=-1)
    out = np.empty((M, n, 3))
    if perms.shape[0] == 1 and np.array_equal(perms[0], np.arange(n)):
        for i in range(M):
            sq = R_d_desc[i] ** 2                       # D x 3, each pair feeds both atoms
            acc = np.zeros((n, 3))
            np.add.at(acc, t_at, sq)
            np.add.at(acc, s_at, sq)
            out[i] = -(5.0 / (3.0 * sig ** 2)) * acc
        return out.reshape(-1)
    P = np.array([desc_perm(p) for p in perms])
    sqrt5 = np.sqrt(5.0)
    for i in range(M):
        J = d_desc_from_comp(R_d_desc[i], n)            # D x 3n
        diff = R_desc[i][None, :] - R_desc[i][P]        # n_perms x D
        norm = sqrt5 * np.linalg.norm(diff, axis=1)
        m = np.exp(-norm / sig) * 5.0 / (3.0 * sig ** 4)
        w = (sig ** 2 + sig * norm) * m
        O = np.zeros((D, 3 * n))
        for p in range(P.shape[0]):
            Jp = J[P[p]]                                # rows permuted: J_i[P_p]
            O += 5.0 * m[p] * np.outer(diff[p], diff[p] @ Jp) - w[p] * Jp
        out[i] = np.einsum("dk,dk->k", J, O).reshape(n, 3)
    return out.reshape(-1)


def energies_matrix_free(R_desc, R_d_desc, perms, sig, alphas):
    """Training-set energies of the model with coefficients alphas, E_F[0] of
    GDMLPredict's _predict_wkr (predict.py:172-220) before the std scale and the
    integration constant: E_i = sum_jp a_ijp (sig + norm) exp(-norm/sig) 5/(3 sig^3),
    a_ijp = (Rd_i - Rd_j[P_p]) . (J_j alpha_j)[P_p], norm = sqrt5 |Rd_i - Rd_j[P_p]|."""
    R_desc = np.asarray(R_desc, dtype=np.float64)
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    perms = np.atleast_2d(perms)
    P = np.array([desc_perm(p) for p in perms])
    s_at, t_at = np.tril_indices(n, k=-1)
    A = np.asarray(alphas, dtype=np.float64).reshape(M, n, 3)
    z = np.einsum("mdc,mdc->md", R_d_desc, A[:, t_at, :] - A[:, s_at, :])
    Rt, Zt = R_desc[:, P], z[:, P]
    E = np.empty(M)
    for i in range(M):
        diff = R_desc[i][None, None, :] - Rt
        norm = np.sqrt(5.0) * np.linalg.norm(diff, axis=2)
        base = np.exp(-norm / sig) * 5.0 / (3.0 * sig ** 3) * (norm + sig)
        a = np.einsum("jpd,jpd->jp", diff, Zt)
        E[i] = np.sum(a * base)
    return E
