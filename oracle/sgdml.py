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


def assemble_kernel(R_desc, R_d_desc, tril_perms_lin_, sig):
    """GDMLTrain._assemble_kernel_mat with col_idxs = all (train.py:81-236, 1121-1308)."""
    M, D = R_desc.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    dim_i = 3 * n
    n_perms = int(len(tril_perms_lin_) / D)
    K = np.empty((M * dim_i, M * dim_i))
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
    return K
