"""Synthetic SPD RBF kernel and the rule-of-thumb preconditioner size.

TEST INFRASTRUCTURE (see oracle/__init__.py).
"""
from __future__ import annotations

import numpy as np
from scipy.spatial.distance import pdist, squareform


def rbf_kernel(X, length_scale=1.0, jitter=0.0):
    """sklearn RBF(length_scale)(X) (+ jitter I) as in tools/utils.py:181-186:
    exp(-0.5 * sqeuclidean(X / l)), diagonal 1."""
    X = np.asarray(X, dtype=np.float64)
    d = pdist(X / length_scale, metric="sqeuclidean")
    K = np.exp(-0.5 * d)
    K = squareform(K)
    np.fill_diagonal(K, 1)
    if jitter:
        K += jitter * np.eye(K.shape[0])
    return K


def get_params(dataset_name):
    """plot_data.get_params(old=False) (plot_data.py:677-706): (slope m, k_unity, prefactor)."""
    table = {
        "default": (1, 100), "ethanol": (0.87, 10), "uracil": (1.07, 32),
        "C6H5CH3": (1.01, 44), "toluene": (1.01, 44), "aspirin": (1.14, 236),
        "azobenzene_new": (1.02, 62), "azobenzene": (1.02, 62),
        "aims_catcher": (1.02, 316), "catcher": (1.02, 316),
        "larger_aims_nanotube": (0.73, 89), "nanotube": (0.73, 89),
    }
    if dataset_name not in table:
        raise NotImplementedError(f"dataset_name = {dataset_name} is not specified. ")
    m, k = table[dataset_name]
    return m, k, 1


def rule_of_thumb(n, k_min, m):
    """plot_data.py:1254-1258."""
    res = (k_min ** m * m * n ** 2 / 2) ** (1 / (2 + m))
    if isinstance(n, int):
        res = int(np.floor(res))
    return res
