"""Synthetic inputs for the benchmark configurations.

The reference's datasets (ethanol_dft.npz, larger_aims_nanotube.npz) are
downloaded over HTTP and absent here, so geometries are generated:
  * ethanol-like: 9 atoms z = [6, 6, 8, 1 x 6], seeded Gaussian perturbations of
    a fixed equilibrium frame;
  * nanotube-like: 370 atoms (300 C on a cylinder r = 6 A, 30 A long, 70 H
    capping both ends), seeded perturbations;
  * RBF points x ~ U[0,1)^d (seed 0, numpy default_rng), b = sum(x^2)
    (tools/utils.py:19-23 test_function).
Forces are seeded Gaussian labels (only their normalised ravel enters the solve,
train.py:837-845).
"""
from __future__ import annotations

import numpy as np

ETHANOL_Z = np.array([6, 6, 8, 1, 1, 1, 1, 1, 1])
_ETHANOL_FRAME = np.array([
    [0.000, 0.000, 0.000],    # C
    [1.520, 0.000, 0.000],    # C
    [2.000, 1.350, 0.000],    # O
    [-0.390, 1.030, 0.000],   # H
    [-0.390, -0.510, 0.890],  # H
    [-0.390, -0.510, -0.890], # H
    [1.910, -0.510, 0.890],   # H
    [1.910, -0.510, -0.890],  # H
    [2.960, 1.300, 0.000],    # H
])


def ethanol_like(M: int, seed: int = 0, scale: float = 0.08):
    rng = np.random.default_rng(seed)
    R = _ETHANOL_FRAME[None, :, :] + scale * rng.standard_normal((M, 9, 3))
    F = rng.standard_normal((M, 9, 3))
    E = rng.standard_normal(M)
    return {"R": R, "z": ETHANOL_Z.copy(), "F": F, "E": E}


def ethanol_harmonic(M: int, seed: int = 0, scale: float = 0.08, k: float = 1.0):
    """ethanol_like geometries with CONSISTENT labels: E = k/2 sum_{a<b} (r_ab - r0_ab)^2
    over all atom pairs (r0 = the frame), F = -grad E.  The reference's integration-
    constant recovery (train.py:972-1119) needs energies that the forces integrate to."""
    rng = np.random.default_rng(seed)
    R = _ETHANOL_FRAME[None, :, :] + scale * rng.standard_normal((M, 9, 3))
    a, b = np.triu_indices(9, k=1)
    r0 = np.linalg.norm(_ETHANOL_FRAME[a] - _ETHANOL_FRAME[b], axis=1)
    d = R[:, a, :] - R[:, b, :]                    # M x P x 3
    r = np.linalg.norm(d, axis=2)
    E = 0.5 * k * np.sum((r - r0) ** 2, axis=1)
    g = (k * (r - r0) / r)[:, :, None] * d          # dE/dR_a for each pair
    F = np.zeros_like(R)
    np.add.at(F, (slice(None), a), -g)
    np.add.at(F, (slice(None), b), g)
    return {"R": R, "z": ETHANOL_Z.copy(), "F": F, "E": E}


def nanotube_frame():
    ring_n, rings, radius, length = 15, 20, 6.0, 30.0
    pts = []
    for r in range(rings):
        zc = r * length / (rings - 1)
        phase = 0.5 * (r % 2)
        for a in range(ring_n):
            th = 2 * np.pi * (a + phase) / ring_n
            pts.append([radius * np.cos(th), radius * np.sin(th), zc])
    for zc in (-1.1, length + 1.1):
        for a in range(35):
            th = 2 * np.pi * a / 35
            pts.append([(radius + 0.4) * np.cos(th), (radius + 0.4) * np.sin(th), zc])
    z = np.array([6] * 300 + [1] * 70)
    return np.array(pts), z


def nanotube_like(M: int, seed: int = 0, scale: float = 0.05):
    frame, z = nanotube_frame()
    rng = np.random.default_rng(seed)
    R = frame[None, :, :] + scale * rng.standard_normal((M, frame.shape[0], 3))
    F = rng.standard_normal((M, frame.shape[0], 3))
    E = rng.standard_normal(M)
    return {"R": R, "z": z, "F": F, "E": E}


def labels(F: np.ndarray):
    """y = F.ravel() / std (train.py:837-845, use_E_cstr = False)."""
    y = F.ravel().copy()
    y_std = np.std(y)
    return y / y_std, y_std


def rbf_points(n: int, d: int = 3, seed: int = 0):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    return X, np.sum(X ** 2, axis=1)
