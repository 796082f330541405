"""Debug helper: the persistent pivoted Cholesky against the launch sequence (dense rows of an
RBF-like matrix and the configs[1]-like nanotube); prints the first step where they part."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."),
                os.path.join(os.path.dirname(__file__), "..", "..", "mlff-preconditioner_amd")]
import sgdml_amd  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402


def build(setup, n, k, env):
    for key in ("MLFF_PIV_G", "MLFF_PIVCHOL_PERSIST"):
        os.environ.pop(key, None)
    os.environ.update(env)
    with sgdml_amd.KernelSolver(n) as s:
        setup(s)
        piv, sec = s.precon_pivchol(k, build_woodbury=False)
        return piv, s.precon_panel(), sec


def compare(tag, setup, n, k):
    ref = build(setup, n, k, {"MLFF_PIVCHOL_PERSIST": "0"})
    for G in ("256", "64"):
        got = build(setup, n, k, {"MLFF_PIV_G": G})
        dp = np.nonzero(got[0][:k] != ref[0][:k])[0]
        dl = np.nonzero(np.any(got[1][:k] != ref[1][:k], axis=1))[0]
        msg = f"{tag} k={k} G={G}: first pivot diff {dp[:3]}, first L row diff {dl[:3]}"
        if dl.size:
            m = dl[0]
            d = np.nonzero(got[1][m] != ref[1][m])[0]
            rel = np.abs(got[1][m, d] - ref[1][m, d]) / np.maximum(np.abs(ref[1][m, d]), 1e-300)
            msg += f"; row {m}: {d.size} entries, max rel {rel.max():.2e}, first cols {d[:5]}"
        print(msg, flush=True)


n = 3000
rng = np.random.default_rng(3)
X = rng.uniform(size=(n, 3))
K = np.exp(-((X[:, None, :] - X[None, :, :]) ** 2).sum(-1) / (2 * 0.3 ** 2)) + 1e-6 * np.eye(n)


def dense(s):
    s.set_matrix(K)
    s.set_operator(1.0, 1e-6)


compare("dense", dense, n, 400)
ds = synthetic.nanotube_like(14, seed=0)
Rd, Rdd = sgdml_amd.sgdml_descriptors(ds["R"])


def nano(s):
    s.sgdml_operator(Rd, Rdd, np.arange(370)[None, :], 10.0)
    s.set_operator(-1.0, 1e-10)


compare("nanotube", nano, 15540, 1000)
