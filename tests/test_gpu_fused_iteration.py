"""The nanotube PCG iteration in four launches against the six-launch form.

The folds keep the reference's arithmetic (scipy 1.7.3 CG: p = z + beta p, x += alpha p,
r -= alpha q with the same fma bits); only the ||r||^2 partials of the stop test are summed in
another fixed order.  So the two forms must produce the same iterates to rounding level, the
same iteration count and the same stop decisions, also across chunk boundaries (where the last
iteration of a chunk keeps its own k_update_xr + k_stoptest) and through the true-residual
recheck.  MLFF_FUSE_P / MLFF_FUSE_XR are read when a context is created.
"""
import os

import numpy as np
import pytest

from tests.test_gpu_golden import NANOTUBE, load, run_dropin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


@pytest.fixture(scope="module")
def nanotube(sg, golden_dir):
    f = load(golden_dir, NANOTUBE)
    return f, sg.sgdml_descriptors(f["R"])


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


FORMS = {"four": {}, "five": {"MLFF_FUSE_XR": "0"}, "six": {"MLFF_FUSE_P": "0"}}


def _kernel_solve(sg, f, desc, chunk, env):
    Rd, Rdd = desc
    n, lam, sig = f["y"].size, float(f["lam"]), float(f["sig"])
    k = int(f["k_rot"])
    with _env(**env), sg.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, f["perms"], sig)
        s.set_operator(-1.0, lam)
        assert s.storage_info()[0] == "matfree"
        s.precon_pivchol(k)
        assert s.precon_apply_traffic()[0] == 1  # the one-pass rows apply: the fused form runs
        res = s.pcg(f["y"], tol=1e-10, chunk=chunk)
    return res


@pytest.mark.parametrize("chunk", [0, 7])
def test_fused_iteration_matches_separate_launches(sg, nanotube, chunk):
    """Kernel-level solve (pivoted Cholesky k = 873, the rows apply) to 1e-10 in the 4-, 5- and
    6-launch forms; chunk 7 puts a chunk boundary (standalone k_update_xr + stop test) every
    seventh iteration."""
    f, desc = nanotube
    out = {name: _kernel_solve(sg, f, desc, chunk, env) for name, env in FORMS.items()}
    ref = out["six"]
    for name in ("four", "five"):
        r = out[name]
        assert r.iters == ref.iters and r.info == ref.info, (name, r.iters, ref.iters)
        t, tr = np.asarray(r.trace), np.asarray(ref.trace)
        assert t.shape == tr.shape
        assert np.max(np.abs(t - tr) / np.abs(tr)) <= 1e-12, name
        assert np.linalg.norm(r.x - ref.x) <= 1e-12 * np.linalg.norm(ref.x), name


def test_fused_dropin_recheck_matches(sg, nanotube):
    """The golden drop-in solve (tol 1e-6 ends in the true-residual recheck) in both forms: the
    reference's 322 iterations, traces equal to rounding."""
    f, desc = nanotube
    res = {}
    for name in ("four", "six"):
        with _env(**FORMS[name]):
            res[name] = run_dropin(f, NANOTUBE, "cholesky", desc)
    (a4, it4, *_r4, info4), (a6, it6, *_r6, info6) = res["four"], res["six"]
    assert it4 == it6 == int(f["cholesky__num_iters"])
    t4, t6 = np.asarray(info4["resid_trace"]), np.asarray(info6["resid_trace"])
    assert t4.shape == t6.shape
    assert np.max(np.abs(t4 - t6) / np.abs(t6)) <= 1e-12
    assert np.linalg.norm(a4 - a6) <= 1e-12 * np.linalg.norm(a6)
