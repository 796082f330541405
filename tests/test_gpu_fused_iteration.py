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
    same count, inside the reference's measured band (its 322 iterations, b_it 1: the device took
    exactly 322 with the fp64 matrix-core Gram of rounds 3-4 and takes 321 with the double-double
    Gram of round 5), traces equal to rounding."""
    from tests.parity import noise_band

    f, desc = nanotube
    res = {}
    for name in ("four", "six"):
        with _env(**FORMS[name]):
            res[name] = run_dropin(f, NANOTUBE, "cholesky", desc)
    (a4, it4, *_r4, info4), (a6, it6, *_r6, info6) = res["four"], res["six"]
    b = noise_band(f"{NANOTUBE}/cholesky")
    ref = int(f["cholesky__num_iters"])
    print(f"drop-in: {it4} iterations (four launches), {it6} (six), reference {ref} (b_it {b['band_iters']})")
    assert it4 == it6 and abs(it4 - ref) <= 2 * b["band_iters"] + 2, (it4, it6, ref)
    t4, t6 = np.asarray(info4["resid_trace"]), np.asarray(info6["resid_trace"])
    assert t4.shape == t6.shape
    assert np.max(np.abs(t4 - t6) / np.abs(t6)) <= 1e-12
    assert np.linalg.norm(a4 - a6) <= 1e-12 * np.linalg.norm(a6)


def test_fused_dropin_checkpoints(sg, nanotube, monkeypatch):
    """The drop-in's progress / checkpoint chunking (iterative_solver.py:874-965) on the fused
    iteration: chunks end on the checkpoint iterations, where the last iteration keeps its own
    k_update_xr + stop test.  Every checkpoint's alphas are -x_j of an independent solve stopped
    at j (bit for bit, with its stop-test residual), and the final model equals the one of a
    solve without callbacks."""
    from sgdml_amd import model as mdl
    from sgdml_amd.solvers import iterative_solver as its

    f, _ = nanotube
    Rd, Rdd = sg.host_descriptors(f["R"])  # the trainer's descriptors (model.train)
    M = f["R"].shape[0]
    task = {"type": "t", "dataset_name": "nanotube", "dataset_theory": "synthetic", "z": f["z"],
            "R_train": f["R"], "F_train": f["F"], "E_train": f["E"], "idxs_train": np.arange(M),
            "md5_train": "0", "idxs_valid": np.arange(0), "md5_valid": "0", "sig": 10,
            "lam": 1e-15, "use_E": True, "use_E_cstr": False, "use_sym": False,
            "use_cprsn": False, "solver_name": "cg", "solver_tol": 1e-4,
            "n_inducing_pts_init": 25, "interact_cut_off": None, "perms": f["perms"],
            "truncated_cholesky": 1500}
    monkeypatch.setattr(its._CGStatus, "CHECKPOINT_S", 2e-3)
    monkeypatch.setattr(its._CGStatus, "PROGRESS_S", 5e-4)
    n = f["y"].size
    k = int(f["k_rot"])
    saved = []
    m = mdl.train(task, save_progr_callback=lambda mod: saved.append(dict(mod)),
                  callback=lambda *a, **kw: None, break_percentage=k / n,
                  str_preconditioner="cholesky")
    m_plain = mdl.train(task, break_percentage=k / n, str_preconditioner="cholesky")
    np.testing.assert_array_equal(m["alphas_F"], m_plain["alphas_F"])
    assert m["solver_iters"] == m_plain["solver_iters"]
    assert len(saved) >= 2, len(saved)

    y = f["F"].ravel().copy()
    y /= np.std(y)
    with sg.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.atleast_2d(f["perms"]), 10.0)
        s.set_operator(-1.0, 1e-10)
        s.precon_pivchol(k)
        assert s.precon_apply_traffic()[0] == 1  # the rows apply: the fused iteration runs
        last = 0
        for mod in saved:
            j = int(mod["solver_iters"])
            assert j > last
            last = j
            s.pcg_start(y, None, 1e-4, 5 * n)
            s.pcg_run(j)
            assert s.pcg_result()[0] == j
            np.testing.assert_array_equal(mod["alphas_F"], -s.pcg_x())
            assert mod["solver_resid"] == s.pcg_trace()[j]


@pytest.mark.parametrize("perms", ["identity", "group2"])
@pytest.mark.parametrize("chunk", [0, 7])
def test_pair_tile_fused_iteration_matches_separate_launches(sg, chunk, perms):
    """The few-atom iteration (pair-tile operator) with the same folds: k_mf_z
    forms p = z + beta p_old for the entries it reads and runs the previous iteration's stop test,
    k_pt_fin writes p (k_update_p's bits), and k_update_xr moves into the next rows apply -- four
    launches fewer per iteration than the seven-launch form (MLFF_FUSE_P=0), the same iterates,
    counts and stop decisions (chunk 7: a chunk boundary every seventh iteration).  A
    two-element permutation group exercises the permuted Zt gathers."""
    from sgdml_amd import synthetic

    ds = synthetic.ethanol_harmonic(200, seed=4)
    P = np.arange(9)[None, :] if perms == "identity" else np.array([np.arange(9),
                                                                     [0, 1, 2, 4, 3, 5, 6, 7, 8]])
    Rd, Rdd = sg.sgdml_descriptors(ds["R"])
    y, _ = synthetic.labels(ds["F"])
    n = y.size
    out = {}
    for name, env in FORMS.items():
        with _env(**env), sg.KernelSolver(n) as s:
            s.sgdml_operator(Rd, Rdd, P, 10.0)
            s.set_operator(-1.0, 1e-10)
            assert s.storage_info()[0] == "matfree" and s.operator_form() == "pt"
            s.precon_pivchol(800)
            assert s.precon_apply_traffic()[0] == 1  # rows apply: the x / r fold applies
            out[name] = s.pcg(y, tol=1e-8, maxiter=3000, chunk=chunk)
    ref = out["six"]
    assert ref.info == 0
    for name in ("four", "five"):
        r = out[name]
        assert r.iters == ref.iters and r.info == ref.info, (name, r.iters, ref.iters)
        t, tr = np.asarray(r.trace), np.asarray(ref.trace)
        assert t.shape == tr.shape
        assert np.max(np.abs(t - tr) / np.abs(tr)) <= 1e-12, name
        assert np.linalg.norm(r.x - ref.x) <= 1e-12 * np.linalg.norm(ref.x), name
