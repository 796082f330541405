"""Drop-in Iterative.solve sharded over several ranks from ONE process
(sgdml_amd.sharded.ShardedKernelSolver), the way the reference spreads its GPU operator
with DataParallel (predict.py:335-341).  On the one-GPU test box the ranks share cuda:0
through the library's in-process transport (RCCL refuses two ranks on one device); on a
node each rank has its own GPU and the transport is RCCL.  Criteria: tests/parity.py
against the reference's own solves (tests/golden)."""
import numpy as np
import pytest

from tests.parity import assert_pcg_parity
from tests.test_gpu_golden import SEEDS, load, task_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


def run(f, name, precon, devices, desc=None):
    """(solve result, type and world of the solver it used); the solver's contexts are
    released before returning, pass or fail."""
    from sgdml_amd.solvers import Iterative

    n = f["y"].size
    Rd, Rdd = desc if desc is not None else (f["R_desc"], f["R_d_desc"])
    np.random.seed(1000 + SEEDS[name])
    with Iterative(None, None, devices=devices) as it:
        out = it.solve(task_of(f), Rd, Rdd, f["tril_perms_lin"], f["y"], float(f["y_std"]),
                       break_percentage=int(f["k_rot"]) / n, str_preconditioner=precon)
        return out, (type(it.solver), getattr(it.solver, "world", 1))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,precon,world", [
    ("sgdml_ethanol_n621", "cholesky", 2), ("sgdml_ethanol_n621", "random_scores", 3),
    ("sgdml_ethanol_n2997", "cholesky", 4), ("sgdml_ethanol_n270", "lev_random", 2),
    ("sgdml_nanotube_n3330", "cholesky", 2)])
def test_sharded_dropin_vs_reference(sg, golden_dir, name, precon, world):
    f = load(golden_dir, name)
    desc = sg.sgdml_descriptors(f["R"]) if "R_desc" not in f.files else None
    (alphas, num_iters, resid, rmse, idxs, is_conv, info), (kind, w) = run(
        f, name, precon, [0] * world, desc)
    assert kind is sg.ShardedKernelSolver and w == world
    assert info["n_gpus"] == world
    assert is_conv
    if precon != "lev_random":
        assert np.array_equal(idxs, f[f"{precon}__inducing_pts_idxs"])
    if precon == "cholesky":
        assert np.array_equal(info["index_columns"], f["cholesky__index_columns"])
    assert_pcg_parity(num_iters, info["resid_trace"][1:], alphas, int(f[f"{precon}__num_iters"]),
                      f[f"{precon}__trace"], f[f"{precon}__alphas"], case=f"{name}/{precon}")


@pytest.mark.timeout(300)
def test_sharded_dropin_eigen(sg, golden_dir):
    """eigvec_precon: the truncated eigensolver runs on the sharded matrix-free operator."""
    name = "sgdml_ethanol_n270"
    f = load(golden_dir, name)
    (alphas, num_iters, resid, rmse, idxs, is_conv, info), (kind, w) = run(
        f, name, "eigvec_precon", [0, 0])
    assert kind is sg.ShardedKernelSolver and w == 2 and info["n_gpus"] == 2
    assert is_conv
    assert_pcg_parity(num_iters, info["resid_trace"][1:], alphas,
                      int(f["eigvec_precon__num_iters"]), f["eigvec_precon__trace"],
                      f["eigvec_precon__alphas"], case=f"{name}/eigvec_precon")


@pytest.mark.timeout(300)
def test_sharded_solver_gathers(sg):
    """Global-array semantics of ShardedKernelSolver against one KernelSolver."""
    from sgdml_amd import synthetic

    n = 1500
    X, b = synthetic.rbf_points(n, 3, 7)
    v = np.random.default_rng(3).standard_normal(n)
    with sg.KernelSolver(n, device=0) as s1:
        s1.gen_rbf(X, 0.2)
        s1.set_operator(1.0, 1e-2)
        y1, d1 = s1.matvec(v), s1.diag()
        s1.precon_pivchol(60)
        z1 = s1.precon_apply(v)
        r1 = s1.pcg(b, tol=1e-8, maxiter=5 * n)
    with sg.ShardedKernelSolver(n, [0, 0, 0]) as s3:
        s3.gen_rbf(X, 0.2)
        s3.set_operator(1.0, 1e-2)
        y3, d3 = s3.matvec(v), s3.diag()
        s3.precon_pivchol(60)
        z3 = s3.precon_apply(v)
        seen = []
        r3 = s3.pcg(b, tol=1e-8, maxiter=5 * n, callback=lambda x, it, res: seen.append(x.size),
                    cb_every=2)
    np.testing.assert_allclose(y3, y1, rtol=1e-13, atol=1e-13 * np.abs(y1).max())
    np.testing.assert_array_equal(d3, d1)
    np.testing.assert_allclose(z3, z1, rtol=1e-9, atol=1e-9 * np.abs(z1).max())
    assert r3.info == r1.info == 0 and abs(r3.iters - r1.iters) <= 1
    assert np.linalg.norm(r3.x - r1.x) <= 1e-7 * np.linalg.norm(r1.x)
    assert seen and all(s == n for s in seen)
