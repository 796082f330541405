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
    # 3 ranks vs one: two summation orders of a chaotic solve (the one-step Woodbury panel,
    # iterative_cholesky.py:141-148): the generic chaotic rule of tests/parity.py
    from tests.parity import assert_pcg_parity

    assert r3.info == r1.info == 0
    assert_pcg_parity(r3.iters, r3.trace[1:], r3.x, r1.iters, r1.trace[1:], r1.x, mode="chaotic")
    assert seen and all(s == n for s in seen)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_atomic_interactions_mask(sg, golden_dir, world):
    """eigvec_precon_atomic_interactions (iterative_solver.py:1238-1253) sharded: every rank
    masks its rows of the dense K with the global max|K| (the per-rank maxima all-gathered)
    and the truncated eigensolver runs on the sharded masked operator.  Against one rank: the
    top-k eigenvalues to 1e-10 and the Woodbury apply to 1e-9; the drop-in solve against the
    reference's (which stops at 5N iterations on this system, as in
    test_gpu_golden.py::test_dropin_solve_eigen_masks): the first residuals within 1e-6 in
    log10."""
    from tests.test_gpu_golden import EIGMASK

    f = load(golden_dir, EIGMASK)
    n = f["y"].size
    k = int(int(f["k_rot"]) / n * n)
    dim_i = 3 * f["R"].shape[1]
    v = np.random.default_rng(4).standard_normal(n)
    out = {}
    for w in (1, world):
        s = sg.KernelSolver(n, device=0) if w == 1 else sg.ShardedKernelSolver(n, [0] * w)
        try:
            s.assemble_sgdml(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]))
            s.set_operator(-1.0, float(f["lam"]))
            ev, _ = s.precon_eig(k, mask_mode=2, dim_i=dim_i, want_evals=True)
            out[w] = (ev, s.precon_apply(v))
        finally:
            s.close()
    np.testing.assert_allclose(out[world][0], out[1][0], rtol=1e-10)
    z1, zw = out[1][1], out[world][1]
    assert np.linalg.norm(zw - z1) <= 1e-9 * np.linalg.norm(z1)
    precon = "eigvec_precon_atomic_interactions"
    (alphas, num_iters, resid, rmse, idxs, is_conv, info), (kind, w) = run(
        f, EIGMASK, precon, [0] * world)
    assert kind is sg.ShardedKernelSolver and w == world
    assert is_conv == bool(f[f"{precon}__is_conv"])
    ref_tr = f[f"{precon}__trace"]
    assert np.max(np.abs(np.log10(info["resid_trace"][1:9] / ref_tr[:8]))) <= 1e-6
