"""GPU parity against the REFERENCE's own outputs (tests/golden/*.npz).

The product path is exercised exactly as the reference's GDMLTrain.train calls
its solver (train.py:859-890): sgdml_amd.solvers.Iterative.solve(task, R_desc,
R_d_desc, tril_perms_lin, y, y_std, break_percentage, str_preconditioner) with the
same numpy RNG seed the fixture generator used, so the host-side column
selection draws the same indices.  Criteria: tests/parity.py.
"""
import numpy as np
import pytest

from tests.parity import assert_pcg_parity

pytestmark = pytest.mark.gpu


def load(golden_dir, name):
    return np.load(golden_dir / f"{name}.npz", allow_pickle=False)


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


def task_of(f):
    M, n = f["R"].shape[:2]
    return {"R_train": f["R"], "F_train": f["F"], "E_train": f["E"], "z": f["z"],
            "perms": f["perms"], "sig": float(f["sig"]), "lam": float(f["lam"]),
            "solver_tol": float(f["solver_tol"]), "truncated_cholesky": 1500,
            "n_inducing_pts_init": 25, "use_E_cstr": False, "use_E": True}


SEEDS = {"sgdml_ethanol_n270": 3, "sgdml_ethanol_n270_perms": 5, "sgdml_ethanol_n621": 7,
         "sgdml_ethanol_n2997": 9, "sgdml_ethanol_n270_nongroup": 5, "sgdml_nanotube_n3330": 4,
         "sgdml_ethanol_n270_eigmask": 3}
NANOTUBE = "sgdml_nanotube_n3330"


@pytest.mark.parametrize("name", ["sgdml_ethanol_n270", "sgdml_ethanol_n621",
                                  "sgdml_ethanol_n270_perms", "sgdml_ethanol_n270_nongroup"])
def test_assembly_operator_diag(sg, golden_dir, name):
    f = load(golden_dir, name)
    n = f["y"].size
    with sg.KernelSolver(n) as s:
        s.assemble_sgdml(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]))
        K = s.get_matrix_rows()
        s.set_operator(-1.0, float(f["lam"]))
        Av = s.matvec(f["v"])
        d = s.diag()
    scale = np.abs(f["K"]).max()
    assert np.max(np.abs(K - f["K"])) <= 1e-13 * scale
    np.testing.assert_array_equal(d, -np.diag(K))
    np.testing.assert_allclose(d, f["diag_K"], rtol=1e-12)
    if not name.endswith("nongroup"):
        # matrix-free reference operator K_op(v) = K v - lam v; ours is A v = -K v + lam v
        assert np.linalg.norm(-Av - f["Kop_v"]) <= 1e-13 * np.linalg.norm(f["Kop_v"])
        if name.endswith("_perms"):
            # diagonal blocks are stored transposed (train.py:172-210): symmetric to rounding
            np.testing.assert_allclose(K, K.T, rtol=0, atol=1e-15 * scale)
        else:
            np.testing.assert_array_equal(K, K.T)  # mirrored assembly is exactly symmetric


def test_assembly_n2997_rows(sg, golden_dir):
    f = load(golden_dir, "sgdml_ethanol_n2997")
    n = f["y"].size
    with sg.KernelSolver(n) as s:
        s.assemble_sgdml(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]))
        K = s.get_matrix_rows(0, 64)
    assert np.max(np.abs(K - f["K_rows"])) <= 1e-13 * np.abs(f["K_rows"]).max()


@pytest.mark.parametrize("name", ["sgdml_ethanol_n270", "sgdml_ethanol_n621"])
@pytest.mark.parametrize("variant", [0, 1])
def test_nystrom_apply_vs_reference(sg, golden_dir, name, variant):
    f = load(golden_dir, name)
    n = f["y"].size
    with sg.KernelSolver(n) as s:
        s.assemble_sgdml(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]))
        s.set_operator(-1.0, float(f["lam"]))
        s.precon_nystrom(f["nys_idx"], variant=variant)
        z = s.precon_apply(f["v"])
    ref = f[f"nys{variant}_z"]
    assert np.linalg.norm(z - ref) <= 1e-6 * np.linalg.norm(ref)


def run_dropin(f, name, precon, desc=None):
    from sgdml_amd.solvers import Iterative

    n = f["y"].size
    bp = int(f["k_rot"]) / n
    Rd, Rdd = desc if desc is not None else (f["R_desc"], f["R_d_desc"])
    np.random.seed(1000 + SEEDS[name])
    with Iterative(None, None, device=0) as it:  # contexts released when the solve returns
        return it.solve(task_of(f), Rd, Rdd, f["tril_perms_lin"], f["y"],
                        float(f["y_std"]), break_percentage=bp, str_preconditioner=precon)


@pytest.fixture(scope="module")
def nanotube(sg, golden_dir):
    """370-atom nanotube-like fixture: descriptors are computed here on the GPU (the
    fixture stores only R; D = 68265)."""
    f = load(golden_dir, NANOTUBE)
    return f, sg.sgdml_descriptors(f["R"])


def test_nanotube_operator_vs_reference(sg, nanotube):
    f, (Rd, Rdd) = nanotube
    n, lam, sig = f["y"].size, float(f["lam"]), float(f["sig"])
    with sg.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, f["perms"], sig)
        s.set_operator(-1.0, lam)
        assert s.storage_info()[0] == "matfree"
        Av = s.matvec(f["v"])
        d = s.diag()
        zs = []
        for variant in (0, 1):
            s.precon_nystrom(f["nys_idx"], variant=variant)
            zs.append(s.precon_apply(f["v"]))
    assert np.linalg.norm(-Av - f["Kop_v"]) <= 1e-13 * np.linalg.norm(f["Kop_v"])
    np.testing.assert_allclose(d, f["diag_K"], rtol=1e-12)
    for variant, z in enumerate(zs):
        ref = f[f"nys{variant}_z"]
        assert np.linalg.norm(z - ref) <= 1e-6 * np.linalg.norm(ref)
    with sg.KernelSolver(n) as s:
        s.assemble_sgdml(Rd, Rdd, f["perms"], sig)
        K = s.get_matrix_rows(0, 16)
    assert np.max(np.abs(K - f["K_rows"])) <= 1e-13 * np.abs(f["K_rows"]).max()


@pytest.mark.parametrize("precon", ["cholesky", "random_scores"])
def test_dropin_solve_nanotube(sg, nanotube, precon):
    """Residual curve and coefficients against the reference's own solve on the
    nanotube molecule (rule-of-thumb rank k = 873 at N = 3330)."""
    f, desc = nanotube
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, NANOTUBE, precon, desc)
    assert is_conv and bool(f[f"{precon}__is_conv"])
    assert np.array_equal(idxs, f[f"{precon}__inducing_pts_idxs"])
    if precon == "cholesky":
        assert np.array_equal(info["index_columns"], f["cholesky__index_columns"])
    assert_pcg_parity(num_iters, info["resid_trace"][1:], alphas, int(f[f"{precon}__num_iters"]),
                      f[f"{precon}__trace"], f[f"{precon}__alphas"], case=f"{NANOTUBE}/{precon}")


PRECONS = ["cholesky", "random_scores", "lev_scores", "inverse_lev", "lev_random",
           "truncated_cholesky", "truncated_cholesky_custom", "rank_k_lev_scores",
           "rank_k_lev_scores_custom", "eigvec_precon"]


@pytest.mark.parametrize("precon", PRECONS)
def test_dropin_solve_n270(sg, golden_dir, precon):
    name = "sgdml_ethanol_n270"
    f = load(golden_dir, name)
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, name, precon)
    assert is_conv and bool(f[f"{precon}__is_conv"])
    if precon not in ("lev_random", "rank_k_lev_scores", "rank_k_lev_scores_custom"):
        # p-weighted sampling may flip where a score differs by rounding
        assert np.array_equal(idxs, f[f"{precon}__inducing_pts_idxs"])
    if precon == "cholesky":
        assert np.array_equal(info["index_columns"], f["cholesky__index_columns"])
        assert info["L.shape"] == (f["y"].size, int(f["k_rot"]))
    assert_pcg_parity(num_iters, info["resid_trace"][1:], alphas, int(f[f"{precon}__num_iters"]),
                      f[f"{precon}__trace"], f[f"{precon}__alphas"], case=f"{name}/{precon}")
    assert resid <= float(f["solver_tol"]) * np.linalg.norm(f["y"])
    assert abs(rmse - resid / np.sqrt(f["y"].size)) == 0


EIGMASK = "sgdml_ethanol_n270_eigmask"


@pytest.mark.parametrize("precon", ["eigvec_precon_block_diagonal",
                                    "eigvec_precon_atomic_interactions"])
def test_dropin_solve_eigen_masks(sg, golden_dir, precon):
    """The masked eigen preconditioners (iterative_solver.py:1238-1268) against the
    reference's own solves: block_diagonal zeroes all of K (L = 0, P = I / lam: plain CG),
    atomic_interactions keeps the 3 x 3 atom blocks; neither reaches tol 1e-4 within
    5N iterations here, in the reference as on the GPU."""
    f = load(golden_dir, EIGMASK)
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, EIGMASK, precon)
    assert is_conv == bool(f[f"{precon}__is_conv"])
    assert np.array_equal(idxs, f[f"{precon}__inducing_pts_idxs"])
    ref_it, ref_tr = int(f[f"{precon}__num_iters"]), f[f"{precon}__trace"]
    if is_conv:
        assert_pcg_parity(num_iters, info["resid_trace"][1:], alphas, ref_it, ref_tr,
                          f[f"{precon}__alphas"], mode="chaotic")
    else:  # both stop at maxiter; the early curve agrees before rounding takes over
        assert num_iters == ref_it == 5 * f["y"].size
        assert np.max(np.abs(np.log10(info["resid_trace"][1:9] / ref_tr[:8]))) <= 1e-6


@pytest.mark.parametrize("name,precon", [("sgdml_ethanol_n621", "cholesky"),
                                         ("sgdml_ethanol_n621", "random_scores"),
                                         ("sgdml_ethanol_n621", "truncated_cholesky"),
                                         ("sgdml_ethanol_n2997", "cholesky"),
                                         ("sgdml_ethanol_n2997", "random_scores")])
def test_dropin_solve_larger(sg, golden_dir, name, precon):
    f = load(golden_dir, name)
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, name, precon)
    assert is_conv
    assert np.array_equal(idxs, f[f"{precon}__inducing_pts_idxs"])
    assert_pcg_parity(num_iters, info["resid_trace"][1:], alphas, int(f[f"{precon}__num_iters"]),
                      f[f"{precon}__trace"], f[f"{precon}__alphas"], case=f"{name}/{precon}")


def test_dropin_unpreconditioned_maxiter(sg, golden_dir):
    """No preconditioner: the reference hits maxiter = 5N (info = maxiter, 5N callbacks)."""
    f = load(golden_dir, "sgdml_ethanol_n270")
    n = f["y"].size
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, "sgdml_ethanol_n270", "none")
    assert not is_conv
    assert num_iters == int(f["none_1e-04__callbacks"]) == 5 * n
    ref = f["none_1e-04__trace"]
    assert np.max(np.abs(np.log10(info["resid_trace"][1:9] / ref[:8]))) <= 1e-6


@pytest.mark.parametrize("precon", ["cholesky", "random_scores", "truncated_cholesky_custom"])
def test_dropin_solve_perm_group(sg, golden_dir, precon):
    name = "sgdml_ethanol_n270_perms"
    f = load(golden_dir, name)
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, name, precon)
    assert is_conv
    assert np.array_equal(idxs, f[f"{precon}__inducing_pts_idxs"])
    assert_pcg_parity(num_iters, info["resid_trace"][1:], alphas, int(f[f"{precon}__num_iters"]),
                      f[f"{precon}__trace"], f[f"{precon}__alphas"], case=f"{name}/{precon}")


def test_error_semantics(sg):
    """Non-PSD pivot -> AssertionError (incomplete_cholesky.py:62); singular K_mm in the
    Nystrom build -> LinAlgError (scipy cho_factor)."""
    n = 200
    rng = np.random.default_rng(0)
    A = rng.standard_normal((n, n))
    indef = (A + A.T) / 2
    with sg.KernelSolver(n) as s:
        s.set_matrix(indef)
        s.set_operator(1.0, 1e-6)
        with pytest.raises(AssertionError):
            s.precon_pivchol(50)
    negdef = -np.eye(n) - 0.01 * np.ones((n, n))  # S_mm negative definite: no Cholesky
    for variant in (0, 1):
        with sg.KernelSolver(n) as s:
            s.set_matrix(negdef)
            s.set_operator(1.0, 1e-10)
            with pytest.raises(np.linalg.LinAlgError):
                s.precon_nystrom(np.arange(0, 200, 10), variant=variant)


def test_dropin_unknown_preconditioner(sg, golden_dir):
    f = load(golden_dir, "sgdml_ethanol_n270")
    with pytest.raises(NotImplementedError):
        run_dropin(f, "sgdml_ethanol_n270", "does_not_exist")


def test_rbf_reference_generator_and_preconditioner(sg, golden_dir):
    """tools/utils.create_kernel_mat (sklearn RBF, l = 1, d = 2, + 1e-10 I; utils.py:173-187)
    generated on the device, the reference's pivoted Cholesky on it (incomplete_cholesky.py
    :24-93, index order and L), and IterativeCholesky._init_precon_operator's Woodbury
    apply (iterative_cholesky.py:115-150) on the l = 0.2 kernel."""
    f = load(golden_dir, "rbf_reference")
    n = f["X"].shape[0]
    k = int(f["k"])
    with sg.KernelSolver(n) as s:
        s.gen_rbf(f["X"], length_scale=1.0, jitter=1e-10)
        K = s.get_matrix_rows()
        np.testing.assert_allclose(K, f["K"], rtol=0, atol=2e-15)
        s.set_operator(1.0, 1e-10)
        piv, _ = s.precon_pivchol(k, build_woodbury=False)
        np.testing.assert_array_equal(piv[:k], f["index_columns"][:k])
        Lt = s.precon_panel()
    np.testing.assert_allclose(Lt.T, f["L"], rtol=0, atol=1e-12 * np.abs(f["L"]).max())
    lam, k3 = float(f["lam"]), int(f["k3"])
    with sg.KernelSolver(n) as s:
        s.gen_rbf(f["X3"], length_scale=0.2, jitter=0.0)
        np.testing.assert_allclose(s.get_matrix_rows(), f["K3"], rtol=0, atol=2e-15)
        s.set_operator(1.0, lam)
        piv3, _ = s.precon_pivchol(k3)
        np.testing.assert_array_equal(piv3[:k3], f["index_columns3"][:k3])
        z = s.precon_apply(f["r"])
    np.testing.assert_allclose(z, f["z"], rtol=1e-9, atol=1e-9 * np.abs(f["z"]).max())


def test_dropin_info_dict_schema(sg, golden_dir, tmp_path):
    """The info dict carries the reference's keys (iterative_solver.py:1094-1105, plus the
    pivoted-Cholesky info of incomplete_cholesky.py:86-88), so the reference's consumers
    work unchanged: create_model/model.update (train.py:925-940), tools/create_data.cg_steps
    (create_data.py:117-148) and store_model's np.savez_compressed (train_models.py:152-154)."""
    name = "sgdml_ethanol_n270"
    f = load(golden_dir, name)
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, name, "cholesky")
    ref_keys = {"is_conv", "total_time_cholesky", "total_time_cg", "total_time_solve",
                "total_time_preconditioner", "time_cholesky", "L.shape", "index_columns"}
    assert ref_keys <= set(info)
    k = int(f["k_rot"])
    n = f["y"].size
    t = info["time_cholesky"]
    assert t.shape == (k,) and np.all(t > 0)
    # per-column device times (event stamps every 4 columns), not one uniform average
    assert np.unique(t).size > 1 and info["time_woodbury"] > 0
    assert info["operator_storage"] == "matfree" and info["gbps_matvec"] > 0
    # cg_steps' arithmetic
    t_begin, t_end = np.median(t[:20]), np.median(t[20:])
    assert np.isfinite(t_end / t_begin - 1)
    assert info["total_time_cg"] / num_iters > 0
    assert len(idxs) / len(alphas) == k / n
    # store_model: the solver's fields and info values round-trip through savez_compressed
    model = dict(info, alphas_F=alphas, solver_iters=num_iters, solver_resid=resid,
                 inducing_pts_idxs=idxs, norm_y_train=np.linalg.norm(f["y"]))
    path = tmp_path / "model.npz"
    np.savez_compressed(path, **model)
    back = np.load(path, allow_pickle=False)
    np.testing.assert_array_equal(back["alphas_F"], alphas)
    np.testing.assert_array_equal(back["index_columns"], info["index_columns"])
    assert tuple(back["L.shape"]) == (n, k)


def test_dropin_warm_start(sg, golden_dir):
    """task['alphas0_F'] / task['solver_iters'] (iterative_solver.py:650-660, 995-1005): the
    solve restarts from -alphas0_F and the iteration count continues the previous one."""
    from sgdml_amd.solvers import Iterative

    name = "sgdml_ethanol_n270"
    f = load(golden_dir, name)
    n = f["y"].size
    a_ref = f["cholesky__alphas"]
    task = dict(task_of(f), alphas0_F=a_ref * (1 + 1e-3 * np.random.default_rng(0).standard_normal(n)),
                solver_iters=1000)
    with Iterative(None, None, device=0) as it:
        alphas, num_iters, resid, rmse, idxs, is_conv, info = it.solve(
            task, f["R_desc"], f["R_d_desc"], f["tril_perms_lin"], f["y"], float(f["y_std"]),
            break_percentage=int(f["k_rot"]) / n, str_preconditioner="cholesky")
    assert is_conv
    assert num_iters == 1000 + max(info["cg_iterations"], 1)
    assert resid <= float(f["solver_tol"]) * np.linalg.norm(f["y"])
    assert np.linalg.norm(alphas - a_ref) <= 1e-3 * np.linalg.norm(a_ref)
