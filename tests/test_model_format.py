"""Host side of the training entry point and the on-disk model format
against the reference's own GDMLTrain.train output (tests/golden/sgdml_model_ethanol_n621,
make_golden.py fx_model).  CPU only: the model fields are computed from the fixture's
coefficients; the GPU end-to-end run is tests/test_gpu_model.py."""
import numpy as np

from oracle.sgdml import descriptors, energies_matrix_free
from oracle.sgdml import tril_perms_lin as oracle_tpl
from sgdml_amd import model as mdl


def load(golden_dir):
    return np.load(golden_dir / "sgdml_model_ethanol_n621.npz", allow_pickle=False)


def test_tril_perms_lin_matches_reference_and_oracle(golden_dir):
    f = load(golden_dir)
    np.testing.assert_array_equal(mdl.tril_perms_lin(f["perms"]), f["model__tril_perms_lin"])
    rng = np.random.default_rng(0)
    perms = np.array([np.arange(12), rng.permutation(12), rng.permutation(12)])
    np.testing.assert_array_equal(mdl.tril_perms_lin(perms), oracle_tpl(perms))


def test_create_model_and_int_const(golden_dir):
    f = load(golden_dir)
    Rd, Rdd = descriptors(f["R"])
    alphas = f["model__alphas_F"]
    M = f["R"].shape[0]
    task = {"dataset_name": f["model__dataset_name"], "dataset_theory": f["model__dataset_theory"],
            "solver_tol": float(f["model__solver_tol"]), "n_inducing_pts_init": 25, "z": f["z"],
            "idxs_train": np.arange(M), "md5_train": "0", "idxs_valid": np.arange(0),
            "md5_valid": "0", "interact_cut_off": None, "sig": 10, "lam": 1e-10,
            "perms": f["perms"], "use_E": True, "use_E_cstr": False, "use_cprsn": False}
    m = mdl.create_model(task, "cg", Rd, Rdd, mdl.tril_perms_lin(f["perms"]),
                         float(f["model__std"]), alphas,
                         solver_resid=float(f["model__solver_resid"]),
                         solver_iters=int(f["model__solver_iters"]),
                         norm_y_train=float(f["model__norm_y_train"]),
                         inducing_pts_idxs=f["model__inducing_pts_idxs"])
    ref_keys = set(f["model_keys"])
    info_keys = {"is_conv", "total_time_cholesky", "total_time_cg", "total_time_solve",
                 "total_time_preconditioner", "time_cholesky", "L.shape", "index_columns"}
    assert set(m) | info_keys == ref_keys
    for key in ["R_desc", "R_d_desc_alpha"]:
        np.testing.assert_allclose(m[key], f[f"model__{key}"], rtol=1e-13,
                                   atol=1e-13 * np.abs(f[f"model__{key}"]).max())
    for key in ["type", "code_version", "solver_name", "dataset_name", "use_E", "use_cprsn",
                "n_test", "sig", "lam"]:
        assert np.asarray(m[key]) == f[f"model__{key}"], key
    # training-set energies (c = 0) as the reference predicts them, then its constant
    E = energies_matrix_free(Rd, Rdd, f["perms"], 10.0, alphas) * float(f["model__std"])
    np.testing.assert_allclose(E, f["E_pred_c0"], rtol=1e-12)
    c = mdl.recov_int_const(f["E_pred_c0"], f["E"])
    assert c == float(f["model__c"])
    # the reference's refusals
    assert mdl.recov_int_const(-f["E_pred_c0"], f["E"]) is None            # gradients
    assert mdl.recov_int_const(np.random.default_rng(1).standard_normal(M), f["E"]) is None
    assert mdl.recov_int_const(2.0 * f["E_pred_c0"], f["E"]) is None       # scale


def test_store_model_layout(golden_dir, tmp_path):
    from datetime import datetime

    f = load(golden_dir)
    model = {k[len("model__"):]: f[k] for k in f.files if k.startswith("model__")}
    model.update(hardware="mi355x", n_datapoints=23, str_preconditioner="cholesky",
                 f_err={"mae": np.nan, "rmse": np.nan}, md5_test=None)
    out = mdl.store_model(model, tmp_path, now=datetime(2026, 10, 16, 9, 30))
    assert out == (tmp_path / "data_new" / "models" / "mi355x" / "ethanol" / "cholesky" / "n=23"
                   / "k=132" / "2026-10-16_0930.npz")
    back = np.load(out, allow_pickle=True)  # our own file (dict / None fields, as the reference)
    np.testing.assert_array_equal(back["alphas_F"], f["model__alphas_F"])
    assert float(back["c"]) == float(f["model__c"])
    assert back["f_err"].item()["mae"] != back["f_err"].item()["mae"]  # nan


def test_cg_steps_record_schema():
    """create_data.cg_steps' record (create_data.py:116-155) from a model dict."""
    n, k = 120, 30
    model = {"alphas_F": np.zeros(n), "inducing_pts_idxs": np.arange(k), "solver_iters": 40,
             "time_cholesky": np.linspace(1.0, 2.0, k), "total_time_cg": 2.0, "is_conv": True,
             "total_time_preconditioner": 0.5, "total_time_solve": 2.6}
    task = {"dataset_name": "ethanol", "sig": 10, "lam": 1e-10, "solver_tol": 1e-4}
    rec = mdl.cg_steps_record(task, model, 5, k / n, "cholesky")
    t = model["time_cholesky"]
    assert rec["k"] == k and rec["n_kernel"] == n and rec["K.shape"] == (n, n)
    assert rec["cholesky_percentage"] == k / n and rec["cholesky_cgsteps"] == 40
    assert rec["time_cg_step"] == 2.0 / 40
    assert rec["chol_t_correction"] == np.median(t[20:]) / np.median(t[:20]) - 1
    assert rec["lam"] == 1e-10 and rec["n_datapoints"] == 5 and rec["task"] is task
    rec2 = mdl.cg_steps_record(task, model, 5, k / n, "random_scores")
    assert "t_cholesky" not in rec2 and rec2["random_scores_cgsteps"] == 40
    model["is_conv"] = False
    import pytest

    with pytest.raises(RuntimeError):
        mdl.cg_steps_record(task, model, 5, k / n, "cholesky")
