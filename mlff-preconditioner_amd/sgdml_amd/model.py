"""Training entry point and the reference's on-disk model format.

`train(task, ...)` is GDMLTrain.train for solver 'cg' (src/sGDML/sgdml/train.py:707-970)
with the solve on the MI355X: label vector y = F / std(F) (:837-845), lambda = 1e-10
(:866), `Iterative.solve` (the drop-in, :868-890), `create_model` (:597-702),
`model.update(info)` (:938-939) and the integration constant `_recov_int_const`
(:972-1119) from the training-set energies predicted on the GPU
(`mlff_sgdml_energies`, the E part of GDMLPredict, predict.py:172-220).  The returned
dict has the reference model's keys and meanings, so `store_model` (train_models.py
:127-154) writes the same `.npz` that the reference's analysis scripts read.

Not covered (out of the solve path): symmetry compression (`use_cprsn`),
energy constraints (`use_E_cstr`), periodic lattices, the 'analytic' solver.
"""
from __future__ import annotations

import os
import platform
from datetime import datetime
from pathlib import Path

import numpy as np

from .solver import host_descriptors, sgdml_descriptors  # noqa: F401

CODE_VERSION = "0.4.10"  # the sGDML model format the reference writes (sgdml/__init__.py:25)


def desc_perm(perm: np.ndarray) -> np.ndarray:
    """Atom permutation -> permutation of the D = n(n-1)/2 inverse-distance entries
    (Desc.perm, desc.py:360-389): entry (a, b), a > b, at a(a-1)/2 + b, maps to the entry
    of the atom pair {perm[a], perm[b]}."""
    perm = np.asarray(perm, dtype=np.int64)
    n = perm.size
    a, b = np.tril_indices(n, -1)
    pa, pb = perm[a], perm[b]
    hi, lo = np.maximum(pa, pb), np.minimum(pa, pb)
    return hi * (hi - 1) // 2 + lo


def tril_perms_lin(perms: np.ndarray) -> np.ndarray:
    """train.py:783-790: the descriptor permutations of all symmetries, offset by
    p * D and interleaved ('F' order) as GDMLTrain passes them to the solvers."""
    perms = np.atleast_2d(np.asarray(perms))
    n_perms, n = perms.shape
    D = n * (n - 1) // 2
    tril = np.array([desc_perm(p) for p in perms])
    return (tril + np.arange(n_perms)[:, None] * D).flatten("F")


def r_d_desc_alpha(R_d_desc: np.ndarray, alphas_F: np.ndarray) -> np.ndarray:
    """create_model's Jacobian-coefficient product (train.py:642-649):
    sum_c R_d_desc[k, d, c] (alpha_k[t_d, c] - alpha_k[s_d, c]), pair d = (s > t)."""
    n_train, D = R_d_desc.shape[:2]
    n_atoms = int((1 + np.sqrt(8 * D + 1)) / 2)
    s, t = np.tril_indices(n_atoms, k=-1)
    a = np.asarray(alphas_F).reshape(-1, n_atoms, 3)
    return np.einsum("kji,kji->kj", R_d_desc, a[:, t, :] - a[:, s, :])


def create_model(task, solver, R_desc, R_d_desc, tril_perms_lin_, std, alphas_F, alphas_E=None,
                 solver_resid=None, solver_iters=None, norm_y_train=None,
                 inducing_pts_idxs=None):
    """GDMLTrain.create_model (train.py:597-702)."""
    if "cprsn_keep_atoms_idxs" in task:
        raise NotImplementedError("symmetry compression (use_cprsn) is not supported")
    model = {
        "type": "m",
        "code_version": CODE_VERSION,
        "dataset_name": task["dataset_name"],
        "dataset_theory": task["dataset_theory"],
        "solver_name": solver,
        "solver_tol": task["solver_tol"],
        "norm_y_train": norm_y_train,
        "n_inducing_pts_init": task["n_inducing_pts_init"],
        "z": task["z"],
        "idxs_train": task["idxs_train"],
        "md5_train": task["md5_train"],
        "idxs_valid": task["idxs_valid"],
        "md5_valid": task["md5_valid"],
        "n_test": 0,
        "md5_test": None,
        "f_err": {"mae": np.nan, "rmse": np.nan},
        "R_desc": np.asarray(R_desc).T,
        "R_d_desc_alpha": r_d_desc_alpha(np.asarray(R_d_desc), alphas_F),
        "interact_cut_off": task["interact_cut_off"],
        "c": 0.0,
        "std": std,
        "sig": task["sig"],
        "lam": task["lam"],
        "alphas_F": alphas_F,
        "perms": task["perms"],
        "tril_perms_lin": tril_perms_lin_,
        "use_E": task["use_E"],
        "use_cprsn": task["use_cprsn"],
    }
    if solver_resid is not None:
        model["solver_resid"] = solver_resid
    if solver_iters is not None:
        model["solver_iters"] = solver_iters
    if inducing_pts_idxs is not None:
        model["inducing_pts_idxs"] = inducing_pts_idxs
    if task["use_E"]:
        model["e_err"] = {"mae": np.nan, "rmse": np.nan}
        if task.get("use_E_cstr", False):
            model["alphas_E"] = alphas_E
    if "lattice" in task:
        model["lattice"] = task["lattice"]
    if "r_unit" in task and "e_unit" in task:
        model["r_unit"] = task["r_unit"]
        model["e_unit"] = task["e_unit"]
    return model


def recov_int_const(E_pred: np.ndarray, E_ref: np.ndarray):
    """The decision and estimate of GDMLTrain._recov_int_const (train.py:972-1119) given
    the predicted training-set energies (c = 0): None when the labels look like
    gradients (negative scale), are inconsistent (correlation < 0.95) or scaled (|scale
    - 1| > 0.1); otherwise the least-squares constant mean(E_ref - E_pred)."""
    E_pred = np.asarray(E_pred, dtype=np.float64)
    E_ref = np.squeeze(np.asarray(E_ref, dtype=np.float64))
    e_fact = np.linalg.lstsq(np.column_stack((E_pred, np.ones(E_ref.shape))), E_ref,
                             rcond=-1)[0][0]
    corrcoef = np.corrcoef(E_ref, E_pred)[0, 1]
    if np.sign(e_fact) == -1:
        return None
    if corrcoef < 0.95:
        return None
    if np.abs(e_fact - 1) > 1e-1:
        return None
    return np.sum(E_ref - E_pred) / E_ref.shape[0]


class _ModelFactory:
    """Stands in for GDMLTrain where the solver's checkpoint needs create_model."""

    create_model = staticmethod(create_model)


def train(task, cprsn_callback=None, save_progr_callback=None, callback=None,
          break_percentage=0.1, n_columns=None, str_preconditioner="", flag_eigvals=False,
          device=None, devices=None, gdml_train=None):
    """GDMLTrain.train (train.py:707-970) for solver 'cg' on the MI355X."""
    from .solvers import Iterative

    task = dict(task)
    solver_name = task["solver_name"]
    if solver_name != "cg":
        raise NotImplementedError(f"solver '{solver_name}': only the iterative 'cg' path runs here")
    if task.get("use_cprsn", False) or "lattice" in task:
        raise NotImplementedError("symmetry compression / periodic lattices are not supported")
    if task.get("use_E", False) and task.get("use_E_cstr", False):
        # as the reference's train -> Iterative.solve (see Iterative.solve)
        raise ValueError("use_E_cstr: the reference's iterative solve cannot run with energy "
                         "constraints (operator sized 3 n M, labels 3 n M + M)")
    n_train, n_atoms = task["R_train"].shape[:2]
    perms = np.atleast_2d(np.asarray(task["perms"]))
    tpl = tril_perms_lin(perms)
    # the descriptors as the reference's trainer forms them, on the host (Desc.from_R): the
    # reference's system bit for bit (sgdml_descriptors forms them on the GPU, equal to rounding)
    R_desc, R_d_desc = host_descriptors(np.asarray(task["R_train"], dtype=np.float64))
    y = task["F_train"].ravel().copy()                    # train.py:837-845
    y_std = np.std(y)
    y /= y_std
    if n_columns is not None:
        break_percentage = n_columns / len(y)
    assert 0 <= break_percentage <= 1, "break_percentage is too large"
    task["lam"] = 1e-10                                   # train.py:866
    # the 2-minute progress checkpoint of the solver builds its model with create_model
    it = Iterative(gdml_train or _ModelFactory(), None, callback=callback, device=device,
                   devices=devices)
    with it:  # the device contexts are released on every exit path
        alphas, num_iters, resid, train_rmse, inducing_pts_idxs, is_conv, info = it.solve(
            task, R_desc, R_d_desc, tpl, y, y_std, save_progr_callback=save_progr_callback,
            break_percentage=break_percentage, str_preconditioner=str_preconditioner,
            flag_eigvals=flag_eigvals)
        model = create_model(task, "cg", R_desc, R_d_desc, tpl, y_std, alphas,
                             solver_resid=resid, solver_iters=num_iters,
                             norm_y_train=np.linalg.norm(y), inducing_pts_idxs=inducing_pts_idxs)
        model.update(info)
        if model["use_E"]:
            _, E = it.solver.sgdml_energies(alphas)
            c = recov_int_const(E * y_std, task["E_train"])
            if c is None:
                model["use_E"] = False
            else:
                model["c"] = c
    return model


def train_model(task, name_dataset: str, n_datapoints: int, preconditioner: str,
                hardware: str = "mi355x", devices=None) -> dict:
    """The solve part of src/train_models.py:train_model (:68-124) for a task the caller
    built (dataset download and GDMLTrain.create_task stay with the reference):
    rule-of-thumb preconditioner size (:95-97), train, and the bookkeeping keys
    store_model and the analysis scripts read (:104-113)."""
    import timeit

    from .rule_of_thumb import get_params, rule_of_thumb

    task = dict(task)
    task["truncated_cholesky"] = 1500
    task["str_preconditioner"] = preconditioner
    n = task["F_train"].size
    m, k_min, _ = get_params(name_dataset)
    k_rot = int(rule_of_thumb(n=n, k_min=k_min, m=m))
    strength = k_rot / n
    t0 = timeit.default_timer()
    model = train(task, break_percentage=strength, str_preconditioner=preconditioner,
                  devices=devices)
    model["solver_runtime_s"] = timeit.default_timer() - t0
    model["truncated_cholesky"] = 1500
    model["str_preconditioner"] = preconditioner
    model["n_datapoints"] = n_datapoints
    model["kernel_size"] = n
    model["preconditioner_strength"] = strength
    model["task"] = task
    model["hardware"] = hardware
    return model


def store_model(model: dict, path_to_script: str | os.PathLike, now: datetime | None = None) -> Path:
    """src/train_models.py:127-154: data_new/models/<hardware>/<dataset>/<precon>/n=<n>/k=<k>/
    <date>_<HHMM>.npz via np.savez_compressed(**model) (model['hardware'],
    ['n_datapoints'] and ['str_preconditioner'] as train_model sets them)."""
    now = now or datetime.now()
    name_dataset = str(model["dataset_name"])
    folder = Path(os.path.abspath(path_to_script)) / "data_new" / "models" / model["hardware"] / name_dataset
    solver = model["solver_name"]
    file_name = f"{now.date()}_{now.strftime('%H%M')}.pickle"
    if solver == "analytic":
        path = folder / "analytic" / f"n={model['n_datapoints']}" / file_name
    elif solver == "cg":
        k = np.asarray(model["inducing_pts_idxs"]).size
        path = folder / model["str_preconditioner"] / f"n={model['n_datapoints']}" / f"k={k}" / file_name
    else:
        raise ValueError(f"solver = {solver}")
    model["platform"] = platform.uname()
    path.parent.mkdir(exist_ok=True, parents=True)
    out = path.with_suffix(".npz")
    np.savez_compressed(out, **model)
    return out


CG_STEPS_INFO_KEYS = ("dataset_name", "sig", "lam", "solver_tol")  # create_data.py:20


def cg_steps_record(task: dict, model: dict, n_datapoints: int, preconditioner_strength: float,
                    preconditioner: str, flag_eigvals: bool = False) -> dict:
    """The measurement dict of tools/create_data.cg_steps (create_data.py:100-155) from a
    trained model: Cholesky step timings and their begin/end medians (:123-131), the
    preconditioner size actually used (:116-120), CG step count and the solver's timings
    (:142-149), the task and its info keys (:150-152)."""
    n = len(model["alphas_F"])
    actual = len(model["inducing_pts_idxs"]) / n
    k = int(actual * n)
    rec: dict = {}
    if preconditioner == "cholesky":
        t = np.asarray(model["time_cholesky"])
        t_begin, t_end = np.median(t[:20]), np.median(t[20:])
        rec["t_cholesky"] = t
        rec["time_cg_step"] = model["total_time_cg"] / model["solver_iters"]
        rec["chol_t_begin"] = t_begin
        rec["chol_t_end"] = t_end
        rec["chol_t_correction"] = t_end / t_begin - 1
    if flag_eigvals:  # create_data.py:133-135
        rec[f"eigvals_{preconditioner}_{preconditioner_strength * 100:.2f}"] = model["eigvals"]
        rec[f"eigvals_{preconditioner}_{0}"] = model["eigvals_K"]
    if model["is_conv"] is False and flag_eigvals is False:  # :137 (not for eigvals runs)
        raise RuntimeError("Solver is not converged.")
    rec[f"{preconditioner}_percentage"] = actual
    rec[f"{preconditioner}_cgsteps"] = model["solver_iters"]
    rec["K.shape"] = (n, n)
    rec["n_kernel"] = n
    rec["k"] = k
    for key in ("total_time_preconditioner", "total_time_solve", "total_time_cg"):
        rec[key] = model[key]
    rec["task"] = task
    for label in CG_STEPS_INFO_KEYS:
        rec[label] = task[label]
    rec["platform"] = platform.uname()
    rec["n_datapoints"] = n_datapoints
    return rec


def cg_steps(task: dict, n_datapoints: int, preconditioner_strength: float, preconditioner: str,
             flag_eigvals: bool = False, path_to_script: str | os.PathLike = "",
             devices=None, now: datetime | None = None) -> Path:
    """tools/create_data.cg_steps (create_data.py:100-168) with the solve on the MI355X:
    trains with `truncated_cholesky` = 1500, then pickles the record to
    data_new/<dataset>/<precon>/n = <n>/<date>_<HHMM>_k = <k>.pickle, the file
    scripts/main_plot.py reads."""
    import pickle

    task = dict(task)
    task["truncated_cholesky"] = 1500
    task["str_preconditioner"] = preconditioner
    model = train(task, break_percentage=preconditioner_strength, callback=lambda *a, **kw: None,
                  str_preconditioner=preconditioner, flag_eigvals=flag_eigvals, devices=devices)
    rec = cg_steps_record(task, model, n_datapoints, preconditioner_strength, preconditioner,
                          flag_eigvals)
    now = now or datetime.now()
    folder = (Path(os.path.abspath(path_to_script)) / "data_new" / str(task["dataset_name"])
              / preconditioner / f"n = {n_datapoints}")
    folder.mkdir(exist_ok=True, parents=True)
    path = folder / f"{now.date()}_{now.strftime('%H%M')}_k = {rec['k']}.pickle"
    with open(path, "wb") as fh:
        pickle.dump(rec, fh)
    return path
