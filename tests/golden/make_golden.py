"""Generate the golden fixtures of tests/golden/ by running the REFERENCE itself.

Run in the development container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden.py [--only NAME ...]

The reference (bluecher31/mlff-preconditioner, Python) is imported from
/root/reference with four behaviour-preserving shims for the newer NumPy/SciPy of
this image:
  1. np.int = int                         (desc.py:260 uses the removed alias)
  2. scipy.linalg.eigh(eigvals=(a,b))  -> subset_by_index=[a,b]   (iterative_solver.py:577)
  3. scipy.sparse.linalg.cg            -> a transliteration of scipy 1.7.3's cg
     (pinned by environment.yml:11): python reverse-communication driver + the
     CGREVCOM Fortran state machine, with the caller-frame local `resid` that
     _cg_status reads (iterative_solver.py:884); it also records ||r_k||.
  4. GDMLPredict.prepare_parallel -> no-op (it writes a cache file into the
     read-only package directory, predict.py:895-925).
Only inputs and outputs are written (npz, allow_pickle=False).  Nothing from the
reference is copied into this repository.
"""
from __future__ import annotations

import argparse
import inspect
import os
import sys
import time
from pathlib import Path

sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path("/root/reference")
sys.path[:0] = [str(REPO / "mlff-preconditioner_amd")]

import numpy as np  # noqa: E402
import scipy  # noqa: E402
import scipy.linalg  # noqa: E402
import scipy.sparse.linalg  # noqa: E402
from scipy.sparse.linalg._isolve.utils import make_system  # noqa: E402

# ---------------------------------------------------------------- shim 1
np.int = int  # type: ignore[attr-defined]

# ---------------------------------------------------------------- shim 2
_eigh = scipy.linalg.eigh


def _eigh_compat(a, *args, eigvals=None, **kw):
    if eigvals is not None:
        kw["subset_by_index"] = [int(eigvals[0]), int(eigvals[1])]
    return _eigh(a, *args, **kw)


scipy.linalg.eigh = _eigh_compat

# ---------------------------------------------------------------- shim 3
TRACE: list[float] = []


def _cgrevcom_1_7_3(b, x, maxit, tol):
    """Generator transliterating scipy 1.7.3 CGREVCOM.f.src.  Yields requests
    (ijob, ITER) and receives the stop-test INFO after ijob 4."""
    n = b.size
    work = {"R": b.copy(), "Z": np.zeros(n), "P": np.zeros(n), "Q": np.zeros(n)}
    it = maxit  # ITER keeps MAXIT until label 2 resets it
    if np.linalg.norm(x) != 0.0:
        yield 3, it, work  # R = R - A x
    if np.linalg.norm(work["R"]) < tol:
        return 0, it
    it = 0
    rho1 = None
    while True:
        it += 1
        yield 2, it, work  # Z = M R   (PSOLVE)
        rho = float(np.dot(work["R"], work["Z"]))
        if it > 1:
            beta = rho / rho1
            work["Z"] = work["Z"] + beta * work["P"]
            work["P"] = work["Z"].copy()
        else:
            work["P"] = work["Z"].copy()
        yield 1, it, work  # Q = A P   (MATVEC)
        alpha = rho / float(np.dot(work["P"], work["Q"]))
        x += alpha * work["P"]
        work["R"] = work["R"] + (-alpha) * work["Q"]
        info = yield 4, it, work  # stop test
        if info == 1:
            return 0, it
        if it == maxit:
            return 1, it
        rho1 = rho


def cg_scipy_1_7_3(A, b, x0=None, tol=1e-05, maxiter=None, M=None, callback=None, atol=None):
    A, M, x, b, postprocess = make_system(A, M, x0, b)
    n = len(b)
    if maxiter is None:
        maxiter = n * 10
    matvec = A.matvec
    psolve = M.matvec
    bnrm2 = np.linalg.norm(b)
    # _get_atol, legacy mode
    if atol is None:
        resid0 = np.linalg.norm(matvec(x) - b)
        if resid0 <= tol:
            TRACE[:] = [resid0]
            return postprocess(x), 0
        atol = tol if bnrm2 == 0 else tol * float(bnrm2)
    else:
        atol = max(float(atol), tol * float(bnrm2))
    resid = atol
    TRACE[:] = []
    gen = _cgrevcom_1_7_3(b, x, maxiter, atol)
    iter_ = maxiter
    info = 0
    send = None
    while True:
        olditer = iter_
        try:
            ijob, iter_, work = gen.send(send)
        except StopIteration as stop:
            code, iter_ = stop.value
            info = 0 if code == 0 else 1
            if callback is not None:
                callback(x)
            break
        send = None
        if callback is not None and iter_ > olditer:
            callback(x)
        if ijob == 1:
            work["Q"] = matvec(work["P"])
        elif ijob == 2:
            work["Z"] = psolve(work["R"])
        elif ijob == 3:
            if not TRACE:
                pass
            work["R"] = work["R"] + (-1.0) * matvec(x)
        elif ijob == 4:
            resid = np.linalg.norm(work["R"])
            info4 = 1 if resid <= atol else 0
            if info4 == 1 and iter_ > 1:
                work["R"] = b - matvec(x)
                resid = np.linalg.norm(work["R"])
                info4 = 1 if resid <= atol else 0
            TRACE.append(float(resid))
            send = info4
    if info > 0 and iter_ == maxiter and not (resid <= atol):
        info = iter_
    return postprocess(x), info


scipy.sparse.linalg.cg = cg_scipy_1_7_3

# ------------------------------------------------------------ import the reference
sys.path += [str(REF / "src" / "sGDML"), str(REF / "src")]
import sgdml.predict  # noqa: E402

sgdml.predict.GDMLPredict.prepare_parallel = lambda self, *a, **k: None  # shim 4
import sgdml.train  # noqa: E402
from sgdml.solvers import incomplete_cholesky, iterative_cholesky, iterative_solver  # noqa: E402
from sgdml.utils.desc import Desc  # noqa: E402

sys.path.insert(0, str(REF / "src"))
from tools import plot_data  # noqa: E402
from tools import utils as tools_utils  # noqa: E402

from sgdml_amd import synthetic  # noqa: E402  (input generation only)

_TRAIN = None


def gdml_train():
    global _TRAIN
    if _TRAIN is None:
        _TRAIN = sgdml.train.GDMLTrain(max_processes=1)
    return _TRAIN


def make_task(ds, perms=None, dataset_name="ethanol", solver_tol=1e-4):
    M, n = ds["R"].shape[:2]
    return {
        "type": "t", "dataset_name": np.array(dataset_name), "dataset_theory": np.array("synthetic"),
        "z": ds["z"], "R_train": ds["R"], "F_train": ds["F"], "E_train": ds["E"],
        "idxs_train": np.arange(M), "md5_train": "0", "idxs_valid": np.arange(0),
        "md5_valid": "0", "sig": 10, "lam": 1e-10, "use_E": True, "use_E_cstr": False,
        "use_sym": perms is not None, "use_cprsn": False, "solver_name": "cg",
        "solver_tol": solver_tol, "n_inducing_pts_init": 25, "interact_cut_off": None,
        "perms": np.arange(n)[None, :] if perms is None else np.asarray(perms),
        "truncated_cholesky": 1500,
    }


def prepare(task):
    """train.py:775-845 (descriptors, tril_perms_lin, y)."""
    n_train, n_atoms = task["R_train"].shape[:2]
    desc = Desc(n_atoms, interact_cut_off=None, max_processes=1)
    n_perms = task["perms"].shape[0]
    tril_perms = np.array([desc.perm(p) for p in task["perms"]])
    perm_offsets = np.arange(n_perms)[:, None] * desc.dim
    tril_perms_lin = (tril_perms + perm_offsets).flatten("F")
    R = task["R_train"].reshape(n_train, -1)
    R_desc, R_d_desc = desc.from_R(R, lat_and_inv=None, callback=None)
    y = task["F_train"].ravel().copy()
    y_std = np.std(y)
    y /= y_std
    return desc, tril_perms_lin, R_desc, R_d_desc, y, y_std


def noop(*a, **k):
    pass


def run_solver(task, desc, tril_perms_lin, R_desc, R_d_desc, y, y_std, precon, bp, seed,
               flag_eigvals=False):
    """Iterative.solve exactly as GDMLTrain.train calls it (train.py:859-890)."""
    iterative_solver.glob_U = None
    iterative_solver.glob_s = None
    iterative_solver.global_type_delet = None
    task = dict(task)
    task["str_preconditioner"] = precon
    np.random.seed(seed)
    it = iterative_solver.Iterative(gdml_train(), desc, callback=noop, max_processes=1, use_torch=False)
    t0 = time.time()
    out = it.solve(task, R_desc, R_d_desc, tril_perms_lin, y, y_std, save_progr_callback=None,
                   break_percentage=bp, str_preconditioner=precon, flag_eigvals=flag_eigvals)
    alphas, num_iters, resid, train_rmse, idxs, is_conv, info = out
    res = {
        "alphas": np.asarray(alphas), "num_iters": np.int64(num_iters), "resid": np.float64(resid),
        "train_rmse": np.float64(train_rmse), "inducing_pts_idxs": np.asarray(idxs, dtype=np.int64),
        "is_conv": np.bool_(is_conv), "trace": np.array(TRACE), "seconds": np.float64(time.time() - t0),
    }
    if precon == "cholesky":
        res["index_columns"] = np.asarray(info["index_columns"], dtype=np.int64)
    if flag_eigvals:
        res["eigvals"] = np.asarray(info["eigvals"])
        res["eigvals_K"] = np.asarray(info["eigvals_K"])
    return res


def run_direct_cg(K_op_neg, y, tol, maxiter):
    """Unpreconditioned legacy cg on -K_op (tools/utils.py:139-143 'direct CG')."""
    calls = [0]

    def cb(xk):
        calls[0] += 1

    x, info = scipy.sparse.linalg.cg(K_op_neg, y, tol=tol, atol=None, maxiter=maxiter, callback=cb)
    return {"x": x, "info": np.int64(info), "trace": np.array(TRACE), "callbacks": np.int64(calls[0])}


def kernel_operator(task, desc, R_desc, R_d_desc, tril_perms_lin, n):
    it = iterative_solver.Iterative(gdml_train(), desc, callback=noop, max_processes=1, use_torch=False)
    K_op = it._init_kernel_operator(task, R_desc, R_d_desc, tril_perms_lin, task["lam"], n,
                                    callback=None)
    return it, K_op


def save(name, **arrays):
    path = HERE / f"{name}.npz"
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({path.stat().st_size / 1024:.0f} KiB)", flush=True)


# ----------------------------------------------------------------------- fixtures
def fx_descriptors():
    ds = synthetic.ethanol_like(4, seed=11)
    desc = Desc(9, interact_cut_off=None, max_processes=1)
    R_desc, R_d_desc = desc.from_R(ds["R"].reshape(4, -1))
    perm = np.array([0, 1, 2, 4, 5, 3, 7, 6, 8])
    save("descriptors_ethanol", R=ds["R"], R_desc=R_desc, R_d_desc=R_d_desc, perm=perm,
         desc_perm=desc.perm(perm), d_desc_full=desc.d_desc_from_comp(R_d_desc[0])[0])


def fx_rule_of_thumb():
    names = ["ethanol", "uracil", "toluene", "aspirin", "azobenzene", "catcher", "nanotube"]
    ns = [270, 621, 2997, 15540, 65536]
    table = np.array([[plot_data.rule_of_thumb(n=n, k_min=plot_data.get_params(nm)[1],
                                               m=plot_data.get_params(nm)[0]) for n in ns]
                      for nm in names], dtype=np.int64)
    params = np.array([plot_data.get_params(nm)[:2] for nm in names], dtype=np.float64)
    save("rule_of_thumb", names=np.array(names), ns=np.array(ns), k=table, params=params)


def fx_rbf():
    """tools/utils.create_kernel_mat (sklearn RBF, l = 1, d = 2, + 1e-10 I) and the
    reference pivoted Cholesky / Woodbury preconditioner on it."""
    n = 300
    np.random.seed(0)
    K, f = tools_utils.create_kernel_mat(n=n, dim=2)
    np.random.seed(0)
    X = np.random.random_sample((n, 2))
    k = 12
    L, index_columns, _ = incomplete_cholesky.pivoted_cholesky(
        get_col=lambda i: K[:, i].copy(), diagonal=np.diag(K).copy(), max_rank=k)
    # ell = 0.2 in 3-d: a better conditioned SPD kernel, Woodbury preconditioner via the
    # reference's IterativeCholesky._init_precon_operator on a dense operator
    rng = np.random.default_rng(1)
    X3 = rng.random((n, 3))
    import sklearn.gaussian_process as gp

    K3 = gp.kernels.RBF(length_scale=0.2)(X3)
    lam = 1e-6
    task = {"R_train": np.zeros((n // 3, 1, 3))}
    ic = iterative_cholesky.Iterative(gdml_train(), None, task)
    K_op = scipy.sparse.linalg.LinearOperator((n, n), matvec=lambda v: K3 @ v + lam * v)
    k3 = 40
    P_op, info = ic._init_precon_operator(np.diag(K3).copy(), K_op, lam_regularization=lam,
                                          break_percentage=k3 / n)
    r = rng.standard_normal(n)
    z = P_op.matvec(r)
    save("rbf_reference", X=X, K=K, f=f, k=np.int64(k), L=L, index_columns=index_columns,
         X3=X3, K3=K3, lam=np.float64(lam), k3=np.int64(k3),
         index_columns3=np.asarray(info["index_columns"], dtype=np.int64), r=r, z=z)


def _nystrom_apply(it, task, R_desc, R_d_desc, tril_perms_lin, idx, variant, r):
    if variant == 0:
        P_op = it._init_precon_operator(task, R_desc, R_d_desc, tril_perms_lin, idx, callback=noop)
    else:
        P_op = it._init_precon_operator_sb(task, R_desc, R_d_desc, tril_perms_lin, idx, callback=noop)
    return P_op.matvec(r)


def fx_sgdml(M, name, precons, seed=3, perms=None, with_K=True, none_tol=(1e-4,), geom="ethanol",
             k_rows=64):
    """geom: 'ethanol' (9 atoms) or 'nanotube' (370 atoms, D = 68265: descriptors are not
    stored, the consumer recomputes them from R with its own tested descriptor code)."""
    ds = (synthetic.ethanol_like if geom == "ethanol" else synthetic.nanotube_like)(M, seed=seed)
    task = make_task(ds, perms=perms, dataset_name=geom)
    desc, tpl, R_desc, R_d_desc, y, y_std = prepare(task)
    n = y.size
    out = {"R": ds["R"], "F": ds["F"], "E": ds["E"], "z": ds["z"], "perms": task["perms"],
           "tril_perms_lin": tpl, "y": y,
           "y_std": np.float64(y_std), "sig": np.float64(10.0), "lam": np.float64(1e-10),
           "solver_tol": np.float64(task["solver_tol"])}
    if geom == "ethanol":
        out["R_desc"], out["R_d_desc"] = R_desc, R_d_desc
    K = gdml_train()._assemble_kernel_mat(R_desc, R_d_desc, tpl, 10, desc, use_E_cstr=False,
                                          col_idxs=np.s_[:], callback=noop)
    if with_K:
        out["K"] = np.array(K)
    else:  # too large to commit: keep a row sample for the assembly check
        out["K_rows"] = np.array(K[:k_rows])
    # operator and preconditioner applies on a fixed vector
    it, K_op = kernel_operator(task, desc, R_desc, R_d_desc, tpl, n)
    rng = np.random.default_rng(seed + 100)
    v = rng.standard_normal(n)
    out["v"] = v
    out["Kop_v"] = K_op.matvec(v)        # K_asm v - lam v (matrix-free)
    ic = iterative_cholesky.Iterative(gdml_train(), desc, task)
    out["diag_K"] = ic._assemble_kernel_mat_diag(tril_perms_lin=tpl, sig=10, R_desc=R_desc,
                                                 R_d_desc=R_d_desc, n=n)
    k_app = max(8, n // 10)
    idx = np.sort(rng.choice(n, k_app, replace=False))
    out["nys_idx"] = idx
    for variant in (0, 1):
        try:
            out[f"nys{variant}_z"] = _nystrom_apply(it, dict(task, lam=1e-10), R_desc, R_d_desc, tpl,
                                                    idx, variant, v)
        except np.linalg.LinAlgError as e:  # the reference raises: record it
            out[f"nys{variant}_error"] = np.array(type(e).__name__)
    # solves at the boundary (Iterative.solve)
    m, kmin, _ = plot_data.get_params(geom)
    k_rot = int(plot_data.rule_of_thumb(n=n, k_min=kmin, m=m))
    bp = k_rot / n
    out["k_rot"] = np.int64(k_rot)
    for p in precons:
        t0 = time.time()
        try:
            res = run_solver(task, desc, tpl, R_desc, R_d_desc, y, y_std, p, bp, seed=1000 + seed)
        except (np.linalg.LinAlgError, AssertionError) as e:
            out[f"{p}__error"] = np.array(type(e).__name__)
            print(f"  {name} {p}: reference raised {type(e).__name__}: {e}", flush=True)
            continue
        for key, val in res.items():
            out[f"{p}__{key}"] = val
        print(f"  {name} {p}: iters={res['num_iters']} resid={res['resid']:.3e} "
              f"({time.time() - t0:.1f}s)", flush=True)
    for tol in none_tol:
        t0 = time.time()
        _, K_op2 = kernel_operator(task, desc, R_desc, R_d_desc, tpl, n)
        res = run_direct_cg(-K_op2, y, tol, 5 * n)
        tag = f"none_{tol:.0e}"
        for key, val in res.items():
            out[f"{tag}__{key}"] = val
        print(f"  {name} none tol={tol}: info={res['info']} callbacks={res['callbacks']} "
              f"iters={len(res['trace'])} ({time.time() - t0:.1f}s)", flush=True)
    # the revcom transliteration on the dense operator (-K + lam I): the oracle's own
    # CG loop must reproduce it bit for bit (two independent restatements of scipy 1.7.3)
    A = scipy.sparse.linalg.LinearOperator((n, n), matvec=lambda v: -(K @ v) + 1e-10 * v,
                                           dtype=np.float64)
    xd, infod = scipy.sparse.linalg.cg(A, y, tol=1e-4, atol=None, maxiter=min(5 * n, 400))
    out["dense_none__x"] = xd
    out["dense_none__info"] = np.int64(infod)
    out["dense_none__trace"] = np.array(TRACE)
    save(name, **out)


def fx_lev_scores():
    """_lev_scores with the approximating columns recorded (np.random replay)."""
    ds = synthetic.ethanol_like(12, seed=21)
    task = make_task(ds)
    desc, tpl, R_desc, R_d_desc, y, y_std = prepare(task)
    n = y.size
    it, _ = kernel_operator(task, desc, R_desc, R_d_desc, tpl, n)
    n_inducing = 8
    dim_i = 27
    dim_m = max(1, n_inducing // 4) * dim_i
    np.random.seed(77)
    cols = np.sort(np.random.choice(12 * dim_i, dim_m, replace=False))
    np.random.seed(77)
    lev, order = it._lev_scores(R_desc, R_d_desc, tpl, 10, 1e-10, False, n_inducing,
                                callback=lambda *a, **k: None)
    K = gdml_train()._assemble_kernel_mat(R_desc, R_d_desc, tpl, 10, desc, use_E_cstr=False,
                                          col_idxs=np.s_[:], callback=noop)
    save("lev_scores_ethanol", R=ds["R"], K=np.array(K), cols=cols, lev=lev, order=order,
         lam=np.float64(1e-10))


def fx_cho_stable():
    """_cho_factor_stable's eigenvalue sign test (iterative_solver.py:555-583) on a nearly
    singular K_mm: ethanol-like M = 10 plus a copy of geometry 0 moved by `delta` (point 10),
    27 inducing columns that hold 4 columns of point 0 and the same 4 of its copy.  The
    smallest eigenvalue of -K_mm then shrinks like delta^2: delta = 3e-7 puts it in
    (0, 1e-15), where the reference shifts by -1e-15 and its Cholesky fails (LinAlgError from
    the Nystrom build and from _lev_scores); delta = 1e-6 / 1e-5 put it just above 1e-15 /
    well above; delta = 0 is an exact duplicate (lo_eig at the rounding level: recorded, not
    a parity case).  Recorded per delta: the reference's K_mm (from its own column-panel
    assembly, :112-124), lo_eig of -K_mm (eigh as at :577), the Nystrom variant-0 apply P_op v
    (:95-322) or its exception, the _lev_scores output (:447-552, the columns forced through
    idxs_ordered_by_lev_score) or its exception, and the oracle's apply distance to the
    reference's (the NumPy restatement's own rounding spread)."""
    if str(REPO) not in sys.path:
        sys.path.append(str(REPO))
    from oracle.precon import apply_panel, nystrom_panel

    pairs = [0, 1, 5, 13]
    other = np.linspace(27, 269, 19).astype(np.int64)
    idx = np.sort(np.r_[pairs, [270 + i for i in pairs], other]).astype(np.int64)
    assert idx.size == 27 and np.unique(idx).size == 27
    out = {"idx": idx, "deltas": np.array([0.0, 3e-7, 1e-6, 1e-5])}
    for t, delta in enumerate(out["deltas"]):
        ds = synthetic.ethanol_like(10, seed=3)
        shift = np.random.default_rng(9).standard_normal(ds["R"][0].shape)
        for key in ("R", "F", "E"):
            ds[key] = np.concatenate([ds[key], ds[key][:1]])
        ds["R"][10] = ds["R"][10] + delta * shift
        task = make_task(ds)
        desc, tpl, R_desc, R_d_desc, y, y_std = prepare(task)
        n = y.size
        K_nm = gdml_train()._assemble_kernel_mat(R_desc, R_d_desc, tpl, 10, desc, use_E_cstr=False,
                                                 col_idxs=idx, callback=noop)
        M = -np.array(K_nm)[idx, :]
        lo = float(scipy.linalg.eigh(M, eigvals_only=True, eigvals=(0, 0))[0])
        it, _ = kernel_operator(task, desc, R_desc, R_d_desc, tpl, n)
        v = np.random.default_rng(31).standard_normal(n)
        out[f"R_{t}"], out[f"Kmm_{t}"], out[f"lo_eig_{t}"] = ds["R"], M, np.float64(lo)
        out[f"v_{t}"] = v
        try:
            z = _nystrom_apply(it, dict(task, lam=1e-10), R_desc, R_d_desc, tpl, idx, 0, v)
            out[f"nys0_z_{t}"] = z
            B, sp = nystrom_panel(-np.array(K_nm), idx, 1e-10, 0)
            zo = apply_panel(B, sp, 1e-10, v)
            out[f"nys0_oracle_rel_{t}"] = np.float64(np.linalg.norm(zo - z) / np.linalg.norm(z))
        except np.linalg.LinAlgError as e:
            out[f"nys0_error_{t}"] = np.array(type(e).__name__)
        order = np.r_[np.setdiff1d(np.arange(n), idx), idx]  # the last dim_m = 27 are idx
        try:
            lev, _ = it._lev_scores(R_desc, R_d_desc, tpl, 10, 1e-10, False, 4,
                                    idxs_ordered_by_lev_score=order,
                                    callback=lambda *a, **k: None)
            out[f"lev_{t}"] = lev
        except np.linalg.LinAlgError as e:
            out[f"lev_error_{t}"] = np.array(type(e).__name__)
        print(f"  delta={delta:.0e} lo_eig={lo:.3e} nys0={'z' if f'nys0_z_{t}' in out else 'error'} "
              f"lev={'ok' if f'lev_{t}' in out else 'error'}", flush=True)
    save("cho_stable_ethanol", **out)


def fx_model():
    """GDMLTrain.train end to end for solver 'cg' (train.py:707-970: label normalisation,
    lam = 1e-10, Iterative.solve, create_model :597-702, model.update(info),
    _recov_int_const :972-1119) on harmonic-labelled ethanol geometries (energies the
    forces integrate to), plus the reference's training-set energy prediction with c = 0
    (GDMLPredict.predict, predict.py:997-1110) that the constant is regressed on."""
    from sgdml.predict import GDMLPredict

    M = 23
    ds = synthetic.ethanol_harmonic(M, seed=13)
    task = make_task(ds)
    desc, tpl, R_desc, R_d_desc, y, y_std = prepare(task)
    n = y.size
    m, kmin, _ = plot_data.get_params("ethanol")
    k_rot = int(plot_data.rule_of_thumb(n=n, k_min=kmin, m=m))
    np.random.seed(2024)
    model = gdml_train().train(task, callback=noop, break_percentage=k_rot / n,
                               str_preconditioner="cholesky")
    gdml = GDMLPredict(dict(model, c=0.0), max_processes=1)
    E_pred, F_pred = gdml.predict(task["R_train"].reshape(M, -1), R_desc=R_desc, R_d_desc=R_d_desc)
    out = {"R": ds["R"], "F": ds["F"], "E": ds["E"], "z": ds["z"], "perms": task["perms"],
           "k_rot": np.int64(k_rot), "E_pred_c0": np.asarray(E_pred), "F_pred_c0": np.asarray(F_pred),
           "model_keys": np.array(sorted(model.keys()))}
    for key, val in model.items():
        if isinstance(val, dict) or val is None:
            continue
        if isinstance(val, (str, np.str_)):
            out[f"model__{key}"] = np.array(str(val))
        elif isinstance(val, tuple):
            out[f"model__{key}"] = np.asarray(val)
        else:
            a = np.asarray(val)
            if a.dtype == object:
                continue
            out[f"model__{key}"] = a
    print(f"  model: use_E={model['use_E']} c={model.get('c')} iters={model['solver_iters']}", flush=True)
    save("sgdml_model_ethanol_n621", **out)


def fx_ecstr(M, name, seed, perms=None):
    """use_E_cstr (energy constraints in the kernel, train.py:212-236, 837-845): the
    assembled (N + M) x (N + M) kernel, the matrix-free operator with energy coefficients
    (iterative_solver.py:416-443: GDMLPredict with alphas_E, predict.py:206-218) on a fixed
    vector, and what the reference's Iterative.solve does with it (records the exception)."""
    ds = synthetic.ethanol_like(M, seed=seed)
    task = dict(make_task(ds, perms=perms), use_E_cstr=True)
    desc, tpl, R_desc, R_d_desc, _, _ = prepare(task)
    n = 3 * M * ds["R"].shape[1]
    y = task["F_train"].ravel().copy()
    E_train = task["E_train"].ravel().copy()
    y = np.hstack((y, -E_train + np.mean(E_train)))
    y_std = np.std(y)
    y /= y_std
    K = gdml_train()._assemble_kernel_mat(R_desc, R_d_desc, tpl, 10, desc, use_E_cstr=True,
                                          col_idxs=np.s_[:], callback=noop)
    # _init_kernel_operator cannot be built at the system size n + M (create_model reshapes
    # the n + M dummy alphas to forces and raises), and at size n its LinearOperator
    # rejects an (n + M)-vector; the closure _K_vec itself (iterative_solver.py:416-443)
    # splits v into forces and energies as intended, so it is called directly
    _, K_op = kernel_operator(task, desc, R_desc, R_d_desc, tpl, n)
    rng = np.random.default_rng(seed + 200)
    v = rng.standard_normal(n + M)
    out = {"R": ds["R"], "F": ds["F"], "E": ds["E"], "z": ds["z"], "perms": task["perms"],
           "tril_perms_lin": tpl, "R_desc": R_desc, "R_d_desc": R_d_desc, "y": y,
           "y_std": np.float64(y_std), "sig": np.float64(10.0), "lam": np.float64(1e-10),
           "K": np.array(K), "v": v, "Kop_v": K_op._matvec(v)}
    # the solve entry point with use_E_cstr: record what the reference does
    for precon in ("cholesky", "eigvec_precon"):
        try:
            run_solver(task, desc, tpl, R_desc, R_d_desc, y, y_std, precon, 0.2, seed=1)
            out[f"{precon}__error"] = np.array("")
        except Exception as e:  # noqa: BLE001 - the reference's failure mode is the datum
            out[f"{precon}__error"] = np.array(f"{type(e).__name__}: {e}")
            print(f"  {name} {precon}: reference raised {type(e).__name__}: {e}", flush=True)
    save(name, **out)


def fx_eigvals(M, name, seed, precons):
    """Iterative.solve(flag_eigvals=True) (iterative_solver.py:978-989, 1002, 1100-1102):
    the spectra of P_op K and of K (dev_utils.get_eigvals, complex, LAPACK order) and the
    10-iteration CG it runs instead of a full solve."""
    iterative_solver.glob_eigvals_K = None
    ds = synthetic.ethanol_like(M, seed=seed)
    task = make_task(ds)
    desc, tpl, R_desc, R_d_desc, y, y_std = prepare(task)
    n = y.size
    m, kmin, _ = plot_data.get_params("ethanol")
    k_rot = int(plot_data.rule_of_thumb(n=n, k_min=kmin, m=m))
    out = {"R": ds["R"], "F": ds["F"], "E": ds["E"], "z": ds["z"], "perms": task["perms"],
           "tril_perms_lin": tpl, "R_desc": R_desc, "R_d_desc": R_d_desc, "y": y,
           "y_std": np.float64(y_std), "sig": np.float64(10.0), "lam": np.float64(1e-10),
           "solver_tol": np.float64(task["solver_tol"]), "k_rot": np.int64(k_rot)}
    for p in precons:
        iterative_solver.glob_eigvals_K = None  # the reference caches eigvals_K module-wide
        res = run_solver(task, desc, tpl, R_desc, R_d_desc, y, y_std, p, k_rot / n,
                         seed=1000 + seed, flag_eigvals=True)
        for key, val in res.items():
            out[f"{p}__{key}"] = val
        print(f"  {name} {p}: iters={res['num_iters']} eig range "
              f"{np.abs(res['eigvals']).min():.3e}..{np.abs(res['eigvals']).max():.3e}", flush=True)
    save(name, **out)


FIXTURES = {
    "eigvals_n270": lambda: fx_eigvals(10, "sgdml_ethanol_n270_eigvals", 3,
                                       ["cholesky", "random_scores", "eigvec_precon"]),
    "ecstr_n270": lambda: fx_ecstr(10, "sgdml_ethanol_n270_ecstr", seed=3),
    "ecstr_n270_perms": lambda: fx_ecstr(
        10, "sgdml_ethanol_n270_perms_ecstr", seed=5,
        perms=[np.arange(9), [0, 1, 2, 4, 5, 3, 6, 7, 8], [0, 1, 2, 5, 3, 4, 6, 7, 8]]),
    "model": fx_model,
    "descriptors": fx_descriptors,
    "rule_of_thumb": fx_rule_of_thumb,
    "rbf": fx_rbf,
    "lev": fx_lev_scores,
    "sgdml_n270": lambda: fx_sgdml(
        10, "sgdml_ethanol_n270",
        ["cholesky", "random_scores", "lev_scores", "inverse_lev", "lev_random",
         "truncated_cholesky", "truncated_cholesky_custom", "rank_k_lev_scores",
         "rank_k_lev_scores_custom", "eigvec_precon"], seed=3, none_tol=(1e-4, 1e-6)),
    # the two masked eigen preconditioners (iterative_solver.py:1238-1268) on the n270 geometry
    "sgdml_n270_eigmask": lambda: fx_sgdml(
        10, "sgdml_ethanol_n270_eigmask",
        ["eigvec_precon_block_diagonal", "eigvec_precon_atomic_interactions"], seed=3,
        with_K=False, none_tol=()),
    # a permutation GROUP (rotations of the methyl hydrogens), as sGDML's find_perms returns
    "sgdml_n270_perms": lambda: fx_sgdml(
        10, "sgdml_ethanol_n270_perms", ["cholesky", "random_scores", "truncated_cholesky_custom"],
        seed=5, perms=[np.arange(9), [0, 1, 2, 4, 5, 3, 6, 7, 8], [0, 1, 2, 5, 3, 4, 6, 7, 8]],
        none_tol=()),
    # not a group: the reference's mirrored assembly and its matrix-free operator then
    # disagree; kept for the assembly semantics (diagonal blocks stored transposed) only
    "sgdml_n270_nongroup": lambda: fx_sgdml(
        10, "sgdml_ethanol_n270_nongroup", [], seed=5,
        perms=[np.arange(9), [0, 1, 2, 4, 5, 3, 6, 7, 8], [0, 1, 2, 5, 3, 4, 7, 6, 8]],
        none_tol=()),
    "sgdml_n2997": lambda: fx_sgdml(
        111, "sgdml_ethanol_n2997", ["cholesky", "random_scores"], seed=9, with_K=False,
        none_tol=(1e-4,)),
    # nanotube-like geometry (370 atoms, BASELINE configs[1] molecule), M = 3 -> N = 3330,
    # nanotube rule-of-thumb rank; the reference's K_op costs ~0.1 s here
    "sgdml_nanotube_n3330": lambda: fx_sgdml(
        3, "sgdml_nanotube_n3330", ["cholesky", "random_scores"], seed=4, with_K=False,
        none_tol=(), geom="nanotube", k_rows=16),
    "cho_stable": fx_cho_stable,
    "sgdml_n621": lambda: fx_sgdml(
        23, "sgdml_ethanol_n621", ["cholesky", "random_scores", "truncated_cholesky"], seed=7,
        none_tol=(1e-4,)),
}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    a = ap.parse_args()
    names = a.only or list(FIXTURES)
    for nm in names:
        t0 = time.time()
        print(f"== {nm}", flush=True)
        FIXTURES[nm]()
        print(f"== {nm} done in {time.time() - t0:.1f}s", flush=True)
