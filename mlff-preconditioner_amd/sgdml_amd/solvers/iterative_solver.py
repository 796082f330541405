"""Drop-in replacement of the reference's iterative solver on MI355X.

Mirrors `sgdml.solvers.iterative_solver.Iterative`
(src/sGDML/sgdml/solvers/iterative_solver.py:75-1108): same constructor, same
`solve(...)` signature, same preconditioner strings (`str_preconditioner`,
`break_percentage`), same return tuple
`(alphas, num_iters, resid, train_rmse, inducing_pts_idxs, is_conv, info)` and
the same exceptions (NotImplementedError for an unknown preconditioner,
AssertionError for a non-PSD pivot, LinAlgError for a failed Cholesky).

What runs where:
  * the operator is the reference's matrix-free K_op (:383-445) evaluated on the GPU
    from R_desc/R_d_desc; preconditioner builds fetch their columns through it (as
    IterativeCholesky does) and the eigen preconditioners' truncated eigensolver applies
    it block-wise, so no N x N matrix is formed -- except for
    eigvec_precon_atomic_interactions, whose masked K is formed from the assembled K;
  * every preconditioner build (pivoted Cholesky, Nystrom, _sb, leverage
    scores, eigen-decomposition) and the PCG iterations run in libmlffpcg.so;
  * column *selection* stays on the host with NumPy's global RNG exactly as in the
    reference (:683-757), so a seeded run draws the same indices;
  * several GPUs (`devices=[0, 1, ...]`, or MLFF_DEVICES="0,1,..." / "all"): the rows of
    the operator and of the preconditioner panel are sharded over the devices from this
    one process (sgdml_amd.sharded, RCCL), as the reference spreads its GPU operator
    with DataParallel (predict.py:335-341).  The atomic-interactions eigen preconditioner
    masks every device's rows of the dense K (assembled sharded).
"""
from __future__ import annotations

import collections
import os
import timeit
import warnings
from functools import partial

import numpy as np

from .. import _native as nat
from ..sharded import ShardedKernelSolver
from ..solver import KernelSolver, PCGResult

DONE, NOT_DONE = 1, 0  # sgdml/__init__.py:31-32 (the progress callback's first argument)

LEV_SCORES_KEYS = ["lev_scores", "random_scores", "inverse_lev", "lev_random",
                   "truncated_cholesky", "truncated_cholesky_custom", "rank_k_lev_scores",
                   "rank_k_lev_scores_custom"]
EIGVEC_KEYS = ["eigvec_precon", "eigvec_precon_block_diagonal",
               "eigvec_precon_atomic_interactions"]


class Iterative(object):
    def __init__(self, gdml_train, desc, callback=None, max_processes=None, use_torch=False,
                 device=None, devices=None):
        self.gdml_train = gdml_train
        self.desc = desc
        self.callback = callback
        self._max_processes = max_processes
        self._use_torch = use_torch
        self.device = device
        if devices is None:
            env = os.environ.get("MLFF_DEVICES", "").strip()
            if env == "all":
                devices = list(range(nat.device_count()))
            elif env:
                devices = [int(d) for d in env.split(",")]
        self.devices = None if devices is None or len(devices) < 2 else [int(d) for d in devices]
        self.solver = None  # KernelSolver of the last solve (kept for inspection)

    def close(self):
        """Release the device context(s) of the last solve (a new solve does so too)."""
        solver, self.solver = self.solver, None
        if solver is not None:
            solver.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ helpers
    def _kernel_solver(self, task, R_desc, R_d_desc, tril_perms_lin, n, dense, one_device=False):
        """dense: assemble K on the device (the atomic-interactions mask is formed from it);
        otherwise only the matrix-free operator (the reference's K_op) is set up and
        the preconditioner builds fetch their columns through it, as the reference's
        IterativeCholesky does (iterative_cholesky.py:152-156): no N^2 memory.
        one_device: the solve runs on the first device even when several are configured
        (the dense flag_eigvals spectra are one-GPU computations)."""
        if self.devices is not None and not one_device:
            s = ShardedKernelSolver(n, self.devices)
        else:
            s = KernelSolver(n, device=self.devices[0] if self.devices is not None else self.device)
        perms = np.atleast_2d(np.asarray(task["perms"]))
        D = R_desc.shape[1]
        if len(tril_perms_lin) != perms.shape[0] * D:
            raise ValueError("tril_perms_lin does not match task['perms']")
        if dense:
            s.assemble_sgdml(R_desc, R_d_desc, perms, float(task["sig"]))
        else:
            s.sgdml_operator(R_desc, R_d_desc, perms, float(task["sig"]))
        # sGDML: K is negative semidefinite, the solved system is (-K + lam I) x = y
        s.set_operator(-1.0, float(task["lam"]))
        return s

    def _lev_scores(self, solver, n_train, dim_i, lam, n_inducing_pts,
                    idxs_ordered_by_lev_score=None):
        """_lev_scores (iterative_solver.py:447-552): host column choice, GPU numerics."""
        dim_m = np.maximum(1, n_inducing_pts // 4) * dim_i
        if idxs_ordered_by_lev_score is None:
            lev_approx_idxs = np.sort(np.random.choice(n_train * dim_i, dim_m, replace=False))
        else:
            assert len(idxs_ordered_by_lev_score) == n_train * dim_i
            lev_approx_idxs = np.sort(idxs_ordered_by_lev_score[-dim_m:])
        lev_scores = solver.lev_scores(lev_approx_idxs.astype(np.int64), lam)
        return lev_scores, np.argsort(lev_scores)

    def _eigvec_factor(self, solver, k, name, dim_i):
        """_init_precon_operator_eigvals (iterative_solver.py:1177-1329) on the device."""
        mask = {"eigvec_precon": 0, "eigvec_precon_block_diagonal": 1,
                "eigvec_precon_atomic_interactions": 2}[name]
        solver.precon_eig(k, mask_mode=mask, dim_i=dim_i, build_woodbury=True)
        _warn_eig(solver)

    # --------------------------------------------------------------- solve
    def solve(self, task, R_desc, R_d_desc, tril_perms_lin, y, y_std, save_progr_callback=None,
              break_percentage=None, str_preconditioner="", flag_eigvals=False):
        start_solve_routine = timeit.default_timer()
        n_train, n_atoms = task["R_train"].shape[:2]
        dim_i = 3 * n_atoms
        n = 3 * n_train * n_atoms
        lam = task["lam"]
        if task.get("use_E_cstr", False):
            # the reference's solve cannot run either: its K_op and preconditioners are built
            # at n = 3 n_train n_atoms (iterative_solver.py:638, 827-830) while y carries the
            # n_train energy labels too (train.py:837-845), so scipy's cg (or create_model)
            # raises ValueError (tests/golden/*_ecstr.npz).  The energy-constrained operator
            # and assembly themselves are available on KernelSolver (use_E_cstr=True).
            raise ValueError(f"use_E_cstr: the system has {n + n_train} entries (forces and "
                             f"energies) but the reference's solve builds its operator and "
                             f"preconditioner at {n}")

        alphas0_F = task["alphas0_F"] if "alphas0_F" in task else None
        num_iters0 = task["solver_iters"] if "solver_iters" in task else 0
        if break_percentage is None:
            n_inducing_pts_init = int(task["n_inducing_pts_init"])
        else:
            n_inducing_pts_init = int(max(np.ceil(break_percentage * n_train), 1))
        if "inducing_pts_idxs" in task:
            n_inducing_pts_init = len(task["inducing_pts_idxs"]) // (3 * n_atoms)
        n_inducing_pts = min(n_train, n_inducing_pts_init)

        # only the atomic-interactions mask is formed from the dense K; the truncated
        # eigensolver of the other eigen preconditioners runs on the matrix-free operator
        dense = str_preconditioner == "eigvec_precon_atomic_interactions"
        self.close()  # the previous solve's contexts (operator tables, panel, communicator)
        solver = self._kernel_solver(task, np.asarray(R_desc), np.asarray(R_d_desc),
                                     tril_perms_lin, n, dense, one_device=bool(flag_eigvals))
        self.solver = solver
        start_preconditioner = timeit.default_timer()
        info_cholesky = None
        if str_preconditioner in LEV_SCORES_KEYS:
            k = int(break_percentage * n)
            if "inducing_pts_idxs" in task:
                raise AssertionError("Nor applicable in this setting")
            if str_preconditioner == "random_scores":
                inducing_pts_idxs = np.sort(np.random.choice(np.arange(n), size=k, replace=False))
            elif str_preconditioner in ["truncated_cholesky", "truncated_cholesky_custom"]:
                k_truncate = task["truncated_cholesky"]
                k_truncate = k_truncate if k_truncate < k else k
                k_chol = int(float(k_truncate / n) * n)  # iterative_cholesky.py:135
                index_columns, _ = solver.precon_pivchol(k_chol, build_woodbury=False)
                inducing_pts_cholesky = index_columns[:k_truncate]
                k_random = int(k - k_truncate) if k_truncate < k else 0
                inducing_pts_random = np.random.choice(index_columns[k_truncate:], size=k_random,
                                                       replace=False)
                inducing_pts_idxs = np.sort(np.concatenate([inducing_pts_cholesky,
                                                            inducing_pts_random]))
            elif str_preconditioner in ["rank_k_lev_scores", "rank_k_lev_scores_custom"]:
                leverage_scores = self._rank_k_leverage_scores(solver, break_percentage, n)
                p = leverage_scores / leverage_scores.sum()
                inducing_pts_idxs = np.sort(np.random.choice(np.arange(n), size=k, replace=False,
                                                             p=p))
            else:  # lev_scores / inverse_lev / lev_random
                lev_scores, order = self._lev_scores(solver, n_train, dim_i, lam, n_inducing_pts)
                if str_preconditioner == "inverse_lev":
                    inducing_pts_idxs = np.sort(order[:k])
                elif str_preconditioner == "lev_scores":
                    inducing_pts_idxs = np.sort(order[-k:])
                else:
                    p = lev_scores / lev_scores.sum()
                    inducing_pts_idxs = np.sort(np.random.choice(np.arange(n), size=k,
                                                                 replace=False, p=p))
            assert inducing_pts_idxs.shape == (k,), "Incorrect number of inducing points."
            variant = 1 if str_preconditioner in ["truncated_cholesky_custom",
                                                  "rank_k_lev_scores_custom"] else 0
            solver.precon_nystrom(np.asarray(inducing_pts_idxs, dtype=np.int64), variant=variant)
        elif str_preconditioner == "cholesky":
            k = int(break_percentage * n)
            index_columns, sec = solver.precon_pivchol(k, build_woodbury=True)
            # per-column device times of the build (incomplete_cholesky.py:48-80), the
            # Woodbury build (iterative_cholesky.py:141-143) reported on its own
            t_cols, t_woodbury = solver.pivchol_times(k)
            info_cholesky = {"time_cholesky": t_cols, "time_woodbury": t_woodbury,
                             "L.shape": (n, k), "index_columns": index_columns}
            inducing_pts_idxs = np.arange(int(break_percentage * n))
        elif str_preconditioner in EIGVEC_KEYS:
            k = int(np.max([int(break_percentage * n), 1]))
            self._eigvec_factor(solver, k, str_preconditioner, dim_i)
            inducing_pts_idxs = np.arange(k)
        elif str_preconditioner == "none":
            solver.precon_none()
            inducing_pts_idxs = np.arange(0)
        else:
            raise NotImplementedError(f"str_preconditioner = {str_preconditioner}")
        stop_preconditioner = timeit.default_timer()
        total_time_preconditioner = stop_preconditioner - start_preconditioner

        eig_info = None
        if flag_eigvals:
            # iterative_solver.py:978-989 (dev_utils.get_eigvals): the spectra of P_op K and
            # of K, K = -K_op (the PCG operator), dense on the device (mlff_spectrum); real
            # and descending here, complex in LAPACK order in the reference
            if getattr(solver, "world", 1) > 1:
                raise NotImplementedError("flag_eigvals: the dense spectrum runs on one GPU")
            eig_info = {"eigvals": solver.spectrum(True), "eigvals_K": solver.spectrum(False)}
        x0 = None if alphas0_F is None else -np.asarray(alphas0_F, dtype=np.float64)
        # the reference stops the CG after 10 iterations when the spectra are requested (:1002)
        maxiter = 3 * n_atoms * n_train * 5 if not flag_eigvals else 10
        cb = None
        if self.callback is not None:  # :820-823, :852-853
            cb = partial(self.callback, disp_str="Initializing solver")
            cb(NOT_DONE, sec_disp_str=None)
        status = _CGStatus(self, task, R_desc, R_d_desc, tril_perms_lin, y, y_std,
                           inducing_pts_idxs, num_iters0, n_inducing_pts, save_progr_callback, cb)
        op_storage, op_bytes = solver.storage_info()
        solver.timing(True)
        solver.timing_reset()
        tic = timeit.default_timer()
        res = status.run(solver, np.asarray(y, dtype=np.float64), x0, float(task["solver_tol"]),
                         maxiter)
        total_time_cg = timeit.default_timer() - tic
        t = solver.timing_read()
        alphas = -res.x
        is_conv = res.info == 0
        num_iters = num_iters0 + res.callbacks
        resid = res.resid
        total_time_solve = timeit.default_timer() - start_solve_routine
        info = {"is_conv": is_conv,
                "total_time_cholesky": total_time_preconditioner,
                "total_time_cg": total_time_cg,
                "total_time_solve": total_time_solve,
                "total_time_preconditioner": total_time_preconditioner,
                # additions of this backend
                "resid_trace": res.trace,
                "cg_iterations": res.iters,
                # algorithmic bytes of the operator in the storage it ran on (matrix-free:
                # the descriptor tables; tiles: 4 N^2) over its mean HIP-event time
                "gbps_matvec": op_bytes / (t["gemv_ms"] / t["gemv_count"]) / 1e6
                if t["gemv_count"] else float("nan"),
                "operator_storage": op_storage,
                "n_gpus": getattr(solver, "world", 1)}
        if info_cholesky is not None:
            info.update(info_cholesky)
        if eig_info is not None:
            info.update(eig_info)  # iterative_solver.py:1100-1102
        if cb is not None:  # :1074-1086
            cb(DONE, disp_str="Training on {:,} points{}".format(
                n_train, "" if is_conv else " (NOT CONVERGED)"),
               sec_disp_str="{:d} iter @ {} iter/s".format(
                   num_iters, "{:.1f}".format(num_iters / status.avg_tt)
                   if status.avg_tt > 0 else "--"),
               done_with_warning=not is_conv)
        train_rmse = resid / np.sqrt(len(y))
        return alphas, num_iters, resid, train_rmse, inducing_pts_idxs, is_conv, info

    def _rank_k_leverage_scores(self, solver, break_percentage, n):
        """_rank_k_leverage_scores (iterative_solver.py:1110-1175): ||U[:, :k] row||."""
        k = int(np.max([int(break_percentage * n), 1]))
        _, rowlev = solver.precon_eig(k, mask_mode=0, build_woodbury=False, want_rowlev=True)
        _warn_eig(solver)
        return rowlev


def _warn_eig(solver):
    """The truncated eigensolver's pairs were accepted at a looser tolerance (mlff_eig_info)."""
    converged, rel = solver.eig_info()
    if not converged:
        warnings.warn(f"truncated eigensolver: the leading Ritz pairs reached a relative residual of "
                      f"{rel:.1e} (target 1e-11) within the iteration cap; the preconditioner is "
                      f"built from them", RuntimeWarning, stacklevel=3)


class _CGStatus:
    """The reference's per-iteration CG callback `_cg_status` (iterative_solver.py:874-965)
    around the chunked device PCG.

    scipy 1.7.3 calls it once per iteration with the iterate x_j (j = 1 ... m; the caller-frame
    `resid` it reads is the stop-test residual of that iterate, trace[j]).  In it the
    reference keeps (module globals) num_iters (= num_iters0 + calls so far), the per-call
    wall time tt, avg_tt = sum tt, and the last CG_STEPS_HIST_LEN = 100 residual steps, and
      * once per second -- when tt > 0 and num_iters % ceil(1 / tt) == 0 -- calls
        callback(NOT_DONE, disp_str='Training error (RMSE): forces ...',
        sec_disp_str='<num_iters> iter @ <1/tt> iter/s [eff: <eff>%] k: <n_inducing_pts>'),
        eff = (int(100 * ratio) - 50) * 2, ratio = -sum(negative steps) / sum |steps|;
      * every two minutes -- num_iters % ceil(120 / tt) == 0 -- builds the unconverged model
        of -x_j (create_model, solver_iters = num_iters + 1, solver_resid = resid), its
        integration constant c = sum(E_ref - E_pred) / M from a prediction of the training
        energies with those coefficients (:942-951), and hands it to save_progr_callback.
    Here the iterations run on the device in chunks that end exactly on the iterations where
    one of the two conditions holds for the per-iteration time measured over the previous
    chunk (tt of every call in a chunk = that chunk's average; the first call has tt = 0 as
    in the reference); the bookkeeping of every call inside a chunk is replayed from the
    device's residual trace, so eff and num_iters are the reference's.  Without a callback
    and save_progr_callback the PCG runs in one piece."""

    HIST_LEN = 100          # CG_STEPS_HIST_LEN (iterative_solver.py:57-59)
    PROGRESS_S = 1.0        # "once per second" (:899)
    CHECKPOINT_S = 120.0    # "once every 2 minutes" (:919-920)
    FIRST_CHUNK = 8         # iterations timed before the first planned stop

    def __init__(self, it, task, R_desc, R_d_desc, tril_perms_lin, y, y_std, idxs, iters0,
                 n_inducing_pts, save_progr_callback, cb):
        self.it, self.task = it, task
        self.R_desc, self.R_d_desc, self.tpl = R_desc, R_d_desc, tril_perms_lin
        self.y, self.y_std, self.idxs = y, y_std, idxs
        self.iters0, self.k = int(iters0), int(n_inducing_pts)
        self.save = save_progr_callback if it.gdml_train is not None else None
        self.cb = cb
        self.num_iters = int(iters0)
        self.resid = 0.0
        self.avg_tt = 0.0
        self.calls = 0
        self.hist = collections.deque(maxlen=self.HIST_LEN)
        self.eff = 0
        self.checkpoints = []  # (iterate j, solver_iters) of every model handed over

    @property
    def active(self):
        return self.cb is not None or self.save is not None

    def _period(self, tt, seconds):
        return int(np.ceil(seconds / tt))

    def _next_stop(self, j, tt, maxiter):
        """Smallest iterate index > j whose call has num_iters = iters0 + index - 1 divisible
        by the progress or the checkpoint period (of the per-iteration time tt)."""
        cand = [maxiter]
        for sec, on in ((self.PROGRESS_S, self.cb is not None), (self.CHECKPOINT_S, self.save is not None)):
            if on:
                P = self._period(tt, sec)
                base = self.iters0 + j  # num_iters of the call of iterate j + 1
                cand.append(j + 1 + (-base) % P)
        return min(cand)

    def _replay(self, trace, j0, j1, tt):
        """Bookkeeping of the calls of iterates j0 + 1 ... j1 (everything except the displays),
        per chunk rather than per call: only the last HIST_LEN steps reach the history and eff
        is that of the chunk's last call, so the host work between device chunks is O(HIST_LEN)
        (the per-call wall time is summed call by call, as the reference accumulates it)."""
        if j1 <= j0:
            return
        n_calls = j1 - j0
        for _ in range(n_calls):
            self.avg_tt += 0.0 if self.calls == 0 else tt
            self.calls += 1
        # call of iterate j: num_iters = num_iters(j0 + 1) + (j - j0 - 1); its step is
        # trace[j] - (previous call's resid), 0 when that num_iters is 0
        nfirst = self.num_iters
        for j in range(max(j0 + 1, j1 - self.HIST_LEN + 1), j1 + 1):
            old = self.resid if j == j0 + 1 else float(trace[j - 1])
            self.hist.append(0.0 if nfirst + (j - j0 - 1) == 0 else float(trace[j]) - old)
        self.resid = float(trace[j1])
        self.num_iters = nfirst + n_calls - 1
        h = np.asarray(self.hist)
        tot = np.abs(h).sum()
        ratio = (-h.clip(max=0).sum() / tot) if tot > 0 else 1
        self.eff = 0 if self.num_iters == 0 else (int(100 * ratio) - 50) * 2
        # num_iters is now that of the call of iterate j1 (incremented after it by the caller)

    def _at_stop(self, solver, j, tt):
        if tt <= 0.0:
            return
        if self.cb is not None and self.num_iters % self._period(tt, self.PROGRESS_S) == 0:
            rmse = self.resid / np.sqrt(len(self.y))
            self.cb(NOT_DONE, disp_str="Training error (RMSE): forces {:.4f}".format(rmse),
                    sec_disp_str="{:d} iter @ {} iter/s [eff: {:d}%] k: {:d}".format(
                        self.num_iters, "{:.1f}".format(1.0 / tt), self.eff, self.k))
        if self.save is not None and self.num_iters % self._period(tt, self.CHECKPOINT_S) == 0:
            self.save(self.checkpoint_model(solver.pcg_x(), solver))
            self.checkpoints.append((j, self.num_iters + 1))

    def checkpoint_model(self, x, solver):
        """:922-951: the unconverged model of -x and its integration constant."""
        alphas_F = -np.asarray(x)
        model = self.it.gdml_train.create_model(
            self.task, "cg", self.R_desc, self.R_d_desc, self.tpl, self.y_std, alphas_F,
            alphas_E=None, solver_resid=self.resid, solver_iters=self.num_iters + 1,
            norm_y_train=np.linalg.norm(self.y), inducing_pts_idxs=self.idxs)
        _, E = solver.sgdml_energies(alphas_F)  # GDMLPredict with these alphas, c = 0, std 1
        E_pred = E * self.y_std
        E_ref = np.squeeze(self.task["E_train"])
        model["c"] = np.sum(E_ref - E_pred) / E_ref.shape[0]
        return model

    def run(self, solver, y, x0, tol, maxiter):
        if not self.active:
            return solver.pcg(y, x0, tol=tol, maxiter=maxiter)
        early = solver.pcg_start(y, x0, tol, maxiter)
        j, status, _, _ = solver.pcg_result()
        tt = 0.0
        while status == nat.PCG_RUNNING:
            stop = min(maxiter, j + self.FIRST_CHUNK) if tt <= 0.0 else \
                self._next_stop(j, tt, maxiter)
            t0 = timeit.default_timer()
            solver.pcg_run(stop - j)
            el = timeit.default_timer() - t0
            j1, status, _, _ = solver.pcg_result()
            tr = solver.pcg_trace()
            tt_chunk = el / max(j1 - j, 1)
            if j1 > j:
                self._replay(tr, j, j1, tt if tt > 0.0 else tt_chunk)
                if j1 == stop:
                    self._at_stop(solver, j1, tt)
                self.num_iters += 1
            j, tt = j1, tt_chunk
        it, status, resid, info = solver.pcg_result()
        return PCGResult(x=solver.pcg_x(), info=info, iters=it, resid=resid,
                         trace=solver.pcg_trace(), early_exit=early,
                         callbacks=0 if early else max(it, 1))
