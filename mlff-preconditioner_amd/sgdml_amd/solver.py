"""KernelSolver: one GPU (one rank) of the MI355X PCG solver.

Thin object wrapper over the C ABI (include/mlffpcg.h).  It owns a device
context holding this rank's row block of the dense kernel matrix K, the operator
A = sigma_K * K + lam * I, an optional low-rank preconditioner and the PCG state.

    s = KernelSolver(n)                       # single GPU
    s.gen_rbf(X, length_scale=0.2)            # or set_matrix / assemble_sgdml
    s.set_operator(sigma_K=+1.0, lam=1e-6)
    s.precon_nystrom(idx)                     # or precon_pivchol(k) / precon_none()
    res = s.pcg(b, tol=1e-6, maxiter=5 * n)

Multi-GPU: one process per GPU; every rank constructs KernelSolver(n, rank=r,
world=W, comm_id=id) with the same RCCL id (sgdml_amd.distributed.make_comm_id)
and passes its own row block (row_range()).
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass, field

import numpy as np

from . import _native as nat


@dataclass
class PCGResult:
    x: np.ndarray            # local solution block
    info: int                # scipy convention: 0 converged, maxiter otherwise
    iters: int               # CG iterations performed (scipy ITER)
    resid: float             # last stop-test ||r|| (true residual after the recheck)
    trace: np.ndarray        # ||r_0||, ||r_1||, ..., ||r_iters||
    early_exit: bool = False  # legacy pre-check ||A x0 - b|| <= tol ended the solve
    callbacks: int = 0       # number of scipy callback invocations this solve maps to
    extra: dict = field(default_factory=dict)


class KernelSolver:
    def __init__(self, n: int, device: int | None = None, rank: int = 0, world: int = 1,
                 comm_id: bytes | None = None):
        self._lib = nat.load_library()
        self._close_lock = threading.Lock()
        self.n = int(n)
        self.rank, self.world = int(rank), int(world)
        if device is None:
            ndev = nat.device_count()
            device = rank % max(ndev, 1)
        self.device = int(device)
        ctx = ctypes.c_void_p()
        cid = None if comm_id is None else ctypes.c_char_p(bytes(comm_id))
        nat.check(self._lib.mlff_ctx_create(self.device, self.rank, self.world, cid, self.n,
                                            ctypes.byref(ctx)), None, "mlff_ctx_create")
        self._ctx = ctx
        r0, nr = ctypes.c_int64(), ctypes.c_int64()
        self._call("mlff_shard_range", ctypes.byref(r0), ctypes.byref(nr))
        self.row0, self.nrows = r0.value, nr.value

    # ------------------------------------------------------------------ basics
    def _call(self, name, *args):
        rc = getattr(self._lib, name)(self._ctx, *args)
        if rc != nat.MLFF_OK and self.world > 1 and rc not in (nat.MLFF_ERR_NOT_PSD,
                                                                nat.MLFF_ERR_LINALG):
            # a failure on one rank would leave its peers waiting in the next collective
            # (mlff_comm_abort); NOT_PSD / LINALG are reached by every rank together
            try:
                nat.check(rc, self._ctx, name)
            finally:
                self._lib.mlff_comm_abort(self._ctx)
        nat.check(rc, self._ctx, name)

    def close(self):
        """Destroy the device context (idempotent, safe from any thread)."""
        lock = getattr(self, "_close_lock", None)
        if lock is None:
            return
        with lock:
            ctx = getattr(self, "_ctx", None)
            self._ctx = None
            if ctx is not None and ctx.value is not None:
                self._lib.mlff_ctx_destroy(ctx)

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def row_range(self) -> tuple[int, int]:
        return self.row0, self.row0 + self.nrows

    def synchronize(self):
        self._call("mlff_synchronize")

    def stream_handle(self) -> int:
        p = ctypes.c_void_p()
        self._call("mlff_stream", ctypes.byref(p))
        return p.value or 0

    # ------------------------------------------------------------------ matrix
    def set_matrix(self, K_local: np.ndarray):
        """K_local: this rank's rows (nrows x N) of K."""
        K_local = np.ascontiguousarray(K_local, dtype=np.float64)
        if K_local.shape != (self.nrows, self.n):
            raise ValueError(f"K_local must have shape {(self.nrows, self.n)}, got {K_local.shape}")
        self._call("mlff_set_matrix_host", nat.dptr(K_local), self.n)

    def get_matrix_rows(self, r0: int = 0, nr: int | None = None) -> np.ndarray:
        nr = self.nrows - r0 if nr is None else nr
        out = np.empty((nr, self.n))
        self._call("mlff_get_matrix_rows", int(r0), int(nr), nat.dptr(out), self.n)
        return out

    def gen_rbf(self, X: np.ndarray, length_scale: float = 1.0, jitter: float = 0.0):
        X = np.ascontiguousarray(X, dtype=np.float64)
        if X.ndim != 2 or X.shape[0] != self.n:
            raise ValueError("X must be N x d")
        self._call("mlff_gen_rbf", nat.dptr(X), int(X.shape[1]), float(length_scale), float(jitter))

    def sgdml_operator(self, R_desc: np.ndarray, R_d_desc: np.ndarray, perms: np.ndarray,
                       sig: float, use_E_cstr: bool = False):
        """Matrix-free sGDML operator (the reference's K_op) without assembling K.
        use_E_cstr: the solver's N is 3 n_atoms M + M and the operator is the reference's
        _K_vec with energy coefficients (iterative_solver.py:416-443); one rank only."""
        self._call("mlff_set_energy_constraints", int(bool(use_E_cstr)))
        R_desc = np.ascontiguousarray(R_desc, dtype=np.float64)
        R_d_desc = np.ascontiguousarray(R_d_desc, dtype=np.float64)
        perms = np.ascontiguousarray(np.atleast_2d(perms), dtype=np.int32)
        M, D = R_desc.shape
        n_atoms = perms.shape[1]
        if R_d_desc.shape != (M, D, 3) or D != n_atoms * (n_atoms - 1) // 2:
            raise ValueError("R_desc / R_d_desc / perms shapes do not match")
        self._call("mlff_sgdml_operator", nat.dptr(R_desc), nat.dptr(R_d_desc), M, n_atoms,
                   nat.i32ptr(perms), perms.shape[0], float(sig))

    def assemble_sgdml(self, R_desc: np.ndarray, R_d_desc: np.ndarray, perms: np.ndarray,
                       sig: float, use_E_cstr: bool = False):
        """Dense sGDML kernel (_assemble_kernel_mat, train.py:81-236, 1121-1308) and the
        matrix-free operator of the same inputs; use_E_cstr appends the M energy rows /
        columns (train.py:212-236; N = 3 n_atoms M + M, one rank only)."""
        self._call("mlff_set_energy_constraints", int(bool(use_E_cstr)))
        R_desc = np.ascontiguousarray(R_desc, dtype=np.float64)
        R_d_desc = np.ascontiguousarray(R_d_desc, dtype=np.float64)
        perms = np.ascontiguousarray(np.atleast_2d(perms), dtype=np.int32)
        M, D = R_desc.shape
        n_atoms = perms.shape[1]
        if R_d_desc.shape != (M, D, 3) or D != n_atoms * (n_atoms - 1) // 2:
            raise ValueError("R_desc / R_d_desc / perms shapes are inconsistent")
        self._call("mlff_assemble_sgdml", nat.dptr(R_desc), nat.dptr(R_d_desc), int(M),
                   int(n_atoms), nat.i32ptr(perms), int(perms.shape[0]), float(sig))

    def sgdml_energies(self, alphas: np.ndarray) -> tuple[int, np.ndarray]:
        """Training-set energies (GDMLPredict's E before std scale and constant) of the
        model with coefficients `alphas` (global N-vector): (i0, E[i0 : i0 + ni]) for the
        training points this rank's rows touch (all M on one rank)."""
        alphas = np.ascontiguousarray(alphas, dtype=np.float64)
        if alphas.shape != (self.n,):
            raise ValueError("alphas must have N entries")
        E = np.empty(self.n)  # >= M entries
        i0, ni = ctypes.c_int64(), ctypes.c_int64()
        self._call("mlff_sgdml_energies", nat.dptr(alphas), nat.dptr(E), ctypes.byref(i0),
                   ctypes.byref(ni))
        return i0.value, E[: ni.value].copy()

    def set_operator(self, sigma_K: float, lam: float):
        self._call("mlff_set_operator", float(sigma_K), float(lam))

    def set_storage(self, mode: str):
        """Operator storage: 'dense' (row GEMV), 'sym' (lower block triangle in
        512 x 512 tiles, half the bytes), 'matfree' (sGDML operator evaluated from
        the descriptors, no N^2 bytes), 'auto' (default: the cheapest available)."""
        code = {"dense": nat.STORAGE_DENSE, "sym": nat.STORAGE_SYMTILE,
                "auto": nat.STORAGE_AUTO, "matfree": nat.STORAGE_MATFREE}[mode]
        self._call("mlff_set_storage", code)

    def storage_info(self) -> tuple[str, float]:
        """(storage in use, algorithmic HBM bytes of one operator application on this rank)."""
        mode = ctypes.c_int()
        nbytes = ctypes.c_double()
        self._call("mlff_storage_info", ctypes.byref(mode), ctypes.byref(nbytes))
        name = {nat.STORAGE_SYMTILE: "sym", nat.STORAGE_MATFREE: "matfree"}.get(mode.value,
                                                                                "dense")
        return name, nbytes.value

    def operator_form(self) -> str | None:
        """Form of the matrix-free sGDML operator: 'pair', 'rec' (record-factored, many atoms /
        few points) or 'pt' (pair-tile, few atoms / many points); None without one."""
        f = ctypes.c_int()
        self._call("mlff_operator_form", ctypes.byref(f))
        return {0: "pair", 1: "rec", 2: "pt"}.get(f.value)

    def matvec(self, v: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.float64)
        if v.shape != (self.n,):
            raise ValueError("v must have N entries")
        y = np.empty(self.nrows)
        self._call("mlff_matvec", nat.dptr(v), nat.dptr(y))
        return y

    def spectrum(self, preconditioned: bool = True) -> np.ndarray:
        """Eigenvalues (descending) of P_op A, or of A = sigma_K K + lam I: the flag_eigvals
        diagnostics of Iterative.solve (iterative_solver.py:978-989).  One rank, dense."""
        out = np.empty(self.n)
        self._call("mlff_spectrum", int(bool(preconditioned)), nat.dptr(out))
        return out

    def diag(self) -> np.ndarray:
        d = np.empty(self.nrows)
        self._call("mlff_get_diag", nat.dptr(d))
        return d

    # ------------------------------------------------------------ preconditioner
    def precon_none(self):
        self._call("mlff_precon_none")

    def precon_pivchol(self, k: int, build_woodbury: bool = True):
        """Pivoted Cholesky of S = sigma_K K to rank k (+ Woodbury).  Returns
        (index_columns (N,), seconds)."""
        idx = np.empty(self.n, dtype=np.int64)
        sec = ctypes.c_double()
        self._call("mlff_precon_pivchol", int(k), int(bool(build_woodbury)), nat.i64ptr(idx),
                   ctypes.byref(sec))
        return idx, sec.value

    def pivchol_times(self, k: int) -> tuple[np.ndarray, float]:
        """(device seconds of every column of the last pivoted-Cholesky build, seconds of its
        Woodbury build): the reference's info['time_cholesky'] (incomplete_cholesky.py:48-80)."""
        t = np.empty(int(k))
        w = ctypes.c_double()
        self._call("mlff_pivchol_times", nat.dptr(t), int(k), ctypes.byref(w))
        return t, w.value

    def precon_nystrom(self, idx: np.ndarray, variant: int = 0) -> float:
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        sec = ctypes.c_double()
        self._call("mlff_precon_nystrom", nat.i64ptr(idx), int(idx.size), int(variant),
                   ctypes.byref(sec))
        return sec.value

    def precon_lowrank(self, Lt_local: np.ndarray):
        Lt_local = np.ascontiguousarray(Lt_local, dtype=np.float64)
        k = Lt_local.shape[0]
        if Lt_local.shape != (k, self.nrows):
            raise ValueError("Lt_local must be k x nrows")
        self._call("mlff_precon_lowrank", nat.dptr(Lt_local), int(k))

    def precon_eig(self, k: int, mask_mode: int = 0, dim_i: int = 0, build_woodbury: bool = True,
                   want_evals: bool = False, want_rowlev: bool = False):
        """Top-k eigen-decomposition of S = sigma_K K (see mlff_precon_eig).  Returns
        (evals or None, ||U[i, :k]|| or None)."""
        ev = np.empty(int(k)) if want_evals else None
        rl = np.empty(self.n) if want_rowlev else None
        self._call("mlff_precon_eig", int(k), int(mask_mode), int(dim_i), int(bool(build_woodbury)),
                   nat.dptr(ev), nat.dptr(rl))
        return ev, rl

    def eig_info(self) -> tuple[bool, float]:
        """(converged to 1e-11, worst Ritz residual / |theta_0|) of the last precon_eig."""
        c, r = ctypes.c_int(), ctypes.c_double()
        self._call("mlff_eig_info", ctypes.byref(c), ctypes.byref(r))
        return bool(c.value), r.value

    def precon_info(self) -> tuple[int, int]:
        kind, k = ctypes.c_int(), ctypes.c_int64()
        self._call("mlff_precon_info", ctypes.byref(kind), ctypes.byref(k))
        return kind.value, k.value

    def precon_apply_traffic(self) -> tuple[int, float]:
        """(form, algorithmic HBM bytes of one low-rank apply on this rank); form 0 = two
        passes over the panel, 1 = one pass with a row per workgroup, 2 = one pass with a
        row per cluster of workgroups."""
        one, b = ctypes.c_int(), ctypes.c_double()
        self._call("mlff_precon_apply_traffic", ctypes.byref(one), ctypes.byref(b))
        return one.value, b.value

    def precon_apply(self, r_local: np.ndarray) -> np.ndarray:
        r_local = np.ascontiguousarray(r_local, dtype=np.float64)
        z = np.empty(self.nrows)
        self._call("mlff_precon_apply", nat.dptr(r_local), nat.dptr(z))
        return z

    def precon_panel(self) -> np.ndarray:
        _, k = self.precon_info()
        T = np.empty((k, self.nrows))
        self._call("mlff_precon_get_panel", nat.dptr(T), self.nrows)
        return T

    def cho_factor_stable(self, M: np.ndarray) -> tuple[np.ndarray, float]:
        """Iterative._cho_factor_stable (iterative_solver.py:555-583) on the device: (L, lo_eig)
        with L L^T = M +- 1e-15 I (+ when the smallest eigenvalue lo_eig of M's lower triangle
        is <= 0); LinAlgError when the shifted M is not positive definite."""
        M = np.ascontiguousarray(M, dtype=np.float64)
        if M.ndim != 2 or M.shape[0] != M.shape[1]:
            raise ValueError("M must be square")
        L = np.empty_like(M)
        lo = ctypes.c_double()
        self._call("mlff_cho_factor_stable", nat.dptr(M), M.shape[0], nat.dptr(L), ctypes.byref(lo))
        return L, lo.value

    def sym_min_eig(self, M: np.ndarray, want_tridiag: bool = False):
        """Smallest eigenvalue of M's lower triangle (the eigh of _cho_factor_stable,
        iterative_solver.py:577) on the device; with want_tridiag also the tridiagonal (d, e)."""
        M = np.ascontiguousarray(M, dtype=np.float64)
        if M.ndim != 2 or M.shape[0] != M.shape[1]:
            raise ValueError("M must be square")
        m = M.shape[0]
        lo = ctypes.c_double()
        d = np.empty(m) if want_tridiag else None
        e = np.empty(max(m - 1, 1)) if want_tridiag else None
        self._call("mlff_sym_min_eig", nat.dptr(M), m, ctypes.byref(lo), nat.dptr(d), nat.dptr(e))
        return (lo.value, d, e[: m - 1]) if want_tridiag else lo.value

    def lev_scores(self, idx: np.ndarray, lam: float) -> np.ndarray:
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        out = np.empty(self.n)
        self._call("mlff_lev_scores", nat.i64ptr(idx), int(idx.size), float(lam), nat.dptr(out))
        return out

    # ---------------------------------------------------------------------- PCG
    def pcg_start(self, b_local: np.ndarray, x0_local: np.ndarray | None = None,
                  tol: float = 1e-5, maxiter: int | None = None) -> bool:
        b_local = np.ascontiguousarray(b_local, dtype=np.float64)
        if b_local.shape != (self.nrows,):
            raise ValueError("b_local must have nrows entries")
        x0p = None
        if x0_local is not None:
            x0_local = np.ascontiguousarray(x0_local, dtype=np.float64)
            if x0_local.shape != (self.nrows,):
                raise ValueError("x0_local must have nrows entries")
            x0p = nat.dptr(x0_local)
        maxiter = 10 * self.n if maxiter is None else int(maxiter)
        early = ctypes.c_int()
        self._call("mlff_pcg_start", nat.dptr(b_local), x0p, float(tol), maxiter,
                   ctypes.byref(early))
        self._maxiter = maxiter
        return bool(early.value)

    def pcg_run(self, n_iter: int, chunk: int = 0) -> int:
        st = ctypes.c_int()
        self._call("mlff_pcg_run", int(n_iter), int(chunk), ctypes.byref(st))
        return st.value

    def pcg_result(self) -> tuple[int, int, float, int]:
        it, st, res, info = ctypes.c_int64(), ctypes.c_int(), ctypes.c_double(), ctypes.c_int()
        self._call("mlff_pcg_result", ctypes.byref(it), ctypes.byref(st), ctypes.byref(res),
                   ctypes.byref(info))
        return it.value, st.value, res.value, info.value

    def pcg_x(self) -> np.ndarray:
        x = np.empty(self.nrows)
        self._call("mlff_pcg_get_x", nat.dptr(x))
        return x

    def pcg_trace(self) -> np.ndarray:
        it = self.pcg_result()[0]
        t = np.empty(it + 1)
        self._call("mlff_pcg_get_trace", nat.dptr(t), it + 1)
        return t

    def pcg(self, b_local: np.ndarray, x0_local: np.ndarray | None = None, tol: float = 1e-5,
            maxiter: int | None = None, callback=None, cb_every: int = 0,
            chunk: int = 0) -> PCGResult:
        """Full solve with scipy-1.7.3 `cg(A, b, x0, tol, atol=None, maxiter, M)` semantics.

        callback(x_local, iters, resid) is called every `cb_every` iterations (the
        reference's 2-minute checkpoint / progress hook, iterative_solver.py:874-965)."""
        early = self.pcg_start(b_local, x0_local, tol, maxiter)
        status = self.pcg_result()[1]
        step = int(cb_every) if cb_every and cb_every > 0 else self._maxiter
        while status == nat.PCG_RUNNING:
            status = self.pcg_run(step, chunk)
            if callback is not None and status == nat.PCG_RUNNING:
                it, _, res, _ = self.pcg_result()
                callback(self.pcg_x(), it, res)
        it, status, resid, info = self.pcg_result()
        x = self.pcg_x()
        trace = self.pcg_trace()
        # scipy 1.7.3 calls callback(x) at the start of iterations 2..m and once at the
        # end: m calls for m >= 1 iterations, one call when ||r0|| < atol, none on the
        # legacy early exit.
        callbacks = 0 if early else max(it, 1)
        return PCGResult(x=x, info=info, iters=it, resid=resid, trace=trace,
                         early_exit=early, callbacks=callbacks)

    # ------------------------------------------------------------------- timing
    def timing(self, on: bool | int = True):
        """True / 1: bracket every PCG iteration with timing events; n > 1: every n-th
        iteration only (events cost GPU time); False / 0: off."""
        self._call("mlff_timing_enable", int(on) if not isinstance(on, bool) else int(on))

    def timing_reset(self):
        self._call("mlff_timing_reset")

    def timing_read(self) -> dict:
        gm, gc, im, ic = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
        self._call("mlff_timing_read", ctypes.byref(gm), ctypes.byref(gc), ctypes.byref(im),
                   ctypes.byref(ic))
        pm, pc = ctypes.c_double(), ctypes.c_int64()
        self._call("mlff_timing_read_precon", ctypes.byref(pm), ctypes.byref(pc))
        cm, cc = ctypes.c_double(), ctypes.c_int64()
        self._call("mlff_timing_read_comm", ctypes.byref(cm), ctypes.byref(cc))
        return {"gemv_ms": gm.value, "gemv_count": gc.value, "iter_ms": im.value,
                "iter_count": ic.value, "precon_ms": pm.value, "precon_count": pc.value,
                "comm_ms": cm.value, "comm_count": cc.value}

    def device_memory(self) -> tuple[int, int]:
        """(free, total) bytes of this context's device."""
        fr, tot = ctypes.c_int64(), ctypes.c_int64()
        self._call("mlff_device_memory", ctypes.byref(fr), ctypes.byref(tot))
        return fr.value, tot.value


def host_descriptors(R: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Desc.from_R on the host, the way the reference's trainer forms the descriptors it hands
    to Iterative.solve (desc.py:80-110 scipy pdist, :112-201 1/r and (r_a - r_b)/r^3; no cutoff,
    no PBC): the same bits as the reference's, so a solve from them is the reference's system
    exactly.  R: M x n_atoms x 3.  (sgdml_descriptors forms them on the GPU, equal to rounding.)"""
    R = np.asarray(R, dtype=np.float64)
    a, b = np.tril_indices(R.shape[1], k=-1)
    diff = R[:, a, :] - R[:, b, :]
    r = np.sqrt(np.sum(diff ** 2, axis=2))
    return 1.0 / r, diff / (r ** 3)[:, :, None]


def sgdml_descriptors(R: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Desc.from_R on the GPU (desc.py:292-358; no cutoff, no PBC).  R: M x n_atoms x 3."""
    lib = nat.load_library()
    R = np.ascontiguousarray(R, dtype=np.float64)
    M, n = R.shape[0], R.shape[1]
    D = n * (n - 1) // 2
    Rd = np.empty((M, D))
    Rdd = np.empty((M, D, 3))
    nat.check(lib.mlff_sgdml_descriptors(nat.dptr(R), M, n, nat.dptr(Rd), nat.dptr(Rdd)), None,
              "mlff_sgdml_descriptors")
    return Rd, Rdd
