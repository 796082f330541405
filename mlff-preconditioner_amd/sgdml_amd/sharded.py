"""Several GPUs inside one process: the drop-in's multi-GPU mode.

The reference runs its GPU operator on every GPU of a node from ONE process
(`torch.nn.DataParallel`, src/sGDML/sgdml/predict.py:335-341); `Iterative.solve` is a
single-process API.  `ShardedKernelSolver` keeps that shape: it owns one
`KernelSolver` per device, each driven by its own worker thread (ctypes releases the
GIL, so the ranks' blocking collectives run concurrently), joined by one RCCL
communicator created in-process (`ncclCommInitRank` per thread), or by the library's
in-process transport ("LOCAL:") when two ranks share a device (tests on one GPU).

The methods mirror `KernelSolver` with GLOBAL arrays: inputs are whole N-vectors,
outputs are gathered over the row blocks.  Every call runs on all ranks in the same
order, exactly as the one-process-per-GPU launch of bench.py does.
"""
from __future__ import annotations

import queue
import threading

import numpy as np

from . import _native as nat
from .solver import KernelSolver, PCGResult


class _Worker(threading.Thread):
    def __init__(self, name: str):
        super().__init__(daemon=True, name=name)
        self.q: queue.Queue = queue.Queue()
        self.start()

    def run(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            fn, box, done = item
            try:
                box["value"] = fn()
            except BaseException as e:  # noqa: BLE001 - re-raised by the caller
                box["error"] = e
            done.set()
            # drop the closure while waiting for the next item: it references the
            # ShardedKernelSolver, which must stay collectable
            del item, fn, box, done


class ShardedKernelSolver:
    def __init__(self, n: int, devices, comm: str | None = None):
        devices = [int(d) for d in devices]
        if len(devices) < 2:
            raise ValueError("ShardedKernelSolver needs at least two ranks")
        self.n, self.world, self.devices = int(n), len(devices), devices
        if comm is None:
            comm = "local" if len(set(devices)) < len(devices) else "rccl"
        if comm == "rccl":
            comm_id = nat.comm_unique_id()
        elif comm == "local":
            key = f"LOCAL:sharded-{id(self)}-{np.random.default_rng().integers(1 << 62)}"
            comm_id = key.encode().ljust(128, b"\0")
        else:
            raise ValueError("comm must be 'rccl' or 'local'")
        self.comm = comm
        self._workers = [_Worker(f"mlff-rank{r}-dev{d}") for r, d in enumerate(devices)]
        self.ranks: list[KernelSolver | None] = [None] * self.world
        self._all(lambda r: KernelSolver(n, device=devices[r], rank=r, world=self.world,
                                         comm_id=comm_id), assign=True)
        self.spans = [s.row_range() for s in self.ranks]

    # ------------------------------------------------------------------ dispatch
    def _all(self, fn, assign=False):
        """fn(rank) on every rank's worker thread; returns the per-rank results."""
        boxes, events = [], []
        for r, w in enumerate(self._workers):
            box, done = {}, threading.Event()
            w.q.put((lambda r=r: fn(r), box, done))
            boxes.append(box)
            events.append(done)
        aborted = False
        while not all(e.wait(0.05) for e in events):
            if not aborted and any("error" in b for b in boxes) and self.ranks[0] is not None:
                # a failed rank leaves its peers blocked in a collective: abort their
                # communicators too (the RCCL-documented way to release them)
                aborted = True
                for s in self.ranks:
                    if s is not None and s._ctx is not None:
                        s._lib.mlff_comm_abort(s._ctx)
        for b in boxes:
            if "error" in b:
                raise b["error"]
        out = [b.get("value") for b in boxes]
        if assign:
            self.ranks = out
        return out

    def _each(self, name, *args, **kw):
        return self._all(lambda r: getattr(self.ranks[r], name)(*args, **kw))

    def _gather(self, parts):
        return np.concatenate(parts)

    def _local(self, v, r):
        a, b = self.spans[r]
        return np.ascontiguousarray(v[a:b])

    # --------------------------------------------------------------- lifecycle
    def close(self):
        """Destroy every rank's context and stop the workers.  The contexts are destroyed
        concurrently on the workers (RCCL's communicator teardown waits for the peers);
        from __del__ on a worker thread itself, where that dispatch would wait on the
        calling thread, they are destroyed one by one.  Idempotent."""
        workers = getattr(self, "_workers", None)
        if workers is None:
            return
        try:
            ranks = getattr(self, "ranks", [])
            if threading.current_thread() in workers or any(s is None for s in ranks):
                for s in ranks:
                    if s is not None:
                        s.close()
            else:
                self._each("close")
        finally:
            self._workers = None
            for w in workers:
                w.q.put(None)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ same on all
    def sgdml_operator(self, *a, **k):
        self._each("sgdml_operator", *a, **k)

    def assemble_sgdml(self, *a, **k):
        self._each("assemble_sgdml", *a, **k)

    def gen_rbf(self, *a, **k):
        self._each("gen_rbf", *a, **k)

    def set_operator(self, *a, **k):
        self._each("set_operator", *a, **k)

    def set_storage(self, *a, **k):
        self._each("set_storage", *a, **k)

    def storage_info(self):
        out = self._each("storage_info")
        return out[0][0], float(sum(b for _, b in out))

    def operator_form(self):
        return self._each("operator_form")[0]

    def precon_none(self):
        self._each("precon_none")

    def precon_pivchol(self, k, build_woodbury=True):
        out = self._each("precon_pivchol", k, build_woodbury)
        return out[0]  # index_columns are replicated on every rank

    def pivchol_times(self, k):
        """per-column times of the slowest rank (the build is collective per column)"""
        out = self._each("pivchol_times", k)
        return np.max(np.stack([t for t, _ in out]), axis=0), max(w for _, w in out)

    def precon_nystrom(self, idx, variant=0):
        return max(self._each("precon_nystrom", idx, variant))

    def precon_eig(self, k, mask_mode=0, dim_i=0, build_woodbury=True, want_evals=False,
                   want_rowlev=False):
        """Truncated eigensolver over all ranks (evals and global row norms from rank 0);
        mask_mode 2 masks every rank's rows of the dense K (assemble_sgdml first)."""
        return self._each("precon_eig", k, mask_mode, dim_i, build_woodbury, want_evals,
                          want_rowlev)[0]

    def eig_info(self):
        return self.ranks[0].eig_info()

    def lev_scores(self, idx, lam):
        return self._each("lev_scores", idx, lam)[0]  # global scores on every rank

    def sgdml_energies(self, alphas):
        """(0, E) over all M training points: each point from the first rank that holds
        rows of it (a point split across two ranks is computed by both)."""
        alphas = np.ascontiguousarray(alphas, dtype=np.float64)
        parts = self._each("sgdml_energies", alphas)
        M = max(i0 + e.size for i0, e in parts)
        E = np.full(M, np.nan)
        for i0, e in reversed(parts):
            E[i0:i0 + e.size] = e
        return 0, E

    def timing(self, on=True):
        self._each("timing", on)

    def timing_reset(self):
        self._each("timing_reset")

    def timing_read(self):
        out = self._each("timing_read")
        # the slowest rank bounds the step
        return max(out, key=lambda t: t["iter_ms"])

    # ------------------------------------------------------- gathered results
    def matvec(self, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        return self._gather(self._each("matvec", v))

    def diag(self):
        return self._gather(self._each("diag"))

    def precon_apply(self, r):
        r = np.ascontiguousarray(r, dtype=np.float64)
        return self._gather(self._all(lambda q: self.ranks[q].precon_apply(self._local(r, q))))

    # the PCG primitives of KernelSolver over all ranks (global b / x0 / x): the drop-in's
    # chunked progress / checkpoint loop (solvers/iterative_solver.py _CGStatus) drives these
    def pcg_start(self, b, x0=None, tol=1e-5, maxiter=None):
        b = np.ascontiguousarray(b, dtype=np.float64)
        x0 = None if x0 is None else np.ascontiguousarray(x0, dtype=np.float64)
        early = self._all(lambda r: self.ranks[r].pcg_start(
            self._local(b, r), None if x0 is None else self._local(x0, r), tol, maxiter))[0]
        self._maxiter = self.ranks[0]._maxiter
        return early

    def pcg_run(self, n_iter, chunk=0):
        return self._each("pcg_run", n_iter, chunk)[0]

    def pcg_result(self):
        return self.ranks[0].pcg_result()

    def pcg_x(self):
        return self._gather(self._each("pcg_x"))

    def pcg_trace(self):
        return self.ranks[0].pcg_trace()

    def pcg(self, b, x0=None, tol=1e-5, maxiter=None, callback=None, cb_every=0, chunk=0):
        """KernelSolver.pcg over all ranks (global b / x0 / x); callback(x, iters, resid)
        sees the gathered iterate."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        x0 = None if x0 is None else np.ascontiguousarray(x0, dtype=np.float64)
        early = self._all(lambda r: self.ranks[r].pcg_start(
            self._local(b, r), None if x0 is None else self._local(x0, r), tol, maxiter))[0]
        maxiter = self.ranks[0]._maxiter
        status = self.ranks[0].pcg_result()[1]
        step = int(cb_every) if cb_every and cb_every > 0 else maxiter
        while status == nat.PCG_RUNNING:
            status = self._each("pcg_run", step, chunk)[0]
            if callback is not None and status == nat.PCG_RUNNING:
                it, _, res, _ = self.ranks[0].pcg_result()
                callback(self._gather(self._each("pcg_x")), it, res)
        it, status, resid, info = self.ranks[0].pcg_result()
        x = self._gather(self._each("pcg_x"))
        trace = self.ranks[0].pcg_trace()
        callbacks = 0 if early else max(it, 1)
        return PCGResult(x=x, info=info, iters=it, resid=resid, trace=trace, early_exit=early,
                         callbacks=callbacks)
