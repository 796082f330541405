"""Diagnostic: ragged-shard cases one at a time, with progress lines and thread stacks on a stall.

Usage (GPU box): timeout -k 10 170 python -u scripts/dev/diag_ragged.py [n ...]
"""
import faulthandler
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "mlff-preconditioner_amd"))
import sgdml_amd  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402

faulthandler.dump_traceback_later(40, repeat=True, file=sys.stdout)


def log(*a):
    print(f"[{time.monotonic() - T0:7.2f}]", *a, flush=True)


T0 = time.monotonic()


def run(n, world, storage):
    X, b = synthetic.rbf_points(n, 3, n)
    v = np.random.default_rng(n).standard_normal(n)
    k = max(1, min(40, n // 3))
    key = f"LOCAL:diag-{np.random.default_rng().integers(1 << 62)}".encode().ljust(128, b"\0")
    out = [None] * world

    def body(r):
        try:
            s = sgdml_amd.KernelSolver(n, device=0, rank=r, world=world, comm_id=key if world > 1 else None)
            log(f"  r{r} ctx rows={s.row_range()}")
            s.gen_rbf(X, 0.3)
            s.set_operator(1.0, 0.5)
            s.set_storage(storage)
            y = s.matvec(v)
            log(f"  r{r} matvec ok")
            s.precon_pivchol(k)
            log(f"  r{r} pivchol ok")
            r0, r1 = s.row_range()
            res = s.pcg(np.ascontiguousarray(b[r0:r1]), tol=1e-10, maxiter=5 * n + 5)
            log(f"  r{r} pcg iters={res.iters} info={res.info}")
            s.close()
            out[r] = (y, res.x, res.iters, res.info)
        except BaseException as e:  # noqa: BLE001
            log(f"  r{r} ERROR {type(e).__name__}: {e}")
            out[r] = e

    th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
        if t.is_alive():
            log("  HUNG")
            faulthandler.dump_traceback(file=sys.stdout)
            os._exit(3)
    return out


ns = [int(a) for a in sys.argv[1:]] or [1, 2, 63, 513, 1100, 2049]
for n in ns:
    for world in (1, 2, 5, 8):
        for storage in ("sym", "dense"):
            log(f"n={n} world={world} storage={storage}")
            run(n, world, storage)
log("done")
os._exit(0)
