"""Iteration counts of the ragged-shard matrix-free solve (tests/test_gpu_matfree.py::
test_matfree_ragged_shards) for W = 1 and several W, to tell a rounding lottery from a
W-dependent operator (MLFF_LIB selects a library variant)."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]
import sgdml_amd as sg  # noqa: E402
from tests.test_gpu_multirank import run_ranks  # noqa: E402

f = np.load(REPO / "tests/golden/sgdml_ethanol_n270.npz")
for m in (1, 2, 3):
    Rd, Rdd = f["R_desc"][:m], f["R_d_desc"][:m]
    n, sig = 27 * m, float(f["sig"])
    lam = 1e-3 * float(np.abs(f["diag_K"][:n]).mean())
    y = np.ascontiguousarray(f["y"][:n])
    k = min(6, n)

    def body(rank, w, key):
        with sg.KernelSolver(n, device=0, rank=rank, world=w, comm_id=key if w > 1 else None) as s:
            s.sgdml_operator(Rd, Rdd, f["perms"], sig)
            s.set_operator(-1.0, lam)
            s.precon_pivchol(k)
            r0, r1 = s.row_range()
            res = s.pcg(np.ascontiguousarray(y[r0:r1]), tol=1e-8, maxiter=10 * n)
            return res.iters, res.trace

    out = []
    for w in (1, 2, 5, 7, 8):
        it, tr = run_ranks(w, body, timeout=120)[0]
        out.append(f"W={w}:{it}")
    print(f"m={m}", " ".join(out), flush=True)
