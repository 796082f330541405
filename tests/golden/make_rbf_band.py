"""Noise band and CPU reference solve of the headline RBF system (BASELINE configs[2]).

The bench's `value` workload (bench.py): x ~ U[0,1)^3 (numpy default_rng seed 0), sklearn
RBF with length scale 0.2 (the reference's generator, src/tools/utils.py:173-187), A = K +
1e-6 I, b = sum(x^2), rank-256 Nystrom preconditioner on uniform random columns
(`random_scores`, default_rng(0)), solved to relres 1e-6 by the scipy-1.7.3 CG recurrence
(iterative_solver.py:995-1005; oracle.pcg.cg_legacy).

1. N = 8192 (`--band`, ~10 min on 8 cores): the oracle solve in several summation orders of
   the mat-vec and of the panel apply (tests/golden/make_noise_band.py's idea, applied to the
   dense RBF K, whose mat-vec IS the reference's operator here):
     blas    K @ v, T.T @ (T @ r)                         (NumPy/OpenBLAS: the reference's order)
     rev     columns reversed
     blk7    7 column blocks added in block order
     blk512  512-column tiles (the GPU's tile width)
     pair    np.einsum pairwise sums
     tiles   lower-triangle 512 x 512 tiles, row and column partials (oracle/rbf_tiles.c: the
             GPU's storage) with the panel in 512-column tiles
   The spread against the blas solve is the band (iterations, half-decade crossings of the
   running-minimum residual, ||dx|| / ||x||) -> rbf_band_n8192.npz / .json.
2. N = 65536 (`--full`, ~2-3 h on 8 cores, 17.3 GB of RAM): the oracle solve with the tiled
   mat-vec (a dense 34.4 GB NumPy K does not fit next to the rest) -> rbf_solve_n65536.npz:
   iterations, final relres, trace, x; `--full --order tiles_rev`: the same solve in a second
   summation order (tiles, tile rows and thread partials reversed, panel columns reversed) ->
   rbf_solve_n65536_rev.npz.  The GPU solve of the same system is held to the
   N = 8192 band scaled by the iteration count (tests/test_gpu_rbf_band.py).

CPU only; the reference is not imported (its RBF generator is sklearn's formula, restated in
oracle/rbf.py and oracle/rbf_tiles.c).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

from oracle.pcg import cg_legacy  # noqa: E402
from oracle.precon import apply_panel, nystrom_panel  # noqa: E402
from oracle.rbf import rbf_kernel  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402  (input generation only)

GOLDEN = REPO / "tests" / "golden"
LAM, ELL, K_RANK, TOL = 1e-6, 0.2, 256, 1e-6
sys.path.insert(0, str(GOLDEN))
from make_noise_band import half_decade_crossings, make_gemv  # noqa: E402


def tiles_lib():
    so = REPO / "oracle" / "_build" / "librbftiles.so"
    src = REPO / "oracle" / "rbf_tiles.c"
    if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
        so.parent.mkdir(parents=True, exist_ok=True)
        subprocess.run(["gcc", "-O3", "-fopenmp", "-shared", "-fPIC", str(src), "-o", str(so),
                        "-lm"], check=True)
    lib = ctypes.CDLL(str(so))
    P = ctypes.POINTER(ctypes.c_double)
    I64 = ctypes.c_int64
    lib.rbf_tiles_count.restype = I64
    lib.rbf_tiles_count.argtypes = [I64]
    lib.rbf_tiles_gen.argtypes = [P, I64, ctypes.c_int, P]
    lib.rbf_tiles_cols.argtypes = [P, I64, ctypes.POINTER(I64), I64, P]
    lib.rbf_tiles_symv.argtypes = [P, I64, P, P]
    lib.rbf_tiles_symv_rev.argtypes = [P, I64, P, P]
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class Tiles:
    def __init__(self, X, ell):
        self.lib = tiles_lib()
        self.n = X.shape[0]
        Xs = np.ascontiguousarray(X / ell)
        self.t = np.empty(int(self.lib.rbf_tiles_count(self.n)) * 512 * 512)
        self.lib.rbf_tiles_gen(_p(Xs), self.n, Xs.shape[1], _p(self.t))

    def matvec(self, v, reverse=False):
        v = np.ascontiguousarray(v, dtype=np.float64)
        y = np.empty(self.n)
        (self.lib.rbf_tiles_symv_rev if reverse else self.lib.rbf_tiles_symv)(
            _p(self.t), self.n, _p(v), _p(y))
        return y

    def cols(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        out = np.empty((self.n, idx.size))
        self.lib.rbf_tiles_cols(_p(self.t), self.n,
                                idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), idx.size,
                                _p(out))
        return out


def problem(n):
    X, b = synthetic.rbf_points(n, 3, 0)
    idx = np.sort(np.random.default_rng(0).choice(n, K_RANK, replace=False))
    return X, b, idx


ORDERS = ["blas", "rev", "blk7", "blk512", "pair", "tiles"]


def band(n=8192, orders=None):
    """orders: a subset of ORDERS (always with "blas", the reference's order the band is
    measured from); N = 32768 runs the four orders that take minutes, not hours, at that size
    (rev / pair: ~3 h each)."""
    orders = ORDERS if not orders else ["blas"] + [o for o in orders if o != "blas"]
    X, b, idx = problem(n)
    K = rbf_kernel(X, ELL)
    B, sp = nystrom_panel(K[:, idx], idx, LAM, 0)
    tiles = Tiles(X, ELL)
    panel_order = {"blas": "blas", "rev": "rev", "blk7": "blk7", "blk512": "blk512",
                   "pair": "pair", "tiles": "blk512"}
    runs = {}
    for order in orders:
        t0 = time.time()
        mvK = tiles.matvec if order == "tiles" else make_gemv(K, order)
        mvT = make_gemv(B, panel_order[order])
        mvTt = make_gemv(np.ascontiguousarray(B.T), panel_order[order])
        x, info, tr, it = cg_legacy(lambda v: mvK(v) + LAM * v, b, tol=TOL, maxiter=5 * n,
                                    psolve=lambda r: sp * ((r - mvTt(mvT(r))) / LAM))
        runs[order] = (x, info, tr, it)
        print(f"n={n} {order:7s} iters {it} info {info} ({time.time() - t0:.0f} s)", flush=True)
    x0, _, tr0, it0 = runs["blas"]
    top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
    cr0 = half_decade_crossings(tr0[1:], top)
    variants = {}
    for order, (x, info, tr, it) in runs.items():
        cr = half_decade_crossings(tr[1:], top)
        dc = [abs(cr[k] - cr0[k]) for k in cr0 if k in cr]
        variants[order] = {"iters": int(it), "info": int(info), "d_iters": int(it - it0),
                           "max_d_crossing": int(max(dc) if dc else 0),
                           "rel_dx": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}
    v = variants.values()
    out = {"n": n, "k": K_RANK, "lam": LAM, "ell": ELL, "tol": TOL, "ref_order": "blas",
           "ref_iters": int(it0), "variants": variants,
           "band_iters": int(max(abs(e["d_iters"]) for e in v)),
           "band_crossing": int(max(e["max_d_crossing"] for e in v)),
           "band_rel_dx": float(max(e["rel_dx"] for e in v))}
    out["orders"] = list(runs)
    tiles = {"tiles_x": runs["tiles"][0], "tiles_trace": runs["tiles"][2]} if "tiles" in runs else {}
    np.savez_compressed(GOLDEN / f"rbf_band_n{n}.npz", x=x0, trace=tr0, iters=np.int64(it0),
                        idx=idx, **tiles, **{f"trace_{o}": r[2] for o, r in runs.items()})
    (GOLDEN / f"rbf_band_n{n}.json").write_text(json.dumps(out, indent=1, sort_keys=True))
    print(json.dumps({k: out[k] for k in ("ref_iters", "band_iters", "band_crossing",
                                          "band_rel_dx")}), flush=True)


def extended(n=8192):
    """The N = n system in extended precision (np.longdouble products and sums of the mat-vec
    and of the panel apply, rounded to fp64 once per operator application): where the count lands
    when the operator's rounding error shrinks -- rbf_ld_n{n}.json."""
    X, b, idx = problem(n)
    K = rbf_kernel(X, ELL)
    B, sp = nystrom_panel(K[:, idx], idx, LAM, 0)
    t0 = time.time()
    mvK, mvT = make_gemv(K, "ld"), make_gemv(B, "ld")
    mvTt = make_gemv(np.ascontiguousarray(B.T), "ld")
    x, info, tr, it = cg_legacy(lambda v: mvK(v) + LAM * v, b, tol=TOL, maxiter=5 * n,
                                psolve=lambda r: sp * ((r - mvTt(mvT(r))) / LAM))
    f = np.load(GOLDEN / f"rbf_band_n{n}.npz", allow_pickle=False)
    out = {"n": n, "order": "ld", "iters": int(it), "info": int(info),
           "rel_dx_vs_blas": float(np.linalg.norm(x - f["x"]) / np.linalg.norm(f["x"])),
           "seconds": time.time() - t0}
    (GOLDEN / f"rbf_ld_n{n}.json").write_text(json.dumps(out, indent=1, sort_keys=True))
    print(json.dumps(out), flush=True)


def full(n=65536, order="tiles"):
    """order: 'tiles' (rbf_tiles_symv, the committed rbf_solve_n65536.npz) or 'tiles_rev'
    (rbf_tiles_symv_rev with the panel apply in reversed column order: a second sample of the
    oracle's solve, rbf_solve_n65536_rev.npz)."""
    X, b, idx = problem(n)
    t0 = time.time()
    tiles = Tiles(X, ELL)
    S_nm = tiles.cols(idx)
    B, sp = nystrom_panel(S_nm, idx, LAM, 0)
    del S_nm
    print(f"n={n}: tiles + panel in {time.time() - t0:.0f} s", flush=True)
    t0 = time.time()
    state = {"it": 0}

    def cb(_x):
        state["it"] += 1
        if state["it"] % 250 == 0:
            el = time.time() - t0
            print(f"  iteration {state['it']}  {el:.0f} s ({el / state['it']:.2f} s/it)",
                  flush=True)

    rev = order == "tiles_rev"
    if rev:
        mvT = make_gemv(B, "rev")
        mvTt = make_gemv(np.ascontiguousarray(B.T), "rev")
        psolve = lambda r: sp * ((r - mvTt(mvT(r))) / LAM)  # noqa: E731
    else:
        psolve = lambda r: apply_panel(B, sp, LAM, r)  # noqa: E731
    x, info, tr, it = cg_legacy(lambda v: tiles.matvec(v, reverse=rev) + LAM * v, b, tol=TOL,
                                maxiter=20000, psolve=psolve, callback=cb)
    el = time.time() - t0
    relres = float(np.linalg.norm(b - (tiles.matvec(x) + LAM * x)) / np.linalg.norm(b))
    np.savez_compressed(GOLDEN / f"rbf_solve_n{n}{'_rev' if rev else ''}.npz", x=x, trace=tr,
                        iters=np.int64(it),
                        info=np.int64(info), idx=idx, final_relres=relres,
                        x_norm=np.linalg.norm(x), seconds=el)
    print(json.dumps({"n": n, "iters": int(it), "info": int(info), "final_true_relres": relres,
                      "x_norm": float(np.linalg.norm(x)), "seconds": el}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--band", action="store_true")
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--order", choices=["tiles", "tiles_rev"], default="tiles")
    ap.add_argument("--ld", action="store_true", help="extended-precision solve of --n")
    ap.add_argument("--orders", nargs="+", choices=ORDERS, default=None)
    a = ap.parse_args()
    if a.ld:
        extended(a.n or 8192)
    if a.band:
        band(a.n or 8192, a.orders)
    if a.full:
        full(a.n or 65536, a.order)
