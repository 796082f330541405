"""CPU spread of the random-panel low-rank solves of tests/test_gpu_core.py::test_one_pass_lowrank_apply
across summation orders (the oracle's scipy-1.7.3 CG, oracle/pcg.py, on K + lam I with the
Woodbury panel of the test's random L, oracle/precon.py).

Orders: the mat-vec as one BLAS GEMV or as 512-column tile sums; the apply's t = T r as one GEMV
or as per-segment partials (the cluster apply's member segments: 8192 or 7168 columns) added in
member order.  Prints each order's count and every half-decade crossing of the running-minimum
residual, and the largest crossing difference between any two orders (the chaotic contract of
tests/parity.py compares one such pair).

    python scripts/dev/lowrank_chaotic_band.py --n 20000 --k 400
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "mlff-preconditioner_amd"))

from oracle.pcg import cg_legacy  # noqa: E402
from oracle.precon import woodbury_panel  # noqa: E402
from oracle.rbf import rbf_kernel  # noqa: E402
from parity import envelope  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402


def crossings(trace, top, bot):
    e = envelope(trace)
    out = {}
    for lvl in np.arange(np.floor(top) - 0.5, bot, -0.5):
        out[round(float(lvl), 1)] = int(np.argmax(e <= 10 ** lvl)) if np.any(e <= 10 ** lvl) else len(e)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--k", type=int, default=400)
    ap.add_argument("--save", default="", help="npz of every order's trace")
    args = ap.parse_args()
    n, k, lam = args.n, args.k, 1.0
    X, b = synthetic.rbf_points(n, 3, 0)
    K = rbf_kernel(X, length_scale=0.2)
    rng = np.random.default_rng(n + k)
    L = rng.standard_normal((k, n)) * 0.05
    r_unused = rng.standard_normal(n)  # the test draws r after L (same generator state)
    del r_unused
    T, _ = woodbury_panel(L.T, lam)

    def mv_blas(p):
        return K @ p + lam * p

    def mv_tiles(p):
        y = np.zeros(n)
        for j0 in range(0, n, 512):
            y += K[:, j0:j0 + 512] @ p[j0:j0 + 512]
        return y + lam * p

    def ap_blas(r):
        return (r - T.T @ (T @ r)) / lam

    def ap_seg(seg):
        def f(r):
            t = np.zeros(k)
            for c0 in range(0, n, seg):
                t += T[:, c0:c0 + seg] @ r[c0:c0 + seg]
            return (r - T.T @ t) / lam
        return f

    orders = {"blas/blas": (mv_blas, ap_blas), "tiles/blas": (mv_tiles, ap_blas),
              "tiles/seg8192": (mv_tiles, ap_seg(8192)), "tiles/seg7168": (mv_tiles, ap_seg(7168)),
              "blas/seg4096": (mv_blas, ap_seg(4096))}
    res = {}
    for name, (mv, ps) in orders.items():
        x, info, trace, it = cg_legacy(mv, b, tol=1e-8, maxiter=5 * n, psolve=ps)
        res[name] = (it, trace[1:], x)
        print(f"{name:16s} iters {it} info {info}", flush=True)
    if args.save:
        np.savez(args.save, **{name.replace("/", "_"): v[1] for name, v in res.items()})
    ref = res["blas/blas"]
    top = np.log10(envelope(ref[1])[0])
    bot = min(np.log10(envelope(v[1])[-1]) for v in res.values())
    cr = {name: crossings(v[1], top, bot) for name, v in res.items()}
    for name in res:
        print(name.ljust(16), " ".join(f"{lvl}:{i}" for lvl, i in cr[name].items()))
    names = list(res)
    worst = 0
    for a in range(len(names)):
        for c in range(a + 1, len(names)):
            for lvl in cr[names[a]]:
                worst = max(worst, abs(cr[names[a]][lvl] - cr[names[c]][lvl]))
    x0 = ref[2]
    dx = max(np.linalg.norm(v[2] - x0) / np.linalg.norm(x0) for v in res.values())
    its = [v[0] for v in res.values()]
    print(f"band: iters {min(its)}-{max(its)}, largest crossing difference {worst}, max rel dx {dx:.2e}")


if __name__ == "__main__":
    main()
