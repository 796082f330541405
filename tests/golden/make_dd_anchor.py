"""The exact-sum anchor of configs[2] (GPU script: run on an MI355X through gpurun).

    python tests/golden/make_dd_anchor.py      # -> tests/golden/rbf_dd_n65536.json

The configs[2] system (synthetic RBF N = 65536, x ~ U[0,1)^3 seed 0, length scale 0.2, lambda
1e-6, rank-256 Nystrom random_scores seed 0; bench.py's `value` workload) solved to relres 1e-6
by the scipy-1.7.3 CG recurrence (iterative_solver.py:995-1005) with the operator and the panel
apply in double-double sums rounded once per entry (MLFF_EXACT_SUMS=1, csrc/kernels_dd.hip): the
count the solve takes when the summation order of the mat-vec stops mattering.  The same anchor
at N = 8192 / 16384 is checked against the CPU oracle in np.longdouble (rbf_ld_n*.json,
make_rbf_band.py --ld; tests/test_gpu_exact_sums.py).  Recorded beside it:
  * fp64_distance_fraction: how far fp64 summation orders land from the near-exact count at the
    sizes where both are measured -- |iters - anchor| / anchor of the oracle's six (N = 8192,
    16384) orders against the long-double count, and of the GPU's fp64 solve against the GPU
    anchor (N = 8192, 16384) -- the tolerance tests/test_gpu_exact_sums.py holds the N = 65536
    fp64 solve to;
  * the fp64 GPU solve and the oracle's two N = 65536 orders (rbf_solve_n65536*.npz).
"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]
GOLDEN = REPO / "tests" / "golden"

LAM, ELL, K, TOL = 1e-6, 0.2, 256, 1e-6


def solve(n, exact, maxiter=20000):
    import sgdml_amd
    from sgdml_amd import synthetic

    if exact:
        os.environ["MLFF_EXACT_SUMS"] = "1"
    else:
        os.environ.pop("MLFF_EXACT_SUMS", None)
    X, b = synthetic.rbf_points(n, 3, 0)
    idx = np.sort(np.random.default_rng(0).choice(n, K, replace=False))
    t0 = time.time()
    with sgdml_amd.KernelSolver(n) as s:
        s.gen_rbf(X, ELL)
        s.set_operator(1.0, LAM)
        s.set_storage("dense" if exact else "auto")
        s.precon_nystrom(idx)
        r = s.pcg(b, tol=TOL, maxiter=maxiter)
    os.environ.pop("MLFF_EXACT_SUMS", None)
    print(f"N={n} {'exact' if exact else 'fp64 '}: {r.iters} iterations info {r.info} "
          f"({time.time() - t0:.1f} s)", flush=True)
    return r


def main():
    out = {"n": 65536, "k": K, "lam": LAM, "ell": ELL, "tol": TOL, "order": "double-double sums",
           "fp64_distance_fraction": {}, "anchors": {}}
    for n in (8192, 16384):
        ra, rf = solve(n, True), solve(n, False)
        ld = json.loads((GOLDEN / f"rbf_ld_n{n}.json").read_text())
        bd = json.loads((GOLDEN / f"rbf_band_n{n}.json").read_text())
        out["anchors"][str(n)] = {"gpu_exact": int(ra.iters), "oracle_long_double": ld["iters"],
                                  "gpu_fp64": int(rf.iters),
                                  "oracle_fp64": {o: v["iters"] for o, v in bd["variants"].items()}}
        fr = out["fp64_distance_fraction"]
        fr[f"gpu_fp64_n{n}"] = abs(rf.iters - ra.iters) / ra.iters
        fr[f"oracle_fp64_n{n}"] = max(abs(v["iters"] - ld["iters"]) for v in bd["variants"].values()) \
            / ld["iters"]
    ra = solve(65536, True)
    rf = solve(65536, False)
    out.update(iters=int(ra.iters), info=int(ra.info), final_relres=float(ra.trace[-1] / ra.trace[0]),
               x_norm=float(np.linalg.norm(ra.x)), gpu_fp64_iters=int(rf.iters),
               gpu_fp64_rel_dx=float(np.linalg.norm(rf.x - ra.x) / np.linalg.norm(ra.x)))
    orc = {}
    for name in ("rbf_solve_n65536.npz", "rbf_solve_n65536_rev.npz"):
        if (GOLDEN / name).exists():
            f = np.load(GOLDEN / name, allow_pickle=False)
            orc[name] = int(f["iters"])
            if name == "rbf_solve_n65536.npz":
                out["oracle_rel_dx"] = float(np.linalg.norm(f["x"] - ra.x) / np.linalg.norm(ra.x))
    out["oracle_fp64_iters"] = orc
    dest = Path(os.environ.get("MLFF_GOLDEN_OUT", GOLDEN))  # gpurun: a gpurun_out/ directory
    dest.mkdir(parents=True, exist_ok=True)
    (dest / "rbf_dd_n65536.json").write_text(json.dumps(out, indent=1, sort_keys=True))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
