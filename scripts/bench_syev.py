"""Cost of the device eigenvalue step of _cho_factor_stable (iterative_solver.py:555-583) at
build sizes: sym_min_eig alone (kernels_syev.hip: dsytd2-style tridiagonalisation + Sturm
bisection) against the Nystrom build it sits in (two calls per build, iterative_solver.py:218,
235), on the nanotube geometry at the rule-of-thumb ranks k = 2701 (N = 15540, M = 14) and
k = 14670 (N = 156510, M = 141).

    python scripts/bench_syev.py [--m 14 141]

Prints one JSON line per size: wall seconds of sym_min_eig (median of 3; includes the host ->
device copy of the k x k matrix, so run it under rocprofv3 --kernel-trace --stats for the
kernels' own time), of the whole Nystrom build (random_scores columns, variant 0) and the ratio.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[14, 141])
    a = ap.parse_args()
    import sgdml_amd
    from sgdml_amd import synthetic
    from sgdml_amd.rule_of_thumb import get_params, rule_of_thumb

    for M in a.m:
        ds = synthetic.nanotube_like(M, seed=0)
        n = 3 * 370 * M
        mm, kmin, _ = get_params("nanotube")
        k = int(rule_of_thumb(n=n, k_min=kmin, m=mm))
        Rd, Rdd = sgdml_amd.sgdml_descriptors(ds["R"])
        idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False)).astype(np.int64)
        rng = np.random.default_rng(1)
        B = rng.standard_normal((k, k))
        S = (B + B.T) * 0.5 + k * np.eye(k)   # symmetric, O(k^2) to form
        with sgdml_amd.KernelSolver(n) as s:
            s.sgdml_operator(Rd, Rdd, np.arange(370)[None, :], 10.0)
            s.set_operator(-1.0, 1e-10)
            t_eig = []
            for _ in range(3):
                s.synchronize()
                t0 = time.perf_counter()
                s.sym_min_eig(S)
                t_eig.append(time.perf_counter() - t0)
            t_nys = s.precon_nystrom(idx, variant=0)
        te = sorted(t_eig)[1]
        print(json.dumps({"M": M, "n": n, "k": k, "sym_min_eig_s": te, "sym_min_eig_samples": t_eig,
                          "nystrom_build_s": t_nys, "two_calls_over_build": 2 * te / t_nys}),
              flush=True)


if __name__ == "__main__":
    main()
