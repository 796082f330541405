"""The random-panel solve of tests/test_gpu_core.py::test_one_pass_lowrank_apply[20000-400-0] on the
GPU with the one-pass (cluster) apply and with two passes: traces saved for comparison with the
CPU orders of scripts/dev/lowrank_chaotic_band.py (run under MLFF_LC_CFG to pick the cluster form).

    python scripts/dev/diag_lowrank_20000.py gpurun_out/r04/lr20000_<tag>.npz
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "mlff-preconditioner_amd"))

import sgdml_amd  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402


def main():
    out = sys.argv[1]
    n, k, lam = 20000, 400, 1.0
    X, b = synthetic.rbf_points(n, 3, 0)
    rng = np.random.default_rng(n + k)
    L = rng.standard_normal((k, n)) * 0.05
    traces = {}
    for mode in ("0", "1"):
        os.environ["MLFF_LR_ROWS"] = mode
        with sgdml_amd.KernelSolver(n) as s:
            s.gen_rbf(X, length_scale=0.2)
            s.set_operator(1.0, lam)
            s.precon_lowrank(L)
            form, _ = s.precon_apply_traffic()
            res = s.pcg(b, tol=1e-8, maxiter=5 * n)
            traces[f"form{form}"] = res.trace[1:]
            print(f"mode {mode} form {form} iters {res.iters}", flush=True)
    np.savez(out, **traces)
    for name, t in traces.items():
        e = np.minimum.accumulate(t)
        print(name, "iters", len(t), "envelope at 60..100:",
              " ".join(f"{i}:{np.log10(e[i]):.4f}" for i in range(60, 100, 3)))


if __name__ == "__main__":
    main()
