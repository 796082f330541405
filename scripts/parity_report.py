"""Parity report: the drop-in Iterative.solve on the GPU against the reference's own
solves stored in tests/golden/ (iterations, residual curve, coefficients).

    python scripts/parity_report.py > profiles/r02/parity_report.txt   (on the GPU box)

Columns band_it / band_dx: the CPU oracle's own spread under a change of summation order
(tests/golden/noise_band.json); tests/parity.py holds |it_gpu - it_ref| <= 2 band_it + 2.
"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

import sgdml_amd  # noqa: E402
from tests.parity import noise_band  # noqa: E402
from tests.test_gpu_golden import PRECONS, SEEDS, run_dropin  # noqa: E402

CASES = [("sgdml_ethanol_n270", p) for p in PRECONS] + [
    ("sgdml_ethanol_n270_perms", p) for p in ["cholesky", "random_scores", "truncated_cholesky_custom"]] + [
    ("sgdml_ethanol_n621", p) for p in ["cholesky", "random_scores", "truncated_cholesky"]] + [
    ("sgdml_ethanol_n2997", p) for p in ["cholesky", "random_scores"]] + [
    ("sgdml_nanotube_n3330", p) for p in ["cholesky", "random_scores"]]


def main():
    gd = REPO / "tests" / "golden"
    print(f"{'fixture':28s} {'preconditioner':26s} {'N':>5s} {'k':>4s} {'it_ref':>6s} {'it_gpu':>6s} "
          f"{'dlog10 r[:8]':>12s} {'|da|/|a|':>9s} {'resid_gpu/tol|y|':>16s} {'band_it':>7s} {'band_dx':>8s}")
    for name, precon in CASES:
        f = np.load(gd / f"{name}.npz", allow_pickle=False)
        desc = sgdml_amd.sgdml_descriptors(f["R"]) if "R_desc" not in f.files else None
        alphas, it, resid, rmse, idxs, conv, info = run_dropin(f, name, precon, desc)
        ref_tr = f[f"{precon}__trace"]
        tr = info["resid_trace"][1:]
        m = min(8, len(tr), len(ref_tr))
        d = np.max(np.abs(np.log10(tr[:m] / ref_tr[:m])))
        ra = f[f"{precon}__alphas"]
        da = np.linalg.norm(alphas - ra) / np.linalg.norm(ra)
        n = f["y"].size
        b = noise_band(f"{name}/{precon}")
        print(f"{name:28s} {precon:26s} {n:5d} {int(f['k_rot']):4d} {int(f[f'{precon}__num_iters']):6d} "
              f"{it:6d} {d:12.1e} {da:9.1e} {resid / (float(f['solver_tol']) * np.linalg.norm(f['y'])):16.3f} "
              f"{b['band_iters']:7d} {b['band_rel_dalpha']:8.1e}",
              flush=True)


if __name__ == "__main__":
    main()
