"""Parity report: the drop-in Iterative.solve on the GPU against the reference's own
solves stored in tests/golden/ (iterations, residual curve, coefficients).

    python scripts/parity_report.py > profiles/r01/parity_report.txt   (on the GPU box)
"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

import sgdml_amd  # noqa: E402
from tests.test_gpu_golden import PRECONS, SEEDS, run_dropin  # noqa: E402

CASES = [("sgdml_ethanol_n270", p) for p in PRECONS] + [
    ("sgdml_ethanol_n270_perms", p) for p in ["cholesky", "random_scores", "truncated_cholesky_custom"]] + [
    ("sgdml_ethanol_n621", p) for p in ["cholesky", "random_scores", "truncated_cholesky"]] + [
    ("sgdml_ethanol_n2997", p) for p in ["cholesky", "random_scores"]] + [
    ("sgdml_nanotube_n3330", p) for p in ["cholesky", "random_scores"]]


def main():
    gd = REPO / "tests" / "golden"
    print(f"{'fixture':28s} {'preconditioner':26s} {'N':>5s} {'k':>4s} {'it_ref':>6s} {'it_gpu':>6s} "
          f"{'dlog10 r[:8]':>12s} {'|da|/|a|':>9s} {'resid_gpu/tol|y|':>16s}")
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
        print(f"{name:28s} {precon:26s} {n:5d} {int(f['k_rot']):4d} {int(f[f'{precon}__num_iters']):6d} "
              f"{it:6d} {d:12.1e} {da:9.1e} {resid / (float(f['solver_tol']) * np.linalg.norm(f['y'])):16.3f}",
              flush=True)


if __name__ == "__main__":
    main()
