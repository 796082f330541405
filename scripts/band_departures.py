"""Where the configs[2] oracle orders leave each other (tests/golden/rbf_band_n16384.npz: the
residual traces of the six summation orders of make_rbf_band.py --band --n 16384).

    python scripts/band_departures.py [--n 16384]

For every order against the BLAS-order solve: the first iteration at which the stop-test
residuals differ by more than 1e-14 / 1e-12 / 1e-10 / 1e-6 / 1e-3 in log10.  CPU only (reads the
committed fixture).
"""
from __future__ import annotations

import argparse
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]


def first_departure(tr, ref, tol):
    m = min(len(tr), len(ref))
    d = np.abs(np.log10(np.asarray(tr[1:m]) / np.asarray(ref[1:m])))
    hit = np.nonzero(d > tol)[0]
    return int(hit[0]) + 1 if hit.size else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    a = ap.parse_args()
    f = np.load(REPO / "tests" / "golden" / f"rbf_band_n{a.n}.npz", allow_pickle=False)
    ref = f["trace_blas"]
    tols = (1e-14, 1e-12, 1e-10, 1e-6, 1e-3)
    print(f"N = {a.n}: first iteration with |log10(r / r_blas)| above " + " / ".join(map(str, tols)))
    for o in ("rev", "blk7", "blk512", "pair", "tiles"):
        tr = f[f"trace_{o}"]
        print(f"  {o:7s} {len(tr) - 1:5d} iterations: "
              + " / ".join(str(first_departure(tr, ref, t)) for t in tols))


if __name__ == "__main__":
    main()
