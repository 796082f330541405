"""Per-kernel medians of rocprofv3 --pmc passes over the solve phase of a bench run.

    python scripts/pmc_kernel_medians.py OUT.csv AFTER_KERNEL DIR [DIR ...]

Each DIR holds one pass's *counter_collection.csv (scripts/gpu_pmc_nt.sh writes
gpurun_out/r02_nt_{FETCH_SIZE,WRITE_SIZE,TCC_HIT_sum}).  Dispatches after the last one
whose name contains AFTER_KERNEL (the end of the preconditioner build) are the solve
phase; the medians per (kernel, counter) are written to OUT.csv in kB for the *_SIZE
counters and in requests for the TCC_* counters.
"""
from __future__ import annotations

import csv
import statistics
import sys
from pathlib import Path


def short_name(name: str) -> str:
    k = name.replace("(anonymous namespace)::", "").replace("mlff::", "").replace("void ", "")
    return k.split("(")[0]


def main():
    out, after, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    acc: dict[str, dict[str, list[float]]] = {}
    for d in dirs:
        f = next(Path(d).rglob("*counter_collection.csv"))
        rs = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        last = max((i for i, r in enumerate(rs) if after in r["Kernel_Name"]), default=-1)
        for r in rs[last + 1:]:
            acc.setdefault(short_name(r["Kernel_Name"]), {}).setdefault(
                r["Counter_Name"], []).append(float(r["Counter_Value"]))
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "counter", "median_per_launch", "launches"])
        for k in sorted(acc):
            for c in sorted(acc[k]):
                v = acc[k][c]
                w.writerow([k, c, statistics.median(v), len(v)])
                print(f"{k:40s} {c:14s} {statistics.median(v):14.1f} x{len(v)}")


if __name__ == "__main__":
    main()
