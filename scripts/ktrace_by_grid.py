"""Per-(kernel, grid size) launch counts and durations from a rocprofv3 kernel_trace.csv.

The default bench command launches the operator kernels at three sizes (the timed N = 65536
iterations, the N = 8192 parity solve, the CPU-baseline copy), so the kernel_stats average
mixes them; this splits them by grid so the N = 65536 average can be compared with the
HIP-event time in the bench line.
    python scripts/ktrace_by_grid.py TRACE.csv [TOP]
"""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
d = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("mlff::", "")
    name = name.replace("void ", "").split("(")[0][-48:]
    d[(name, int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':48s} {'grid':>10s} {'calls':>6s} {'mean us':>10s} {'median us':>10s} {'total ms':>10s}")
for (name, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{name:48s} {g:10d} {len(v):6d} {statistics.mean(v):10.2f} {statistics.median(v):10.2f} "
          f"{sum(v) / 1e3:10.2f}")
