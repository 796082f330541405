"""Per-kernel durations of the solve phase from a rocprofv3 kernel_trace.csv: the
dispatches after the last one whose name contains AFTER (default: the pivoted-Cholesky
finisher), so build launches of the same kernels do not mix in.  Also prints the mean
gap between consecutive dispatches (launch overhead the queue does not hide)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
after = sys.argv[2] if len(sys.argv) > 2 else "k_piv_fin"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = max((i for i, r in enumerate(rows) if after in r["Kernel_Name"]), default=-1)
rows = rows[last + 1:]
dur = defaultdict(list)
gaps = []
for a, b in zip(rows, rows[1:]):
    gaps.append(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
    dur[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in dur.values())
print(f"{len(rows)} dispatches after the last '{after}'; busy {tot / 1e3:.1f} us")
for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{name:62s} {len(v):6d} avg {sum(v) / len(v) / 1e3:8.2f} us  med {v[len(v) // 2] / 1e3:8.2f}")
if gaps:
    gaps.sort()
    print(f"gap between dispatches: mean {sum(gaps) / len(gaps) / 1e3:.2f} us, median {gaps[len(gaps) // 2] / 1e3:.2f} us")
