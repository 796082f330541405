"""Print a rocprofv3 kernel_stats.csv as name / calls / average us (top entries)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
    print(f"{name:62s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:10.1f} us")
