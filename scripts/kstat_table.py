"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg us, total ms)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:n]:
    name = r["Name"].split("(")[0].replace("mlff::", "").replace("(anonymous namespace)::", "")
    print(f"{name[:58]:58s} {r['Calls']:>7s} {float(r['AverageNs']) / 1e3:9.2f}us "
          f"{float(r['TotalDurationNs']) / 1e6:9.2f}ms")
