"""Per-iteration kernels of a rocprofv3 --kernel-trace --stats run: the kernels called once per
PCG step (calls within +-4 of the step count), their mean / min durations and their sum.

    python scripts/kstat_iter.py <kernel_stats.csv> <steps>
"""
import csv
import sys


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = 0.0
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        if abs(int(r["Calls"]) - steps) <= 4:
            a = float(r["AverageNs"]) / 1e3
            tot += a
            print(f"  {r['Name'][:96]:96s} calls {r['Calls']:>6s} avg {a:8.2f} us "
                  f"min {float(r['MinNs']) / 1e3:7.2f}")
    print(f"  sum {tot:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
