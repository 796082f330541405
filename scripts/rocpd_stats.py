"""Per-kernel duration statistics (count, mean, median, total) from a rocprofv3 rocpd
SQLite database (`rocprofv3 --kernel-trace -d DIR -o NAME` writes NAME_results.db when no
--output-format is given), split by grid size like scripts/ktrace_by_grid.py.

    python scripts/rocpd_stats.py gpurun_out/rec_prof/nt_results.db [--top 30]
"""
import argparse
import sqlite3
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    d = defaultdict(list)
    for kid, gx, t0, t1 in c.execute(
            "select kernel_id, grid_size_x, start, end from rocpd_kernel_dispatch"):
        d[(names.get(kid, str(kid)), gx)].append((t1 - t0) / 1e3)
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'kernel':52s} {'grid':>8s} {'calls':>6s} {'mean us':>9s} {'median us':>10s} {'total ms':>9s}")
    for (k, gx), v in rows[:a.top]:
        print(f"{k[:52]:52s} {gx:8d} {len(v):6d} {statistics.mean(v):9.2f} "
              f"{statistics.median(v):10.2f} {sum(v) / 1e3:9.2f}")


if __name__ == "__main__":
    main()
