"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of a kernel GROUP (one launch of each
kernel per CG iteration, e.g. the low-rank apply's T r, T^T t and finisher) into
profiles/pmc_traffic.json, counting only the solve phase: the dispatches after the last one
whose name contains AFTER (the build calls some of the same kernels at other sizes).

    python scripts/pmc_group.py KEY FETCH_DIR WRITE_DIR ALG_BYTES AFTER "SUB1|SUB2|..." [note]

HBM bytes per group launch = sum over the group's kernels of the per-kernel medians of
2 * FETCH_SIZE + WRITE_SIZE (kB -> B), per MI355X_MICROARCH.md (HBM section: on gfx950
FETCH_SIZE reports 1/2 of wide coalesced streaming reads)."""
import csv
import json
import statistics
import sys
from pathlib import Path

key, fdir, wdir, alg, after, subs = sys.argv[1:7]
note = sys.argv[7] if len(sys.argv) > 7 else None
subs = subs.split("|")


def per_kernel(d):
    rows = sorted(csv.DictReader(open(Path(d) / "bench_counter_collection.csv")),
                  key=lambda r: int(r["Dispatch_Id"]))
    last = max((i for i, r in enumerate(rows) if after and after in r["Kernel_Name"]), default=-1)
    rows = rows[last + 1:]
    out = {}
    for s in subs:
        v = [float(r["Counter_Value"]) for r in rows if s in r["Kernel_Name"]]
        if not v:
            raise SystemExit(f"no solve-phase dispatch of '{s}' in {d}")
        out[s] = (statistics.median(v), len(v))
    return out


f = per_kernel(fdir)
w = per_kernel(wdir)
parts = {s: {"FETCH_SIZE_kB_median": f[s][0], "WRITE_SIZE_kB_median": w[s][0], "launches": f[s][1],
             "hbm_bytes": 2 * f[s][0] * 1024 + w[s][0] * 1024} for s in subs}
hbm = sum(p["hbm_bytes"] for p in parts.values())
p = Path(__file__).resolve().parents[1] / "profiles" / "pmc_traffic.json"
d = json.loads(p.read_text()) if p.exists() else {}
d[key] = {"kernel": " + ".join(subs), "per_kernel": parts,
          "correction": "hbm = sum_k (2 * FETCH_SIZE_k + WRITE_SIZE_k) * 1024 (MI355X_MICROARCH.md HBM: "
                        "FETCH_SIZE reads 1/2 of wide coalesced streaming reads on gfx950)",
          "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": float(alg),
          "traffic_over_algorithmic": hbm / float(alg),
          "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), {fdir}, {wdir}; "
                    f"solve-phase dispatches after the last '{after}'"}
if note:
    d[key]["note"] = note
p.write_text(json.dumps(d, indent=1) + "\n")
print(key, d[key]["traffic_over_algorithmic"], hbm)
