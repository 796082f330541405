"""PMC HBM traffic of the bench's dominant kernel groups at the CURRENT sources.

    python scripts/pmc_head.py [--out gpurun_out/pmc_head] [--workloads rbf nanotube]

Runs on the GPU box (the parent never touches the GPU; every profiled program is a child):
for each workload, `python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve ...` under
`rocprofv3 --pmc FETCH_SIZE` and, in a separate pass, `--pmc WRITE_SIZE`
(MI355X_MICROARCH.md: one TCC counter group per pass), each under its own `timeout -s KILL`.
Then folds, per kernel group of the bench line (operator; low-rank apply in the form that
ran), the medians over the timed PCG iterations' dispatches:

    hbm bytes per launch = sum_k (2 * FETCH_SIZE_k + WRITE_SIZE_k) * 1024

(FETCH_SIZE reports 1/2 of wide coalesced streaming reads on gfx950, same guide, HBM
section), next to the algorithmic bytes the bench line reports for the same launch, and
stamps each entry with the content hash of the library sources (bench.csrc_hash()).  The
result, <out>/pmc_traffic.json, is copied to profiles/pmc_traffic.json; bench.py uses an
entry only while its hash matches the sources it runs (else traffic = null + the reason).
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import bench  # noqa: E402  (csrc_hash only; bench imports nothing GPU-side at module level)

STEPS, WARMUP = 6, 1
WORKLOADS = {
    "rbf": ["--configs3-n", "0"],
    "nanotube": ["--workload", "nanotube"],
    # the reference's N = 156510 point (M = 141: Zt stored by k_mf_z, cluster apply)
    "nanotube_m141": ["--workload", "nanotube", "--m", "141"],
    # the many-point ethanol shape (pair-tile operator): configs[0]'s M = 111 and the
    # reference's N = 74979 point
    "ethanol_m111": ["--workload", "ethanol", "--m", "111", "--storage", "matfree"],
    "ethanol_m583": ["--workload", "ethanol", "--m", "583", "--storage", "matfree"],
    "ethanol_m2777": ["--workload", "ethanol", "--m", "2777", "--storage", "matfree"],
}
GROUPS = {
    "sym": ["k_symv_dyn", "k_sym_reduce"],
    "dense": ["k_gemv<4, 4, 1>"],
    "matfree": ["k_mf_z?", "k_rec_g", "k_rec_fin"],  # ?: launched only where it runs
    "matfree_pt": ["k_mf_z", "k_pt_pair", "k_pt_fin"],
    "precon0": ["k_gemv<4, 2, 0>", "k_colgemv_part", "k_precon_fin"],
    "precon1": ["k_lr_rows", "k_lr_fin"],
    "precon2": ["k_lr_cluster", "k_lr_fin"],
}


def kname(full: str) -> str:
    """'void mlff::k_lr_rows<16>(double const*, ...)' -> 'k_lr_rows<16>'."""
    s = full.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
    return s.split("::")[-1]


def matches(full: str, want: str) -> bool:
    """'k_gemv<4, 2, 0>' matches k_gemv<4, 2, 0> and its instantiations with further template
    arguments (k_gemv<4, 2, 0, false>: the load-policy flag of a panel that fits the MALL)."""
    k = kname(full)
    if "<" in want:
        return k == want or k.startswith(want[:-1] + ",")
    return re.sub(r"<.*", "", k) == want


# counters are collected for the measured groups' kernels only (the builds launch ~20k other
# kernels, each of which a --pmc pass would serialize)
KERNEL_REGEX = "|".join(sorted({k.split("<")[0].rstrip("?") for g in GROUPS.values() for k in g}))


def run_pass(wl: str, counter: str, out: Path) -> dict:
    import time

    d = out / f"{wl}_{counter.lower()}"
    d.mkdir(parents=True, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "300", "rocprofv3", "--pmc", counter,
           "--kernel-include-regex", KERNEL_REGEX, "-d", str(d), "-o", "pmc",
           "--output-format", "csv", "--", sys.executable, str(REPO / "bench.py"), "--steps",
           str(STEPS), "--warmup", str(WARMUP), "--no-cpu", "--no-solve", *WORKLOADS[wl]]
    t0 = time.time()
    with open(d / "bench_stdout.txt", "w") as fo:
        p = subprocess.Popen(cmd, stdout=fo, stderr=subprocess.STDOUT, cwd=REPO)
        while p.poll() is None:  # a heartbeat: the pass itself writes its files at the end
            time.sleep(5)
            print(f"  {wl} {counter}: {time.time() - t0:.0f} s", flush=True)
        rc = p.returncode
    if rc != 0:
        raise SystemExit(f"{wl} {counter}: rocprofv3 pass failed (rc {rc}), see {d}")
    lines = [json.loads(x) for x in (d / "bench_stdout.txt").read_text().splitlines()
             if x.startswith("{") and '"metric"' in x]
    return lines[-1]


def medians(d: Path, kernels: list[str]) -> dict:
    f = next(d.rglob("*counter_collection.csv"))
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    out = {}
    for k in kernels:
        opt = k.endswith("?")
        k = k.rstrip("?")
        v = [float(r["Counter_Value"]) for r in rows if matches(r["Kernel_Name"], k)]
        if not v and opt:
            continue
        if not v:
            raise SystemExit(f"no dispatch of {k} in {f}")
        v = v[-STEPS:]  # the timed iterations (the last launches of the bench)
        out[k] = (statistics.median(v), len(v))
    return out


def fold(out: Path, wl: str, line: dict, table: dict, sha: str):
    cfg = line["config"]
    storage, world = cfg["storage"], line["n_gpus"]
    workload = cfg["workload"]
    og = "matfree_pt" if cfg.get("operator_form") == "pt" else storage
    groups = [(f"{workload}/{storage}/gpus{world}", GROUPS[og], line["operator_roofline"])]
    pre = line.get("precon_roofline")
    if pre is not None:
        form = 2 if "k_lr_cluster" in pre["kernel"] else 1 if "k_lr_rows" in pre["kernel"] else 0
        groups.append((f"{workload}/precon{form}/{storage}/gpus{world}", GROUPS[f"precon{form}"], pre))
    for key, kernels, roof in groups:
        fm = medians(out / f"{wl}_fetch_size", kernels)
        wm = medians(out / f"{wl}_write_size", kernels)
        parts = {k: {"FETCH_SIZE_kB_median": fm[k][0], "WRITE_SIZE_kB_median": wm[k][0],
                     "launches": fm[k][1], "hbm_bytes": (2 * fm[k][0] + wm[k][0]) * 1024}
                 for k in fm}
        hbm = sum(p["hbm_bytes"] for p in parts.values())
        alg = float(roof["bytes_per_launch"])  # (the pair-tile line: its algorithmic bytes)
        table[key] = {
            "kernel": " + ".join(parts), "per_kernel": parts,
            "correction": "hbm = sum_k (2 * FETCH_SIZE_k + WRITE_SIZE_k) * 1024 (MI355X_MICROARCH.md "
                          "HBM: FETCH_SIZE reads 1/2 of wide coalesced streaming reads on gfx950)",
            "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg,
            "traffic_over_algorithmic": hbm / alg, "csrc_sha": sha,
            "source": f"scripts/pmc_head.py: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate "
                      f"passes) of bench.py --steps {STEPS} --warmup {WARMUP} --no-cpu --no-solve "
                      f"{' '.join(WORKLOADS[wl])}; medians of the last {STEPS} dispatches"}
        print(f"{key}: {hbm / 1e6:.1f} MB per launch = {hbm / alg:.4f} x algorithmic", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(REPO / "gpurun_out" / "pmc_head"))
    ap.add_argument("--workloads", nargs="*", default=list(WORKLOADS))
    ap.add_argument("--fold-only", action="store_true")
    a = ap.parse_args()
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    sha = bench.csrc_hash()
    prof = REPO / "profiles" / "pmc_traffic.json"
    table = json.loads(prof.read_text()) if prof.exists() else {}
    for wl in a.workloads:
        if a.fold_only:
            line = [json.loads(x) for x in (out / f"{wl}_fetch_size" / "bench_stdout.txt")
                    .read_text().splitlines() if x.startswith("{") and '"metric"' in x][-1]
        else:
            line = run_pass(wl, "FETCH_SIZE", out)
            run_pass(wl, "WRITE_SIZE", out)
        fold(out, wl, line, table, sha)
    (out / "pmc_traffic.json").write_text(json.dumps(table, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
