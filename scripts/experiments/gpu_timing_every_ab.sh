#!/bin/bash
# Timed-region event brackets on every iteration (MLFF_BENCH_TIMING_EVERY=1) vs every 8th
# (default): configs[2] (no CPU leg, no solve), nanotube, W = 8 per-rank floor; 2 rounds.
set -u
mkdir -p gpurun_out
L=gpurun_out/timing_every_ab.log
: > $L
run() { echo "=== $1" >> $L; shift; timeout -k 10 300 "$@" >> $L 2>&1 || { echo "failed $*"; tail -20 $L; exit 1; }; }
for rep in 1 2; do
  for e in 8 1; do
    run "rbf every=$e" env MLFF_BENCH_TIMING_EVERY=$e python3 bench.py --no-cpu --no-solve --configs3-n 0
    run "nt every=$e" env MLFF_BENCH_TIMING_EVERY=$e python3 bench.py --workload nanotube --no-cpu --no-solve
    run "solo8 every=$e" env MLFF_BENCH_TIMING_EVERY=$e python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 50 --warmup 5
  done
done
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/timing_every_ab.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line)
        if d.get('solo_profile'):
            print(f"{cur:20s} wall {d['ms_per_iter_wall']*1e3:7.1f} us dev {d['iter_device_ms']*1e3:7.1f} us op {d['operator_ms']*1e3:7.1f} us")
        else:
            p=d.get('precon_roofline') or {}; o=d.get('operator_roofline') or {}; r=d.get('roofline') or {}
            print(f"{cur:20s} {d['value']:8.1f} it/s step {d['ms_per_step']*1e3:8.1f} us op {o.get('mean_launch_ms',0)*1e3:7.1f} apply {p.get('mean_launch_ms',0)*1e3:6.1f} frac {r.get('frac',0):.3f}")
PY
