#!/bin/bash
# Timing events without the system-scope fence (default now) vs with it (MLFF_EVENT_FENCE=1):
# default bench (configs[2], no CPU leg, no solve), nanotube, and the W = 8 SOLO rank floor,
# interleaved, 2 rounds.
set -u
mkdir -p gpurun_out
L=gpurun_out/event_ab.log
: > $L
run() { echo "=== $1" >> $L; shift; timeout -k 10 300 "$@" >> $L 2>&1 || { echo "failed $*"; tail -20 $L; exit 1; }; }
for rep in 1 2; do
  for f in "X=0" "MLFF_EVENT_FENCE=1"; do
    run "rbf $f" env $f python3 bench.py --no-cpu --no-solve --configs3-n 0
    run "nt $f" env $f python3 bench.py --workload nanotube --no-cpu --no-solve
    run "solo8 $f" env $f python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 50 --warmup 5
  done
done
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/event_ab.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line)
        if d.get('solo_profile'):
            print(f"{cur:28s} wall {d['ms_per_iter_wall']*1e3:7.1f} us dev {d['iter_device_ms']*1e3:7.1f} us op {d['operator_ms']*1e3:7.1f} us")
        else:
            p=d.get('precon_roofline') or {}; o=d.get('operator_roofline') or {}
            print(f"{cur:28s} {d['value']:8.1f} it/s step {d['ms_per_step']*1e3:8.1f} us op {o.get('mean_launch_ms',0)*1e3:7.1f} apply {p.get('mean_launch_ms',0)*1e3:6.1f} build {d.get('setup_s',{}).get('pivoted_cholesky_build')}")
PY
