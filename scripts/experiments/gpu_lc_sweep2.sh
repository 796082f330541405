#!/bin/bash
# Member cap of the cluster apply: nanotube M = 200 (N = 222000, C = 28) and M = 300
# (N = 333000, C = 41), cluster (MLFF_LC_MAXC=64) vs two passes; heartbeat every 30 s.
set -u
mkdir -p gpurun_out
L=gpurun_out/lc_sweep2.log
: > $L
for M in 200 300; do
  for v in "MLFF_LC_MAXC=64" "MLFF_LR_ROWS=0"; do
    echo "=== M=$M $v" >> $L
    timeout -k 10 500 env $v python3 bench.py --workload nanotube --m $M --steps 10 --warmup 2 --no-cpu --no-solve >> $L 2>&1 &
    pid=$!
    while kill -0 $pid 2> /dev/null; do sleep 30; echo "M=$M $v alive $(date +%T)"; done
    wait $pid || { echo "failed M=$M $v"; tail -20 $L; exit 1; }
  done
done
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/lc_sweep2.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line); p=d.get('precon_roofline') or {}
        print(f"{cur:28s} N={d['config']['n']:7d} k={d['config']['k']:6d} step {d['ms_per_step']:.4f} ms apply {p.get('mean_launch_ms',0):.4f} ms {p.get('kernel','')[:14]}")
PY
