#!/bin/bash
# Where does the cluster one-pass apply beat two passes?  Nanotube M = 15, 20, 30, 60, 100
# (N = 16650 ... 111000, rule-of-thumb k), default vs MLFF_LR_ROWS=0, bench without CPU/solve.
set -u
mkdir -p gpurun_out
L=gpurun_out/lc_sweep.log
: > $L
for M in 15 20 30 60 100; do
  for v in "X=0" "MLFF_LR_ROWS=0"; do
    echo "=== M=$M $v" >> $L
    timeout -k 10 300 env $v python3 bench.py --workload nanotube --m $M --steps 20 --warmup 3 --no-cpu --no-solve >> $L 2>&1 || { echo "failed M=$M $v"; tail -20 $L; exit 1; }
    echo "M=$M $v done $(date +%T)"
  done
done
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/lc_sweep.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line); p=d.get('precon_roofline') or {}
        print(f"{cur:28s} N={d['config']['n']:7d} k={d['config']['k']:6d} step {d['ms_per_step']:.4f} ms apply {p.get('mean_launch_ms',0):.4f} ms {p.get('kernel','')[:14]}")
PY
