#!/bin/bash
# One-pass apply A/B (nanotube configs[1], interleaved, 2 rounds): MALL-cached rows per group
# (MLFF_LR_CACHE_ROWS) instead of whole groups, non-temporal partial stores (MLFF_LR_NT_STORE).
set -u
mkdir -p gpurun_out
L=gpurun_out/lr_ab3.log
: > $L
NT="python3 bench.py --workload nanotube --no-cpu --no-solve"
for rep in 1 2; do
  for v in "X=0" "MLFF_LR_CACHE_ROWS=4" "MLFF_LR_CACHE_ROWS=5" "MLFF_LR_NT_STORE=1" "MLFF_LR_CACHE_ROWS=4 MLFF_LR_NT_STORE=1"; do
    echo "=== $v" >> $L
    timeout -k 10 300 env $v $NT >> $L 2>&1 || { echo "failed: $v"; tail -20 $L; exit 1; }
  done
done
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/lr_ab3.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line); p=d.get('precon_roofline') or {}
        print(f"{cur:40s} {d['value']:7.0f} it/s step {d['ms_per_step']*1e3:6.1f} apply {p.get('mean_launch_ms',0)*1e3:5.1f}")
PY
