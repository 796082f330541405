#!/bin/bash
# k_lr_fin waves per workgroup (MLFF_LR_FIN_WAVES 4 / 8 / 16): nanotube (configs[1]) and the
# N = 156510 point, interleaved, 2 rounds; rocprof stats of the 8-wave nanotube run.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
L=gpurun_out/fin_ab.log
: > $L
run() { echo "=== $1" >> $L; shift; timeout -k 10 400 "$@" >> $L 2>&1 || { echo "failed $*"; tail -20 $L; exit 1; }; }
for rep in 1 2; do
  for w in 4 8 16; do
    run "nt w=$w" env MLFF_LR_FIN_WAVES=$w python3 bench.py --workload nanotube --no-cpu --no-solve
  done
done
for w in 4 16; do
  run "m141 w=$w" env MLFF_LR_FIN_WAVES=$w python3 bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
done
timeout -k 10 300 env MLFF_LR_FIN_WAVES=16 rocprofv3 --kernel-trace --stats -d gpurun_out/fin16 -o bench --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve > gpurun_out/fin16.log 2>&1 || exit 1
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/fin_ab.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line); p=d.get('precon_roofline') or {}
        print(f"{cur:12s} {d['value']:8.1f} it/s step {d['ms_per_step']*1e3:8.1f} us apply {p.get('mean_launch_ms',0)*1e3:7.1f} us")
PY
