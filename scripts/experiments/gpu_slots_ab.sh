#!/bin/bash
# Resident workgroups of the tile mat-vec (MLFF_SYM_SLOTS: default 512; -1 = fewest slots that
# cover the tiles in whole rounds; 258): per-rank floors at W = 8 / 4 (SOLO) and the 1-GPU
# configs[2] line, interleaved, 2 rounds.
set -u
mkdir -p gpurun_out
L=gpurun_out/slots_ab.log
: > $L
run() { echo "=== $1" >> $L; shift; timeout -k 10 300 "$@" >> $L 2>&1 || { echo "failed $*"; tail -20 $L; exit 1; }; }
for rep in 1 2; do
  for v in "X=0" "MLFF_SYM_SLOTS=-1" "MLFF_SYM_SLOTS=258"; do
    run "solo8 $v" env $v python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 50 --warmup 5
    run "solo4 $v" env $v python3 bench.py --solo-world 4 --solo-rank 0 --n 65536 --steps 50 --warmup 5
  done
  for v in "X=0" "MLFF_SYM_SLOTS=-1"; do
    run "rbf $v" env $v python3 bench.py --no-cpu --no-solve --configs3-n 0
  done
done
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/slots_ab.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line)
        if d.get('solo_profile'):
            print(f"{cur:28s} wall {d['ms_per_iter_wall']*1e3:7.1f} us op {d['operator_ms']*1e3:7.1f} us {d['operator_gbs']:.0f} GB/s")
        else:
            o=d.get('operator_roofline') or {}
            print(f"{cur:28s} {d['value']:8.1f} it/s step {d['ms_per_step']*1e3:8.1f} us op {o.get('mean_launch_ms',0)*1e3:7.1f}")
PY
