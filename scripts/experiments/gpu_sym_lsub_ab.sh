#!/bin/bash
# A/B of the tile mat-vec tail slicing (MLFF_SYM_LSUB=2: quarters, as before; 4 at W = 8 / 4, 3 at W = 1: the
# 16 / 8 slices, what an adaptive choice would pick): SOLO W = 8 / W = 4 rank 0 of configs[2] and the 1-GPU step,
# interleaved A B A B, bench JSON lines + rocprofv3 kernel stats per run.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/lsub
run() {  # tag env-value args...
  local tag=$1 lv=$2; shift 2
  if [ "$lv" = auto ]; then unset MLFF_SYM_LSUB; else export MLFF_SYM_LSUB=$lv; fi
  timeout -k 10 240 python3 bench.py "$@" --no-cpu --no-solve > gpurun_out/lsub/$tag.log 2>&1 || { tail -20 gpurun_out/lsub/$tag.log; return 1; }
  echo "$tag $(grep '^{' gpurun_out/lsub/$tag.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d.get("value"), d.get("ms_per_step", d.get("ms_per_iter_wall")), d.get("operator_ms", d.get("iter_device_ms")))')"
}
prof() {
  local tag=$1 lv=$2; shift 2
  if [ "$lv" = auto ]; then unset MLFF_SYM_LSUB; else export MLFF_SYM_LSUB=$lv; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/lsub/prof_$tag -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-solve > gpurun_out/lsub/prof_$tag.log 2>&1 || { tail -20 gpurun_out/lsub/prof_$tag.log; return 1; }
}
S8="--solo-world 8 --solo-rank 0 --n 65536 --steps 200 --warmup 10"
S4="--solo-world 4 --solo-rank 0 --n 65536 --steps 200 --warmup 10"
G1="--steps 100 --warmup 10"
run w8_q 2 $S8 && run w8_a 4 $S8 && run w8_q2 2 $S8 && run w8_a2 4 $S8 &&
run w4_q 2 $S4 && run w4_a 4 $S4 && run w4_q2 2 $S4 && run w4_a2 4 $S4 &&
run g1_q 2 $G1 && run g1_a 3 $G1 && run g1_q2 2 $G1 && run g1_a2 3 $G1 &&
prof w8_q 2 $S8 && prof w8_a 4 $S8 && prof g1_q 2 $G1 && prof g1_a 3 $G1 &&
echo done
