#!/bin/bash
# Default bench line (N=1, configs[2]) + SOLO per-rank floors of configs[3] (N=131072, W=8 / 4 / 2)
set -u
mkdir -p gpurun_out
L=gpurun_out/bench_round.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -30 $L; exit $rc; fi
}
step 600 bench python bench.py
for W in 8 4 2; do
  step 300 solo$W python bench.py --solo-world $W --solo-rank 0 --n 131072 --steps 20 --warmup 3
done
grep -v "^===" $L | tail -8
