#!/bin/bash
# sweep one env knob on a bench workload, interleaved repeats: VAR=MLFF_X VALS="a b c"
set -u
mkdir -p gpurun_out
L=gpurun_out/sweep_env.log
: > $L
for rep in 1 2; do
  for v in $VALS; do
    echo "=== $VAR=$v rep=$rep" >> $L
    env $VAR=$v timeout -k 10 150 python bench.py --workload ${WORKLOAD:-nanotube} --steps ${STEPS:-300} --warmup 20 --no-cpu --no-solve >> $L 2>&1 || exit 1
  done
done
echo done >> $L
