#!/bin/bash
set -u
mkdir -p gpurun_out
L=gpurun_out/split.log
: > $L
for sr in -1 0 1 2 4 100; do
  for n in 16384 23040 65536; do
    echo "=== sr=$sr n=$n" >> $L
    MLFF_SYM_SPLIT_ROUNDS=$sr timeout -k 10 120 python bench.py --n $n --steps 40 --warmup 5 --no-cpu --no-solve >> $L 2>&1 || exit 1
  done
done
echo done >> $L
