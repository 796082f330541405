#!/bin/bash
set -u
mkdir -p gpurun_out
L=gpurun_out/sched.log
: > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_symtile.py tests/test_gpu_fullsize.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread >> $L 2>&1 || exit 1
for sched in quarter persist quarter persist; do
  for n in 16384 23040 65536; do
    echo "=== sched=$sched n=$n" >> $L
    MLFF_SYM_SCHED=$sched timeout -k 10 120 python bench.py --n $n --steps 40 --warmup 5 --no-cpu --no-solve >> $L 2>&1 || exit 1
  done
done
echo done >> $L
