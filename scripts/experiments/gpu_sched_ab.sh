#!/bin/bash
# correctness of a tile schedule (MLFF_SYM_SCHED) + interleaved A/B against the default
set -u
mkdir -p gpurun_out
L=gpurun_out/sched_ab.log
: > $L
S=${SCHED:-dyn}
MLFF_SYM_SCHED=$S timeout -k 10 900 python -u -m pytest tests/test_gpu_symtile.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -x -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread >> $L 2>&1 || exit 1
for rep in 1 2 3; do
  for sch in default $S; do
    for n in ${NS:-16384 23040 65536}; do
      echo "=== s=$sch n=$n rep=$rep" >> $L
      if [ $sch = default ]; then e=""; else e=$sch; fi
      MLFF_SYM_SCHED=$e timeout -k 10 120 python bench.py --n $n --steps 40 --warmup 5 --no-cpu --no-solve >> $L 2>&1 || exit 1
    done
  done
done
echo done >> $L
