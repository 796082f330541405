#!/bin/bash
# A/B of library variants (MLFF_LIB) on the bench operator; interleaved repeats
set -u
mkdir -p gpurun_out
L=gpurun_out/ab.log
: > $L
V=${VARIANTS:-base}
for rep in ${REPS:-1 2}; do
  for v in $V; do
    for n in ${NS:-23040 65536}; do
      echo "=== v=$v n=$n rep=$rep" >> $L
      if [ "$v" = base ]; then lib=""; else lib=mlff-preconditioner_amd/lib/variants/$v.so; fi
      MLFF_LIB=$lib timeout -k 10 120 python bench.py --n $n --steps ${STEPS:-40} --warmup 5 --no-cpu --no-solve >> $L 2>&1 || exit 1
    done
  done
done
echo done >> $L
