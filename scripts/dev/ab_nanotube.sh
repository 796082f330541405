#!/bin/bash
# A/B of library variants on the nanotube bench (matrix-free operator + rank-2701 apply);
# VARIANTS names files under lib/variants ("base" = the in-tree library); interleaved
set -u
mkdir -p gpurun_out
L=gpurun_out/ab_nt.log
: > $L
for rep in 1 2 3; do
  for v in ${VARIANTS:-base}; do
    echo "=== v=$v rep=$rep" >> $L
    if [ "$v" = base ]; then lib=""; else lib=mlff-preconditioner_amd/lib/variants/$v.so; fi
    MLFF_LIB=$lib timeout -k 10 150 python bench.py --workload nanotube --steps 300 --warmup 20 --no-cpu --no-solve >> $L 2>&1 || exit 1
  done
done
echo done >> $L
