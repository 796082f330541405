#!/bin/bash
# split-factor sweep of the low-rank apply (MLFF_TSPLIT / MLFF_ZSPLIT) on one box;
# CFGS="ts,zs ts,zs ..."
set -u
mkdir -p gpurun_out
L=gpurun_out/sweep_split.log
: > $L
W=${WORKLOAD:-nanotube}
for rep in 1 2; do
  for cfg in ${CFGS:-1,29 3,29 1,33 3,33 2,33 1,25 1,41}; do
    ts=${cfg%,*}; zs=${cfg#*,}
    echo "=== ts=$ts,zs=$zs rep=$rep" >> $L
    MLFF_TSPLIT=$ts MLFF_ZSPLIT=$zs timeout -k 10 150 python bench.py --workload $W --steps 300 --warmup 20 --no-cpu --no-solve >> $L 2>&1 || exit 1
  done
done
echo done >> $L
