#!/bin/bash
# round 6: finer tile units at W = 8 again, now that the owned-slot reduction batches the split
# planes' loads (k_sym_reduce_wl): SOLO W = 8 A/B of MLFF_SYM_WHOLE_ROUNDS / MLFF_SYM_LSUB, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/units2
for rep in 1 2; do
  for cfg in "default::" "r1:MLFF_SYM_WHOLE_ROUNDS=1:" "r0:MLFF_SYM_WHOLE_ROUNDS=0:" "r0l1:MLFF_SYM_WHOLE_ROUNDS=0:MLFF_SYM_LSUB=1" "r1l1:MLFF_SYM_WHOLE_ROUNDS=1:MLFF_SYM_LSUB=1"; do
    name=${cfg%%:*}; rest=${cfg#*:}; e1=${rest%%:*}; e2=${rest#*:}
    env $e1 $e2 timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 \
      > gpurun_out/r06/units2/${name}_$rep.json 2> gpurun_out/r06/units2/${name}_$rep.err || exit 1
  done
done
