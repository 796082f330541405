#!/bin/bash
# round 6: the W = 8 per-rank floor -- finer tile units for the dynamic
# schedule (MLFF_SYM_WHOLE_ROUNDS, MLFF_SYM_LSUB) A/B, interleaved, and the SOLO kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/w8
for rep in 1 2; do
  for cfg in "default::" "r1:MLFF_SYM_WHOLE_ROUNDS=1:" "r0:MLFF_SYM_WHOLE_ROUNDS=0:" "r0l1:MLFF_SYM_WHOLE_ROUNDS=0:MLFF_SYM_LSUB=1" "r1l3:MLFF_SYM_WHOLE_ROUNDS=1:MLFF_SYM_LSUB=3"; do
    name=${cfg%%:*}; rest=${cfg#*:}; e1=${rest%%:*}; e2=${rest#*:}
    env $e1 $e2 MLFF_SYM_TRACE=30 timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 \
      > gpurun_out/r06/w8/${name}_$rep.json 2> gpurun_out/r06/w8/${name}_$rep.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/w8/prof -o solo -- \
  python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 > gpurun_out/r06/w8/prof.json 2>&1 || exit 1
