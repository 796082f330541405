#!/bin/bash
# round 6: the owned-slot reduction from the flat load list
# (k_sym_reduce_wl) -- its bitwise test, the SOLO W = 8 per-rank floor A/B against
# k_sym_reduce_w (MLFF_SYM_REDUCE_LIST=0), interleaved, and the SOLO kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/reduce
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_multirank.py -k "reduce_list or pq_publish or fused_p_update" \
  > gpurun_out/r06/reduce/tests.log 2>&1 || exit 1
for rep in 1 2; do
  for cfg in list1:1:0 list0:0:0 list1sep:1:1; do
    name=${cfg%%:*}; rest=${cfg#*:}; lst=${rest%%:*}; sep=${rest#*:}
    MLFF_SYM_REDUCE_LIST=$lst MLFF_PQ_PUBLISH=$sep timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 \
      > gpurun_out/r06/reduce/w8_${name}_$rep.json 2> gpurun_out/r06/reduce/w8_${name}_$rep.err || exit 1
  done
done
for lst in 1 0; do
  MLFF_SYM_REDUCE_LIST=$lst timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 0 --n 131072 --steps 20 \
    > gpurun_out/r06/reduce/w8_n131072_list${lst}.json 2> gpurun_out/r06/reduce/w8_n131072_list${lst}.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/reduce/prof -o solo -- \
  python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 > gpurun_out/r06/reduce/prof.json 2>&1 || exit 1
