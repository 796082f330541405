#!/bin/bash
# round 6: where the per-rank tile stream's time goes -- the workgroup trace
# of one k_symv_dyn launch (MLFF_SYM_TRACE) at W = 1 and for one rank of W = 8 (SOLO transport),
# and the SOLO per-rank floors
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/symtrace
for i in 1 2; do
  MLFF_SYM_TRACE=30 timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-solve --configs3-n 0 \
    > gpurun_out/r06/symtrace/w1_$i.json 2> gpurun_out/r06/symtrace/w1_$i.err || exit 1
  MLFF_SYM_TRACE=30 timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 \
    > gpurun_out/r06/symtrace/w8_n65536_$i.json 2> gpurun_out/r06/symtrace/w8_n65536_$i.err || exit 1
  MLFF_SYM_TRACE=30 timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 3 --n 65536 --steps 40 \
    > gpurun_out/r06/symtrace/w8r3_n65536_$i.json 2> gpurun_out/r06/symtrace/w8r3_n65536_$i.err || exit 1
  MLFF_SYM_TRACE=30 timeout -k 10 300 python -u bench.py --solo-world 8 --solo-rank 0 --steps 40 \
    > gpurun_out/r06/symtrace/w8_n131072_$i.json 2> gpurun_out/r06/symtrace/w8_n131072_$i.err || exit 1
done
