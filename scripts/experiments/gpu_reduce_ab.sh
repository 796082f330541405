#!/bin/bash
# slot-reduction change: multirank tests, RBF bench kernel trace, and the 8-rank bench
# rehearsal under a kernel trace (k_sym_reduce_w durations on one GPU)
set -u
mkdir -p gpurun_out
L=gpurun_out/reduce_ab.log
: > $L
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_symtile.py tests/test_gpu_core.py -q -p no:cacheprovider --timeout 200 --timeout-method thread >> $L 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_rbf_stats -o bench --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu --no-solve >> $L 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_w8_stats -o t --output-format csv -- python3 -m pytest tests/test_gpu_multirank.py -q -p no:cacheprovider -k eight_ranks >> $L 2>&1 || exit 3
echo done >> $L
