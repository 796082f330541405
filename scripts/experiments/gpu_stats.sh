#!/bin/bash
# rocprofv3 kernel stats of the bench (ARGS) + summary into gpurun_out/stats.log
set -u
mkdir -p gpurun_out
L=gpurun_out/stats.log
: > $L
export TMPDIR=/tmp
D=gpurun_out/${TAG:-stats}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o bench --output-format csv -- python3 bench.py ${ARGS:---steps 30 --warmup 3 --no-cpu --no-solve} >> $L 2>&1 || exit 1
python3 scripts/kstats.py $D/bench_kernel_stats.csv 25 >> $L
