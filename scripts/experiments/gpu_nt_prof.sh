#!/bin/bash
# rocprofv3 kernel stats of the nanotube bench (matrix-free operator + rank-2701 apply)
set -u
mkdir -p gpurun_out
L=gpurun_out/nt_prof.log
: > $L
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-r01}_nt_stats -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 200 --warmup 10 --no-cpu --no-solve >> $L 2>&1
echo "rc=$?" >> $L
