#!/bin/bash
# Per-rank kernel breakdown of the sharded PCG iteration: rank 0 of a W = 8 row split of the
# configs[2] problem (N = 65536) alone on one GPU (SOLO transport), rocprofv3 stats + trace.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 50 --warmup 5 > gpurun_out/solo8.log 2>&1 || { tail -20 gpurun_out/solo8.log; exit 1; }
grep '^{' gpurun_out/solo8.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/solo8_prof -o bench --output-format csv -- python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 50 --warmup 5 > gpurun_out/solo8_prof.log 2>&1 || { tail -20 gpurun_out/solo8_prof.log; exit 1; }
echo done
