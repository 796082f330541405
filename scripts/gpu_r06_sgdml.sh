#!/bin/bash
# round 6: the sGDML bench lines (configs[1] nanotube, ethanol N = 15741, configs[0] geometry)
# at the current library, and the nanotube line under rocprofv3 (build + iteration split)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u bench.py --workload nanotube > gpurun_out/r06/bench_nt.json 2> gpurun_out/r06/bench_nt.err || exit 1
timeout -k 10 300 python -u bench.py --workload ethanol --m 583 > gpurun_out/r06/bench_eth583.json 2> gpurun_out/r06/bench_eth583.err || exit 1
timeout -k 10 300 python -u bench.py --workload ethanol --m 111 > gpurun_out/r06/bench_eth111.json 2> gpurun_out/r06/bench_eth111.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_nt -o nt -- \
  python3 bench.py --workload nanotube --steps 40 --warmup 5 --no-cpu \
  > gpurun_out/r06/bench_nt_prof.json 2> gpurun_out/r06/bench_nt_prof.err || exit 1
