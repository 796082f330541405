#!/bin/bash
# round 6, final library: the reference's large published points with the one-step default panel
# (host descriptors): ethanol N = 157491 (M = 5833) and nanotube N = 156510 (M = 141)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/large
timeout -k 10 500 python -u bench.py --workload ethanol --m 5833 --no-cpu > gpurun_out/r06/large/bench_eth5833.json 2> gpurun_out/r06/large/bench_eth5833.err || exit 1
timeout -k 10 500 python -u bench.py --workload nanotube --m 141 --no-cpu > gpurun_out/r06/large/bench_nt141.json 2> gpurun_out/r06/large/bench_nt141.err || exit 1
