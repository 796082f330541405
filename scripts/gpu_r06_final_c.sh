#!/bin/bash
# round 6, final library, after the ethanol N = 74979 fixture (tests/golden/make_ethanol_75k.py):
# its fixture test, the N = 74979 bench line against it, the PMC entries of configs[0]'s geometry,
# and the self-launched 8-rank bench flow on one GPU (SOLO ranks, MLFF_BENCH_REHEARSE=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/final
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  tests/test_gpu_configs.py -k "n74979" > gpurun_out/r06/final/eth75k_test.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload ethanol --m 2777 > gpurun_out/r06/final/bench_eth2777.json 2> gpurun_out/r06/final/bench_eth2777.err || exit 1
timeout -k 10 300 python -u scripts/pmc_head.py --out gpurun_out/r06/final/pmc111 --workloads ethanol_m111 \
  > gpurun_out/r06/final/pmc_head_111.log 2>&1 || exit 1
MLFF_BENCH_REHEARSE=1 timeout -k 10 300 python -u bench.py --gpus 8 --steps 10 --warmup 2 \
  > gpurun_out/r06/final/selflaunch_rehearse_w8.txt 2>&1 || exit 1
