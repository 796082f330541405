#!/bin/bash
# round 6: the sGDML bench lines on host descriptors (the fixtures' exact systems), and the ethanol
# k = 554 fixture test with the one-pass rows apply forced (MLFF_LR_ROWS=1; the default keeps two
# passes below k = 768 at N_loc > 4096)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/hostdesc
MLFF_LR_ROWS=1 timeout -k 10 300 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "ethanol_full_size and 554 and onestep" > gpurun_out/r06/hostdesc/k554_rows.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload nanotube > gpurun_out/r06/hostdesc/bench_nt.json 2> gpurun_out/r06/hostdesc/bench_nt.err || exit 1
timeout -k 10 300 python -u bench.py --workload ethanol --m 583 > gpurun_out/r06/hostdesc/bench_eth583.json 2> gpurun_out/r06/hostdesc/bench_eth583.err || exit 1
timeout -k 10 300 python -u bench.py --workload ethanol --m 111 > gpurun_out/r06/hostdesc/bench_eth111.json 2> gpurun_out/r06/hostdesc/bench_eth111.err || exit 1
