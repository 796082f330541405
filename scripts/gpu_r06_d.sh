#!/bin/bash
# round 6: the Woodbury build (BK = 32 dd Gram stages, triangular POTRF update): numerics suites,
# then the nanotube build split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/d
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_core.py tests/test_gpu_golden.py tests/test_gpu_fused_iteration.py tests/test_gpu_configs.py \
  > gpurun_out/r06/d/suites.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/d/prof_nt -o nt -- \
  python3 bench.py --workload nanotube --steps 20 --warmup 5 --no-cpu \
  > gpurun_out/r06/d/bench_nt_prof.json 2> gpurun_out/r06/d/bench_nt_prof.err || exit 1
