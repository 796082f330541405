#!/bin/bash
# round 6: POTRF one-wave diagonal / pipelined dd Gram checks, then the W = 8 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_core.py tests/test_gpu_pivchol_persist.py tests/test_gpu_golden.py \
  "tests/test_gpu_configs.py::test_config1_full_size_against_oracle_fixture" \
  > gpurun_out/r06/potrf.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload nanotube --no-cpu > gpurun_out/r06/bench_nt2.json 2> gpurun_out/r06/bench_nt2.err || exit 1
bash scripts/gpu_r06_w8.sh
