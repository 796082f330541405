#!/bin/bash
# round 6: the rank-counting candidate merge (k_spec_top_merge) -- the pivoted-Cholesky tests
# (persistent / launch sequence bit-identity, configs[1] and ethanol pivots against the oracle),
# the nanotube bench line and its rocprof kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/piv
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_pivchol_persist.py tests/test_gpu_configs.py -k "not n74979" \
  > gpurun_out/r06/piv/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload nanotube > gpurun_out/r06/piv/bench_nt.json 2> gpurun_out/r06/piv/bench_nt.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/piv/prof_nt -o nt -- \
  python3 bench.py --workload nanotube --steps 40 --warmup 5 --no-cpu \
  > gpurun_out/r06/piv/bench_nt_prof.json 2> gpurun_out/r06/piv/bench_nt_prof.err || exit 1
