#!/bin/bash
# round 6: the fused one-rank p update's bitwise test, the configs[2] bench line, its kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_symtile.py tests/test_gpu_exact_sums.py::test_configs2_fp64_count_held_to_exact_anchor \
  > gpurun_out/r06/symtile.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r06/bench_default.json 2> gpurun_out/r06/bench_default.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_bench -o bench -- \
  python3 bench.py --steps 40 --warmup 5 --no-cpu --no-solve --configs3-n 0 \
  > gpurun_out/r06/bench_prof.json 2> gpurun_out/r06/bench_prof.err || exit 1
