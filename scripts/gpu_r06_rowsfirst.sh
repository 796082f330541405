#!/bin/bash
# round 6: the first tile rows requested before the fused p update's rho sum (k_symv_dyn):
# symmetric-tile and sharded bitwise tests, SOLO W = 8 floor, configs[2] one-GPU step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/rowsfirst
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_symtile.py tests/test_gpu_multirank.py > gpurun_out/r06/rowsfirst/tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 \
    > gpurun_out/r06/rowsfirst/w8_$rep.json 2> gpurun_out/r06/rowsfirst/w8_$rep.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-solve --configs3-n 0 \
  > gpurun_out/r06/rowsfirst/c2.json 2> gpurun_out/r06/rowsfirst/c2.err || exit 1
