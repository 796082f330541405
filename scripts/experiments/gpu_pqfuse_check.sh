#!/bin/bash
# Sharded-iteration checks after folding the p.q share publish into k_sym_reduce_w:
# the LOCAL-transport multi-rank suite (bitwise-equal traces across ranks, parity with
# one rank) + the SOLO W = 8 / 4 per-rank step with rocprof kernel stats.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pqf
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_sharded_dropin.py tests/test_gpu_configs.py > gpurun_out/pqf/tests.log 2>&1 || { tail -30 gpurun_out/pqf/tests.log; exit 1; }
tail -2 gpurun_out/pqf/tests.log
for W in 8 4 8 4; do
  timeout -k 10 200 python3 bench.py --solo-world $W --solo-rank 0 --n 65536 --steps 200 --warmup 10 > gpurun_out/pqf/solo$W.log 2>&1 || { tail -20 gpurun_out/pqf/solo$W.log; exit 1; }
  echo "W=$W $(grep '^{' gpurun_out/pqf/solo$W.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["ms_per_iter_wall"], d["iter_device_ms"], d["operator_ms"])')"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pqf/prof_w8 -o run --output-format csv -- python3 bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 200 --warmup 10 > gpurun_out/pqf/prof_w8.log 2>&1 || { tail -20 gpurun_out/pqf/prof_w8.log; exit 1; }
echo done
