#!/bin/bash
# round 6, final library: smoke, the driver's GPU suite, and the bench lines (configs[2] default,
# configs[1] nanotube, ethanol N = 15741 and configs[0]'s geometry with the rank-398 preconditioner)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/final
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/final/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread -k "not n74979" \
  > gpurun_out/r06/final/suite.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r06/final/bench_configs2.json 2> gpurun_out/r06/final/bench_configs2.err || exit 1
timeout -k 10 300 python -u bench.py --workload nanotube > gpurun_out/r06/final/bench_nt.json 2> gpurun_out/r06/final/bench_nt.err || exit 1
timeout -k 10 300 python -u bench.py --workload ethanol --m 583 > gpurun_out/r06/final/bench_eth583.json 2> gpurun_out/r06/final/bench_eth583.err || exit 1
timeout -k 10 300 python -u bench.py --workload ethanol --m 111 > gpurun_out/r06/final/bench_eth111.json 2> gpurun_out/r06/final/bench_eth111.err || exit 1
