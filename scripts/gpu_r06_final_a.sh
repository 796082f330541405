#!/bin/bash
# round 6, final library: PMC HBM traffic of the bench kernel groups (scripts/pmc_head.py: separate
# FETCH_SIZE / WRITE_SIZE passes), and the rocprofv3 kernel split of the configs[2] bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/final
timeout -k 10 700 python -u scripts/pmc_head.py --out gpurun_out/r06/final/pmc \
  --workloads rbf nanotube ethanol_m583 ethanol_m2777 > gpurun_out/r06/final/pmc_head.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/final/prof_c2 -o bench -- \
  python3 bench.py --steps 40 --warmup 5 --no-cpu --no-solve --configs3-n 0 \
  > gpurun_out/r06/final/bench_c2_prof.json 2> gpurun_out/r06/final/bench_c2_prof.err || exit 1
