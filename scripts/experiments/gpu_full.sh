#!/bin/bash
# GPU suite + smoke + default bench line + rocprofv3 kernel stats + nanotube + parity report;
# stops on a crash/timeout.
set -u
mkdir -p gpurun_out
L=gpurun_out/full.log
: > $L
export TMPDIR=/tmp
TAG=${TAG:-r01}
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)" >> $L; exit $rc; fi
  return 0
}
step 1200 gputests python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider -rf --timeout 600 --timeout-method thread
step 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
step 900 bench python bench.py
step 600 stats rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_sym_stats -o bench --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu --no-solve
step 600 nanotube python bench.py --workload nanotube --steps 30 --warmup 3
step 600 parity python scripts/parity_report.py
echo done >> $L
