#!/bin/bash
# GPU suite + smoke + nanotube bench line + nanotube rocprof stats; stops on a crash/timeout.
set -u
mkdir -p gpurun_out
L=gpurun_out/verify.log
: > $L
export TMPDIR=/tmp
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; exit $rc; fi
  return 0
}
step 900 gputests python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider -rf --timeout 600 --timeout-method thread
step 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
step 600 nanotube python bench.py --workload nanotube --steps 30 --warmup 3
step 600 nt_stats rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-r01}_nt_stats -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 30 --warmup 3 --no-cpu
echo done >> $L
