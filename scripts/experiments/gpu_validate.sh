#!/bin/bash
# GPU suite + smoke + default bench line; stops on a crash/timeout.
set -u
mkdir -p gpurun_out
L=gpurun_out/validate.log
: > $L
export TMPDIR=/tmp
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc $(date +%T)" >> $L
  if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)" >> $L; exit $rc; fi
  return 0
}
step 800 gputests python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider -rf --timeout 300 --timeout-method thread
step 200 smoke python -c "import __graft_entry__ as g; g.smoke()"
step 300 bench python bench.py
echo done >> $L
