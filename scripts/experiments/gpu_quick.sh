#!/bin/bash
# Selected GPU tests (args: pytest selection) + the nanotube bench line; stops on failure.
set -u
mkdir -p gpurun_out
L=gpurun_out/quick.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -40 $L; exit $rc; fi
  return 0
}
step 600 tests python -u -m pytest ${TESTS:-tests/} -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
if [ -n "${BENCH:-}" ]; then step 600 bench python bench.py $BENCH; fi
tail -15 $L
