#!/bin/bash
# Third-session re-entry check at HEAD: driver-exact GPU suite, smoke, default bench line.
set -u
mkdir -p gpurun_out
L=gpurun_out/r02_s3_verify.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -30 $L; exit $rc; fi
}
step 700 suite bash scripts/gpu_driver_repro.sh
step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke()"
step 600 bench python3 bench.py
grep -E '^\{|passed|smoke' $L | cut -c1-400
