#!/bin/bash
# Round-2 evidence: default bench line, rocprofv3 kernel stats of the same command,
# nanotube bench line + stats, parity report.  Each GPU step under its own time limit;
# stop at the first failure.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
L=gpurun_out/r02_profiles.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -30 $L; exit $rc; fi
}
step 600 rbf_stats rocprofv3 --kernel-trace --stats -d gpurun_out/r02_rbf_stats -o bench --output-format csv -- python3 bench.py
step 300 nt_stats rocprofv3 --kernel-trace --stats -d gpurun_out/r02_nt_stats -o bench --output-format csv -- python3 bench.py --workload nanotube
step 600 parity python3 scripts/parity_report.py
grep '^{' $L | cut -c1-400
