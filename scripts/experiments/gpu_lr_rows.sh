#!/bin/bash
# One-pass low-rank apply: its GPU tests, nanotube bench A/B (MLFF_LR_ROWS=1 default vs 0,
# interleaved), rocprof stats of the nanotube timed region, then the driver-exact suite,
# smoke and the default bench line.  Stops at the first failure.
set -u
mkdir -p gpurun_out
L=gpurun_out/lr_rows.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -30 $L; exit $rc; fi
}
step 400 unit python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_core.py -k "one_pass or pivchol"
for rep in 1 2; do
  step 300 nt_on$rep python3 bench.py --workload nanotube --no-cpu --no-solve
  step 300 nt_off$rep env MLFF_LR_ROWS=0 python3 bench.py --workload nanotube --no-cpu --no-solve
done
step 300 nt_prof rocprofv3 --kernel-trace --stats -d gpurun_out/lr_nt -o bench --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve
step 700 suite bash scripts/gpu_driver_repro.sh
step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke()"
step 600 bench python3 bench.py
grep -E '^\{|passed|smoke|rc=' $L | cut -c1-600
