#!/bin/bash
# Record-factored matrix-free operator: GPU suite, nanotube bench (configs[1]) plain and
# under rocprofv3 kernel stats, the N = 156510 nanotube step, and the pair-path A/B.
set -u
mkdir -p gpurun_out
L=gpurun_out/rec.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -40 $L; exit $rc; fi
}
export TMPDIR=/tmp
step 300 matfree python3 -u -m pytest tests/test_gpu_matfree.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step 600 suite bash scripts/gpu_driver_repro.sh
step 300 nt python3 bench.py --workload nanotube
step 300 nt_pairpath env MLFF_MF_REC=0 python3 bench.py --workload nanotube --no-cpu --no-solve
step 300 nt_prof rocprofv3 --kernel-trace --stats -d gpurun_out/rec_prof -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve
step 400 nt141 python3 bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
grep -E '^\{' $L | cut -c1-200
grep -E "passed|failed" $L
