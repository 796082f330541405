#!/bin/bash
# One-pass low-rank apply, second pass: unit tests, nanotube A/B of the MALL-cached row
# groups (MLFF_LR_CACHE_WGS 0 / default / all) and of the two-pass apply, rocprof stats,
# PMC (FETCH_SIZE, WRITE_SIZE; separate passes) of k_lr_rows + k_lr_fin.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
L=gpurun_out/lr_rows2.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -30 $L; exit $rc; fi
}
NT="python3 bench.py --workload nanotube --no-cpu --no-solve"
step 400 unit python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_core.py -k "one_pass or pivchol"
for rep in 1 2; do
  step 300 nt_def$rep $NT
  step 300 nt_c0_$rep env MLFF_LR_CACHE_WGS=0 $NT
  step 300 nt_call$rep env MLFF_LR_CACHE_WGS=1000 $NT
  step 300 nt_off$rep env MLFF_LR_ROWS=0 $NT
done
step 300 nt_prof rocprofv3 --kernel-trace --stats -d gpurun_out/lr2_nt -o bench --output-format csv -- $NT
RX='k_lr_rows|k_lr_fin|k_trsm_diag_wide'
for C in FETCH_SIZE WRITE_SIZE; do
  step 180 pmc_$C rocprofv3 --pmc $C --kernel-include-regex "$RX" -d gpurun_out/lr2_pmc_$C -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 10 --warmup 2 --no-cpu --no-solve
done
grep -E '^\{|passed|rc=' $L | cut -c1-300
