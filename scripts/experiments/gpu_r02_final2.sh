#!/bin/bash
# Round-2 closing evidence (second session): driver-exact GPU suite, smoke, the default bench
# line plain and under rocprofv3 (full command + the timed-region-only command), the nanotube
# line and its kernel stats, SOLO per-rank floors of the N = 65536 strong-scaling problem,
# and the multi-rank bench rehearsal.  Stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r02_final2.log
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
step 600 bench_prof rocprofv3 --kernel-trace --stats -d gpurun_out/f2_rbf -o bench --output-format csv -- python3 bench.py
step 300 bench_prof_timed rocprofv3 --kernel-trace --stats -d gpurun_out/f2_rbf_timed -o bench --output-format csv -- python3 bench.py --no-solve --no-cpu --configs3-n 0
step 300 nanotube python3 bench.py --workload nanotube
step 300 nanotube_prof rocprofv3 --kernel-trace --stats -d gpurun_out/f2_nt -o bench --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve
for W in 8 4 2; do
  step 300 solo$W python3 bench.py --solo-world $W --solo-rank 0 --n 65536 --steps 20 --warmup 3
done
step 600 rehearse env WS=8 bash scripts/gpu_rehearse_multirank.sh
grep -E '^\{|passed|smoke' $L | cut -c1-300
