#!/bin/bash
# Round-2 closing evidence: driver-exact GPU suite, smoke, default bench line, nanotube line,
# SOLO floors at configs[3], multi-rank rehearsal.  Stops at the first failure.
set -u
mkdir -p gpurun_out
L=gpurun_out/r02_final.log
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
step 300 nanotube python3 bench.py --workload nanotube
for W in 8 4 2; do
  step 300 solo$W python3 bench.py --solo-world $W --solo-rank 0 --n 131072 --steps 20 --warmup 3
done
step 600 rehearse bash scripts/gpu_rehearse_multirank.sh
grep -E '^\{|passed|smoke' $L | cut -c1-300
