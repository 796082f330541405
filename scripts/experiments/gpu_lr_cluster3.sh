#!/bin/bash
# Cluster one-pass apply (row waves + a sync wave): GPU tests, large nanotube points with the
# cluster apply (M = 141 with the solve, M = 455 bench only) and M = 141 two-pass A/B.
set -u
mkdir -p gpurun_out
L=gpurun_out/lr_cluster3.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1 &
  local pid=$!
  while kill -0 $pid 2> /dev/null; do sleep 30; echo "$name alive $(date +%T)"; done
  wait $pid
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -40 $L; exit $rc; fi
}
step 400 unit python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_core.py -k "one_pass"
step 300 m141 python3 bench.py --workload nanotube --m 141 --steps 20 --warmup 3 --no-cpu
step 300 m141_off env MLFF_LR_ROWS=0 python3 bench.py --workload nanotube --m 141 --steps 20 --warmup 3 --no-cpu --no-solve
step 600 m455 python3 bench.py --workload nanotube --m 455 --steps 10 --warmup 2 --no-cpu --no-solve
grep -E '^\{|passed|failed|rc=' $L | cut -c1-300
