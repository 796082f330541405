#!/bin/bash
# Cluster one-pass apply: GPU tests, A/B of hand-off slack vs load distance (MLFF_LC_MODE 0:
# D = 1, L = 2; 1: D = 2, L = 1) on the large nanotube points, two-pass reference at M = 141.
set -u
mkdir -p gpurun_out
L=gpurun_out/lr_cluster4.log
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
for md in 0 1; do
  step 300 m141_mode$md env MLFF_LC_MODE=$md python3 bench.py --workload nanotube --m 141 --steps 20 --warmup 3 --no-cpu --no-solve
done
step 600 m455_mode0 env MLFF_LC_MODE=0 python3 bench.py --workload nanotube --m 455 --steps 10 --warmup 2 --no-cpu --no-solve
grep -E '^\{|passed|failed|rc=' $L | cut -c1-300
