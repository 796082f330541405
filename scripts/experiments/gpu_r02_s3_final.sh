#!/bin/bash
# Round-2 third-session evidence at HEAD: driver-exact GPU suite, smoke, default bench line,
# nanotube (configs[1]) line + rocprof stats of its timed region, the N = 156510 nanotube
# point with the cluster one-pass apply (solve to 1e-6) + its rocprof stats.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
L=gpurun_out/r02_s3_final${TAG:-}.log
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
step 700 suite bash scripts/gpu_driver_repro.sh
step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke()"
step 600 bench python3 bench.py
step 300 nanotube python3 bench.py --workload nanotube
step 300 nanotube_prof rocprofv3 --kernel-trace --stats -d gpurun_out/s3_nt -o bench --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve
step 400 m141 python3 bench.py --workload nanotube --m 141 --steps 20 --warmup 3 --no-cpu
step 400 m141_prof rocprofv3 --kernel-trace --stats -d gpurun_out/s3_m141 -o bench --output-format csv -- python3 bench.py --workload nanotube --m 141 --steps 20 --warmup 3 --no-cpu --no-solve
grep -E '^\{|passed|smoke|rc=' $L | cut -c1-300
