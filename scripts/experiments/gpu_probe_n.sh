#!/bin/bash
# tile-count (tail) probe: sym mat-vec rate vs N on one GPU; PMC refresh; nanotube stats
set -u
mkdir -p gpurun_out
L=gpurun_out/probe_n.log
: > $L
export TMPDIR=/tmp
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)" >> $L; exit $rc; fi
  return 0
}
for n in 8192 16384 23040 32768 46080; do
  step 120 n$n python bench.py --n $n --steps 50 --warmup 5 --no-cpu --no-solve
done
step 300 fetch rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r01_sym_fetch -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve
step 300 write rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r01_sym_write -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve
step 300 nt_stats rocprofv3 --kernel-trace --stats -d gpurun_out/r01_nt_stats -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 30 --warmup 3
echo done >> $L
