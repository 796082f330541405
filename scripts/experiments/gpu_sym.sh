#!/bin/bash
# symmetric-tile bring-up: unit tests, then bench (sym vs dense), then the full GPU suite.
set -u
mkdir -p gpurun_out
L=gpurun_out/sym.log
: > $L
step() {  # step <timeout> <name> <cmd...>; stops the script on a crash / timeout
  local t=$1 name=$2; shift 2
  echo "=== $name" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)" >> $L; exit $rc; fi
  return 0
}
step 400 newtests python -m pytest tests/test_gpu_symtile.py tests/test_gpu_matfree.py -q -p no:cacheprovider -rf
step 300 bench_sym python bench.py --steps 30 --warmup 3 --no-cpu --no-solve
step 300 bench_dense python bench.py --steps 30 --warmup 3 --no-cpu --no-solve --storage dense
step 600 nanotube python bench.py --workload nanotube --steps 20 --warmup 2
step 1200 gputests python -m pytest tests/ -q -m gpu -p no:cacheprovider -rf
echo done >> $L
