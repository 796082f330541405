#!/bin/bash
# probe + focused tests + benches + full GPU suite; stops on a crash/timeout.
set -u
mkdir -p gpurun_out
L=gpurun_out/round.log
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
[ -x build_probe/probe_symv ] && step 200 probe ./build_probe/probe_symv 65536
step 600 newtests python -m pytest tests/test_gpu_matfree.py tests/test_gpu_symtile.py -q -p no:cacheprovider -rf
step 300 bench_sym python bench.py --steps 30 --warmup 3 --no-cpu --no-solve
step 600 nanotube python bench.py --workload nanotube --steps 30 --warmup 3
step 1500 gputests python -m pytest tests/ -q -m gpu -p no:cacheprovider -rf
echo done >> $L
