#!/bin/bash
# quick iteration loop: focused GPU tests, then the bench at the proxy sizes
set -u
mkdir -p gpurun_out
L=gpurun_out/iter.log
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
step 900 tests python -u -m pytest ${TESTS:-tests/test_gpu_symtile.py tests/test_gpu_multirank.py tests/test_gpu_core.py} -x -q -m gpu -p no:cacheprovider -rf --timeout 300 --timeout-method thread
for n in ${NS:-23040 65536}; do
  step 120 n$n python bench.py --n $n --steps 50 --warmup 5 --no-cpu --no-solve
done
echo done >> $L
