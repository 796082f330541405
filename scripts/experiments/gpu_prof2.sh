#!/bin/bash
# symv variants probe, rocprofv3 kernel stats (sym RBF + nanotube matfree), PMC of the sym bench.
set -u
mkdir -p gpurun_out
L=gpurun_out/prof2.log
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
step 180 probe ./build_probe/probe_symv 65536
step 400 newtests python -m pytest tests/test_gpu_symtile.py tests/test_gpu_matfree.py -q -p no:cacheprovider -rf
step 600 stats_sym rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sym -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-solve
step 600 stats_nt rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nt -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 20 --warmup 3 --no-solve
step 600 pmc_fetch rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_sym_fetch -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve
step 600 pmc_write rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_sym_write -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve
find gpurun_out/prof_sym gpurun_out/prof_nt gpurun_out/pmc_sym_* -type f >> $L
echo done >> $L
