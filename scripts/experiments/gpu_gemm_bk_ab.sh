#!/bin/bash
# MFMA GEMM K step 32 (MLFF_GEMM_BK=32) vs 16: GEMM layout tests, then build times of the
# nanotube (k = 2701) and N = 156510 (k = 14670) pivoted-Cholesky preconditioners, interleaved.
set -u
mkdir -p gpurun_out
L=gpurun_out/gemm_bk_ab.log
: > $L
MLFF_GEMM_BK=32 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py >> $L 2>&1 || { echo "gemm tests failed"; tail -20 $L; exit 1; }
run() { echo "=== $1" >> $L; shift; timeout -k 10 400 "$@" >> $L 2>&1 || { echo "failed $*"; tail -20 $L; exit 1; }; }
for rep in 1 2; do
  for bk in 32 16; do
    run "nt bk=$bk" env MLFF_GEMM_BK=$bk python3 bench.py --workload nanotube --no-cpu --no-solve --steps 10 --warmup 2
    run "m141 bk=$bk" env MLFF_GEMM_BK=$bk python3 bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 5 --warmup 1
  done
done
grep -E "passed|failed" $L | head -3
python3 - <<'PY'
import json
cur=None
for line in open('gpurun_out/gemm_bk_ab.log'):
    if line.startswith('==='): cur=line[4:].strip()
    if line.startswith('{'):
        d=json.loads(line)
        print(f"{cur:16s} build {d['setup_s']['pivoted_cholesky_build']:.4f} s  step {d['ms_per_step']:.4f} ms")
PY
