#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; separate) of the cluster one-pass apply at N = 156510
# (bench.py --workload nanotube --m 141), solve-phase dispatches after the Woodbury build.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
RX='k_lr_cluster|k_lr_fin|k_trsm_diag_wide'
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d gpurun_out/m141_pmc_$C -o bench --output-format csv -- python3 bench.py --workload nanotube --m 141 --steps 10 --warmup 2 --no-cpu --no-solve > gpurun_out/m141_pmc_$C.log 2>&1 || { echo "pass $C failed"; tail -5 gpurun_out/m141_pmc_$C.log; exit 1; }
  echo "pass $C ok"
done
