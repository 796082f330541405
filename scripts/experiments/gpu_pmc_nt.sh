#!/bin/bash
# PMC passes (separate: FETCH_SIZE, WRITE_SIZE, L2 hit/miss) of the nanotube bench (configs[1])
# restricted to the PCG kernels and the last Woodbury-build kernel (the solve-phase marker)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
T=${TAG:-r02}
RX='k_rec_|k_mf_|k_gemv|k_colgemv_part|k_precon_fin|k_trsm_diag_wide|k_update|k_stoptest'
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d gpurun_out/${T}_nt_$name -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 10 --warmup 2 --no-cpu --no-solve > gpurun_out/${T}_nt_$name.log 2>&1 || { echo "pass $C failed"; tail -5 gpurun_out/${T}_nt_$name.log; exit 1; }
  echo "pass $C ok"
done
