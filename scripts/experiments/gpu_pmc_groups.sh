#!/bin/bash
# PMC HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the default bench (tile
# mat-vec + Nystrom apply) and of the nanotube bench (matrix-free operator + rank-2701
# apply); folded into profiles/pmc_traffic.json by scripts/pmc_summary.py / pmc_group.py.
# The nanotube pass instruments only the iteration's kernel families (the rank-2701
# pivoted-Cholesky build under full --pmc instrumentation crashed in the runtime).
set -u
mkdir -p gpurun_out
L=gpurun_out/pmc.log
: > $L
export TMPDIR=/tmp
T=${TAG:-r01}
RX='k_gemv|k_colgemv_part|k_precon_fin|k_mf_pair|k_mf_h|k_mf_jt'
for c in ${COUNTERS:-FETCH_SIZE WRITE_SIZE}; do
  if [ -z "${SKIP_RBF:-}" ]; then
    timeout -s KILL 150 rocprofv3 --pmc $c -d gpurun_out/${T}_rbf_$c -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve >> $L 2>&1 || exit 1
  fi
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "$RX" -d gpurun_out/${T}_nt_$c -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 6 --warmup 1 --no-cpu --no-solve >> $L 2>&1 || exit 1
done
echo done >> $L
