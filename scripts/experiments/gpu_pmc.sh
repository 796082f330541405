#!/bin/bash
# PMC HBM traffic of the default bench's tile mat-vec: FETCH_SIZE and WRITE_SIZE in
# separate passes (MI355X_MICROARCH.md: one TCC counter group per pass)
set -u
mkdir -p gpurun_out
L=gpurun_out/pmc.log
: > $L
export TMPDIR=/tmp
T=${TAG:-r01}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_sym_fetch -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve >> $L 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_sym_write -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve >> $L 2>&1 || exit 1
echo done >> $L
