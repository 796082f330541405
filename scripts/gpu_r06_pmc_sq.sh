#!/bin/bash
# round 6: what limits the nanotube rows apply (k_lr_rows + k_lr_fin) beside
# the configs[2] tile mat-vec -- SQ wave-state counters and the L2->fabric read requests with their
# DRAM credit stalls, each counter group in a pass of its own (MI355X_MICROARCH.md PMC slots)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/pmcsq
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD"
TCC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_CYCLE_sum"
REGEX="k_lr_rows|k_lr_fin|k_symv_dyn|k_sym_reduce|k_rec_g|k_rec_fin"
for wl in nt c2; do
  if [ $wl = nt ]; then ARGS="--workload nanotube"; else ARGS="--configs3-n 0"; fi
  for grp in sq tcc; do
    if [ $grp = sq ]; then C="$SQ"; else C="$TCC"; fi
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$REGEX" -d $O/${wl}_$grp -o pmc \
      --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve $ARGS \
      > $O/${wl}_$grp.log 2>&1 || exit 1
  done
done
