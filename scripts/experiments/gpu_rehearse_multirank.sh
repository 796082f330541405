#!/bin/bash
# One-GPU rehearsal of the multi-rank bench flow (torchrun, W processes, SOLO library ranks,
# gloo): exercises bench.py's distributed logic (configs[2] value, configs[3] leg, RCCL /
# memory fields, max-over-ranks timing, the single JSON line) -- not RCCL, not a measurement.
set -u
mkdir -p gpurun_out
L=gpurun_out/rehearse.log
: > $L
for W in ${WS:-2 8}; do
  echo "=== W=$W" >> $L
  MLFF_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29500 + W)) \
    bench.py --gpus $W --steps 10 --warmup 2 --no-solve >> $L 2>&1
  rc=$?
  echo "=== W=$W rc=$rc" >> $L
  if [ $rc -ne 0 ]; then tail -40 $L; exit $rc; fi
done
grep -v amdgpu.ids $L | tail -12
