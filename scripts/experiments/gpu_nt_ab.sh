#!/bin/bash
# A/B of a nanotube-bench environment switch: VAR=name, values in VALS (interleaved, 2 rounds)
set -u
mkdir -p gpurun_out
L=gpurun_out/nt_ab.log
: > $L
for round in 1 2; do
  for v in $VALS; do
    echo "=== $VAR=$v round $round" >> $L
    env $VAR=$v timeout -k 10 300 python bench.py --workload nanotube --steps 100 --warmup 5 --no-cpu --no-solve > gpurun_out/ab_tmp.json 2>>$L || exit 1
    python - >> $L <<'PY'
import json
d = [json.loads(l) for l in open("gpurun_out/ab_tmp.json") if l.startswith("{")][-1]
print(f"value {d['value']:.1f} it/s  iter {d['iter_device_ms']*1e3:.1f} us  op {d['operator_roofline']['mean_launch_ms']*1e3:.1f} us  precon {d['precon_roofline']['mean_launch_ms']*1e3:.1f} us  build {d['setup_s']['pivoted_cholesky_build']:.3f} s")
PY
  done
done
cat $L
