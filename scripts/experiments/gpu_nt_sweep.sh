#!/bin/bash
# Nanotube-bench sweep over environment settings: SETTINGS="A=1 A=2,B=3 ..." (comma joins
# several variables of one setting; "-" = defaults), interleaved, 2 rounds.
set -u
mkdir -p gpurun_out
L=gpurun_out/nt_sweep.log
: > $L
for round in 1 2; do
  for setting in $SETTINGS; do
    echo "=== $setting round $round" >> $L
    envs=()
    if [ "$setting" != "-" ]; then IFS=',' read -ra envs <<< "$setting"; fi
    env "${envs[@]}" timeout -k 10 300 python bench.py --workload nanotube --steps 100 --warmup 5 --no-cpu --no-solve ${EXTRA:-} > gpurun_out/ab_tmp.json 2>>$L || exit 1
    python - >> $L <<'PY'
import json
d = [json.loads(l) for l in open("gpurun_out/ab_tmp.json") if l.startswith("{")][-1]
print(f"value {d['value']:.1f} it/s  iter {d['iter_device_ms']*1e3:.1f} us  op {d['operator_roofline']['mean_launch_ms']*1e3:.1f} us  precon {d['precon_roofline']['mean_launch_ms']*1e3:.1f} us  build {d['setup_s']['pivoted_cholesky_build']:.3f} s")
PY
  done
done
grep -v amdgpu.ids $L
