#!/bin/bash
# Quick loop for the record-factored operator: matfree + golden GPU tests, nanotube bench
# (configs[1]) plain and under rocprofv3 kernel stats, and the N = 156510 step.
set -u
mkdir -p gpurun_out
L=gpurun_out/recq.log
: > $L
step() {
  local t=$1 name=$2; shift 2
  echo "=== $name $(date +%T)" >> $L
  timeout -k 10 $t "$@" >> $L 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> $L
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >> $L; tail -40 $L; exit $rc; fi
}
export TMPDIR=/tmp
step 300 tests python3 -u -m pytest tests/test_gpu_matfree.py tests/test_gpu_golden.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step 300 nt python3 bench.py --workload nanotube --no-cpu
step 300 nt_prof rocprofv3 --kernel-trace --stats -d gpurun_out/recq_prof -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve
step 400 nt141 python3 bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
grep -E "passed|failed" $L
python3 - <<'PY'
import json
for l in open("gpurun_out/recq.log"):
    if l.startswith("{"):
        d = json.loads(l); o = d["operator_roofline"]; p = d["precon_roofline"]
        print(d["config"]["workload"], "it/s %.0f" % d["value"], "op_ms %.4f" % o["mean_launch_ms"],
              "pre_ms %.4f" % p["mean_launch_ms"], "iter_dev %.4f" % d["iter_device_ms"], d.get("solve_to_1e-6"))
PY
grep -E "k_rec|k_mf_" gpurun_out/recq_prof/nt_kernel_stats.csv | awk -F'",' '{split($1,a,"("); print a[1], $2}' | cut -c1-140
