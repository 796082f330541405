#!/bin/bash
# rocprofv3 kernel stats of the nanotube bench (configs[1]); output dir gpurun_out/$TAG
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
TAG=${TAG:-r02_nt}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o bench --output-format csv -- python3 bench.py --workload nanotube --steps 30 --warmup 3 --no-cpu ${EXTRA:-} > gpurun_out/$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG.log
find gpurun_out/$TAG -name '*kernel_stats.csv' | head -3
exit $rc
