#!/bin/bash
# rocprofv3 kernel stats of the default bench command at HEAD (the line's roofline kernel,
# k_symv_dyn, must agree with the event-measured mean launch in the same run's JSON line).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_e
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e -o bench --output-format csv -- python3 bench.py > gpurun_out/prof_e/bench.log 2>&1 || { tail -20 gpurun_out/prof_e/bench.log; exit 1; }
grep '^{' gpurun_out/prof_e/bench.log | cut -c1-300
