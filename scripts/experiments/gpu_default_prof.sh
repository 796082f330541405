#!/bin/bash
# rocprofv3 kernel stats of the default bench command and of its timed region alone
# (--no-solve --no-cpu --configs3-n 0: the same operator launches, nothing else at N = 65536).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/def_prof -o bench --output-format csv -- python3 bench.py > gpurun_out/def_prof.log 2>&1 || { tail -20 gpurun_out/def_prof.log; exit 1; }
grep '^{' gpurun_out/def_prof.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/def_prof_timed -o bench --output-format csv -- python3 bench.py --no-solve --no-cpu --configs3-n 0 > gpurun_out/def_prof_timed.log 2>&1 || { tail -20 gpurun_out/def_prof_timed.log; exit 1; }
grep '^{' gpurun_out/def_prof_timed.log | cut -c1-300
