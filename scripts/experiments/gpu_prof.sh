#!/bin/bash
# GPU tests (all, no -x) + rocprofv3 kernel trace/stats + PMC (HBM bytes) of the bench.
set -u
mkdir -p gpurun_out
LOG=gpurun_out/prof.log
: > $LOG
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "=== pytest" >> $LOG
timeout -k 10 900 python -m pytest tests/ -q -m gpu -p no:cacheprovider >> $LOG 2>&1
rc=$?; echo "pytest rc=$rc" >> $LOG
if [ $rc -ge 2 ]; then exit $rc; fi
echo "=== rocprof stats" >> $LOG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o bench --output-format csv -- python3 bench.py --steps 30 --warmup 3 --no-cpu --no-solve >> $LOG 2>&1 || exit 3
echo "=== rocprof pmc FETCH_SIZE" >> $LOG
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve >> $LOG 2>&1 || exit 4
echo "=== rocprof pmc WRITE_SIZE" >> $LOG
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu --no-solve >> $LOG 2>&1 || exit 5
find gpurun_out/prof_* -type f | head -50 >> $LOG
