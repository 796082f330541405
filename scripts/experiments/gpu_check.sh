#!/bin/bash
# One GPU session: tests, smoke, benches.  Every GPU step has its own time limit;
# a crash-class exit (>= 2 for pytest, anything non-zero elsewhere) ends the script.
set -u
mkdir -p gpurun_out
LOG=gpurun_out/check.log
: > $LOG
step() { echo "=== $*" >> $LOG; }
step pytest
timeout -k 10 900 python -m pytest tests/ -q -m gpu -x -p no:cacheprovider >> $LOG 2>&1
rc=$?; echo "pytest rc=$rc" >> $LOG
if [ $rc -ge 2 ]; then exit $rc; fi
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $LOG 2>&1 || exit 3
step bench_small
timeout -k 10 300 python bench.py --n 16384 --steps 20 --warmup 3 --no-cpu >> $LOG 2>&1 || exit 4
step bench_default
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2>> $LOG || exit 5
cat gpurun_out/bench_default.json >> $LOG
