#!/bin/bash
# GPU test suite only (one process), then smoke.
set -u
mkdir -p gpurun_out
LOG=gpurun_out/tests.log
: > $LOG
timeout -k 10 1200 python -m pytest tests/ -q -m gpu -p no:cacheprovider -rf >> $LOG 2>&1
rc=$?; echo "pytest rc=$rc" >> $LOG
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> $LOG 2>&1
echo "smoke rc=$?" >> $LOG
