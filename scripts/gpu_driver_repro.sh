#!/bin/bash
# Runs the round-end driver's exact GPU-suite command (no --timeout, no TMPDIR
# override), keeping the whole log, the per-test progress file and the all-thread
# faulthandler dump under gpurun_out/.
set -u
mkdir -p gpurun_out
rm -f gpurun_out/pytest_progress.log gpurun_out/pytest_faulthandler.log
timeout -k 10 600 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider > gpurun_out/driver_pytest.log 2>&1
rc=$?
echo "driver-command rc=$rc" >> gpurun_out/driver_pytest.log
tail -5 gpurun_out/driver_pytest.log
exit $rc
