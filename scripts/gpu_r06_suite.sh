#!/bin/bash
# round 6: the driver's GPU suite and smoke at the current library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/r06/suite.log 2>&1 || exit 1
