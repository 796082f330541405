#!/bin/bash
# round 6: the driver's GPU suite (every -m gpu test, the N = 74979 fixture test included) and smoke at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/head
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/head/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 500 --timeout-method thread \
  > gpurun_out/r06/head/suite.log 2>&1 || exit 1
