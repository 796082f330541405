#!/bin/bash
# round 6: POTRF readlane diagonal (bitwise + time), nanotube build split, W = 8 reduce A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/c
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_core.py::test_potrf_wave_diag_bitwise" "tests/test_gpu_core.py::test_woodbury_refine_steps" \
  > gpurun_out/r06/c/potrf.log 2>&1 || exit 1
for rep in 1 2; do
  for cfg in "default:" "pqsep:MLFF_PQ_PUBLISH=1" "fusep0:MLFF_FUSE_P=0" "both:MLFF_PQ_PUBLISH=1 MLFF_FUSE_P=0"; do
    name=${cfg%%:*}; ev=${cfg#*:}
    env $ev timeout -k 10 200 python -u bench.py --solo-world 8 --solo-rank 0 --n 65536 --steps 40 \
      > gpurun_out/r06/c/w8_${name}_$rep.json 2> gpurun_out/r06/c/w8_${name}_$rep.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/c/prof_nt -o nt -- \
  python3 bench.py --workload nanotube --steps 20 --warmup 5 --no-cpu --no-solve \
  > gpurun_out/r06/c/bench_nt_prof.json 2> gpurun_out/r06/c/bench_nt_prof.err || exit 1
