#!/bin/bash
# round 6: configs[2] slot partials stored / loaded with default (MALL-allocating) policy instead of
# non-temporal (an A/B library, MLFF_LIB), interleaved with the current library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/slots_ab
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --no-solve --configs3-n 0 \
    > gpurun_out/r06/slots_ab/nt_$rep.json 2> gpurun_out/r06/slots_ab/nt_$rep.err || exit 1
  MLFF_LIB=mlff-preconditioner_amd/lib/ab_slots_cached.so timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --no-solve --configs3-n 0 \
    > gpurun_out/r06/slots_ab/cached_$rep.json 2> gpurun_out/r06/slots_ab/cached_$rep.err || exit 1
done
