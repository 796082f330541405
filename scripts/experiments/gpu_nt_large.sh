#!/bin/bash
# Nanotube at the reference's large published points: M = 141 (N = 156510,
# ref. 2.073 s / PCG step on an A100) and M = 455 (N = 505050, ref. 6.600 s / step), rule-of-
# thumb pivoted-Cholesky rank, matrix-free operator.  A heartbeat line every minute (the
# build of the M = 455 case runs for minutes without output).  M list: MS (default "455").
set -u
mkdir -p gpurun_out
for M in ${MS:-455}; do
  L=gpurun_out/nt_m$M.log
  timeout -k 10 ${TLIM:-1100} python3 bench.py --workload nanotube --m $M --steps 20 --warmup 3 --no-cpu > $L 2>&1 &
  pid=$!
  while kill -0 $pid 2> /dev/null; do sleep 60; echo "M=$M alive $(date +%T)"; done
  wait $pid
  rc=$?
  grep '^{' $L | cut -c1-600
  if [ $rc -ne 0 ]; then tail -20 $L; exit $rc; fi
done
