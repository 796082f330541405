#!/bin/bash
# per-rank compute floor of the sharded iteration (bench.py --solo-world): W = 2, 4, 8, rank 0
# and the last rank; VARIANTS = library variants to interleave ("base" = in-tree)
set -u
mkdir -p gpurun_out
L=gpurun_out/solo.log
: > $L
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=""; else lib=mlff-preconditioner_amd/lib/variants/$v.so; fi
  for w in 1 2 4 8; do
    for r in 0 $((w - 1)); do
      [ $w = 1 ] && [ $r != 0 ] && continue
      echo "=== v=$v w=$w r=$r" >> $L
      if [ $w = 1 ]; then
        MLFF_LIB=$lib timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu --no-solve >> $L 2>&1 || exit 1
      else
        MLFF_LIB=$lib timeout -k 10 150 python bench.py --solo-world $w --solo-rank $r --steps 100 --warmup 10 >> $L 2>&1 || exit 1
      fi
    done
  done
done
if [ -n "${TRACE:-}" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG:-r01}_solo8 -o b --output-format csv -- python3 bench.py --solo-world 8 --solo-rank 0 --steps 100 --warmup 10 >> $L 2>&1 || exit 2
fi
echo done >> $L
