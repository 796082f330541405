# k_rec_g phase timestamps (variant build with -DMLFF_REC_TRACE, lib/variants/rectrace.so)
set -u
mkdir -p gpurun_out/r03
for g in 8 16; do
  MLFF_REC_RG=$g MLFF_LIB=mlff-preconditioner_amd/lib/variants/rectrace.so MLFF_REC_TRACE_FILE=gpurun_out/r03/rectrace_rg$g.txt \
    timeout -k 10 300 python bench.py --workload nanotube --no-cpu --no-solve --steps 20 --warmup 5 > gpurun_out/r03/rectrace_rg$g.log 2>&1 || exit 1
done
echo done
