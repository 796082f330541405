set -u
mkdir -p gpurun_out
for w in nanotube rbf; do
for v in base oldsplit; do
  if [ $v = base ]; then lib=""; else lib=mlff-preconditioner_amd/lib/variants/$v.so; fi
  MLFF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ps_${w}_$v -o bench --output-format csv -- python3 bench.py --workload $w --steps 30 --warmup 3 --no-cpu --no-solve > gpurun_out/ps_$v.log 2>&1 || exit 1
done
done
