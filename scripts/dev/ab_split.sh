set -u
L=gpurun_out/ab2.log; : > $L
for rep in 1 2 3; do for v in base oldsplit; do
  if [ $v = base ]; then lib=""; else lib=mlff-preconditioner_amd/lib/variants/$v.so; fi
  echo "=== v=$v nt rep=$rep" >> $L
  MLFF_LIB=$lib timeout -k 10 200 python bench.py --workload nanotube --steps 40 --warmup 3 --no-cpu --no-solve >> $L 2>&1 || exit 1
  echo "=== v=$v rbf rep=$rep" >> $L
  MLFF_LIB=$lib timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --no-solve >> $L 2>&1 || exit 1
done; done
