set -u
export TMPDIR=/tmp
O=gpurun_out/r03/opctr2; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve --steps 6 --warmup 1 > $O/sq.txt 2>&1
echo "sq rc=$?"
