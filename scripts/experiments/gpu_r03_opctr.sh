set -u
export TMPDIR=/tmp
O=gpurun_out/r03/opctr; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
echo "list rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU -d $O/sq -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve --steps 6 --warmup 1 > $O/sq.txt 2>&1
echo "sq rc=$?"
