#!/bin/bash
# Round-3 GPU session: STEPS (space separated) from
#   suite   driver-exact `pytest -m gpu` (per-test timeout, progress log)
#   smoke   __graft_entry__.smoke()
#   bench   default bench line (python bench.py) -> gpurun_out/r03/bench_default.txt
#   nt      nanotube bench line (configs[1])
#   lrab    interleaved A/B of the low-rank apply form at configs[2] (cluster vs two passes)
#   pmc     scripts/pmc_head.py (FETCH_SIZE / WRITE_SIZE passes, rbf + nanotube)
#   prof    rocprofv3 --kernel-trace --stats of the default bench command
#   preab   k_rec_g first-batch prefetch A/B (nanotube); fpab  fused p update A/B;  ntprof  rocprof stats of the nanotube bench
# every GPU step runs under its own timeout; the first failure ends the script
set -u
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" | tee -a $O/steps.log
  timeout -k 10 $lim "$@" > $O/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)" | tee -a $O/steps.log
  if [ $rc -ne 0 ]; then tail -30 $O/$name.txt; exit $rc; fi
}
for s in ${STEPS:-suite smoke bench}; do
  case $s in
    suite) step suite 1100 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread ${PYTEST_EXTRA:-} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_default 600 python bench.py ;;
    nt) step bench_nanotube 300 python bench.py --workload nanotube ;;
    lrab)
      for r in 1 2 3; do
        step lrab_default_$r 200 python bench.py --no-cpu --no-solve --configs3-n 0
        step lrab_twopass_$r 200 env MLFF_LR_ROWS=0 python bench.py --no-cpu --no-solve --configs3-n 0
      done ;;
    opexp)  # matrix-free operator with the rank-2701 panel streamed between applications vs a
            # rank-16 panel (tables stay cached): is the operator bound by cache residency?
      for r in 1 2; do
        step opexp_k2701_$r 300 python bench.py --workload nanotube --no-cpu --no-solve
        step opexp_k16_$r 300 python bench.py --workload nanotube --no-cpu --no-solve --k 16
      done
      step opexp_prof 300 rocprofv3 --kernel-trace --stats -d $O/opexp_prof -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve ;;
    nocap)  # k_rec_g epilogue rows re-read (MLFF_REC_NOCAP=1) vs captured, interleaved
      for r in 1 2; do
        step nocap_default_$r 300 python bench.py --workload nanotube --no-cpu --no-solve
        step nocap_on_$r 300 env MLFF_REC_NOCAP=1 python bench.py --workload nanotube --no-cpu --no-solve
      done ;;
    oneab)  # k_rec_g one-batch form (default) vs two batches (MLFF_REC_ONE=0), interleaved
      for r in 1 2 3; do
        step oneab_on_$r 300 python bench.py --workload nanotube --no-cpu --no-solve
        step oneab_off_$r 300 env MLFF_REC_ONE=0 python bench.py --workload nanotube --no-cpu --no-solve
      done ;;
    rgab)  # k_rec_g variants, interleaved: default (8-point groups, 16-slot stage) / 32-slot stage /
           # 16-point groups (the round-2 form)
      for r in 1 2 3; do
        step rgab_def_$r 300 python bench.py --workload nanotube --no-cpu --no-solve
        step rgab_wc32_$r 300 env MLFF_REC_WC16=0 python bench.py --workload nanotube --no-cpu --no-solve
        step rgab_rg16_$r 300 env MLFF_REC_RG=16 python bench.py --workload nanotube --no-cpu --no-solve
      done ;;
    ntab)  # nanotube bench, 3 runs (operator A/B against the numbers of the previous session)
      for r in 1 2 3; do
        step ntab_$r 300 python bench.py --workload nanotube --no-cpu --no-solve
      done ;;
    rehearse)  # the multi-rank bench flow on one GPU (torchrun, SOLO ranks over gloo): not RCCL
      for W in 2 8; do
        step rehearse_w$W 400 env MLFF_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29500 + W)) \
          bench.py --gpus $W --steps 10 --warmup 2 --no-solve
      done ;;
    preab)  # k_rec_g: Rdd of the first batch issued with the staging loads (default) vs after
      for r in 1 2; do
        step preab_on_$r 300 python bench.py --workload nanotube --no-cpu --no-solve
        step preab_off_$r 300 env MLFF_REC_PRE=0 python bench.py --workload nanotube --no-cpu --no-solve
      done ;;
    fpab)  # the CG vector updates folded into the nanotube iteration (default: 4 launches) vs
           # k_update_xr on its own (5) vs k_update_p and k_update_xr on their own (6), interleaved
      for r in 1 2; do
        step fpab_on_$r 300 python bench.py --workload nanotube --no-cpu --no-solve
        step fpab_xr0_$r 300 env MLFF_FUSE_XR=0 python bench.py --workload nanotube --no-cpu --no-solve
        step fpab_off_$r 300 env MLFF_FUSE_P=0 python bench.py --workload nanotube --no-cpu --no-solve
      done ;;
    lrg)  # one-pass apply workgroups (partial vectors): 256 (default) / 192 / 128, interleaved
      for r in 1 2; do
        for g in 256 192 128; do
          step lrg_${g}_$r 300 env MLFF_LR_GROUPS=$g python bench.py --workload nanotube --no-cpu --no-solve
        done
      done ;;
    ntprof) step ntprof 300 rocprofv3 --kernel-trace --stats -d $O/ntprof -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve ;;
    tests) step tests 1100 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread ${TESTS} ;;
    pmc) step pmc 900 python scripts/pmc_head.py --out $O/pmc_head ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py ;;
  esac
done
echo "== all done $(date +%T)" | tee -a $O/steps.log
