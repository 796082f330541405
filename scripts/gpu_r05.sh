#!/bin/bash
# Round-5 GPU session: STEPS (space separated) from
#   suite     driver-exact `pytest -m gpu` (per-test timeout, progress log)
#   smoke     __graft_entry__.smoke()
#   bench     default bench line (python bench.py)
#   rehearse  MLFF_BENCH_REHEARSE=1 python bench.py --gpus 8: the self-launched 8-rank flow on
#             one GPU (SOLO ranks, gloo; not a measurement)
#   nt        nanotube bench line (configs[1])
#   tests     pytest of $TESTS (-v -s)
#   prof      rocprofv3 --kernel-trace --stats of the default bench command
#   pmc       scripts/pmc_head.py (FETCH_SIZE / WRITE_SIZE passes)
#   cmd       $CMD (one free-form step, $LIM seconds)
#   eth583    ethanol N = 15741 bench lines, k = 1264 / 554, refined vs one-step Woodbury panel
#   ptmfma    pair-tile operator: matrix-core variants (MLFF_PT_MFMA=$PTMV) vs the VALU default
#   ptvar     pair-tile variant sweep (MLFF_PT_VARIANT=$PTVS) at ethanol M = $PTM
#   ptch      pair-tile chunk count x variant sweep (MLFF_PT_CHUNKS=$PTCH) at ethanol M = $PTM
#   final1/2  evidence at the final library (smoke, rocprof, PMC table; bench lines)
# every GPU step runs under its own timeout; the first failure ends the script
set -u
export TMPDIR=/tmp
O=gpurun_out/r05
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
    rehearse) step rehearse_w8 600 env MLFF_BENCH_REHEARSE=1 python bench.py --gpus 8 --steps 20 --warmup 3 --launch-timeout 500 ;;
    nt) step bench_nanotube 300 python bench.py --workload nanotube ;;
    tests) step tests 1100 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread ${TESTS} ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py ;;
    pmc) step pmc 900 python scripts/pmc_head.py ;;
    cmd) step ${NAME:-cmd} ${LIM:-600} bash -c "$CMD" ;;
    profnt)  # kernel split of the nanotube (configs[1]) and ethanol N = 15741 iterations
      step profnt 300 rocprofv3 --kernel-trace --stats -d $O/profnt -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --no-solve --steps 200 --warmup 10
      step profeth 300 rocprofv3 --kernel-trace --stats -d $O/profeth -o eth --output-format csv -- python3 bench.py --workload ethanol --m 583 --no-cpu --no-solve --steps 200 --warmup 10 ;;
    ethpt)  # the ethanol published points with the pair-tile operator (fused iteration at one rank)
      for m in 583 2777 5833; do
        step ethpt_m$m 300 python bench.py --workload ethanol --m $m --no-cpu --no-solve --steps 50 --warmup 5
      done ;;
    solo)  # per-rank compute floor of the sharded configs[2] / configs[3] iteration (SOLO transport),
           # the p.q publish folded (default) vs its separate launch, two interleaved rounds
      for rep in 1 2; do
        step solo_w8_r$rep 300 python bench.py --solo-world 8 --n 65536 --steps 40 --warmup 5
        step solo_w8_pub_r$rep 300 env MLFF_PQ_PUBLISH=1 python bench.py --solo-world 8 --n 65536 --steps 40 --warmup 5
      done
      step solo_w8_n131072 300 python bench.py --solo-world 8 --n 131072 --steps 40 --warmup 5 ;;
    ptchunks)  # ethanol M = 583: pair-tile chunk count (37 = default: 185 workgroups on 256 CUs)
      for rep in 1 2; do
        for S in 37 52 74; do
          step ptS${S}_r$rep 300 env MLFF_PT_CHUNKS=$S python bench.py --workload ethanol --m 583 --no-cpu --no-solve --steps 200 --warmup 10
        done
      done ;;
    gramab)  # the one-step Woodbury panel with its Gram / POTRF / TRSM GEMMs on the VALU instead
             # of the matrix cores (MLFF_GEMM_VALU=1): nanotube configs[1] and ethanol N = 15741
      step gram_nt_mfma 300 env MLFF_WB_REFINE=0 python bench.py --workload nanotube --no-cpu --steps 20 --warmup 3
      step gram_nt_valu 300 env MLFF_WB_REFINE=0 MLFF_GEMM_VALU=1 python bench.py --workload nanotube --no-cpu --steps 20 --warmup 3
      step gram_nt_valu_ref 300 env MLFF_GEMM_VALU=1 python bench.py --workload nanotube --no-cpu --steps 20 --warmup 3
      step gram_eth_valu 300 env MLFF_WB_REFINE=0 MLFF_GEMM_VALU=1 python bench.py --workload ethanol --m 583 --no-cpu --steps 20 --warmup 3
      step gram_eth_valu_ref 300 env MLFF_GEMM_VALU=1 python bench.py --workload ethanol --m 583 --no-cpu --steps 20 --warmup 3
      step gram_diag_valu 600 env MLFF_GEMM_VALU=1 python -u scripts/dev/diag_config1_gram.py ;;
    gramdd)  # the Woodbury Gram in double-double (MLFF_WB_GRAM=1), one-step and refined panels
      for g in ${GRAMS:-1 0}; do
        step gdd${g}_nt_onestep 300 env MLFF_WB_GRAM=$g MLFF_WB_REFINE=0 python bench.py --workload nanotube --no-cpu --steps 20 --warmup 3
        step gdd${g}_nt_refined 300 env MLFF_WB_GRAM=$g python bench.py --workload nanotube --no-cpu --steps 20 --warmup 3
        step gdd${g}_eth_onestep 300 env MLFF_WB_GRAM=$g MLFF_WB_REFINE=0 python bench.py --workload ethanol --m 583 --no-cpu --steps 20 --warmup 3
        step gdd${g}_eth_refined 300 env MLFF_WB_GRAM=$g python bench.py --workload ethanol --m 583 --no-cpu --steps 20 --warmup 3
        step gdd${g}_eth554_refined 300 env MLFF_WB_GRAM=$g python bench.py --workload ethanol --m 583 --k 554 --no-cpu --steps 20 --warmup 3
        step gdd${g}_eth554_onestep 300 env MLFF_WB_GRAM=$g MLFF_WB_REFINE=0 python bench.py --workload ethanol --m 583 --k 554 --no-cpu --steps 20 --warmup 3
      done ;;
    headlines)  # every bench line at HEAD: nanotube configs[1] and N = 156510, ethanol at the
                # reference's published sizes
      step head_nt 300 python bench.py --workload nanotube
      step head_nt141 600 python bench.py --workload nanotube --m 141 --no-cpu --steps 20 --warmup 3
      for m in 583 2777 5833; do
        step head_eth_m$m 600 python bench.py --workload ethanol --m $m --no-cpu --steps 30 --warmup 3
      done ;;
    rpwab)  # rows apply: at least 7 rows per workgroup (default) vs ceil(k / 256) (MLFF_LR_MIN_RPW=1)
      for rep in 1 2; do
        for r in 7 1; do
          step rpw${r}_eth_r$rep 300 env MLFF_LR_MIN_RPW=$r python bench.py --workload ethanol --m 583 --no-cpu --no-solve --steps 200 --warmup 10
          step rpw${r}_nt_r$rep 300 env MLFF_LR_MIN_RPW=$r python bench.py --workload nanotube --no-cpu --no-solve --steps 200 --warmup 10
        done
      done ;;
    final1)  # evidence at the final library (1/2): smoke, the default bench under rocprofv3
             # --kernel-trace --stats, PMC traffic of the bench's kernel groups
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      step final_bench_prof 600 rocprofv3 --kernel-trace --stats -d $O/final_prof -o bench --output-format csv -- python3 bench.py
      step final_pmc 1000 python scripts/pmc_head.py --out $O/pmc_head ;;
    final2)  # (2/2): the default bench (traffic from the committed PMC table), the nanotube and
             # ethanol N = 15741 lines with their CPU baselines
      step final_bench 600 python bench.py
      step final_nt 300 python bench.py --workload nanotube
      step final_eth583 600 python bench.py --workload ethanol --m 583 ;;
    ptmfma)  # pair-tile force sum on the matrix cores (MLFF_PT_MFMA=1) vs the VALU default, interleaved
      for m in ${PTM:-583 2777 5833}; do
        for r in 1 2; do
          step ptv_m${m}_r$r 300 python bench.py --workload ethanol --m $m --no-cpu --no-solve --steps 50 --warmup 5
          for v in ${PTMV:-1 2}; do
            step ptm${v}_m${m}_r$r 300 env MLFF_PT_MFMA=$v python bench.py --workload ethanol --m $m --no-cpu --no-solve --steps 50 --warmup 5
          done
        done
      done ;;
    ptvar)  # pair-tile variant sweep at small M (MLFF_PT_VARIANT), interleaved
      for m in ${PTM:-583}; do
        for r in 1 2; do
          for v in ${PTVS:-0 7 8}; do
            step ptvar${v}_m${m}_r$r 300 env MLFF_PT_VARIANT=$v python bench.py --workload ethanol --m $m --no-cpu --no-solve --steps 100 --warmup 10
          done
        done
      done ;;
    ptch)  # pair-tile chunk count x variant at small M (MLFF_PT_CHUNKS, MLFF_PT_VARIANT), interleaved
      for m in ${PTM:-111}; do
        for r in 1 2; do
          for v in ${PTVS:-0 8}; do
            for c in ${PTCH:-7 14 28 56}; do
              step ptch_v${v}_c${c}_m${m}_r$r 300 env MLFF_PT_VARIANT=$v MLFF_PT_CHUNKS=$c python bench.py --workload ethanol --m $m --no-cpu --no-solve --steps 100 --warmup 10
            done
          done
        done
      done ;;
    eth583)  # ethanol N = 15741 (harmonic labels) at the rule-of-thumb k and a published k, with the
             # refined (default) and one-step Woodbury panel
      for k in 1264 554; do
        step eth583_k${k} 300 python bench.py --workload ethanol --m 583 --k $k --no-cpu --steps 30 --warmup 3
        step eth583_k${k}_onestep 300 env MLFF_WB_REFINE=0 python bench.py --workload ethanol --m 583 --k $k --no-cpu --steps 30 --warmup 3
      done ;;
  esac
done
echo "== all steps ok"
