#!/bin/bash
# Round-4 GPU session: STEPS (space separated) from
#   suite   driver-exact `pytest -m gpu` (per-test timeout, progress log)
#   smoke   __graft_entry__.smoke()
#   bench   default bench line (python bench.py)
#   nt      nanotube bench line (configs[1])
#   tests   pytest of $TESTS (-v -s)
#   ptvar   pair-tile variants on the ethanol shape (M = 583 / 2777): MLFF_PT_VARIANT sweep
#   eth     ethanol bench lines at the reference's published sizes (M = 583 / 2777 / 5833) with
#           the pair-tile operator, the record-factored one and (M <= 2777) stored K
#   ptprof  rocprofv3 --kernel-trace --stats of the ethanol M = 5833 bench
#   prof    rocprofv3 --kernel-trace --stats of the default bench command
#   pmc     scripts/pmc_head.py (FETCH_SIZE / WRITE_SIZE passes)
# every GPU step runs under its own timeout; the first failure ends the script
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" | tee -a $O/steps.log
  timeout -k 10 $lim "$@" > $O/$name.txt 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)" | tee -a $O/steps.log
  if [ $rc -ne 0 ]; then tail -30 $O/$name.txt; exit $rc; fi
}
EB="python bench.py --workload ethanol --no-cpu --no-solve --steps 30 --warmup 3"
for s in ${STEPS:-suite smoke bench}; do
  case $s in
    suite) step suite 1100 python -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread ${PYTEST_EXTRA:-} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_default 600 python bench.py ;;
    nt) step bench_nanotube 300 python bench.py --workload nanotube ;;
    tests) step tests 1100 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread ${TESTS} ;;
    ptvar)
      for m in 583 2777 5833; do
        for v in ${PTV:-0 5 6 7 8 9}; do
          step ptvar_m${m}_v$v 300 env MLFF_PT_VARIANT=$v $EB --m $m --storage matfree --mf-form pt
        done
      done
      step ptvar_prof 600 rocprofv3 --kernel-trace --stats -d $O/ptvar_prof -o eth --output-format csv -- python3 bench.py --workload ethanol --no-cpu --no-solve --steps 30 --warmup 3 --m 2777 --storage matfree ;;
    eth)
      for m in 583 2777 5833; do
        step eth_m${m}_pt 600 $EB --m $m --storage matfree --mf-form pt
      done
      for m in 583 2777; do
        step eth_m${m}_rec 600 $EB --m $m --storage matfree --mf-form rec
        step eth_m${m}_sym 600 $EB --m $m --storage sym
        step eth_m${m}_dense 600 $EB --m $m --storage dense
      done ;;
    eth111)  # configs[0] geometry (N = 2997): pair-tile vs record-factored, kernel split of both
      step eth111_pt 300 $EB --m 111 --storage matfree --mf-form pt
      step eth111_rec 300 $EB --m 111 --storage matfree --mf-form rec
      step eth111_prof_rec 300 rocprofv3 --kernel-trace --stats -d $O/eth111_rec -o eth --output-format csv -- python3 bench.py --workload ethanol --m 111 --no-cpu --no-solve --steps 30 --warmup 3 --storage matfree --mf-form rec
      step eth111_prof_pt 300 rocprofv3 --kernel-trace --stats -d $O/eth111_pt -o eth --output-format csv -- python3 bench.py --workload ethanol --m 111 --no-cpu --no-solve --steps 30 --warmup 3 --storage matfree --mf-form pt ;;
    solo)  # per-rank compute floors of configs[2] on W = 8 / 4 (SOLO transport), fused p vs not
      for W in 8 4; do
        step solo_w${W} 300 python bench.py --solo-world $W --n 65536 --steps 40 --warmup 5
        step solo_w${W}_nofuse 300 env MLFF_FUSE_P=0 python bench.py --solo-world $W --n 65536 --steps 40 --warmup 5
      done ;;
    diag1) step diag1 600 python -u scripts/dev/diag_config1.py ;;
    diag1b) step diag1b 900 python -u scripts/dev/diag_config1b.py ;;
    diag1c) step diag1c 900 python -u scripts/dev/diag_config1c.py ;;
    diag1qr) step diag1qr 600 python -u scripts/dev/diag_config1c.py --qr ;;
    diag1d) step diag1d 600 python -u scripts/dev/diag_config1d.py ;;
    headlines)  # every bench line at HEAD: ethanol at the reference's published sizes (pair-tile),
                # nanotube configs[1] and the N = 156510 point
      for m in 583 2777 5833; do
        step head_eth_m$m 600 python bench.py --workload ethanol --m $m --no-cpu --steps 30 --warmup 3
      done
      step head_nt 300 python bench.py --workload nanotube
      step head_nt141 600 python bench.py --workload nanotube --m 141 --no-cpu --steps 20 --warmup 3 ;;
    nt141ab)  # nanotube N = 156510 solve to 1e-6 with the Woodbury panel in one CholeskyQR step (the
              # default two-step line is headlines/head_nt141)
      step nt141_onestep 600 env MLFF_WB_REFINE=0 python bench.py --workload nanotube --m 141 --no-cpu --steps 20 --warmup 3 ;;
    lr1024)  # one-pass panel apply with 1024-thread workgroups (8 double2 per thread, 4 waves per
             # SIMD) vs 512 (16 double2, 2 waves per SIMD), interleaved; then the parity tests under it
      for rep in 1 2; do
        for T in 512 1024; do
          step lr${T}_nt_r$rep 300 env MLFF_LR_THREADS=$T python bench.py --workload nanotube --no-cpu --steps 200 --warmup 20
          step lr${T}_eth_r$rep 300 env MLFF_LR_THREADS=$T python bench.py --workload ethanol --m 583 --no-cpu --steps 200 --warmup 20 --no-solve
        done
      done
      step lr1024_prof 300 env MLFF_LR_THREADS=1024 rocprofv3 --kernel-trace --stats -d $O/lr1024prof -o nt --output-format csv -- python3 bench.py --workload nanotube --no-cpu --steps 200 --warmup 20 --no-solve
      step lr1024_tests 600 env MLFF_LR_THREADS=1024 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_fused_iteration.py && step cho_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cho_stable.py ;;
    lccfg)  # cluster apply: hand-off slack D, load distance L, double2 per thread M (MLFF_LC_CFG),
            # interleaved twice at the reference's large published points; then the cluster tests
      for rep in 1 2; do
        for c in ${LCC:-2,1,8 2,2,6 3,1,6 3,2,6 2,2,4 4,2,4 3,3,4 5,1,4}; do
          t=${c//,/_}
          step lc${t}_nt141_r$rep 300 env MLFF_LC_CFG=$c python bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
          step lc${t}_eth5833_r$rep 300 env MLFF_LC_CFG=$c $EB --m 5833
        done
      done
      for c in ${LCT:-3,2,6 4,2,4}; do
        t=${c//,/_}
        step lc${t}_tests 600 env MLFF_LC_CFG=$c python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_core.py -k "one_pass or cluster" tests/test_gpu_configs.py::test_nanotube_cluster_apply_solve
      done ;;
    lcpf)  # cluster apply with the next row's hand-off look issued one step early (MLFF_LC_PREFETCH)
           # vs at the start of its own step, at several D / L / M; then the cluster tests
      for rep in 1 2; do
        for c in ${LCC:-2,1,8 1,1,8 3,1,6 3,2,6 4,2,4}; do
          for pf in 1 0; do
            t=${c//,/_}_pf$pf
            step lc${t}_nt141_r$rep 300 env MLFF_LC_PREFETCH=$pf MLFF_LC_CFG=$c python bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
            step lc${t}_eth5833_r$rep 300 env MLFF_LC_PREFETCH=$pf MLFF_LC_CFG=$c $EB --m 5833
          done
        done
        for pf in 1 0; do
          step lc_pf${pf}_rbf_r$rep 300 env MLFF_LC_PREFETCH=$pf python bench.py --no-cpu --no-solve --steps 50 --warmup 5
        done
      done
      step lcpf_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_core.py -k "one_pass or cluster" tests/test_gpu_configs.py::test_nanotube_cluster_apply_solve ;;
    lcrt)  # cluster apply with 7 row waves (2 waves per SIMD, 256 registers: 3-6 rows in registers)
           # vs 8 (3 per SIMD, 4 rows), interleaved; configs[2]; then the cluster tests on one of them
      for rep in 1 2; do
        for c in ${LCC:-2,1,8,512 2,2,8,448 2,3,8,448 3,2,8,448 3,3,8,448 2,4,8,448}; do
          t=${c//,/_}
          step lc${t}_nt141_r$rep 300 env MLFF_LC_CFG=$c python bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
          step lc${t}_eth5833_r$rep 300 env MLFF_LC_CFG=$c $EB --m 5833
          step lc${t}_rbf_r$rep 300 env MLFF_LC_CFG=$c python bench.py --no-cpu --no-solve --steps 50 --warmup 5
        done
      done
      step lcrt_tests 600 env MLFF_LC_CFG=${LCTEST:-2,3,8,448} python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_core.py -k "one_pass or cluster" tests/test_gpu_configs.py::test_nanotube_cluster_apply_solve ;;
    lcd)  # 7 row waves: hand-off slack D 3 / 4 / 5, interleaved; then the cluster tests (every case)
      for rep in 1 2; do
        for c in ${LCC:-3,2,8,448 4,1,8,448 4,2,8,448 5,1,8,448 3,3,8,448}; do
          t=${c//,/_}
          step lc${t}_nt141_r$rep 300 env MLFF_LC_CFG=$c python bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
          step lc${t}_eth5833_r$rep 300 env MLFF_LC_CFG=$c $EB --m 5833
        done
      done
      timeout -k 10 600 env MLFF_LC_CFG=${LCTEST:-3,2,8,448} python -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests/test_gpu_core.py -k "one_pass or cluster" tests/test_gpu_configs.py::test_nanotube_cluster_apply_solve > $O/lcd_tests.txt 2>&1
      echo "== lcd_tests rc=$?" | tee -a $O/steps.log ;;
    lrdiag)  # the 20000 x 400 random-panel solve's traces, one-pass (default / 7 row waves) and two-pass
      step lrdiag_default 300 python -u scripts/dev/diag_lowrank_20000.py $O/lr20000_default.npz
      step lrdiag_448 300 env MLFF_LC_CFG=4,1,8,448 python -u scripts/dev/diag_lowrank_20000.py $O/lr20000_448.npz ;;
    lrform)  # rows that fit one workgroup: the per-workgroup one-pass apply vs the cluster form
             # (MLFF_LR_FORM was a temporary switch of api.hip, removed after this A/B)
      for rep in 1 2; do
        for f in rows cluster; do
          step lrf_${f}_nt_r$rep 300 env MLFF_LR_FORM=$f python bench.py --workload nanotube --no-cpu --steps 200 --warmup 20
          step lrf_${f}_eth583_r$rep 300 env MLFF_LR_FORM=$f python bench.py --workload ethanol --m 583 --no-cpu --steps 200 --warmup 20 --no-solve
        done
      done
      timeout -k 10 600 env MLFF_LR_FORM=cluster python -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_fused_iteration.py tests/test_gpu_golden.py > $O/lrf_tests.txt 2>&1
      echo "== lrf_tests rc=$?" | tee -a $O/steps.log ;;
    lccache)  # configs[2]'s cluster apply: row loads with default policy (the 134 MB panel stays in
              # the MALL) vs non-temporal, interleaved three times
      for rep in 1 2 3; do
        for c in 1 0; do
          step lcc${c}_rbf_r$rep 300 env MLFF_LC_CACHED=$c python bench.py --no-cpu --no-solve --steps 100 --warmup 10
        done
      done ;;
    lcfin)  # k_lr_fin's waves per workgroup for configs[2]'s Q = 25 cluster partials
      for rep in 1 2; do
        for w in 16 8 4; do
          step lcfin${w}_rbf_r$rep 300 env MLFF_LR_FIN_WAVES=$w python bench.py --no-cpu --no-solve --steps 100 --warmup 10
        done
      done ;;
    redlanes)  # configs[2]'s slot reduction with two lanes per row vs one, interleaved
      for rep in 1 2; do
        for l in 2 1; do
          step red${l}_rbf_r$rep 300 env MLFF_SYM_REDUCE_LANES=$l python bench.py --no-cpu --no-solve --steps 100 --warmup 10
        done
      done ;;
    pmccopy)  # the table just collected, for the bench lines of this same call
      cp $O/pmc_head/pmc_traffic.json profiles/pmc_traffic.json ;;
    bigprof)  # kernel stats of the large published points at HEAD (the 7-row-wave cluster apply)
      step prof_nt141 600 rocprofv3 --kernel-trace --stats -d $O/prof_nt141 -o nt141 --output-format csv -- python3 bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
      step prof_eth5833 600 rocprofv3 --kernel-trace --stats -d $O/prof_eth5833 -o eth --output-format csv -- python3 bench.py --workload ethanol --m 5833 --no-cpu --no-solve --steps 30 --warmup 3 ;;
    rpw)  # rows per workgroup of the one-pass apply (fewer partial vectors vs fewer CUs streaming)
      for rep in 1 2; do
        for r in 1 7 10; do
          step rpw${r}_eth583_r$rep 300 env MLFF_LR_MIN_RPW=$r python bench.py --workload ethanol --m 583 --no-cpu --steps 200 --warmup 20 --no-solve
        done
        for r in 1 14; do
          step rpw${r}_nt_r$rep 300 env MLFF_LR_MIN_RPW=$r python bench.py --workload nanotube --no-cpu --steps 200 --warmup 20 --no-solve
        done
      done ;;
    diageth) step diageth 900 python -u scripts/dev/diag_ethanol_refine.py ;;
    calib)  # FETCH_SIZE calibration of k_rec_g's access widths (scripts/dev/pmc_calib.hip)
      step calib_build 120 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/dev/pmc_calib.hip -o $O/pmc_calib
      step calib_fetch 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib -o calib --output-format csv -- $O/pmc_calib ;;
    ethsolve)  # ethanol N = 15741 solve to 1e-6 with the Woodbury panel in two CholeskyQR steps and in one
      step ethsolve_refine 300 python bench.py --workload ethanol --m 583 --no-cpu --steps 10 --warmup 2 --solve-maxiter 80000
      step ethsolve_onestep 300 env MLFF_WB_REFINE=0 python bench.py --workload ethanol --m 583 --no-cpu --steps 10 --warmup 2 --solve-maxiter 80000 ;;
    lcrr)  # cluster apply: held row (D = 2) vs re-read row (D = 4 / 6 / 8), interleaved, at the
           # reference's large published points (ethanol N = 74979 / 157491, nanotube N = 156510)
      for rep in 1 2; do
        for D in 0 4 6 8; do
          step lcrr_eth5833_D${D}_r$rep 300 env MLFF_LC_REREAD=$D $EB --m 5833 --storage matfree --steps 20
          step lcrr_eth2777_D${D}_r$rep 300 env MLFF_LC_REREAD=$D $EB --m 2777 --storage matfree --steps 20
          step lcrr_nt141_D${D}_r$rep 300 env MLFF_LC_REREAD=$D python bench.py --workload nanotube --m 141 --no-cpu --no-solve --steps 20 --warmup 3
        done
      done ;;
    nysref)  # configs[2] band tests with the Nystrom panel re-orthogonalised and without
      step nysref_on 900 env MLFF_NYS_REFINE=1 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_rbf_band.py -k "in_band or scaled"
      step nysref_off 900 env MLFF_NYS_REFINE=0 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_rbf_band.py -k "in_band or scaled" ;;
    syevfast)  # the Nystrom build with the shifted-Cholesky-first cho_factor_stable (default) and without
      step syev_fast 600 python scripts/bench_syev.py
      step syev_nofast 900 env MLFF_CHO_FAST=0 python scripts/bench_syev.py ;;
    soloxr)  # SOLO floors: every fusion / the x, r fold off / the p fold off, interleaved twice
      for rep in 1 2; do
        for W in 8 4; do
          step solo_w${W}_r$rep 300 python bench.py --solo-world $W --n 65536 --steps 40 --warmup 5
          step solo_w${W}_noxr_r$rep 300 env MLFF_FUSE_XR=0 python bench.py --solo-world $W --n 65536 --steps 40 --warmup 5
          step solo_w${W}_nop_r$rep 300 env MLFF_FUSE_P=0 python bench.py --solo-world $W --n 65536 --steps 40 --warmup 5
        done
      done ;;
    soloprof)  # kernel trace of the W = 8 SOLO iteration (per-kernel times and the gaps between them)
      step soloprof 300 rocprofv3 --kernel-trace --stats -d $O/soloprof -o solo --output-format csv -- python3 bench.py --solo-world 8 --n 65536 --steps 40 --warmup 5 ;;
    rehearse)  # the multi-rank bench flow on one GPU (torchrun, SOLO ranks over gloo): not RCCL
      step rehearse_w8 400 env MLFF_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29508 \
        bench.py --gpus 8 --steps 10 --warmup 2 --no-solve ;;
    ptprof) step ptprof 600 rocprofv3 --kernel-trace --stats -d $O/ptprof -o eth --output-format csv -- python3 bench.py --workload ethanol --m 5833 --no-cpu --no-solve --steps 30 --warmup 3 --storage matfree ;;
    syev)
      step syev_blocked 600 env MLFF_SYEV_BLOCKED=1 python scripts/bench_syev.py
      step syev_unblocked 900 env MLFF_SYEV_BLOCKED=0 python scripts/bench_syev.py
      step syev_prof 900 rocprofv3 --kernel-trace --stats -d $O/syev -o syev --output-format csv -- python3 scripts/bench_syev.py ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py ;;
    pmc) step pmc 900 python scripts/pmc_head.py --out $O/pmc_head ;;
    parity)  # the drop-in on every golden solve, Woodbury panel in two CholeskyQR steps (default) and in one
      step parity_refine 600 python scripts/parity_report.py
      step parity_onestep 600 env MLFF_WB_REFINE=0 python scripts/parity_report.py ;;
    pmcrg)  # nanotube operator traffic with one 16-point group per pair block (each Rdd block read
            # by one workgroup) against the default two 8-point groups
      step pmc_rg16 600 env MLFF_REC_RG=16 python scripts/pmc_head.py --out $O/pmc_rg16 --workloads nanotube
      step pmc_rg8 600 python scripts/pmc_head.py --out $O/pmc_rg8 --workloads nanotube ;;
  esac
done
echo "== all done $(date +%T)" | tee -a $O/steps.log
