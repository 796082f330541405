"""bench.py — PCG iterations/s on the north-star workload (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 65536] [--k 256]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

With --gpus N > 1 and no WORLD_SIZE in the environment (the plain first form), the script
launches its own N ranks: the parent process -- before it imports the library or touches a
GPU -- starts N fresh `python bench.py` children with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT set (one per GPU, rank r on device r), waits for all of
them, stops the rest when one fails and exits with the first failing child's status; rank 0
prints the JSON line to the shared stdout.  Under torchrun (WORLD_SIZE set) it is one rank.

Workload: synthetic SPD RBF kernel, x ~ U[0,1)^3 (numpy default_rng seed 0), length
scale 0.2, A = K + 1e-6 I, b = sum(x^2), rank-256 Nystrom preconditioner on uniform
random columns (`random_scores`, seed 0):
  value:         N = 65536 (BASELINE.json configs[2]) on every
                 --gpus N, so the driver's value_N / value_1 is the strong scaling of ONE
                 problem (the north star's "N=64k 1-GPU ... >=6x strong scaling at 8 GPUs")
  configs3_leg:  N = 131072 (configs[3], "row-sharded mat-vec + RCCL, 8 x MI355X") timed
                 the same way on the same ranks, at N = 1 as well (68.7 GB of tiles fit one
                 GPU), so configs[3]'s own 1 -> 8 GPU speed-up is the ratio
                 of this leg's values across the BENCH / SCALE lines (--configs3-n 0 skips)
K is generated on the GPU straight into the symmetric tiles from the points (inputs
resident in HBM before the timed region; no dense N x N copy).  A step = one PCG
iteration (the fp64 mat-vec over the whole N x N matrix + preconditioner apply + CG
updates); with several GPUs the rows are sharded and the iteration runs three RCCL
collectives (allgather of z, reduce-scatter of the partial K p, allreduce of ||r||^2 | T r).

Prints the JSON line (rank 0) with the driver's keys -- once right after the configs[2] leg,
and once more, identical plus `configs3_leg`, after the configs[3] leg (the last line is the
complete one) -- with
  roofline:     algorithmic bytes/launch of the K mat-vec / its mean HIP-event
                duration, against 8 TB/s; traffic from profiles/ (PMC) or null.  With
                the symmetric tiled storage (default) the bytes are the stored lower
                block triangle (8 * tiles * 512^2 + 16 N_local, ~4 N^2);
                matvec_gbs_dense_equivalent restates the rate against 8 N^2
  cpu_baseline: the NumPy/SciPy oracle (oracle/, a port of the reference's CPU
                path) timed on this host on a bounded number of PCG iterations
                of the same matrix (rank 0, N = 1 only)
  parity:       iterations to relres 1e-6 on GPU vs the CPU oracle on an N = 8192
                instance of the same generator (rank 0, N = 1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]

import numpy as np  # noqa: E402

METRIC = "CG iters/sec + GB/s on N×N fp64 kernel mat-vec; iters-to-1e-6 vs CPU ref"
# MLFF_BENCH_REHEARSE=1 with several ranks: the multi-rank bench flow on ONE GPU (SOLO library
# ranks, gloo) -- checks the script's distributed logic; its numbers are not a measurement
REHEARSE = os.environ.get("MLFF_BENCH_REHEARSE", "0") == "1"
# the reference's published seconds per PCG step for the nanotube
# (its matrix-free PyTorch operator on NVIDIA GPUs): N = 15540 (configs[1], 0.105 s,
# data/data/cg_performance_n=15750/...nanotube_points14_meas31), N ~ 157k (2.073 s on an
# A100-PCIe 40 GB, data/data/rule_of_thumb/n = 157500) and N ~ 505k (6.600 s on a Quadro RTX
# 6000, data/data/rule_of_thumb/n = 500000); here M = 14 / 141 / 455 training geometries
REF_STEP_S = {15540: 0.105, 156510: 2.073, 505050: 6.600}
# and for ethanol (few atoms, many points): N = 15741 (M = 583, 0.130 s,
# data/data/cg_performance_n=15750/2022-03-17_2333_ethanol_points583_meas31), N = 74979 (M = 2777,
# 0.238 s, Quadro RTX 6000, data/data/rule_of_thumb/n = 75000/...ethanol_min2777_max2777) and
# N = 157491 (M = 5833, 0.550 s, A100-PCIe, data/data/rule_of_thumb/n = 157500/...ethanol_min5833)
REF_STEP_S_ETHANOL = {15741: 0.130, 74979: 0.238, 157491: 0.550}
# fp64 vector peak of the MI355X (AMD spec: 78.6 TFLOP/s, half the 157.3 TFLOP/s fp32 vector rate
# of MI355X_MICROARCH.md's chip table): the bound of the pair-tile sGDML operator
FP64_VALU_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# timed region: HIP-event brackets on every TIMING_EVERY-th PCG iteration only
TIMING_EVERY = int(os.environ.get("MLFF_BENCH_TIMING_EVERY", "8"))


def timing_every(steps: int) -> int:
    """Bracket period for a timed region of `steps` iterations: TIMING_EVERY, shortened so
    that at least 4 of the steps (or all of a shorter run) are bracketed."""
    return max(1, min(TIMING_EVERY, steps // 4))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=None,
                    help="kernel size of `value` (default 65536 = configs[2], on any number "
                         "of GPUs)")
    ap.add_argument("--k", type=int, default=None,
                    help="preconditioner rank (rbf: 256; sGDML: the rule of thumb, e.g. 2701 "
                         "for the nanotube; configs[4] uses 1024)")
    ap.add_argument("--configs3-n", type=int, default=131072,
                    help="rbf workload: also time this size (configs[3], N = 131072) on the "
                         "same ranks (configs3_leg); 0 skips it")
    ap.add_argument("--lam", type=float, default=1e-6)
    ap.add_argument("--ell", type=float, default=0.2)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-solve", action="store_true", help="skip the solve-to-1e-6 legs")
    ap.add_argument("--cpu-iters", type=int, default=30,
                    help="PCG iterations per CPU-baseline sample (3 samples, median; ~5 s each "
                         "at N=65536 on 16 cores)")
    ap.add_argument("--cpu-iters-sgdml", type=int, default=20,
                    help="PCG iterations of the CPU baseline of the sGDML workloads (~0.45 s each "
                         "at the nanotube size)")
    ap.add_argument("--cpu-iters-1t", type=int, default=2,
                    help="PCG iterations per single-thread CPU-baseline sample (3 samples)")
    ap.add_argument("--workload", choices=["rbf", "nanotube", "ethanol"], default="rbf",
                    help="rbf: configs[2] (default); nanotube: configs[1] (sGDML N=15540, "
                         "pivoted Cholesky k=2701 built on the GPU); ethanol: configs[0] geometry")
    ap.add_argument("--m", type=int, default=0, help="training points (sGDML workloads)")
    ap.add_argument("--solve-maxiter", type=int, default=20000)
    ap.add_argument("--solo-world", type=int, default=0,
                    help="profiling: run ONE rank (--solo-rank) of a W-way row split alone on "
                         "this GPU, collectives skipped (per-rank compute of the sharded "
                         "iteration; not a bench line)")
    ap.add_argument("--solo-rank", type=int, default=0)
    ap.add_argument("--storage", choices=["auto", "sym", "dense", "matfree"], default="auto",
                    help="operator storage: symmetric 512x512 tiles of the lower block "
                         "triangle (auto/sym, ~4 N^2 bytes), dense rows (8 N^2 bytes) or the "
                         "matrix-free sGDML operator; for the sGDML workloads sym / dense "
                         "assemble K on the GPU first (its time in setup_s)")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="--gpus N > 1 without WORLD_SIZE: seconds the self-launched ranks may "
                         "take before they are stopped (exit 124)")
    ap.add_argument("--desc", choices=["host", "gpu"], default="host",
                    help="sGDML descriptors on the host as the reference's trainer forms them "
                         "(default) or on the device")
    ap.add_argument("--mf-form", choices=["pt", "rec", "pair"], default=None,
                    help="matrix-free sGDML operator form (MLFF_MF_FORM): pair-tile (few atoms), "
                         "record-factored (many atoms) or pair sums; default: the library's "
                         "choice")
    return ap.parse_args()


def free_port() -> int:
    """A TCP port on 127.0.0.1 that nothing listens on now (the rendezvous port)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_plan(argv, n: int, port: int, base_env) -> list:
    """(command, environment) of each of the n rank processes the plain `bench.py --gpus n`
    launches: the same script and arguments, rank r on local device r, the torchrun variables
    (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT)."""
    plans = []
    for r in range(n):
        env = dict(base_env)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plans.append(([sys.executable, "-u", str(Path(__file__).resolve()), *argv], env))
    return plans


def launch_ranks(plans, timeout: float, poll: float = 0.2) -> int:
    """Start every planned rank as a child process (never exec: this process stays the parent),
    wait for all of them; when one exits non-zero, or the timeout passes, stop the others
    (SIGTERM, then SIGKILL after 10 s) and return that status (124 on the timeout), else 0.
    The children share this process's stdout / stderr, so rank 0's JSON line is the
    script's output."""
    procs = []
    stopping = {"sig": None}

    def on_signal(sig, _frame):
        stopping["sig"] = sig

    old = {s_: signal.signal(s_, on_signal) for s_ in (signal.SIGTERM, signal.SIGINT)}
    try:
        for cmd, env in plans:
            procs.append(subprocess.Popen(cmd, env=env))
        deadline = time.monotonic() + timeout
        rc = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                return 0
            if stopping["sig"] is not None:
                rc = 128 + int(stopping["sig"])
                break
            if time.monotonic() > deadline:
                print(f"bench.py: ranks still running after {timeout:.0f} s: stopping them",
                      file=sys.stderr)
                rc = 124
                break
            time.sleep(poll)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.monotonic() + 10.0
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if rc < 0:  # a child killed by a signal: the shell's convention
            rc = 128 - rc
        return rc
    finally:
        for s_, h in old.items():
            signal.signal(s_, h)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if REHEARSE:
            # one-GPU rehearsal of the multi-rank bench flow: every rank is a SOLO rank of
            # the library on device 0 (no data exchange), torch.distributed over gloo
            dist.init_process_group(backend="gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl")
        pg = dist
    return rank, world, local, pg


def barrier(pg, solver):
    solver.synchronize()
    if pg is not None:
        import torch

        torch.cuda.synchronize()
        pg.barrier()  # gloo in a rehearsal


def max_over_ranks(pg, v: float) -> float:
    if pg is None:
        return v
    import torch

    t = torch.tensor([v], dtype=torch.float64, device="cpu" if REHEARSE else "cuda")
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def iteration_bytes(op_bytes: float, precon_bytes: float, nloc: int) -> float:
    """Algorithmic HBM bytes of one PCG iteration on a rank: the operator application in the
    storage and form that ran, the low-rank apply in the form that ran (its r in / z out
    included: mlff_precon_apply_traffic), and the other CG vector streams -- rho / p.q / ||r||
    reads, the p, x and r updates -- 7 N-vectors of 8 bytes (SURVEY 8(d)'s 80 N per iteration
    counts the apply's r, z streams too)."""
    return op_bytes + precon_bytes + 56.0 * nloc


def make_solver(n, rank, world, local, pg):
    import sgdml_amd

    comm_id = None
    if world > 1 and REHEARSE:
        return sgdml_amd.KernelSolver(n, device=0, rank=rank, world=world, comm_id=b"SOLO:")
    if world > 1:
        obj = [sgdml_amd.comm_unique_id() if rank == 0 else None]
        pg.broadcast_object_list(obj, src=0)
        comm_id = obj[0]
    return sgdml_amd.KernelSolver(n, device=local, rank=rank, world=world, comm_id=comm_id)


def csrc_hash() -> str:
    """Content hash of the library sources (csrc/ and include/): PMC traffic figures are
    only valid for the code they were collected on (build_native.src_hash, which the build
    also compiles into the library as mlff_build_hash)."""
    import build_native

    return build_native.src_hash()


def library_hash() -> str | None:
    """The source hash compiled into the loaded libmlffpcg.so (None if it cannot be read)."""
    try:
        from sgdml_amd import _native

        return _native.build_hash()
    except Exception:  # noqa: BLE001
        return None


def pmc_traffic(key: str):
    """(HBM bytes per launch from profiles/pmc_traffic.json, None) when the entry was collected
    on the current sources (scripts/pmc_head.py stamps csrc_sha), else (None, reason)."""
    p = REPO / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None, "no profiles/pmc_traffic.json"
    try:
        e = json.loads(p.read_text()).get(key)
    except Exception as ex:  # noqa: BLE001
        return None, f"unreadable profiles/pmc_traffic.json: {ex!r}"
    if e is None:
        return None, f"no PMC entry for {key}"
    sha = csrc_hash()
    lib_sha = library_hash()
    if lib_sha != sha:
        print(f"warning: libmlffpcg.so was built from sources {lib_sha}, the tree is {sha}: "
              f"PMC traffic refused", file=sys.stderr)
        return None, (f"binary/source mismatch: the loaded library was built from {lib_sha}, "
                      f"these sources are {sha} (rebuild with build_native.py)")
    if e.get("csrc_sha") != sha:
        return None, (f"stale: PMC entry {key} was collected on sources {e.get('csrc_sha')}, "
                      f"these are {sha} (scripts/pmc_head.py re-collects)")
    return float(e["hbm_bytes_per_launch"]), None


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cores() -> dict:
    """Physical cores this process may use: the CPU affinity set (sched_getaffinity) in
    whole cores, capped by the cgroup CPU quota (cpu.max) -- the GPU box allots a CPU
    share per GPU, and BLAS threads beyond it only time-slice."""
    aff = len(os.sched_getaffinity(0))
    tpc = 1
    try:
        sib = open("/sys/devices/system/cpu/cpu0/topology/thread_siblings_list").read().strip()
        tpc = sum((int(b) - int(a) + 1) if "-" in x else 1
                  for x in sib.split(",") for a, b in [((x.split("-") + [x])[:2])])
    except (OSError, ValueError):
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    cores = max(1, aff // max(tpc, 1))
    if quota is not None:
        cores = max(1, min(cores, int(quota)))
    return {"cores": cores, "affinity_cpus": aff, "threads_per_core": tpc,
            "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count()}


def _median_rate(fn, samples=3):
    """fn() -> seconds per iteration; median over `samples` runs (and the spread)."""
    per = sorted(fn() for _ in range(samples))
    return per[len(per) // 2], per


def _time_pcg(mv, psolve, b, m):
    """Seconds per oracle PCG iteration (after one warm-up iteration) and per mat-vec."""
    from oracle.pcg import cg_legacy

    cg_legacy(mv, b, tol=0.0, maxiter=1, psolve=psolve)
    t0 = time.perf_counter()
    cg_legacy(mv, b, tol=0.0, maxiter=m, psolve=psolve)
    el = time.perf_counter() - t0
    # cg_legacy spends one extra mat-vec on the legacy ||A x0 - b|| check
    t_mv = time.perf_counter()
    mv(b)
    t_mv = time.perf_counter() - t_mv
    return max(el - t_mv, 1e-9) / m, t_mv


def cpu_baseline_sgdml(solver, Rd, Rdd, perms, b, lam, iters):
    """The reference's CPU iteration for the sGDML workloads, restated by the oracle: its
    matrix-free K_op (GDMLPredict with alphas = v, predict.py:72-234) and the Woodbury
    apply (iterative_cholesky.py:145-148).  The rank-k panel is the one the GPU built
    (the oracle's own pivoted Cholesky would need k CPU operator applications, ~0.4 s
    each at the nanotube size); the timed sample is the per-iteration work only."""
    import threadpoolctl

    from oracle.precon import apply_panel
    from oracle.sgdml import kernel_matvec_matrix_free

    T = solver.precon_panel()
    cpus = usable_cores()

    def mv(v):
        return -kernel_matvec_matrix_free(Rd, Rdd, perms, 10.0, v) + lam * v

    psolve = lambda r: apply_panel(T, 1.0, lam, r)  # noqa: E731
    with threadpoolctl.threadpool_limits(limits=cpus["cores"], user_api="blas"):
        # a bounded sample (~10 s per timed run): the many-point operator is O(M^2) on the host
        t0 = time.perf_counter()
        mv(b)
        psolve(b)
        one = time.perf_counter() - t0
        iters = max(1, min(iters, int(10.0 / max(one, 1e-6))))
        per_it, spread = _median_rate(lambda: _time_pcg(mv, psolve, b, iters)[0])
        t_mv = _time_pcg(mv, psolve, b, 1)[1]
    return dict({"value": 1.0 / per_it, "unit": "CG iters/s", "cores": cpus["cores"], "kind": "port",
                 "sample": f"median of 3 x {iters} PCG iterations (oracle cg_legacy + matrix-free "
                           f"sGDML K_op + Woodbury apply of the GPU-built rank-{T.shape[0]} panel, "
                           f"NumPy) at N={b.size}",
                 "ms_per_iter": per_it * 1e3, "ms_per_iter_samples": [t * 1e3 for t in spread],
                 "matvec_ms": t_mv * 1e3, "host_cpu": _cpu_model()}, **cpus)


def cpu_baseline(solver, X, b, idx, lam, ell, iters, iters_1t):
    """Oracle PCG iterations (NumPy/SciPy port of the reference CPU path) on the same
    matrix, copied from the device; timed per iteration after one warm-up iteration,
    with all BLAS threads and (a shorter sample) with one thread."""
    import threadpoolctl

    from oracle.precon import apply_panel, nystrom_panel

    n = b.size
    K = solver.get_matrix_rows()
    B, sp = nystrom_panel(K[:, idx], idx, lam, 0)
    cpus = usable_cores()

    def mv(v):
        y = K @ v
        y += lam * v
        return y

    psolve = lambda r: apply_panel(B, sp, lam, r)  # noqa: E731
    with threadpoolctl.threadpool_limits(limits=cpus["cores"], user_api="blas"):
        per_it, spread = _median_rate(lambda: _time_pcg(mv, psolve, b, iters)[0])
        t_mv = _time_pcg(mv, psolve, b, 1)[1]
    one = None
    if iters_1t > 0:
        with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
            p1, s1 = _median_rate(lambda: _time_pcg(mv, psolve, b, iters_1t)[0])
        one = {"value": 1.0 / p1, "cores": 1, "ms_per_iter": p1 * 1e3,
               "ms_per_iter_samples": [t * 1e3 for t in s1],
               "sample": f"median of 3 x {iters_1t} PCG iterations"}
    del K
    return dict({"value": 1.0 / per_it, "unit": "CG iters/s", "cores": cpus["cores"], "kind": "port",
                 "sample": f"median of 3 x {iters} PCG iterations (oracle cg_legacy + Nystrom "
                           f"apply, NumPy/OpenBLAS) on the same N={n} fp64 matrix copied from "
                           f"the GPU",
                 "ms_per_iter": per_it * 1e3, "ms_per_iter_samples": [t * 1e3 for t in spread],
                 "matvec_gbs": (8.0 * n * n) / (t_mv * 1e9),
                 "host_cpu": _cpu_model(),
                 "single_thread": one}, **cpus)


def rbf_band():
    """The measured noise band of the configs[2] generator at N = 8192 (tests/golden/
    make_rbf_band.py: the CPU oracle in six summation orders) and the oracle's own solve of
    the full N = 65536 system (iterations to relres 1e-6), when committed."""
    g = REPO / "tests" / "golden"
    bd = json.loads((g / "rbf_band_n8192.json").read_text()) if (g / "rbf_band_n8192.json").exists() else None
    full = None
    if (g / "rbf_solve_n65536.npz").exists():
        f = np.load(g / "rbf_solve_n65536.npz", allow_pickle=False)
        full = {"iters": int(f["iters"]), "info": int(f["info"]),
                "final_true_relres": float(f["final_relres"]), "x_norm": float(f["x_norm"]),
                "cpu_seconds": float(f["seconds"]), "_x": f["x"]}
        if (g / "rbf_solve_n65536_rev.npz").exists():  # a second summation order of the oracle
            fr = np.load(g / "rbf_solve_n65536_rev.npz", allow_pickle=False)
            full["second_order_iters"] = int(fr["iters"])
            full["second_order_rel_dx"] = float(np.linalg.norm(fr["x"] - f["x"]) /
                                                np.linalg.norm(f["x"]))
    return bd, full


def exact_anchor():
    """The configs[2] exact-sum anchor (tests/golden/rbf_dd_n65536.json) or None."""
    p = REPO / "tests" / "golden" / "rbf_dd_n65536.json"
    return json.loads(p.read_text()) if p.exists() else None


def anchor_tolerance(anchor) -> int:
    """Iterations an fp64 configs[2] solve may land from the exact-sum count: the largest
    distance fp64 orders were measured to land from the near-exact count at N = 8192 / 16384 (as
    a fraction of the count), or the largest distance of the oracle's own committed orders at
    N = 65536, whichever is larger, + 2 (the band contains every oracle order)."""
    frac = max(anchor["fp64_distance_fraction"].values())
    oracle = max(abs(v - anchor["iters"]) for v in anchor["oracle_fp64_iters"].values())
    return max(int(np.ceil(frac * anchor["iters"])), oracle) + 2


SGDML_FIXTURES = {("nanotube", 15540): "nanotube_n15540", ("ethanol", 15741): "ethanol_n15741",
                  ("ethanol", 74979): "ethanol_n74979"}


def first_below(trace, tol) -> int | None:
    """First iteration j >= 1 whose stop-test residual is <= tol * ||r_0|| (x0 = 0: ||b||)."""
    tr = np.asarray(trace)
    hit = np.nonzero(tr[1:] <= tol * tr[0])[0]
    return int(hit[0]) + 1 if hit.size else None


def sgdml_parity(workload, n, k, res):
    """The sGDML solve against the CPU oracle's run of the same system at full size, when one is
    committed (make_nanotube_full.py / make_ethanol_full.py): iterations to tol 1e-6 and (where
    recorded) 1e-4 -- the reference's training tolerance, train.py:309 -- held to the band the
    oracle measured over its own summation orders (|d it| <= 2 b_it + 2, tests/parity.py)."""
    name = SGDML_FIXTURES.get((workload, n))
    g = REPO / "tests" / "golden"
    if name is None or not (g / f"{name}_band.json").exists():
        return None
    fx = json.loads((g / f"{name}_band.json").read_text())
    out = {"source": f"tests/golden/{name}_band.json"}
    if "bands" in fx:
        # the default (one-step, the reference's formula) Woodbury panel against the oracle's
        # one-step solves; the re-orthogonalised panel (MLFF_WB_REFINE=1) against its accurate ones
        refined = os.environ.get("MLFF_WB_REFINE", "0") != "0"
        out["panel"] = "refined (accurate band)" if refined else "one-step (LAPACK band)"
        cases = {}
        for t in (1e-4, 1e-6):
            b = fx["bands"].get(f"k{k}_tol{t:g}")
            cases[t] = (b.get("accurate") if refined else b) if b is not None else None
    else:  # the nanotube fixture: one rank, tol 1e-6 (LAPACK one-step band; "accurate" beside it)
        cases = {1e-6: fx if fx.get("k") == k else None}
        if fx.get("k") == k and "accurate" in fx:
            b = fx["accurate"]
            it = first_below(res.trace, 1e-6)
            out["accurate_panels"] = {
                "gpu_iters": it, "cpu_ref_iters": b["ref_iters"], "band_iters": b["band_iters"],
                "in_band": bool(it is not None and abs(it - b["ref_iters"]) <= 2 * b["band_iters"] + 2)}
    ok = True
    for tol, b in cases.items():
        if b is None:
            continue
        it = first_below(res.trace, tol)
        e = {"gpu_iters": it, "cpu_ref_iters": b["ref_iters"], "band_iters": b["band_iters"],
             "oracle_orders": {o: v["iters"] for o, v in b["variants"].items()}}
        e["in_band"] = bool(it is not None and abs(it - b["ref_iters"]) <= 2 * b["band_iters"] + 2)
        ok = ok and e["in_band"]
        out[f"tol_{tol:g}"] = e
    out["in_band"] = ok
    return out


def parity_small(n, k, lam, ell, tol=1e-6):
    """Same generator at N = 8192: GPU vs CPU-oracle iterations to relres 1e-6, with the
    measured noise band of that count (|d iters| <= 2 b_it + 2 is in band, tests/parity.py)."""
    import sgdml_amd
    from sgdml_amd import synthetic

    from oracle.pcg import cg_legacy
    from oracle.precon import apply_panel, nystrom_panel
    from oracle.rbf import rbf_kernel

    X, b = synthetic.rbf_points(n, 3, 0)
    idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False))
    with sgdml_amd.KernelSolver(n) as s:
        s.gen_rbf(X, ell)
        s.set_operator(1.0, lam)
        s.precon_nystrom(idx)
        r = s.pcg(b, tol=tol, maxiter=min(5 * n, 10000))
    K = rbf_kernel(X, ell)
    B, sp = nystrom_panel(K[:, idx], idx, lam, 0)
    x, info, tr, it = cg_legacy(lambda v: K @ v + lam * v, b, tol=tol, maxiter=min(5 * n, 10000),
                                psolve=lambda v: apply_panel(B, sp, lam, v))
    out = {"n": n, "k": k, "tol": tol, "gpu_iters": int(r.iters), "cpu_iters": int(it),
           "gpu_info": int(r.info), "cpu_info": int(info),
           "rel_dx": float(np.linalg.norm(r.x - x) / np.linalg.norm(x))}
    bd, _ = rbf_band()
    if bd is not None and bd["n"] == n and bd["k"] == k and bd["lam"] == lam and bd["ell"] == ell:
        out["band"] = {"b_iters": bd["band_iters"], "b_rel_dx": bd["band_rel_dx"],
                       "oracle_orders": {o: v["iters"] for o, v in bd["variants"].items()},
                       "source": "tests/golden/rbf_band_n8192.json"}
        ld = REPO / "tests" / "golden" / f"rbf_ld_n{n}.json"
        if ld.exists():  # the oracle with extended-precision sums: the exact-arithmetic proxy
            out["band"]["extended_precision_iters"] = json.loads(ld.read_text())["iters"]
        out["in_band"] = bool(abs(r.iters - it) <= 2 * bd["band_iters"] + 2
                              and out["rel_dx"] <= 10 * bd["band_rel_dx"])
    return out


def sgdml_workload(args, rank, world, local, pg):
    """configs[0]/[1]: synthetic ethanol / nanotube sGDML kernel assembled on the GPU."""
    import sgdml_amd
    from sgdml_amd import synthetic
    from sgdml_amd.rule_of_thumb import get_params, rule_of_thumb

    if args.workload == "nanotube":
        M = args.m or 14
        ds = synthetic.nanotube_like(M, seed=0)
        name = "nanotube"
    else:
        M = args.m or 111
        # energy-consistent labels (F = -grad E of a pair-harmonic potential): random force
        # labels put relres 1e-6 at the system's attainable-accuracy floor
        ds = synthetic.ethanol_harmonic(M, seed=0)
        name = "ethanol"
    n_atoms = ds["R"].shape[1]
    n = 3 * n_atoms * M
    m, kmin, _ = get_params(name)
    k = args.k if args.k else int(rule_of_thumb(n=n, k_min=kmin, m=m))
    y, _ = synthetic.labels(ds["F"])
    if args.mf_form:
        os.environ["MLFF_MF_FORM"] = args.mf_form
    t0 = time.perf_counter()
    # descriptors as the reference's trainer forms them (host Desc.from_R): the exact system of
    # the oracle fixtures at their sizes; --desc gpu forms them on the device (equal to rounding)
    Rd, Rdd = (sgdml_amd.sgdml_descriptors(ds["R"]) if args.desc == "gpu"
               else sgdml_amd.host_descriptors(ds["R"]))
    solver = make_solver(n, rank, world, local, pg)
    if args.storage in ("sym", "dense"):
        # the stored-K forms of the same operator: K assembled on the GPU (train.py:1121-1308)
        solver.assemble_sgdml(Rd, Rdd, np.arange(n_atoms)[None, :], 10.0)
    else:
        # as the drop-in Iterative.solve: the matrix-free operator only (the reference's
        # K_op); the pivoted Cholesky fetches its columns through it (no N^2 assembly)
        solver.sgdml_operator(Rd, Rdd, np.arange(n_atoms)[None, :], 10.0)
    solver.set_operator(-1.0, 1e-10)
    solver.synchronize()
    t_asm = time.perf_counter() - t0
    _, t_chol = solver.precon_pivchol(k)
    # the first build includes one-time costs (code-object loads of its kernels, the scratch
    # arena's first chunks); a second, identical build shows the steady-state cost (skipped
    # where the build itself takes seconds)
    t_warm = solver.precon_pivchol(k)[1] if t_chol < 1.0 else None
    return solver, n, k, y, {"operator_setup_s": t_asm, "pivchol_build_s": t_chol,
                             "pivchol_build_warm_s": t_warm,
                             "assembled": args.storage in ("sym", "dense"),
                             "workload": f"sgdml_{name}_n{n}_pivchol{k}", "M": M,
                             "n_atoms": n_atoms, "desc": (Rd, Rdd),
                             "perms": np.arange(n_atoms)[None, :]}


def precon_rbf(solver, idx) -> float:
    """Rank-k Nystrom build (random_scores) of the rbf workloads; in a rehearsal (SOLO ranks
    exchange nothing, so the Nystrom Gram matrices would be partial) a random panel of the
    same shape stands in."""
    if REHEARSE and solver.world > 1:
        r0, r1 = solver.row_range()
        solver.precon_lowrank(np.random.default_rng(solver.rank).standard_normal(
            (idx.size, r1 - r0)) * 1e-3)
        return 0.0
    return solver.precon_nystrom(idx, variant=0)


def all_ok(pg, ok: bool) -> bool:
    """True when every rank reports ok: a collective verdict before any step that would make a
    rank wait in a barrier or a collective for a peer that has already failed."""
    if pg is None:
        return ok
    import torch

    t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64,
                     device="cpu" if REHEARSE else "cuda")
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item()) == 0.0


def size_leg(args, rank, world, local, pg, n, k, lam, ell):
    """Iterations/s of the rbf workload at size n on all ranks (same generator, Nystrom rank,
    storage and timing as the main leg; no solve, no CPU leg): configs[3] (n = 131072) next
    to the configs[2] `value`, so each bench line carries both problems' numbers.  Failures
    are agreed on collectively between the phases, so every rank skips the rest together."""
    from sgdml_amd import synthetic

    X, b = synthetic.rbf_points(n, 3, 0)
    idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False))
    s, err = None, None
    try:
        s = make_solver(n, rank, world, local, pg)
        s.gen_rbf(X, ell)
        s.set_operator(1.0, lam)
    except Exception as e:  # noqa: BLE001 -- reported in the line
        err = e
    if not all_ok(pg, err is None):
        if s is not None:
            s.close()
        return {"n": n, "value": None, "error": repr(err) if err else "failed on another rank"}
    try:
        try:
            precon_rbf(s, idx)
            s.set_storage(args.storage)
            _, op_bytes = s.storage_info()
        except Exception as e:  # noqa: BLE001
            err = e
        if not all_ok(pg, err is None):
            return {"n": n, "value": None,
                    "error": repr(err) if err else "failed on another rank"}
        r0, r1 = s.row_range()
        s.pcg_start(np.ascontiguousarray(b[r0:r1]), tol=0.0,
                    maxiter=args.warmup + args.steps + 1)
        if args.warmup:
            s.pcg_run(args.warmup, args.warmup)
        s.timing(timing_every(args.steps))
        s.timing_reset()
        barrier(pg, s)
        t0 = time.perf_counter()
        s.pcg_run(args.steps, args.steps)
        barrier(pg, s)
        el = max_over_ranks(pg, time.perf_counter() - t0)
        tm = s.timing_read()
        op_ms = max_over_ranks(pg, tm["gemv_ms"] / max(tm["gemv_count"], 1))
        return {"n": n, "k": k, "value": args.steps / el, "ms_per_step": el / args.steps * 1e3,
                "operator_ms_max_rank": op_ms,
                "operator_gbs_max_rank": op_bytes / (op_ms * 1e-3) / 1e9,
                "operator_bytes_rank": op_bytes,
                "rccl_ms_per_iter": max_over_ranks(pg, tm["comm_ms"] / max(tm["gemv_count"], 1))}
    finally:
        s.close()


def solo_profile(args):
    """One rank of a --solo-world W row split on one GPU with the library's SOLO transport
    (every collective keeps only this rank's contribution): the kernels, sizes and launch
    sequence of rank R's sharded PCG iteration without the RCCL calls.  The numbers it
    computes are meaningless; the per-iteration device time is the compute floor of the
    W-GPU iteration (add the three collectives' latency for the real one).  A random
    rank-k panel stands in for the Nystrom factor (its build needs the collectives)."""
    import sgdml_amd
    from sgdml_amd import synthetic

    W, R = args.solo_world, args.solo_rank
    n, k, ell = (args.n or 131072), (args.k or 256), args.ell
    X, b = synthetic.rbf_points(n, 3, 0)
    s = sgdml_amd.KernelSolver(n, device=0, rank=R, world=W, comm_id=b"SOLO:")
    try:
        s.gen_rbf(X, ell)
        s.set_operator(1.0, args.lam)
        r0, r1 = s.row_range()
        Lt = np.random.default_rng(R).standard_normal((k, r1 - r0)) * 1e-3
        s.precon_lowrank(Lt)
        s.set_storage(args.storage)
        storage, op_bytes = s.storage_info()
        s.pcg_start(np.ascontiguousarray(b[r0:r1]), tol=0.0,
                    maxiter=args.warmup + args.steps + 1)
        if args.warmup:
            s.pcg_run(args.warmup, args.warmup)
        s.timing(timing_every(args.steps))
        s.timing_reset()
        s.synchronize()
        t0 = time.perf_counter()
        s.pcg_run(args.steps, args.steps)
        s.synchronize()
        el = time.perf_counter() - t0
        tm = s.timing_read()
        op_ms = tm["gemv_ms"] / max(tm["gemv_count"], 1)
        print(json.dumps({
            "solo_profile": True, "world": W, "rank": R, "n": n, "k": k, "rows": r1 - r0,
            "storage": storage, "steps": args.steps, "ms_per_iter_wall": el / args.steps * 1e3,
            "iter_device_ms": tm["iter_ms"] / max(tm["iter_count"], 1),
            "operator_ms": op_ms, "operator_bytes": op_bytes,
            "operator_gbs": op_bytes / (op_ms * 1e-3) / 1e9,
            "note": "collectives skipped (SOLO transport): compute floor of one rank"}),
            flush=True)
    finally:
        s.close()


def main():
    args = parse()
    if args.solo_world > 1:
        return solo_profile(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # plain `bench.py --gpus N`: launch the N ranks here (nothing has touched a GPU yet)
        sys.exit(launch_ranks(spawn_plan(sys.argv[1:], args.gpus, free_port(), os.environ),
                              args.launch_timeout))
    rank, world, local, pg = dist_setup(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    import sgdml_amd
    from sgdml_amd import synthetic

    if args.n is None:
        args.n = 65536
    n, k, lam, ell = args.n, (args.k or 256), args.lam, args.ell
    sg_info = None
    if args.workload == "rbf":
        workload = f"rbf_n{n}_nystrom{k}"
        X, b = synthetic.rbf_points(n, 3, 0)
        idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False))
        solver = make_solver(n, rank, world, local, pg)
        t0 = time.perf_counter()
        solver.gen_rbf(X, ell)
        t_gen = time.perf_counter() - t0
        solver.set_operator(1.0, lam)
        t_pre = precon_rbf(solver, idx)
    else:
        solver, n, k, b, sg_info = sgdml_workload(args, rank, world, local, pg)
        workload, lam = sg_info["workload"], 1e-10
        t_gen, t_pre = sg_info["operator_setup_s"], sg_info["pivchol_build_s"]
    solver.set_storage(args.storage)
    t0 = time.perf_counter()
    storage, op_bytes = solver.storage_info()  # builds the symmetric tiles (setup)
    t_pack = time.perf_counter() - t0
    free_b, total_b = solver.device_memory()
    used_gb = max_over_ranks(pg, (total_b - free_b) / 1e9)
    r0, r1 = solver.row_range()
    b_loc = np.ascontiguousarray(b[r0:r1])
    # tol = 0: never converges, so exactly warmup + steps iterations run
    solver.pcg_start(b_loc, tol=0.0, maxiter=args.warmup + args.steps + 1)
    if args.warmup:
        solver.pcg_run(args.warmup, args.warmup)
    # HIP events on every TIMING_EVERY-th iteration of the timed region (each event costs
    # GPU time between the kernels it brackets; the per-kernel averages are over those)
    solver.timing(timing_every(args.steps))
    solver.timing_reset()
    barrier(pg, solver)
    t0 = time.perf_counter()
    solver.pcg_run(args.steps, args.steps)
    barrier(pg, solver)
    el = time.perf_counter() - t0
    el = max_over_ranks(pg, el)
    tm = solver.timing_read()
    gemv_ms = tm["gemv_ms"] / max(tm["gemv_count"], 1)
    iter_ms = tm["iter_ms"] / max(tm["iter_count"], 1)
    comm = None
    if world > 1:
        # HIP-event time of the RCCL collectives on this rank's stream (waits for the
        # slowest peer included): per iteration and per collective, max over ranks
        # the bracketed iterations are those with an operator bracket (gemv_count)
        comm = {"ms_per_iter": max_over_ranks(pg, tm["comm_ms"] / max(tm["gemv_count"], 1)),
                "collectives_per_iter": tm["comm_count"] / max(tm["gemv_count"], 1),
                "ms_per_collective": max_over_ranks(pg, tm["comm_ms"] / max(tm["comm_count"], 1)),
                "operator_ms_max_rank": max_over_ranks(pg, gemv_ms)}
    nloc = r1 - r0
    gemv_bytes = op_bytes  # algorithmic bytes of this rank's operator launch
    achieved = gemv_bytes / (gemv_ms * 1e-3) / 1e9
    dense_equiv = (8.0 * nloc * n + 16.0 * nloc) / (gemv_ms * 1e-3) / 1e9
    roof_op = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": achieved / HBM_PEAK_GBS,
               "traffic": None,
               "kernel": {"sym": "k_symv_dyn + k_sym_reduce (K mat-vec, lower-triangle tiles)",
                          "dense": "k_gemv<4,4,1> (K mat-vec, dense rows)",
                          "matfree": "k_rec_g + k_rec_fin (record-factored matrix-free sGDML "
                                     "operator; k_mf_* when the pair records exceed their cap)"}
               .get(storage, storage),
               "bytes_per_launch": gemv_bytes, "mean_launch_ms": gemv_ms}
    roof_op["traffic"], why = pmc_traffic(f"{workload}/{storage}/gpus{world}")
    if why:
        roof_op["traffic_note"] = why
    mf_form = solver.operator_form() if storage == "matfree" else None
    if mf_form == "pt":
        # the pair-tile operator is bound by the fp64 vector pipe: 9 D + 8 flops per (query
        # point, training point, permutation) -- diff (D), |diff|^2 and diff . Zt (2 x 2D),
        # F += c diff - w Zt (4D), nrm / m / w / c (8; sqrt and exp counted as one each)
        M_, D_ = sg_info["M"], sg_info["n_atoms"] * (sg_info["n_atoms"] - 1) // 2
        ni_ = -(-nloc // (3 * sg_info["n_atoms"]))
        flops = ni_ * M_ * sg_info["perms"].shape[0] * (9.0 * D_ + 8.0)
        tf = flops / (gemv_ms * 1e-3) / 1e12
        roof_op = dict(roof_op, bound="valu_fp64", achieved=tf, peak=FP64_VALU_PEAK_TFLOPS,
                       unit="TFLOP/s", frac=tf / FP64_VALU_PEAK_TFLOPS,
                       kernel="k_mf_z + k_pt_pair + k_pt_fin (pair-tile matrix-free sGDML operator)",
                       flops_per_launch=flops, hbm_gbs_algorithmic=achieved,
                       note="query points in registers, training points streamed through LDS; "
                            "bound by the fp64 vector pipe (78.6 TFLOP/s AMD spec), not by its "
                            "bytes (DESIGN.md 3.8)")
    elif storage == "matfree":
        roof_op["note"] = ("two dependent launches (Zt, G = sum w Zt and J^T G of a pair block in one "
                           "workgroup; the finisher): ~33 MB per application at M = 14, latency- "
                           "not HBM-bound (PMC traffic in profiles/pmc_traffic.json; DESIGN.md 3.2); "
                           "in the one-rank PCG iteration the two launches also form the search "
                           "direction p = z + beta p and the first one runs the previous "
                           "iteration's stop test (DESIGN.md 3.7), inside this time")
    # low-rank apply z = sigma_p (r - T^T T r) / lam.  Two-pass form: T (k x N_loc) read
    # twice + r, z (16 k N + 24 N).  One-pass form (one rank, rows in registers): T read once
    # + the row groups' partial vectors written and read (8 k N + 16 G N + 24 N); the
    # algorithmic bytes are those of the form that ran (the library reports them)
    roof_pre = None
    if tm.get("precon_count"):
        pre_ms = tm["precon_ms"] / tm["precon_count"]
        one_pass, pre_bytes = solver.precon_apply_traffic()
        pre_gbs = pre_bytes / (pre_ms * 1e-3) / 1e9
        two_pass_bytes = 16.0 * k * nloc + 24.0 * nloc
        roof_pre = {"bound": "hbm", "achieved": pre_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": pre_gbs / HBM_PEAK_GBS,
                    "traffic": None,
                    "kernel": {1: "k_lr_rows + k_lr_fin (one-pass low-rank apply: each panel "
                                  "row read once, t_i kept in its workgroup)",
                               2: "k_lr_cluster + k_lr_fin (one-pass low-rank apply: each panel "
                                  "row read once by a cluster of workgroups that hand their "
                                  "partial t_i to each other)"}.get(
                        one_pass, "k_gemv<4,2,0> + k_colgemv_part + k_precon_fin (low-rank apply)"),
                    "bytes_per_launch": pre_bytes, "mean_launch_ms": pre_ms,
                    "two_pass_equivalent_gbs": two_pass_bytes / (pre_ms * 1e-3) / 1e9}
        roof_pre["traffic"], why = pmc_traffic(f"{workload}/precon{one_pass}/{storage}/gpus{world}")
        if why:
            roof_pre["traffic_note"] = why
    per_iter_bytes = iteration_bytes(op_bytes, pre_bytes if roof_pre is not None else 0.0, nloc)
    # the roofline entry is the kernel group with the larger share of the iteration
    roof_dominant = roof_pre if roof_pre is not None and roof_pre["mean_launch_ms"] > gemv_ms \
        else roof_op

    solve = None
    if not args.no_solve:
        solver.timing_reset()
        t1 = time.perf_counter()
        res = solver.pcg(b_loc, tol=1e-6 if sg_info is None else 1e-6,
                         maxiter=min(5 * n, args.solve_maxiter))
        t_solve = max_over_ranks(pg, time.perf_counter() - t1)
        solve = {"tol": 1e-6, "iters": int(res.iters), "info": int(res.info),
                 "seconds": t_solve, "final_relres": float(res.resid / np.linalg.norm(b))}
        if sg_info is not None:
            solve["cpu_ref"] = sgdml_parity(args.workload, n, k, res)
        bd, full = rbf_band()
        if sg_info is None and n == 65536 and k == 256 and full is not None and bd is not None:
            # the CPU oracle's solve of this very system (committed fixture, ~2 h of CPU time:
            # make_rbf_band.py --full; a second summation order beside it)
            x_cpu = full.pop("_x")
            solve["cpu_ref"] = dict(full, source="tests/golden/rbf_solve_n65536.npz")
            anchor = exact_anchor()
            if anchor is not None:
                # the count with exact sums (double-double operator and apply, measured on the
                # GPU: make_dd_anchor.py); an fp64 order is in band when it lands within the
                # distance fp64 orders were MEASURED to land from the exact count at N = 8192 /
                # 16384 (the oracle's six orders against its long-double solve, the GPU's)
                # 16384 (the oracle's six orders against its long-double solve, the GPU's), or
                # within the distance of the oracle's own orders at this size, whichever is larger
                # (so every committed oracle order of the reference's algorithm is in band)
                frac = max(anchor["fp64_distance_fraction"].values())
                tol_it = anchor_tolerance(anchor)
                oracle_d = [full["iters"] - anchor["iters"]] + (
                    [full["second_order_iters"] - anchor["iters"]]
                    if "second_order_iters" in full else [])
                solve["exact_anchor"] = {
                    "iters": anchor["iters"], "source": "tests/golden/rbf_dd_n65536.json",
                    "tolerance_iters": tol_it, "fp64_distance_fraction": frac,
                    "gpu_minus_anchor": int(res.iters) - anchor["iters"],
                    "oracle_minus_anchor": oracle_d,
                    "oracle_in_band": all(abs(d) <= tol_it for d in oracle_d),
                    "gpu_minus_oracle": [int(res.iters) - full["iters"]] + (
                        [int(res.iters) - full["second_order_iters"]]
                        if "second_order_iters" in full else [])}
                ok = abs(res.iters - anchor["iters"]) <= tol_it
            else:  # no anchor committed: the oracle's count with the N = 8192 band scaled
                b_it = int(np.ceil(bd["band_iters"] * full["iters"] / bd["ref_iters"]))
                solve["band_iters_scaled"] = b_it
                ok = abs(res.iters - full["iters"]) <= 2 * b_it + 2
            if world == 1:  # ||dx|| / ||x|| against the oracle's x, and its scaled band
                scale = full["iters"] / bd["ref_iters"]
                solve["rel_dx_vs_cpu_ref"] = float(np.linalg.norm(res.x - x_cpu) /
                                                   np.linalg.norm(x_cpu))
                solve["band_rel_dx_scaled"] = float(bd["band_rel_dx"] * max(1.0, scale))
                ok = ok and solve["rel_dx_vs_cpu_ref"] <= 10 * solve["band_rel_dx_scaled"]
            solve["in_band"] = bool(ok)

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            try:
                if sg_info is None:
                    cpu = cpu_baseline(solver, X, b, idx, lam, ell, args.cpu_iters,
                                       args.cpu_iters_1t)
                else:
                    cpu = cpu_baseline_sgdml(solver, *sg_info["desc"], sg_info["perms"], b, lam,
                                             args.cpu_iters_sgdml)
            except Exception as e:  # a baseline failure must not hide the GPU number
                cpu = {"value": None, "error": repr(e)}
        par = None
        if world == 1 and not args.no_solve and args.workload == "rbf":
            par = parity_small(8192, k, lam, ell)
        out = {
            "metric": METRIC,
            **({"rehearsal": "SOLO ranks on one GPU: not a measurement"} if REHEARSE else {}),
            "value": args.steps / el,
            "unit": "CG iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            # BASELINE.md publishes a CG step time only for the nanotube (0.105 s/step at
            # N = 15540, data/data/cg_performance_n=15750/..._nanotube_points14_meas31)
            "vs_baseline": (args.steps / el) / (1.0 / REF_STEP_S[n])
            if args.workload == "nanotube" and n in REF_STEP_S else
            (args.steps / el) / (1.0 / REF_STEP_S_ETHANOL[n])
            if args.workload == "ethanol" and n in REF_STEP_S_ETHANOL else None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": workload,
                       "baseline_config": ("configs[3]" if n == 131072 else
                                           "configs[2]" if n == 65536 else None)
                       if sg_info is None else (None if n != 15540 else
                                                ("configs[4]" if k == 1024 and world > 1
                                                 else "configs[1]")),
                       "n": n, "k": k, "lambda": lam,
                       "length_scale": ell if sg_info is None else 10.0,
                       "precon": "random_scores (Nystrom, iterative_solver.py:95-322)"
                       if sg_info is None else
                       "cholesky (pivoted Cholesky + Woodbury, iterative_cholesky.py:115-150)",
                       "storage": storage,
                       **({"operator_form": mf_form} if mf_form else {}),
                       **({"descriptors": args.desc} if sg_info is not None else {}),
                       "parallelism": f"row-shard x{world} (RCCL allgather/allreduce"
                       + ("/reduce-scatter)" if storage == "sym" else ")")},
            "roofline": roof_dominant,
            "operator_roofline": roof_op,
            "precon_roofline": roof_pre,
            "matvec_gbs": achieved,
            # with half storage also report against the dense 8 N^2 bytes
            "matvec_gbs_dense_equivalent": dense_equiv,
            "iter_device_ms": iter_ms,
            "timing_events_every": timing_every(args.steps),
            "rccl": comm,
            "device_memory_used_gb_max_rank": used_gb,
            "iter_gbs_algorithmic": per_iter_bytes / (iter_ms * 1e-3) / 1e9,
            "cpu_baseline": cpu,
            "solve_to_1e-6": solve,
            "parity_n8192": par,
            # the reference's own headline for this path is the total solve (preconditioner + CG,
            # data/rule_of_thumb.csv:9,15): the device's build (pivoted Cholesky + Woodbury) and
            # CG to 1e-6 beside the reference's published per-column / per-step times
            "time_to_solution": None if sg_info is None or solve is None else {
                "precon_build_s": t_pre, "cg_to_1e-6_s": solve["seconds"],
                "total_s": t_pre + solve["seconds"],
                "precon_build_warm_s": sg_info.get("pivchol_build_warm_s"),
                "reference_published": {
                    "pivchol_s_per_column_nanotube_k3885": [0.076, 0.178],
                    "cg_step_s": REF_STEP_S.get(n) if args.workload == "nanotube" else
                    REF_STEP_S_ETHANOL.get(n),
                    "total_solve_min_n75k": {"ethanol": 2.7, "nanotube": 60}.get(args.workload),
                    "source": "BASELINE.md 1 (nanotube pickle t_cholesky; data/rule_of_thumb.csv:9,15)"}},
            "setup_s": dict({"gen_rbf": t_gen, "nystrom_build": t_pre} if sg_info is None else
                            {("descriptors_and_assembly" if sg_info["assembled"] else
                              "descriptors_and_operator"): t_gen, "pivoted_cholesky_build": t_pre},
                            storage_pack=t_pack),
        }
    solver.close()
    if out is not None:
        # the headline line first: a later leg that fails or hangs cannot take it away
        print(json.dumps(out), flush=True)
    if args.workload == "rbf" and args.configs3_n and args.configs3_n != n:
        try:
            leg = size_leg(args, rank, world, local, pg, args.configs3_n, k, lam, ell)
        except Exception as e:  # the configs[2] line above is already printed
            leg = {"n": args.configs3_n, "value": None, "error": repr(e)}
        if out is not None:
            out["configs3_leg"] = dict(leg, baseline_config=(
                "configs[3]" if args.configs3_n == 131072 else None),
                n_gpus=world, scaling="strong", note=(
                    "the configs[3] problem on the same ranks: its value at N GPUs over its "
                    "value in the N=1 bench line is configs[3]'s strong scaling (BASELINE.md "
                    "2: >=6x at 8 GPUs); `value` above is configs[2] (N=65536) on N GPUs"))
            # the same line again with the configs[3] leg added (the last line supersedes)
            print(json.dumps(out), flush=True)
    if pg is not None:
        pg.barrier()
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
