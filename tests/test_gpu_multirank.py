"""Multi-rank code path on one GPU.

RCCL refuses two ranks on one device, so here W contexts of one process (one
host thread each, all on cuda:0) are joined by the library's in-process
transport (comm_id "LOCAL:<key>").  Everything rank-dependent runs exactly as on
W GPUs — row sharding with padded blocks (uneven for W = 3), the elementwise
all-reduce of partial sums, the all-gather of the search direction, the
all-reduced low-rank apply, the distributed pivot search of the pivoted
Cholesky — only the transport differs.  Results must match the W = 1 solve.
"""
import threading

import numpy as np
import pytest

from tests.parity import assert_pcg_parity, noise_band

pytestmark = pytest.mark.gpu


def run_ranks(world, fn, timeout=300):
    results = [None] * world
    errors = [None] * world
    key = f"LOCAL:test-{np.random.default_rng().integers(1 << 62)}".encode().ljust(128, b"\0")

    def body(r):
        try:
            results[r] = fn(r, world, key)
        except BaseException as e:  # noqa: BLE001
            errors[r] = e

    threads = [threading.Thread(target=body, args=(r,), daemon=True, name=f"rank{r}of{world}")
               for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout)
        assert not t.is_alive(), "rank thread hung"
    for e in errors:
        if e is not None:
            raise e
    return results


def problem(n=1003, seed=3):
    from sgdml_amd import synthetic

    return synthetic.rbf_points(n, 3, seed)


def solve_case(rank, world, key, n, precon, lam=1e-1, k=150, tol=1e-8, storage="auto"):
    import sgdml_amd

    X, b = problem(n)
    idx = np.sort(np.random.default_rng(5).choice(n, k, replace=False))
    s = sgdml_amd.KernelSolver(n, device=0, rank=rank, world=world,
                               comm_id=key if world > 1 else None)
    try:
        s.gen_rbf(X, 0.2)
        s.set_operator(1.0, lam)
        s.set_storage(storage)
        mode, _ = s.storage_info()
        assert mode == ("dense" if storage == "dense" else "sym")
        piv = None
        if precon == "pivchol":
            piv, _ = s.precon_pivchol(k)
        elif precon == "nystrom":
            s.precon_nystrom(idx, variant=0)
        else:
            s.precon_none()
        r0, r1 = s.row_range()
        z = s.precon_apply(np.ascontiguousarray(b[r0:r1]))
        y = s.matvec(b)
        res = s.pcg(np.ascontiguousarray(b[r0:r1]), tol=tol, maxiter=5 * n, chunk=5)
        lev = s.lev_scores(idx, 1e-8)
        return {"r": (r0, r1), "x": res.x, "iters": res.iters, "trace": res.trace, "piv": piv,
                "z": z, "y": y, "lev": lev, "info": res.info}
    finally:
        s.close()


def gather(outs, key):
    return np.concatenate([o[key] for o in outs])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,precon,storage", [
    (2, "none", "auto"), (3, "none", "auto"), (2, "nystrom", "auto"), (3, "nystrom", "auto"),
    (2, "pivchol", "auto"), (3, "pivchol", "auto"), (2, "none", "dense"),
    (3, "pivchol", "dense"), (8, "nystrom", "auto"), (8, "none", "dense")])
def test_sharded_solve_matches_single_rank(world, precon, storage):
    """auto = symmetric tiles (reduce-scatter of the partial products), dense = row GEMV."""
    n = 1003
    ref = run_ranks(1, lambda r, w, key: solve_case(r, w, key, n, precon, storage=storage))[0]
    outs = run_ranks(world, lambda r, w, key: solve_case(r, w, key, n, precon, storage=storage))
    spans = [o["r"] for o in outs]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for a, b in zip(spans, spans[1:]):
        assert a[1] == b[0]
    # every rank runs the same number of iterations with the same residual curve
    for o in outs[1:]:
        assert o["iters"] == outs[0]["iters"]
        np.testing.assert_array_equal(o["trace"], outs[0]["trace"])
        np.testing.assert_array_equal(o["lev"], outs[0]["lev"])
        if precon == "pivchol":
            np.testing.assert_array_equal(o["piv"], outs[0]["piv"])
    if precon == "pivchol":
        np.testing.assert_array_equal(outs[0]["piv"][:150], ref["piv"][:150])
    np.testing.assert_allclose(gather(outs, "y"), ref["y"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(gather(outs, "z"), ref["z"], rtol=1e-9,
                               atol=1e-9 * np.abs(ref["z"]).max())
    np.testing.assert_allclose(outs[0]["lev"], ref["lev"], rtol=1e-8, atol=1e-12)
    assert outs[0]["info"] == ref["info"] == 0
    # W ranks vs one rank: two samples of the summation-order distribution whose spread the
    # oracle measured on this very system (noise_band.json "rbf_n1003/<precon>")
    band = noise_band(f"rbf_n1003/{'none' if precon == 'none' else precon}")
    assert_pcg_parity(outs[0]["iters"], outs[0]["trace"][1:], gather(outs, "x"), ref["iters"],
                      ref["trace"][1:], ref["x"], band=band)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("lsub", ["3", "4"])
def test_sharded_sym_row_slices(lsub, monkeypatch):
    """Split tiles as 8 / 16 row slices (MLFF_SYM_LSUB; below one round of resident
    workgroups every tile is split): the owned-slot reduction sums 7 / 15 partial planes
    per split slot; the sharded mat-vec and solve must match the single-rank one."""
    monkeypatch.setenv("MLFF_SYM_LSUB", lsub)
    n = 1003
    ref = run_ranks(1, lambda r, w, key: solve_case(r, w, key, n, "nystrom"))[0]
    outs = run_ranks(3, lambda r, w, key: solve_case(r, w, key, n, "nystrom"))
    np.testing.assert_allclose(gather(outs, "y"), ref["y"], rtol=1e-13, atol=1e-13)
    assert outs[0]["info"] == ref["info"] == 0
    assert_pcg_parity(outs[0]["iters"], outs[0]["trace"][1:], gather(outs, "x"), ref["iters"],
                      ref["trace"][1:], ref["x"], band=noise_band("rbf_n1003/nystrom"))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,precon", [(2, "nystrom"), (3, "none"), (8, "nystrom")])
def test_sharded_fused_p_update_bitwise(world, precon, monkeypatch):
    """The sharded tiled iteration with p = z + beta p formed inside k_symv_dyn and written by
    the slot reduction (default) against the separate k_update_p_gathered launch
    (MLFF_FUSE_P=0): the same arithmetic on the same operands, so iterates, residual curve and
    stop decisions are bit-identical."""
    n = 1003
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("MLFF_FUSE_P", fuse)
        out[fuse] = run_ranks(world, lambda r, w, key: solve_case(r, w, key, n, precon))
    for a, b in zip(out["1"], out["0"]):
        assert a["iters"] == b["iters"] and a["info"] == b["info"] == 0
        np.testing.assert_array_equal(a["trace"], b["trace"])
        np.testing.assert_array_equal(a["x"], b["x"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,precon", [(2, "nystrom"), (3, "pivchol"), (8, "nystrom")])
def test_sharded_pq_publish_folded_bitwise(world, precon, monkeypatch):
    """The p.q share publish folded into k_sym_reduce_w's last-arriving workgroup (default)
    against the separate k_pq_publish launch (MLFF_PQ_PUBLISH=1, read at context creation): the
    same sums in the same order, so the shares, iterates, residual curve and stop decisions are
    bit-identical."""
    n = 1003
    out = {}
    for sep in ("1", "0"):
        monkeypatch.setenv("MLFF_PQ_PUBLISH", sep)
        out[sep] = run_ranks(world, lambda r, w, key: solve_case(r, w, key, n, precon))
    for a, b in zip(out["1"], out["0"]):
        assert a["iters"] == b["iters"] and a["info"] == b["info"] == 0
        np.testing.assert_array_equal(a["trace"], b["trace"])
        np.testing.assert_array_equal(a["x"], b["x"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,precon,n,lsub", [(2, "nystrom", 1003, "2"), (3, "pivchol", 1003, "2"),
                                                 (8, "nystrom", 1003, "2"), (3, "nystrom", 1003, "4"),
                                                 (4, "none", 9000, "2")])
def test_sharded_sym_reduce_list_bitwise(world, precon, n, lsub, monkeypatch):
    """The owned-slot reduction from the flat load list (k_sym_reduce_wl, default since round 6:
    a row's slot and split-plane loads in batches of 32 with the next batch in flight) against
    k_sym_reduce_w (MLFF_SYM_REDUCE_LIST=0, read at the operator's build): the same additions
    in the same order, so iterates, residual curve and stop decisions are bit-identical.  Below
    one round of resident workgroups every tile is split, so every slot carries 3 (lsub 2) or
    15 (lsub 4) planes."""
    monkeypatch.setenv("MLFF_SYM_LSUB", lsub)
    out = {}
    for lst in ("1", "0"):
        monkeypatch.setenv("MLFF_SYM_REDUCE_LIST", lst)
        out[lst] = run_ranks(world, lambda r, w, key: solve_case(r, w, key, n, precon))
    for a, b in zip(out["1"], out["0"]):
        assert a["iters"] == b["iters"] and a["info"] == b["info"] == 0
        np.testing.assert_array_equal(a["trace"], b["trace"])
        np.testing.assert_array_equal(a["x"], b["x"])
        np.testing.assert_array_equal(a["y"], b["y"])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,precon,n", [(2, "nystrom", 1003), (3, "pivchol", 1003),
                                            (8, "nystrom", 1003), (2, "nystrom", 9000),
                                            (3, "pivchol", 9000)])
def test_sharded_fused_xr_update_bitwise(world, precon, n, monkeypatch):
    """The sharded tiled iteration with k_update_xr_shares folded into the next apply's T r
    pass (k_gemv_xr: r_new staged in LDS, x / r / rr partials written by row group 0, r and
    the spare vector swapped; MLFF_FUSE_XR_RANKS=1) against the separate launch (default):
    the same arithmetic, so iterates, residual curve and stop decisions are bit-identical.
    n = 9000 runs the T r pass in 6-9 column splits (n = 1003: one); chunk = 5 puts
    iterations gated after the stop test inside chunks."""
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("MLFF_FUSE_XR_RANKS", fuse)
        out[fuse] = run_ranks(world, lambda r, w, key: solve_case(r, w, key, n, precon))
    for a, b in zip(out["1"], out["0"]):
        assert a["iters"] == b["iters"] and a["info"] == b["info"] == 0
        np.testing.assert_array_equal(a["trace"], b["trace"])
        np.testing.assert_array_equal(a["x"], b["x"])
        np.testing.assert_array_equal(a["lev"], b["lev"])


@pytest.mark.timeout(300)
def test_sharded_sgdml_assembly_rows():
    import sgdml_amd
    from oracle.sgdml import descriptors
    from sgdml_amd import synthetic

    d = synthetic.ethanol_like(9, seed=8)
    Rd, Rdd = descriptors(d["R"])
    P = np.array([np.arange(9), [0, 1, 2, 4, 5, 3, 6, 7, 8], [0, 1, 2, 5, 3, 4, 6, 7, 8]])
    n = 9 * 27

    def body(rank, world, key):
        s = sgdml_amd.KernelSolver(n, device=0, rank=rank, world=world,
                                   comm_id=key if world > 1 else None)
        try:
            s.assemble_sgdml(Rd, Rdd, P, 10.0)
            return s.get_matrix_rows()
        finally:
            s.close()

    ref = run_ranks(1, body)[0]
    for world in (2, 4):
        rows = np.concatenate(run_ranks(world, body))
        np.testing.assert_array_equal(rows, ref)


@pytest.mark.timeout(900)
def test_bench_config_eight_ranks():
    """The bench's 8-GPU configuration (N = 65536 RBF, rank-256 Nystrom, symmetric tiles,
    8 row blocks of 8192, ~1032 tiles per rank) rehearsed as 8 ranks on one GPU, against
    the one-rank run.  This system is chaotic under summation order: the one-rank DENSE vs
    SYMTILE storages themselves drift apart ~10x per 3 iterations (1e-12 at 12, 3e-9 at
    21, 6e-6 at 27; scripts/dev/diag_ranks.py), and 8 ranks drift the same way.  So: 16
    iterations, residuals within 1e-7 relative, iterates within 1e-7."""
    import sgdml_amd
    from sgdml_amd import synthetic

    n, k, lam, ell, iters = 65536, 256, 1e-6, 0.2, 16
    X, b = synthetic.rbf_points(n, 3, 0)
    idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False))

    def body(rank, world, key):
        s = sgdml_amd.KernelSolver(n, device=0, rank=rank, world=world,
                                   comm_id=key if world > 1 else None)
        try:
            s.gen_rbf(X, ell)
            s.set_operator(1.0, lam)
            s.precon_nystrom(idx, variant=0)
            mode, _ = s.storage_info()
            r0, r1 = s.row_range()
            res = s.pcg(np.ascontiguousarray(b[r0:r1]), tol=0.0, maxiter=iters)
            return mode, res.trace, res.x
        finally:
            s.close()

    ref = run_ranks(1, body)[0]
    outs = run_ranks(8, body, timeout=800)
    assert ref[0] == "sym" and all(o[0] == "sym" for o in outs)
    for o in outs[1:]:
        np.testing.assert_array_equal(o[1], outs[0][1])
    np.testing.assert_allclose(outs[0][1], ref[1], rtol=1e-7)
    x = np.concatenate([o[2] for o in outs])
    assert np.linalg.norm(x - ref[2]) <= 1e-7 * np.linalg.norm(ref[2])


@pytest.mark.timeout(300)
def test_sharded_x0_matches_single_rank():
    """A warm start sliced over 3 ranks (padded blocks) equals the one-rank solve."""
    import sgdml_amd

    n = 1003
    X, b = problem(n)
    x0 = 0.05 * np.random.default_rng(8).standard_normal(n)

    def body(rank, world, key):
        s = sgdml_amd.KernelSolver(n, device=0, rank=rank, world=world,
                                   comm_id=key if world > 1 else None)
        try:
            s.gen_rbf(X, 0.2)
            s.set_operator(1.0, 1e-1)
            s.precon_pivchol(150)
            r0, r1 = s.row_range()
            res = s.pcg(np.ascontiguousarray(b[r0:r1]), np.ascontiguousarray(x0[r0:r1]), tol=1e-8,
                        maxiter=5 * n)
            return res.x, res.iters, res.trace
        finally:
            s.close()

    ref = run_ranks(1, body)[0]
    outs = run_ranks(3, body)
    assert all(o[1] == outs[0][1] for o in outs)
    # ||b - A x0|| over the sharded operator (the warm-start residual itself)
    np.testing.assert_allclose(outs[0][2][0], ref[2][0], rtol=1e-12)
    x = np.concatenate([o[0] for o in outs])
    assert_pcg_parity(outs[0][1], outs[0][2][1:], x, ref[1], ref[2][1:], ref[0],
                      band=noise_band("rbf_n1003/pivchol"))


@pytest.mark.parametrize("n", [1, 2, 63, 513, 1100, 2049])
@pytest.mark.parametrize("world", [2, 5, 8])
def test_sharded_ragged_sizes(n, world):
    """Ragged shards (N not a multiple of W, ranks with no rows, one-tile problems) through
    the three-collective iteration, both operator storages: the sharded mat-vec equals the
    one-rank one, and the solve agrees with the one-rank solve."""
    import sgdml_amd
    from sgdml_amd import synthetic

    X, b = synthetic.rbf_points(n, 3, n)
    v = np.random.default_rng(n).standard_normal(n)
    k = max(1, min(40, n // 3))

    def body(rank, w, key, storage):
        s = sgdml_amd.KernelSolver(n, device=0, rank=rank, world=w, comm_id=key if w > 1 else None)
        try:
            s.gen_rbf(X, 0.3)
            s.set_operator(1.0, 0.5)
            s.set_storage(storage)
            y = s.matvec(v)
            s.precon_pivchol(k)
            r0, r1 = s.row_range()
            res = s.pcg(np.ascontiguousarray(b[r0:r1]), tol=1e-10, maxiter=5 * n + 5)
            return y, res.x, res.iters, res.info
        finally:
            s.close()

    for storage in ("sym", "dense"):
        ref = run_ranks(1, lambda r, w, key: body(r, w, key, storage))[0]
        outs = run_ranks(world, lambda r, w, key: body(r, w, key, storage))
        y = np.concatenate([o[0] for o in outs])
        np.testing.assert_allclose(y, ref[0], rtol=1e-13, atol=1e-13 * np.abs(ref[0]).max())
        x = np.concatenate([o[1] for o in outs])
        assert all(o[3] == 0 for o in outs) and ref[3] == 0
        assert all(o[2] == outs[0][2] for o in outs)
        assert abs(outs[0][2] - ref[2]) <= 2
        assert np.linalg.norm(x - ref[1]) <= 1e-8 * max(np.linalg.norm(ref[1]), 1e-300)


def test_rank_failure_aborts_group():
    """A failure on one rank (here: an argument error only rank 1 makes) aborts the
    in-process group: its peer returns from the collective with an error instead of
    waiting forever, and the aborted contexts refuse further calls."""
    import sgdml_amd

    n = 300
    X, b = problem(n)

    def body(rank, world, key):
        s = sgdml_amd.KernelSolver(n, device=0, rank=rank, world=world, comm_id=key)
        try:
            s.gen_rbf(X, 0.2)
            s.set_operator(1.0, 0.1)
            with pytest.raises((ValueError, RuntimeError)):
                s.precon_pivchol(10 if rank == 0 else n + 5)
            with pytest.raises(RuntimeError, match="aborted"):
                s.matvec(np.ones(n))
            return True
        finally:
            s.close()

    assert run_ranks(2, body, timeout=60) == [True, True]


@pytest.mark.timeout(1100)
def test_configs3_eight_ranks_full_size():
    """BASELINE configs[3] at its full size: N = 131072 RBF (the bench's generator), rank-256
    Nystrom, 8 row blocks of 16384 on the symmetric tiles (8.6 GB of tiles per rank, 69 GB in
    all), as 8 in-process ranks on one GPU.  (a) the sharded mat-vec on 256 sampled rows
    against rows of K evaluated on the host with the sklearn RBF formula of the reference's
    generator; (b) 16 PCG iterations against the one-rank run (same rule as the N = 65536
    rehearsal above: the system is chaotic under summation order); (c) every rank holds the
    same residual trace; the device memory in use with all 8 ranks resident is printed."""
    import sgdml_amd
    from sgdml_amd import synthetic

    n, k, lam, ell, iters = 131072, 256, 1e-6, 0.2, 16
    X, b = synthetic.rbf_points(n, 3, 0)
    idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False))
    v = np.random.default_rng(11).standard_normal(n)
    mem = {}

    def body(rank, world, key):
        s = sgdml_amd.KernelSolver(n, device=0, rank=rank, world=world,
                                   comm_id=key if world > 1 else None)
        try:
            s.gen_rbf(X, ell)
            s.set_operator(1.0, lam)
            s.precon_nystrom(idx, variant=0)
            mode, op_bytes = s.storage_info()
            y = s.matvec(v)
            r0, r1 = s.row_range()
            res = s.pcg(np.ascontiguousarray(b[r0:r1]), tol=0.0, maxiter=iters)
            free_b, total_b = s.device_memory()
            mem[(world, rank)] = (total_b - free_b) / 1e9
            return mode, (r0, r1), y, res.trace, res.x, op_bytes
        finally:
            s.close()

    ref = run_ranks(1, body, timeout=600)[0]
    outs = run_ranks(8, body, timeout=1000)
    assert ref[0] == "sym" and all(o[0] == "sym" for o in outs)
    assert [o[1] for o in outs] == [(r * 16384, (r + 1) * 16384) for r in range(8)]
    print(f"device memory in use: 1 rank {mem[(1, 0)]:.1f} GB, 8 ranks resident "
          f"{max(mem[(8, r)] for r in range(8)):.1f} GB; operator bytes per rank "
          f"{[round(o[5] / 1e9, 2) for o in outs]} GB")
    y = np.concatenate([o[2] for o in outs])
    np.testing.assert_allclose(y, ref[2], rtol=1e-12, atol=1e-12 * np.abs(ref[2]).max())
    rows = np.sort(np.random.default_rng(12).choice(n, 256, replace=False))
    Xs = X / ell
    Kr = np.exp(-0.5 * ((Xs[rows, None, :] - Xs[None, :, :]) ** 2).sum(-1))
    Kr[np.arange(rows.size), rows] = 1.0
    y_host = Kr @ v + lam * v[rows]
    np.testing.assert_allclose(y[rows], y_host, rtol=0, atol=1e-11 * np.abs(y_host).max())
    for o in outs[1:]:
        np.testing.assert_array_equal(o[3], outs[0][3])
    np.testing.assert_allclose(outs[0][3], ref[3], rtol=1e-7)
    x = np.concatenate([o[4] for o in outs])
    assert np.linalg.norm(x - ref[4]) <= 1e-7 * np.linalg.norm(ref[4])


@pytest.mark.parametrize("count", [1, 3, 1000003, 1 << 22])
def test_rccl_transport_one_rank(count):
    """The RCCL branches of comm_allreduce / comm_allgather / comm_reduce_scatter
    (api.hip rccl_*), the transport the 8-GPU bench and drop-in run on, driven on a
    one-rank communicator: in-place and out-of-place forms, odd and multi-chunk counts,
    each collective between a producing kernel and a consuming copy on the context's
    stream.  A one-rank sum or gather is the identity, so any deviation is a count,
    datatype, buffer or stream-ordering error in the call itself."""
    from sgdml_amd import _native

    assert _native.comm_selftest(0, count) == 0.0
