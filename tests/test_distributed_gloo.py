"""World-size-2 checks of the row-sharded PCG protocol on CPU (gloo).

The GPU library runs this exact protocol with RCCL (api.hip launch_iteration_ranks):
every rank owns a contiguous, padded row block; dots are fixed-length partial-sum
arrays; per iteration there are three collectives:
  1. allgather(z_g | rho partials of r_g.z_g) -> every rank sums all ranks' partials
     in the same order (bit-identical rho) and forms the whole p = z + beta p;
  2. symmetric tiles: reduce-scatter(partial K p rows of the tiles this rank owns |
     p.q shares, rank g's share in tail slot g only) -> q rows and the exact vector of
     shares (x + 0 is exact), summed in rank order on every rank;
     dense rows: allreduce(p.q partials);
  3. allreduce(r.r partials | T r of the next iteration) (low-rank preconditioner).
Here the same protocol runs in NumPy over gloo and must reproduce the single-process
oracle solve.  gloo has no reduce-scatter; an allreduce followed by taking this rank's
block stands in for it (same sums, same exactness of the shares).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.parity import assert_pcg_parity

NPART = 8
TS = 32  # tile edge of the symmetric storage in this restatement (512 on the GPU)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _partials(a, b):
    """fixed-length partial sums of a.b over this rank's rows (device layout: grid-stride)"""
    out = np.zeros(NPART)
    for g in range(NPART):
        out[g] = np.dot(a[g::NPART], b[g::NPART])
    return out


def _allreduce(arr):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(arr))
    dist.all_reduce(t)
    return t.numpy()


def _allgather(block, world):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(block))
    out = [torch.zeros(block.size, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(out, t)
    return np.stack([o.numpy() for o in out])


def _owner(I, J, tpr):
    """tile (I, J), I >= J -> rank (kernels_sym.hip owner_of)"""
    a, c = I // tpr, J // tpr
    if a == c:
        return a
    return a if (I + J) & 1 else c


def sharded_pcg(rank, world, K, b, T, lam, sigma_p, tol, maxiter, storage):
    from sgdml_amd.distributed import shard_range

    n = b.size
    rows_per = (n + world - 1) // world
    blk = -(-rows_per // TS) * TS
    ld = world * blk
    pos = np.array([(g // rows_per) * blk + g % rows_per for g in range(n)])
    Kp = np.zeros((ld, ld))
    Kp[np.ix_(pos, pos)] = K
    r0, nr = shard_range(n, world, rank)
    lo = rank * blk
    Kl = Kp[lo:lo + blk]
    Tl = None
    if T is not None:
        Tl = np.zeros((T.shape[0], blk))
        Tl[:, :nr] = T[:, r0:r0 + nr]
    nb, tpr = ld // TS, blk // TS
    tiles = [(I, J) for I in range(nb) for J in range(I + 1) if _owner(I, J, tpr) == rank]
    bl = np.zeros(blk)
    bl[:nr] = b[r0:r0 + nr]
    x = np.zeros(blk)
    r = bl.copy()
    p_full = np.zeros(ld)
    bnorm = np.sqrt(_allreduce(_partials(bl, bl)).sum())
    atol = tol * bnorm
    trace = [bnorm]
    rho1 = None
    t_next = None
    it = 0

    def apply_op(v_full, v_loc):
        if storage == "dense":
            return Kl @ v_full + lam * v_loc, None
        yg = np.zeros(ld)
        for I, J in tiles:
            A = Kp[I * TS:(I + 1) * TS, J * TS:(J + 1) * TS]
            yg[I * TS:(I + 1) * TS] += A @ v_full[J * TS:(J + 1) * TS]
            if I != J:
                yg[J * TS:(J + 1) * TS] += A.T @ v_full[I * TS:(I + 1) * TS]
        share = v_full @ yg + lam * (v_loc @ v_loc)
        send = np.zeros((world, blk + world))
        send[:, :blk] = yg.reshape(world, blk)
        send[:, blk + rank] = share
        recv = _allreduce(send)[rank]  # reduce-scatter stand-in
        return recv[:blk] + lam * v_loc, recv[blk:]

    while True:
        it += 1
        if T is not None:
            t = t_next if t_next is not None else _allreduce(Tl @ r)
            z = sigma_p * ((1.0 / lam) * (r - Tl.T @ t))
        else:
            z = r.copy()
        g = _allgather(np.concatenate([z, _partials(r, z)]), world)  # 1
        rho = g[:, blk:].sum()
        z_full = g[:, :blk].reshape(-1)
        p_full = z_full + (rho / rho1) * p_full if it > 1 else z_full.copy()
        p = p_full[lo:lo + blk]
        q, shares = apply_op(p_full, p)                                 # 2
        pq = _allreduce(_partials(p, q)).sum() if shares is None else sum(shares)
        alpha = rho / pq
        x = x + alpha * p
        r = r - alpha * q
        if T is not None:                                              # 3
            red = _allreduce(np.concatenate([_partials(r, r), Tl @ r]))
            rr, t_next = red[:NPART].sum(), red[NPART:]
        else:
            rr = _allreduce(_partials(r, r)).sum()
        resid = np.sqrt(rr)
        if resid <= atol and it > 1:
            xg = _allgather(x, world).reshape(-1)
            r = bl - apply_op(xg, x)[0]
            resid = np.sqrt(_allreduce(_partials(r, r)).sum())
            t_next = None
        trace.append(resid)
        if resid <= atol or it == maxiter:
            break
        rho1 = rho
    return x[:nr], it, np.array(trace)


def _worker(rank, world, port, path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path[:0] = [str(path), str(path / "mlff-preconditioner_amd")]
    from oracle.precon import nystrom_panel
    from oracle.rbf import rbf_kernel
    from sgdml_amd import synthetic

    n, k, lam = 333, 40, 1.0
    X, b = synthetic.rbf_points(n, 3, 4)
    K = rbf_kernel(X, 0.2)
    idx = np.sort(np.random.default_rng(1).choice(n, k, replace=False))
    B, sp = nystrom_panel(K[:, idx], idx, lam, 0)
    out = {}
    rows_per = (n + world - 1) // world
    for name, T in [("none", None), ("nystrom", B)]:
        for storage in ("dense", "sym"):
            x, it, tr = sharded_pcg(rank, world, K, b, T, lam, sp, 1e-8, 5 * n, storage)
            xs = _allgather(np.pad(x, (0, rows_per - x.size)), world).reshape(-1)
            xs = np.concatenate([xs[q * rows_per: q * rows_per + min(rows_per, n - q * rows_per)]
                                 for q in range(world)])
            out[f"{name}-{storage}"] = (xs, it, tr)
    np.savez(path / "tests" / f".gloo_out_w{world}_r{rank}.npz",
             **{f"{k_}_{i}": v for k_, tup in out.items() for i, v in enumerate(tup)})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_protocol_matches_single_process(world, tmp_path):
    from pathlib import Path

    from oracle.pcg import cg_legacy
    from oracle.precon import apply_panel, nystrom_panel
    from oracle.rbf import rbf_kernel
    from sgdml_amd import synthetic

    repo = Path(__file__).resolve().parent.parent
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, repo), nprocs=world, join=True,
                       start_method="spawn")
    n, k, lam = 333, 40, 1.0
    X, b = synthetic.rbf_points(n, 3, 4)
    K = rbf_kernel(X, 0.2)
    idx = np.sort(np.random.default_rng(1).choice(n, k, replace=False))
    B, sp = nystrom_panel(K[:, idx], idx, lam, 0)
    precons = [("none", None), ("nystrom", lambda r: apply_panel(B, sp, lam, r))]
    for name, ps in [(f"{a}-{st}", f) for a, f in precons for st in ("dense", "sym")]:
        x_ref, info, tr_ref, it_ref = cg_legacy(lambda v: K @ v + lam * v, b, tol=1e-8,
                                                maxiter=5 * n, psolve=ps)
        outs = []
        for rank in range(world):
            f = np.load(repo / "tests" / f".gloo_out_w{world}_r{rank}.npz")
            outs.append((f[f"{name}_0"], int(f[f"{name}_1"]), f[f"{name}_2"]))
        # every rank ends with the same iterate, count and residual curve
        for o in outs[1:]:
            np.testing.assert_array_equal(o[0], outs[0][0])
            assert o[1] == outs[0][1]
            np.testing.assert_array_equal(o[2], outs[0][2])
        x, it, tr = outs[0]
        assert_pcg_parity(it, tr[1:], x, it_ref, tr_ref[1:], x_ref, mode="chaotic", x_tol=1e-7)
    for rank in range(world):
        (repo / "tests" / f".gloo_out_w{world}_r{rank}.npz").unlink()


def test_shard_ranges_partition_rows():
    from sgdml_amd.distributed import padded_block, shard_range

    for n in [1, 7, 64, 1000, 65536, 131072, 15540]:
        for world in [1, 2, 3, 4, 8]:
            spans = [shard_range(n, world, r) for r in range(world)]
            covered = np.concatenate([np.arange(r0, r0 + nr) for r0, nr in spans])
            assert np.array_equal(covered, np.arange(n))
            assert padded_block(n, world) % 64 == 0
            assert padded_block(n, world) >= max(nr for _, nr in spans)
