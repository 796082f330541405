"""World-size-2 checks of the row-sharded PCG protocol on CPU (gloo).

The GPU library runs this exact protocol with RCCL (api.hip launch_iteration):
every rank owns a contiguous row block; dots are reduced as fixed-length
partial-sum arrays that are all-reduced ELEMENTWISE and then summed in a fixed
order on every rank (so every rank computes bit-identical scalars); the search
direction is all-gathered before the local mat-vec; the low-rank apply
all-reduces the k-vector T r.  Here the same protocol runs in NumPy over gloo and
must reproduce the single-process oracle solve.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.parity import assert_pcg_parity

NPART = 8


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


def _allgather(block, nblk, world):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(block))
    out = [torch.zeros(nblk, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(out, t)
    return np.concatenate([o.numpy() for o in out])


def sharded_pcg(rank, world, K, b, T, lam, sigma_p, tol, maxiter):
    from sgdml_amd.distributed import shard_range

    n = b.size
    r0, nr = shard_range(n, world, rank)
    rows_per = (n + world - 1) // world
    Kl = K[r0:r0 + nr]
    Tl = T[:, r0:r0 + nr] if T is not None else None
    bl = b[r0:r0 + nr].copy()
    x = np.zeros(nr)
    r = bl.copy()
    p = np.zeros(nr)
    bnorm = np.sqrt(_allreduce(_partials(bl, bl)).sum())
    atol = tol * bnorm
    trace = [bnorm]
    rho1 = None
    it = 0
    while True:
        it += 1
        if T is not None:
            t = _allreduce(Tl @ r)
            z = sigma_p * ((1.0 / lam) * (r - Tl.T @ t))
        else:
            z = r
        rho = _allreduce(_partials(r, z)).sum()
        p = z + (rho / rho1) * p if it > 1 else z.copy()
        pad = np.zeros(rows_per)
        pad[:nr] = p
        p_full = _allgather(pad, rows_per, world)
        p_full = np.concatenate([p_full[q * rows_per: q * rows_per + shard_range(n, world, q)[1]]
                                 for q in range(world)])
        q = Kl @ p_full + lam * p
        pq = _allreduce(_partials(p, q)).sum()
        alpha = rho / pq
        x = x + alpha * p
        r = r - alpha * q
        resid = np.sqrt(_allreduce(_partials(r, r)).sum())
        if resid <= atol and it > 1:
            pad = np.zeros(rows_per)
            pad[:nr] = x
            xg = _allgather(pad, rows_per, world)
            xg = np.concatenate([xg[qq * rows_per: qq * rows_per + shard_range(n, world, qq)[1]]
                                 for qq in range(world)])
            r = bl - (Kl @ xg + lam * x)
            resid = np.sqrt(_allreduce(_partials(r, r)).sum())
        trace.append(resid)
        if resid <= atol or it == maxiter:
            break
        rho1 = rho
    return x, it, np.array(trace)


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
    for name, T in [("none", None), ("nystrom", B)]:
        x, it, tr = sharded_pcg(rank, world, K, b, T, lam, sp, 1e-8, 5 * n)
        xs = _allgather(np.pad(x, (0, (n + world - 1) // world - x.size)), (n + world - 1) // world, world)
        out[name] = (xs[:n] if world == 1 else np.concatenate(
            [xs[q * ((n + world - 1) // world): q * ((n + world - 1) // world)
                + min((n + world - 1) // world, n - q * ((n + world - 1) // world))]
             for q in range(world)]), it, tr)
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
    for name, ps in [("none", None), ("nystrom", lambda r: apply_panel(B, sp, lam, r))]:
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
