"""One process per GPU: row sharding and RCCL communicator bootstrap.

The C library shards the N rows of K (and every N-vector) into contiguous
blocks of ceil(N / world) rows (mlff_ctx_create); this module mirrors that rule
on the host so callers can slice their right-hand sides, and exchanges the RCCL
unique id over an existing torch.distributed process group (any backend).
"""
from __future__ import annotations


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Rows [row0, row0 + nrows) owned by `rank` (same rule as mlff_ctx_create)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    rows_per = (n + world - 1) // world
    row0 = min(rank * rows_per, n)
    nrows = max(0, min(rows_per, n - row0))
    return row0, nrows


def padded_block(n: int, world: int) -> int:
    """Padded per-rank length of the device vectors (mlff_ctx_create: a multiple of 64
    doubles on one rank, of the 512-row tile edge on several)."""
    rows_per = (n + world - 1) // world
    q = 64 if world == 1 else 512
    return (rows_per + q - 1) // q * q


def broadcast_comm_id(pg, rank: int) -> bytes:
    """Rank 0 creates the RCCL unique id, every rank receives it via `pg`
    (torch.distributed module with an initialised default group)."""
    from . import _native

    obj = [_native.comm_unique_id() if rank == 0 else None]
    pg.broadcast_object_list(obj, src=0)
    return obj[0]


def make_solver(n: int, pg=None, rank: int = 0, world: int = 1, device: int | None = None):
    """KernelSolver for this rank; world > 1 bootstraps the RCCL communicator."""
    from .solver import KernelSolver

    comm_id = broadcast_comm_id(pg, rank) if world > 1 else None
    return KernelSolver(n, device=device, rank=rank, world=world, comm_id=comm_id)
