"""Multi-GPU layout of the batched QP solve: one process per GPU, the global batch
split into contiguous per-rank blocks of one counter-based stream, no data-path collective, and one
gather of the applied moves (U after ``controllerStep``) to rank 0 — the path's only exchange
(RCCL over xGMI with the ``nccl`` backend on the GPU box; ``gloo`` in the CPU tests)."""
from __future__ import annotations

import os


def world_from_env(default_world: int = 1) -> tuple[int, int, int]:
    """(rank, world_size, local_rank) as torch.distributed.run exports them."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(default_world)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def weak_block(per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns QPs [r * per_rank, (r + 1) * per_rank) of the global stream."""
    return rank * per_rank, per_rank


def strong_block(total: int, rank: int, world: int) -> tuple[int, int]:
    """Strong scaling: a fixed global batch split into near-equal contiguous blocks."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def gather_moves(dist, moves, world: int, rank: int, gathered=None):
    """Gather every rank's applied moves to rank 0 (``dist.gather``; equal block sizes).  Returns the
    list of per-rank tensors on rank 0 and None elsewhere."""
    if world == 1:
        return [moves]
    if rank == 0 and gathered is None:
        gathered = [moves.new_empty(moves.shape) for _ in range(world)]
    dist.gather(moves, gathered if rank == 0 else None, dst=0)
    return gathered if rank == 0 else None
