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


def unpad(gathered, total: int, world: int):
    """Rank 0's gathered blocks of a strong-scaling job (each padded to the longest block for the equal-size
    gather) trimmed and joined: the moves of global QPs 0 .. total - 1 in order."""
    import torch

    return torch.cat([t[:strong_block(total, r, world)[1]] for r, t in enumerate(gathered)])


def gather_moves(dist, moves, world: int, rank: int, gathered=None):
    """Gather every rank's applied moves to rank 0 (``dist.gather``; equal block sizes).  Returns the
    list of per-rank tensors on rank 0 and None elsewhere."""
    if world == 1:
        return [moves]
    if rank == 0 and gathered is None:
        gathered = [moves.new_empty(moves.shape) for _ in range(world)]
    dist.gather(moves, gathered if rank == 0 else None, dst=0)
    return gathered if rank == 0 else None


class PipelinedGather:
    """The per-step gather of the applied moves, overlapped with the next step.  Step i writes its moves
    into one of two buffers that alternate and issues their gather asynchronously (``async_op=True``: on
    RCCL the collective runs on the communicator's own stream, ordered after the kernels that produced the
    moves), so step i + 1's solve runs while step i's moves travel over xGMI.  A buffer is written again
    only after its previous gather has been made a dependency of the current stream (``work.wait()``: no
    host stall on RCCL).  World size 1: one buffer, nothing to gather."""

    def __init__(self, dist, world: int, rank: int, like):
        self.dist, self.world, self.rank = dist, world, rank
        self.bufs = [like] if world == 1 else [like, like.clone()]
        self.work = [None] * len(self.bufs)
        self.gathered = ([[like.new_empty(like.shape) for _ in range(world)] for _ in self.bufs]
                         if rank == 0 and world > 1 else None)
        self.k = 0
        self.last = 0

    def buffer(self):
        """The buffer this step writes its moves into (its previous gather is waited on first)."""
        if self.work[self.k] is not None:
            self.work[self.k].wait()
            self.work[self.k] = None
        return self.bufs[self.k]

    def gather(self):
        """Issue this step's gather (rank 0 receives into its per-buffer list); returns that list on rank
        0, None elsewhere (world 1: [moves])."""
        k = self.k
        self.last = k
        self.k = (k + 1) % len(self.bufs)
        if self.world == 1:
            return [self.bufs[k]]
        self.work[k] = self.dist.gather(self.bufs[k], self.gathered[k] if self.rank == 0 else None, dst=0,
                                        async_op=True)
        return self.gathered[k] if self.rank == 0 else None

    def finish(self):
        """Wait for every outstanding gather; returns the last step's moves (this rank's buffer)."""
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None
        return self.bufs[self.last]
