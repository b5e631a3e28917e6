"""Multi-GPU layout of the batch path: one process per GPU,
each owning a contiguous shard of whole streams.  Streams share no state
(writer.go:40-45 state is per Writer), so the data path has no collective;
torch.distributed (RCCL on GPUs, gloo on CPU) is used only for the barrier
around the timed region and to reduce the reported numbers.

Weak scaling: every rank owns `per_rank` streams; rank r's synthetic input
is seeded with base_seed + r, so shards are distinct and reproducible."""

from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Rank:
    rank: int
    world: int
    local: int

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def from_env() -> Rank:
    """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run."""
    return Rank(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                int(os.environ.get("LOCAL_RANK", "0")))


def shard(per_rank: int, r: Rank) -> tuple[int, int]:
    """Global stream range [first, last) owned by rank r (weak scaling)."""
    return r.rank * per_rank, (r.rank + 1) * per_rank


def seed(base: int, r: Rank) -> int:
    return base + r.rank


def reduce_max(values, r: Rank, device=None) -> list[float]:
    """Element-wise max over ranks (timing: the job ends with its slowest rank)."""
    if r.world == 1:
        return [float(v) for v in values]
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def reduce_sum(values, r: Rank, device=None) -> list[int]:
    """Element-wise sum over ranks (bytes processed / produced by the job)."""
    if r.world == 1:
        return [int(v) for v in values]
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return [int(v) for v in t.tolist()]


def barrier(r: Rank):
    if r.world > 1:
        import torch.distributed as dist

        dist.barrier()
