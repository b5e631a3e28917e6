"""Multi-GPU data path of the batch codec: one process per GPU,
each owning a contiguous shard of whole streams of ONE global batch.

Streams share no state (the Writer's ring, table and position are per Writer,
writer.go:40-45; a Reader's likewise, reader.go:17-40), so compression and
decompression need no collective.  The one real exchange is the framing of
the global result: each rank knows only its own streams' compressed sizes, and
the packed global output (the streams back to back, as one caller would
concatenate the independent Writers' sink outputs) needs every stream's
global offset.  So:

1. ``shard_range``: rank r owns streams [count*r//N, count*(r+1)//N).
2. ``exchange_sizes``: an all-gather of the per-stream compressed sizes
   (int64, padded to the largest shard; RCCL over xGMI on GPUs, gloo on the
   CPU) gives every rank the global size table; ``global_offsets`` is its
   exclusive scan, and a rank's shard starts at offsets[first].
3. ``gather_payload`` (optional, timed separately by bench.py): grouped
   point-to-point sends of each rank's packed shard to the root, received
   in place at the shard's global offset.

Tensors stay on whatever device the backend needs (CUDA for nccl/RCCL, CPU for
gloo); nothing here copies between host and device."""

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


def _collective(r: Rank) -> bool:
    """Whether the exchanges go through torch.distributed: always with more than one rank,
    and at world size 1 too once a process group exists (so a one-GPU run still drives the
    RCCL all-gather and all-reduce it would use at N GPUs, instead of a local shortcut)."""
    if r.world > 1:
        return True
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized()


def shard_range(count: int, r: Rank) -> tuple[int, int]:
    """Global stream range [first, last) of rank r: contiguous, whole streams,
    sizes differing by at most one stream (strong scaling over one batch)."""
    return count * r.rank // r.world, count * (r.rank + 1) // r.world


def shard_counts(count: int, world: int) -> list[int]:
    return [count * (k + 1) // world - count * k // world for k in range(world)]


def exchange_sizes(local_sizes, count: int, r: Rank):
    """All-gather of per-stream compressed sizes (int64 tensor, this rank's
    shard in stream order) -> the global size table (count,) on every rank."""
    import torch

    if not _collective(r):
        return local_sizes.clone()
    import torch.distributed as dist

    counts = shard_counts(count, r.world)
    assert local_sizes.numel() == counts[r.rank], "local sizes must cover exactly this rank's shard"
    m = max(counts)
    buf = torch.zeros(m, dtype=torch.int64, device=local_sizes.device)
    buf[: local_sizes.numel()] = local_sizes
    allb = torch.empty(r.world * m, dtype=torch.int64, device=local_sizes.device)
    dist.all_gather_into_tensor(allb, buf)
    return torch.cat([allb[k * m : k * m + counts[k]] for k in range(r.world)])


def global_offsets(global_sizes):
    """Exclusive scan: offsets[s] = global packed position of stream s (count+1)."""
    import torch

    z = torch.zeros(1, dtype=torch.int64, device=global_sizes.device)
    return torch.cat([z, torch.cumsum(global_sizes, 0)])


def rank_bytes(offsets, count: int, world: int) -> list[tuple[int, int]]:
    """(base, length) of every rank's packed shard in the global output."""
    o = offsets.cpu().tolist() if hasattr(offsets, "cpu") else list(offsets)
    res = []
    for k in range(world):
        a, b = count * k // world, count * (k + 1) // world
        res.append((int(o[a]), int(o[b]) - int(o[a])))
    return res


def gather_payload(packed_local, offsets, count: int, r: Rank, out=None, root: int = 0):
    """Rank `root` receives every rank's packed shard (packed_local[:length])
    at its global offset into `out` (allocated if None, offsets[-1] bytes);
    other ranks send.  Returns `out` on the root, None elsewhere."""
    import torch

    spans = rank_bytes(offsets, count, r.world)
    if r.rank == root:
        if out is None:
            out = torch.empty(max(1, spans[-1][0] + spans[-1][1]), dtype=torch.uint8, device=packed_local.device)
        base, n = spans[root]
        out[base : base + n].copy_(packed_local[:n])
    if not _collective(r) or r.world == 1:
        return out
    import torch.distributed as dist

    ops = []
    if r.rank == root:
        for k, (base, n) in enumerate(spans):
            if k != root and n:
                ops.append(dist.P2POp(dist.irecv, out[base : base + n], k))
    else:
        n = spans[r.rank][1]
        if n:
            ops.append(dist.P2POp(dist.isend, packed_local[:n], root))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return out if r.rank == root else None


def reduce_max(values, r: Rank, device=None) -> list[float]:
    """Element-wise max over ranks (timing: the job ends with its slowest rank)."""
    if not _collective(r):
        return [float(v) for v in values]
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def reduce_sum(values, r: Rank, device=None) -> list[int]:
    """Element-wise sum over ranks (bytes processed / produced by the job)."""
    if not _collective(r):
        return [int(v) for v in values]
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return [int(v) for v in t.tolist()]


def barrier(r: Rank):
    if _collective(r):
        import torch.distributed as dist

        dist.barrier()
