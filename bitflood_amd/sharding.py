"""Chunk-range sharding across GPUs.

Chunks are independent, so N GPUs take contiguous index ranges of the global
chunk list (files concatenated in EncodeFile order) with no data-path
collective; each rank hashes its range and the digests are assembled in index
order.  The only collectives are for assembly/timing (all_gather of digest
slices, max of elapsed times) -- nothing is exchanged while hashing.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_chunks: int, rank: int, world: int) -> tuple[int, int]:
    """[begin, end) of rank's contiguous share; the first n % world ranks get one more."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_chunks, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def gather_digests(local: np.ndarray, n_chunks: int, world: int, group=None) -> np.ndarray:
    """All ranks' (end-begin, 20) digest slices -> the full (n_chunks, 20) array
    on every rank, in chunk order.  Uses torch.distributed (gloo or nccl)."""
    import torch
    import torch.distributed as dist

    assert local.dtype == np.uint8 and local.ndim == 2 and local.shape[1] == 20
    counts = [shard_range(n_chunks, r, world) for r in range(world)]
    longest = max(e - b for b, e in counts)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    pad = np.zeros((longest, 20), dtype=np.uint8)
    pad[: local.shape[0]] = local
    t = torch.from_numpy(pad).to(dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    out = np.empty((n_chunks, 20), dtype=np.uint8)
    for (b, e), p in zip(counts, parts):
        out[b:e] = p.cpu().numpy()[: e - b]
    return out


def max_over_ranks(x: float, world: int, group=None) -> float:
    """The bench's clock: the slowest rank's time (a collective whenever a
    process group is formed, even of one rank)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        if world != 1:
            raise RuntimeError("max_over_ranks: world > 1 without a process group")
        return float(x)
    import torch
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
