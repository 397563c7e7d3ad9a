"""Multi-GPU sharding of a granule batch.

Streams are independent (the reference decodes each mp3.Decoder serially and
shares nothing between decoders, decode.go:27-33), so a batch shards across
ranks BY STREAM with no data-path collective: rank r decodes a contiguous
block of streams on its own GPU (one process per GPU).  The only collective
is the optional PCM gather to rank 0 over RCCL (xGMI), reported separately
from the decode throughput.

These helpers are backend-agnostic (RCCL on the GPUs, gloo in the CPU tests).
"""
import numpy as np

from . import STREAM_DTYPE

__all__ = ["shard_bounds", "shard_streams", "gather_pcm", "max_over_ranks"]


def shard_bounds(n_items, world, rank):
    """Contiguous block [lo, hi) of `n_items` owned by `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(int(n_items), world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_streams(streams, world, rank):
    """Streams of this rank and the granule range they cover.

    Returns (local_streams, g_lo, g_hi): local_streams is a STREAM_DTYPE table
    rebased so that granule g_lo of the global arrays is local granule 0;
    the rank decodes granules[g_lo:g_hi].  Requires the streams' granule
    ranges to be ascending and non-overlapping (as mp3g.streams_for builds).
    """
    streams = np.ascontiguousarray(streams, dtype=STREAM_DTYPE)
    lo, hi = shard_bounds(len(streams), world, rank)
    mine = streams[lo:hi].copy()
    if len(mine) == 0:
        return mine, 0, 0
    first = mine["first_granule"].astype(np.int64)
    ends = first + mine["n_granules"].astype(np.int64)
    if np.any(first[1:] < ends[:-1]):
        raise ValueError("streams overlap or are not ascending")
    g_lo, g_hi = int(first[0]), int(ends.max())
    mine["first_granule"] = first - g_lo
    return mine, g_lo, g_hi


def max_over_ranks(value, device=None):
    """MAX of a float over all ranks (the bench's timing rule)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_pcm(pcm, dst=0):
    """Gather every rank's PCM (1-D int16/uint8 tensor, sizes may differ) to
    `dst`; returns the concatenation in rank order on dst, None elsewhere.
    One padded collective: sizes first, then a single gather of max-size
    buffers (xGMI is point-to-point, so one large transfer per link beats
    many small ones)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    dtype = pcm.dtype
    flat = pcm.reshape(-1).view(torch.uint8)  # neither gloo nor RCCL has an int16 type
    n = torch.tensor([flat.numel()], dtype=torch.int64, device=flat.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes) if sizes else 0
    buf = torch.zeros(cap, dtype=flat.dtype, device=flat.device)
    buf[:flat.numel()] = flat
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, bufs, dst=dst)
    if rank != dst:
        return None
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)]).view(dtype)
