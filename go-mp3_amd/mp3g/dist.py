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

__all__ = ["shard_bounds", "shard_streams", "shard_frames", "halo_start", "gather_pcm", "max_over_ranks"]


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


def _stereo(headers):
    return ((np.asarray(headers, dtype=np.uint32) >> 6) & 3) != 3  # frameheader.go:86-105 (mode 3 = mono)


def halo_start(granules, g, stream_first=0):
    """First granule a decode must start from, with zero state, so that its
    state at granule `g` equals the serial decode's: the plans' replay rule
    (granule_fast.hip prologue, DESIGN.md "halo").  store after g-1 is a
    function of granule g-1 and vVec of granules g-2 and g-1
    (frame.go:473-476, :637-652), so two granules back -- but a mono granule
    leaves channel 1 untouched (Decode works on ch < nch, frame.go:125-133),
    so channel 1's state comes from the two latest stereo granules before g.
    (Conservative: always covers channel 1.)"""
    g, s0 = int(g), int(stream_first)
    if g <= s0:
        return s0
    start0 = max(s0, g - 2)
    hdr = granules["header"] if granules.dtype.names else granules
    st = _stereo(hdr[s0:g])  # index i <-> granule s0 + i
    if len(st) >= 2 and st[-1] and st[-2]:
        return start0
    idx = np.nonzero(st)[0]
    start1 = s0 + int(idx[-2]) if len(idx) >= 2 else s0
    return min(start0, start1)


def shard_frames(granules, world, rank, stream_first=0, n_granules=None):
    """Contiguous granule ranges of ONE long stream ("for long
    single streams, shard by contiguous frame ranges and duplicate 2 halo
    granules"): rank r outputs granules [lo, hi) of the stream and decodes
    [h, hi) from zero state, h = halo_start(lo), discarding the PCM of the
    halo [h, lo).  Bit-identical to the serial decode in exact mode (and to a
    one-GPU fast decode in fast mode).  A stream with state_in is not
    supported (its halo would need the state at h).  Returns (h, lo, hi) in
    global granule indices."""
    n = len(granules) - int(stream_first) if n_granules is None else int(n_granules)
    lo, hi = shard_bounds(n, world, rank)
    lo += int(stream_first)
    hi += int(stream_first)
    if hi == lo:
        return lo, lo, hi
    return halo_start(granules, lo, stream_first), lo, hi


def max_over_ranks(value, device=None):
    """MAX of a float over all ranks (the bench's timing rule)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# Largest single point-to-point message of gather_pcm: a rank's c4 slice is
# 4.83 GB (2^32 + bytes, more than a 32-bit element count), so every transfer
# goes as pieces of at most this many bytes, matched in order on both sides
# (RCCL and gloo keep the order of messages between one pair of ranks).
GATHER_PIECE_BYTES = 1 << 30


def _pieces(n, piece):
    return [(a, min(a + piece, n)) for a in range(0, n, piece)]


def gather_pcm(pcm, dst=0, out=None, piece_bytes=None):
    """Gather every rank's PCM (a 1-D tensor of any dtype, sizes may differ) to
    `dst`: returns `out` -- the concatenation in rank order, as raw bytes
    viewed as pcm's dtype -- on dst, None elsewhere.

    The sizes go first (one small all_gather); then every other rank sends its
    PCM point-to-point straight into its slice of ONE output buffer on dst
    (preallocated by the caller as `out`, or allocated here), and dst copies
    its own part into place.  No per-rank staging buffers and no concatenation
    copy: at c4 that is 38.65 GB written once on rank 0.  xGMI
    is point-to-point, so the world - 1 transfers run concurrently on rank 0's
    links, each in pieces of at most GATHER_PIECE_BYTES (piece_bytes
    overrides).  Works on GPU tensors under RCCL and on CPU tensors under gloo.
    """
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    if rank == dst and out is not None and not out.is_contiguous():
        # (reshape would receive into a copy and leave `out` unfilled)
        raise ValueError("gather_pcm: out must be contiguous")
    dtype = pcm.dtype
    flat = pcm.contiguous().reshape(-1).view(torch.uint8)  # neither gloo nor RCCL has an int16 type
    n = torch.tensor([flat.numel()], dtype=torch.int64, device=flat.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    piece = int(piece_bytes or GATHER_PIECE_BYTES)
    if rank != dst:
        if flat.numel():
            ops = [dist.P2POp(dist.isend, flat[a:b], dst) for a, b in _pieces(flat.numel(), piece)]
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return None
    total = sum(sizes)
    if out is None:
        out_b = torch.empty(total, dtype=torch.uint8, device=flat.device)
    else:
        out_b = out.reshape(-1).view(torch.uint8)
        if out_b.numel() < total or out_b.device != flat.device:
            raise ValueError(f"gather_pcm: out holds {out_b.numel()} B on {out_b.device}, "
                             f"need {total} B on {flat.device}")
        out_b = out_b[:total]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    ops = [dist.P2POp(dist.irecv, out_b[int(offs[r]) + a:int(offs[r]) + b], r)
           for r in range(world) if r != dst and sizes[r] for a, b in _pieces(sizes[r], piece)]
    reqs = dist.batch_isend_irecv(ops) if ops else []
    out_b[int(offs[dst]):int(offs[dst + 1])].copy_(flat)
    for req in reqs:
        req.wait()
    return out_b.view(dtype) if out is None else out
