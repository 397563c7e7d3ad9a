"""Multi-rank path on CPU (gloo, world_size 2 and 3): stream sharding, the
max-over-ranks timing rule and the PCM gather to rank 0.

The per-rank "decode" here is the oracle (test infrastructure standing in for
the GPU kernel, which the driver exercises over RCCL at round end); what is
checked is the plumbing: shards partition the batch exactly, gathered PCM in
rank order equals the full-batch decode byte for byte.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import mp3g
from mp3g import dist as mdist
from mp3g import synth


def test_shard_bounds_partition():
    for n in (0, 1, 5, 8, 1024, 1025):
        for world in (1, 2, 3, 8):
            spans = [mdist.shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        mdist.shard_bounds(4, 2, 2)


def test_shard_streams_rebases():
    s = mp3g.streams_for([4, 0, 6, 2, 8], mp3g.STATE_OUT)
    seen = []
    for r in range(3):
        loc, lo, hi = mdist.shard_streams(s, 3, r)
        for row in loc:
            seen.append((int(row["first_granule"]) + lo, int(row["n_granules"])))
            assert row["first_granule"] + row["n_granules"] <= hi - lo
    assert seen == [(int(a), int(b)) for a, b in zip(s["first_granule"], s["n_granules"])]
    bad = s.copy()
    bad["first_granule"][2] = 1
    with pytest.raises(ValueError):
        mdist.shard_streams(bad, 1, 0)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        g, c, s = synth.synth_batch(5, 12, seed=3, p_mixed=0.3)
        loc, lo, hi = mdist.shard_streams(s, world, rank)
        pcm, _ = oracle.dsp_streams(g[lo:hi], c[lo:hi], loc) if hi > lo else (np.zeros((0, 576, 2), np.int16), None)
        t = mdist.max_over_ranks(0.5 + rank)
        out = mdist.gather_pcm(torch.from_numpy(np.ascontiguousarray(pcm).reshape(-1)))
        if rank == 0:
            want, _ = oracle.dsp_streams(g, c, s)
            q.put(("ok", t, bool(np.array_equal(out.numpy().reshape(-1, 576, 2), want))))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shard_and_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, t, same = q.get(timeout=5)
    assert status == "ok"
    assert t == 0.5 + (world - 1)  # max over ranks
    assert same, "gathered PCM differs from the full-batch decode"
