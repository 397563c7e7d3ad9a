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
        mine = torch.from_numpy(np.ascontiguousarray(pcm).reshape(-1))
        out = mdist.gather_pcm(mine)
        # the same into one preallocated buffer on rank 0 (larger than needed:
        # the tail stays untouched)
        pre = torch.full((len(g) * 1152 + 99,), 7, dtype=torch.int16) if rank == 0 else None
        out2 = mdist.gather_pcm(mine, out=pre)
        # and in small pieces (each rank's slice as several messages matched
        # in order: the 1-GiB pieces of a c4 slice, scaled down)
        out3 = mdist.gather_pcm(mine, piece_bytes=1000)
        if rank == 0:
            want, _ = oracle.dsp_streams(g, c, s)
            same = np.array_equal(out.numpy().reshape(-1, 576, 2), want)
            same2 = out2 is pre and np.array_equal(pre[:len(g) * 1152].numpy().reshape(-1, 576, 2), want) \
                and bool((pre[len(g) * 1152:] == 7).all())
            same3 = np.array_equal(out3.numpy().reshape(-1, 576, 2), want)
            q.put(("ok", t, bool(same and same2 and same3)))
        else:
            assert out is None and out2 is None and out3 is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 6])  # 6 ranks, 5 streams: one rank sends nothing
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


def test_halo_start_rule():
    g, _, _ = synth.synth_batch(1, 20, seed=4)
    assert mdist.halo_start(g, 0) == 0 and mdist.halo_start(g, 1) == 0
    assert mdist.halo_start(g, 10) == 8  # two stereo granules back
    mono = synth.header(synth.MODE_MONO)
    g2 = g.copy()
    g2["header"][[5, 6, 7, 8, 9]] = mono  # channel 1 last touched by granules 3 and 4
    assert mdist.halo_start(g2, 10) == 3
    assert mdist.halo_start(g2, 8) == 3
    g2["header"][:10] = mono  # no stereo granule before 10: channel 1 is zero from the start
    assert mdist.halo_start(g2, 10) == 0


def test_shard_frames_partition_and_oracle_exact():
    """Frame-range shards of one stream decoded from zero state (the oracle
    as the per-rank decoder here; the GPU test runs the product): the halo
    makes every shard's PCM bit-identical to the serial decode's."""
    import oracle
    parts = [synth.synth_stream(31, 30), synth.synth_stream(32, 9, mode=synth.MODE_MONO),
             synth.synth_stream(33, 25)]
    g = np.concatenate([p[0] for p in parts])
    c = np.concatenate([p[1] for p in parts])
    want, _ = oracle.dsp_streams(g, c, mp3g.streams_for([len(g)]))
    for world in (1, 2, 3, 5, 8):
        got = []
        for r in range(world):
            h, lo, hi = mdist.shard_frames(g, world, r)
            assert h <= lo <= hi
            if hi == lo:
                continue
            pcm, _ = oracle.dsp_streams(g[h:hi], c[h:hi], mp3g.streams_for([hi - h]))
            got.append(pcm[lo - h:])
        assert np.array_equal(np.concatenate(got), want), f"world {world}"


def test_gather_rejects_noncontiguous_out():
    """A non-contiguous `out` would be received into a reshape copy and left
    unfilled: gather_pcm refuses it.  One gloo rank, so the
    refusal cannot leave a peer waiting."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        pcm = torch.arange(64, dtype=torch.int16)
        with pytest.raises(ValueError, match="contiguous"):
            mdist.gather_pcm(pcm, out=torch.zeros((64, 2), dtype=torch.int16)[:, 0])
        out = torch.zeros(64, dtype=torch.int16)
        assert mdist.gather_pcm(pcm[::1], out=out) is out and torch.equal(out, pcm)
        # a non-contiguous source is gathered as its values
        src = torch.arange(128, dtype=torch.int16)[::2]
        assert torch.equal(mdist.gather_pcm(src), src)
    finally:
        dist.destroy_process_group()
