"""Multi-rank run of the PRODUCT path on one GPU (driven by tests/test_gpu_dist.py).

A fresh interpreter that spawns `world` ranks before anything touches the
GPU; every rank joins a gloo process group, decodes its shard through the
C-ABI plans (libmp3g.so, mp3g.Plan) on cuda:0 and gathers the PCM to rank 0
with mp3g.dist.gather_pcm; rank 0 checks the gathered PCM against the oracle
(checker only).  Covered: stream sharding (shard_streams), frame-range
sharding of one long stream with halos (shard_frames) in exact and fast
mode, and the max-over-ranks timing rule.  Prints one JSON line; exit 0 when
every check holds.

  python tests/dist_gpu_worker.py [--world 2]
"""
import argparse
import json
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, "go-mp3_amd"), os.path.join(REPO, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def _decode(mp3g, g, c, streams, mode):
    """Device-resident decode of a shard through mp3g.Plan (the C-ABI plans)."""
    import numpy as np
    import torch
    n = len(g)
    if n == 0:
        return np.zeros((0, 576, 2), np.int16)
    d_g = torch.from_numpy(np.ascontiguousarray(g).view(np.uint8).reshape(-1).copy()).cuda()
    d_c = torch.from_numpy(np.ascontiguousarray(c).reshape(-1).copy()).cuda()
    d_p = torch.zeros(n * 1152, dtype=torch.int16, device="cuda")
    plan = mp3g.Plan(streams, mode=mode)
    plan.execute(d_g, d_c, d_p, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    plan.close()
    return d_p.cpu().numpy().reshape(n, 576, 2)


def _rank(rank, world, port, q):
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mp3g
        from mp3g import dist as mdist
        from mp3g import synth
        res = {}
        # (1) stream sharding: 7 streams of mixed content
        g, c, s = synth.synth_batch(7, 30, seed=41, p_mixed=0.3, p_is=0.3)
        loc, lo, hi = mdist.shard_streams(s, world, rank)
        pcm = _decode(mp3g, g[lo:hi], c[lo:hi], loc, mp3g.MODE_EXACT)
        out = mdist.gather_pcm(torch.from_numpy(np.ascontiguousarray(pcm).reshape(-1)))
        if rank == 0:
            import oracle
            want, _ = oracle.dsp_streams(g, c, s)
            res["streams_exact"] = bool(np.array_equal(out.numpy().reshape(-1, 576, 2), want))
        # (2) one long stream sharded by frame ranges (halo), a mono stretch inside
        parts = [synth.synth_stream(51, 140), synth.synth_stream(52, 25, mode=synth.MODE_MONO),
                 synth.synth_stream(53, 160, p_mixed=0.3)]
        g1 = np.concatenate([p[0] for p in parts])
        c1 = np.concatenate([p[1] for p in parts])
        h, lo, hi = mdist.shard_frames(g1, world, rank)
        for name, mode in (("exact", mp3g.MODE_EXACT), ("fast", mp3g.MODE_FAST)):
            pcm = _decode(mp3g, g1[h:hi], c1[h:hi], mp3g.streams_for([hi - h]), mode)[lo - h:]
            out = mdist.gather_pcm(torch.from_numpy(np.ascontiguousarray(pcm).reshape(-1)))
            if rank == 0:
                import oracle
                got = out.numpy().reshape(-1, 576, 2)
                want, _ = oracle.dsp_streams(g1, c1, mp3g.streams_for([len(g1)]))
                if name == "exact":
                    res["frames_exact"] = bool(np.array_equal(got, want))
                else:
                    one = _decode(mp3g, g1, c1, mp3g.streams_for([len(g1)]), mode)
                    res["frames_fast_equals_one_gpu"] = bool(np.array_equal(got, one))
                    res["frames_fast_max_dpcm"] = int(np.abs(got.astype(np.int32) - want.astype(np.int32)).max())
            res[f"halo_{name}"] = int(lo - h)
        # (3) the bench's timing rule
        res["max_over_ranks"] = mdist.max_over_ranks(1.0 + rank)
        if rank == 0:
            res["world"] = world
            q.put(res)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, args.world, port, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    codes = [p.exitcode for p in procs]
    res = q.get(timeout=10) if all(cd == 0 for cd in codes) else {"exitcodes": codes}
    ok = (all(cd == 0 for cd in codes) and res.get("streams_exact") and res.get("frames_exact")
          and res.get("frames_fast_equals_one_gpu") and res.get("frames_fast_max_dpcm", 9) <= 1
          and res.get("max_over_ranks") == float(args.world))
    res["ok"] = bool(ok)
    print(json.dumps(res), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
