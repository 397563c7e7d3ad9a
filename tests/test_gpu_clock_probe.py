"""mp3g_debug_clock_probe (diagnostic; bench.py's `roofline.box_clock`,
DESIGN.md section 12): one-wave workgroups on a side stream read s_memtime and
s_memrealtime while other work runs and stop on a device flag set after it, or
after max_ms.  The shader clock they report must be a plausible gfx950 clock
and every probe must see the flag; without the flag they end at max_ms."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rows(out, n):
    r = out.view(n, 5).cpu().numpy().astype(np.float64)
    return r[:, 1] - r[:, 0], r[:, 3] - r[:, 2], r[:, 4]


def test_probe_beside_a_plan(gpu):
    import torch
    from mp3g import synth
    dev = torch.device("cuda:0")
    g, c, s = synth.synth_batch(16, 400, seed=3)
    d_g = torch.from_numpy(g.view(np.uint8).copy()).to(dev)
    d_c = torch.from_numpy(c.reshape(-1).copy()).to(dev)
    d_p = torch.empty(len(g) * 1152, dtype=torch.int16, device=dev)
    plan = gpu.Plan(s, mode=gpu.MODE_FAST)
    main, side = torch.cuda.current_stream(dev), torch.cuda.Stream(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.zeros(8 * 5, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    gpu.clock_probe(flag, out, 8, 5000, stream=side.cuda_stream)
    for _ in range(20):
        plan.execute(d_g, d_c, d_p, stream=main.cuda_stream)
    flag.fill_(1)
    torch.cuda.synchronize(dev)
    plan.close()
    dt, dr, seen = _rows(out, 8)
    assert (seen == 1).all() and (dr > 0).all()
    ghz = dt / dr * 0.1
    assert ((ghz > 0.5) & (ghz < 3.0)).all(), ghz
    assert dr.max() < 5000 * 1e5  # ended by the flag, not by max_ms


def test_probe_times_out_without_flag(gpu):
    import torch
    dev = torch.device("cuda:0")
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.zeros(2 * 5, dtype=torch.int64, device=dev)
    gpu.clock_probe(flag, out, 2, 20)
    torch.cuda.synchronize(dev)
    dt, dr, seen = _rows(out, 2)
    assert (seen == 0).all()
    assert ((dr >= 20 * 1e5) & (dr < 20 * 1e5 + 1e6)).all(), dr  # 20 ms of 100-MHz ticks (+ < 10 ms)
    with pytest.raises(ValueError):
        gpu.clock_probe(flag, out, 3, 20)  # 3 probes need 15 words
    with pytest.raises(gpu.Mp3gError):
        gpu.clock_probe(flag, torch.zeros(5 * 2000, dtype=torch.int64, device=dev), 2000, 20)  # > 1024 waves
