"""bench.py's multi-rank branch, rehearsed on one GPU.

The driver runs `bench.py --gpus N` under torch.distributed.run on a whole
8-GPU node with RCCL; that branch (process group, barriers, max over ranks,
the timed PCM gather to rank 0 into one preallocated buffer, the gathered
PCM's parity) is exercised here as 2 ranks sharing cuda:0 over gloo, with
the collectives staged through host memory, and as ONE rank over RCCL (a
one-GPU box cannot hold two RCCL ranks: the process group, the barriers, the
device max over ranks and the gather's size exchange run through RCCL; the
point-to-point sends need a second GPU).  torch.distributed.run starts the
ranks as fresh processes; nothing in this test touches the GPU itself.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("config", ["c2"])
def test_bench_two_ranks_gloo(config):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--config", config, "--backend", "gloo", "--single-mode", "--no-bitstream", "--no-polyphase"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:] + r.stderr[-5000:]
    d = json.loads(lines[0])
    print({k: d[k] for k in ("value", "ms_per_step", "n_gpus", "gather_ms", "max_dpcm_lsb")})
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["scaling"] == "weak"
    # the gather is timed apart from the decode and lands every rank's PCM
    assert d["gather_ms"] > 0 and d["gather"]["bytes"] == 2 * 20000 * 2304
    assert d["gather"]["parity"]["max_dpcm_lsb"] <= 1 and len(d["gather"]["parity"]["per_rank"]) == 2
    # rank 0's own timed output against the oracle
    assert d["max_dpcm_lsb"] <= 1 and d["modes"]["fast"]["parity_granules"] > 0
    assert "cpu_baseline" not in d  # an N = 1 figure


def test_bench_gpus_flag_launches_ranks():
    """Plain `bench.py --gpus 2` (no launcher): bench.py starts the two ranks
    itself; gloo, so both share cuda:0."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--config", "c2", "--backend", "gloo", "--single-mode", "--no-bitstream", "--no-polyphase"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:] + r.stderr[-5000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["gather"]["bytes"] == 2 * 20000 * 2304 and d["gather_ms"] > 0
    assert d["gather"]["parity"]["max_dpcm_lsb"] <= 1
    assert d["max_dpcm_lsb"] <= 1


def test_bench_one_rank_rccl():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
           "--config", "c2", "--backend", "nccl", "--single-mode", "--no-bitstream", "--no-polyphase",
           "--cpu-repeats", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:] + r.stderr[-5000:]
    d = json.loads(lines[0])
    print({k: d[k] for k in ("value", "ms_per_step", "n_gpus", "gather_ms", "max_dpcm_lsb")})
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["gather"]["backend"].startswith("RCCL") and d["gather"]["bytes"] == 20000 * 2304
    assert d["gather"]["parity"]["max_dpcm_lsb"] <= 1
    assert d["max_dpcm_lsb"] <= 1


def test_bench_pinned_budget_guard():
    """bench.py's pinned-memory budget per rank: with a
    budget too small for the bitstream leg's pinned buffers, the PCIe pass
    and the pipelined drop-in are skipped and say so, the device leg and its
    oracle parity still run, and 2 gloo ranks gather into pageable memory."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--config", "c2", "--backend", "gloo", "--single-mode", "--no-polyphase", "--no-hot"]
    env = dict(os.environ, OMP_NUM_THREADS="4", MP3G_BENCH_PINNED_GB="0.01")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:] + r.stderr[-5000:]
    d = json.loads(lines[0])
    hm = d["host_memory"]
    legs = {x["leg"] for x in hm["skipped_legs"]}
    assert "bitstream PCIe pass + pipelined drop-in" in legs, hm
    assert any(x.startswith("gloo gather") for x in legs), hm
    assert hm["peak_pinned_gb_by_bench_max_over_ranks"] <= 0.011
    b = d["bitstream"]
    assert b["end_to_end"]["skipped"] and b["end_to_end"]["pipelined_s"] is None and b["decoder_api"] is None
    assert b["huffman_plus_dsp_ms"] > 0 and b["max_dpcm_lsb_vs_oracle"] <= 1
    assert d["gather"]["parity"]["max_dpcm_lsb"] <= 1
