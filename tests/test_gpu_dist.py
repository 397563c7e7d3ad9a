"""The product path under a process group: ranks that decode
their shards through the C-ABI plans on the GPU and gather the PCM to rank 0.

The ranks run in a fresh interpreter (tests/dist_gpu_worker.py) that spawns
them before anything touches the GPU; they share cuda:0 and a gloo group (the
8-GPU RCCL run is the driver's).  Checked there by rank 0: stream shards
gathered = the oracle's decode byte for byte; frame-range shards of one long
stream with halos (mp3g.dist.shard_frames) = the oracle byte for byte in exact
mode and = the one-GPU fast decode in fast mode (within +-1 LSB of the
oracle); max over ranks.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world", [2, 3])
def test_product_multi_rank(world):
    r = subprocess.run([sys.executable, os.path.join(HERE, "dist_gpu_worker.py"), "--world", str(world)],
                       capture_output=True, text=True, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(lines[-1])
    print(res)
    assert r.returncode == 0 and res["ok"], res
