"""bench.py's launch decision, on the CPU.

`bench.py --gpus N` with no launcher around it starts N ranks through
torch.distributed.run as a child process; the parent must decide that before
anything imports torch (so it never initialises HIP and never execs).  A
WORLD_SIZE that disagrees with --gpus is an error, not a silent N = 1.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_check_world():
    assert bench.check_world(1, {}) == "run"
    assert bench.check_world(8, {}) == "launch"
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) == "run"
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) == "run"
    assert "disagree" in bench.check_world(8, {"WORLD_SIZE": "1"})
    assert "disagree" in bench.check_world(1, {"WORLD_SIZE": "4"})
    assert ">= 1" in bench.check_world(0, {})


_PARENT = r"""
import os, subprocess, sys
sys.path.insert(0, {repo!r})
os.environ.pop("WORLD_SIZE", None)
calls = []
subprocess.call = lambda cmd, **kw: calls.append(cmd) or 7
sys.argv = ["bench.py", "--gpus", "4", "--config", "c2", "--steps", "2"]
import bench
try:
    bench.main()
except SystemExit as e:
    code = e.code
assert code == 7, code                       # the child's exit code is ours
assert "torch" not in sys.modules, "the launching parent imported torch"
(cmd,) = calls
i = cmd.index("torch.distributed.run")
assert cmd[i - 1] == "-m" and "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
assert cmd[cmd.index("--gpus") + 1] == "4" and cmd[-2:] == ["--steps", "2"]
print("ok")
"""


def test_parent_launches_child_without_torch():
    r = subprocess.run([sys.executable, "-c", _PARENT.format(repo=REPO)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_world_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "disagree" in r.stderr, r.stderr
