"""torch.distributed over RCCL ("nccl" backend), the transport bench.py uses for
N > 1 GPUs: a one-rank process group on the one-GPU box, int64 / float32 MIN
all-reduces and the d-sharded WTA protocol with its exchanges forced through RCCL,
bit-identical to asw_WTA.  Runs in a child process so the process group does not
outlive the test."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_one_rank_protocol():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_one_rank.py"), str(_free_port())],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["backend"] == "nccl"
    assert out["int64_min_ok"] and out["f32_min_ok"]
    assert out["protocol_equals_wta"], out
