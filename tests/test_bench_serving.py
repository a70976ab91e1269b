"""bench.py's N > 1 ending on the host (gloo, world_size 2, no GPU): the serving leg runs after
rank 0's resident line is complete, and neither an exception on one rank nor a hang loses that
line.  The ranks run bench.finish -- the code run() ends with -- under
torch.distributed.run, with a stand-in serving step."""

import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

_RANK = r"""
import sys, time
from datetime import timedelta
sys.path.insert(0, {repo!r})
import torch.distributed as dist
import bench
dist.init_process_group("gloo", timeout=timedelta(seconds=60))
rank, world = dist.get_rank(), dist.get_world_size()
line = dict(metric="m", value=123.5, n_gpus=world, config=dict(parallelism="p"), with_scatter=None) if rank == 0 else None
def serving():
    if rank == 1 and {mode!r} == "raise":
        raise RuntimeError("forced serving-step failure")
    if rank == 1 and {mode!r} == "hang":
        time.sleep(60)  # a collective that never completes
    return dict(value=99.0, rank0_tokens_match=True)
bench.finish(line, rank, world, True, serving, lambda: 0, 1.0, grace=3.0)
"""


def _launch(tmp_path, mode):
    script = tmp_path / f"rank_{mode}.py"
    script.write_text(_RANK.format(repo=REPO, mode=mode))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(script)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["ok", "raise", "hang"])
def test_serving_leg_cannot_lose_the_line(tmp_path, mode):
    r, lines = _launch(tmp_path, mode)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] == 123.5
    ws = d["with_scatter"]
    if mode == "ok":
        assert ws == dict(value=99.0, rank0_tokens_match=True)
        assert "serving leg scatters" in d["config"]["parallelism"]
    elif mode == "raise":
        assert "rank 1" in ws["error"] and "forced serving-step failure" not in d["config"]["parallelism"]
        assert "serving leg failed" in d["config"]["parallelism"]
    else:
        assert "exceeded" in ws["error"]
