"""The multi-GPU path on real hardware: RCCL ("nccl") process groups with the real HIP step.

Only one GPU is available to the tests, so the RCCL path runs at world size 1 in a child
process (scatter from rank 0, HIP graphs, gather), and bench.py's launcher is exercised end
to end with --gpus 1 (torch.distributed.run as a child, one rank).  The sharded form at world
size 2 (C3's partitioning: rank r transcribes its own slice of the batch) runs with both ranks
on the one GPU over a gloo group (RCCL refuses two ranks on one device): real HIP steps,
host-side scatter/gather.  The 8-GPU RCCL run is the driver's scaling bench."""

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import PKG_ROOT, REPO, golden_json

pytestmark = pytest.mark.gpu

CHILD = r'''
import json, os, sys
sys.path[:0] = [{pkg!r}, {repo!r}]
import torch, torch.distributed as dist
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
import velocity_asr as va
from velocity_asr import synthetic as S
from velocity_asr.distributed import graphed_step, hip_step, transcribe_sharded
from velocity_asr.pipeline import GraphedTranscriber, token_lists
m = va.VELOCITYASR()
m.load_state_dict({{k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}}, strict=True)
m = m.to(dev).eval()
audio = torch.from_numpy(S.make_audio(2, 160000, seed=1234)).to(dev)
eager = transcribe_sharded(hip_step(m), audio, 2, 160000, dev)
tr = GraphedTranscriber(m, 2, 160000, dev, streams=2)
graphed = transcribe_sharded(graphed_step(tr), audio, 2, 160000, dev, shard=tr.audio)
blocks = transcribe_sharded(graphed_step(tr), audio, 2, 160000, dev, shard=tr.audio, as_lists=False)
print("RESULT " + json.dumps(dict(eager=eager, graphed=graphed, blocks=token_lists(*blocks))), flush=True)
dist.destroy_process_group()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", LOCAL_RANK="0",
               WORLD_SIZE="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def test_rccl_sharded_transcription_world1_matches_reference():
    """transcribe_sharded with the real HIP step (eager and graphed) through an RCCL group:
    tokens equal the reference's greedy lists for the same clips (decode_fwd.json b2_10s)."""
    r = subprocess.run([sys.executable, "-c", CHILD.format(pkg=PKG_ROOT, repo=REPO)], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    exp = golden_json("decode_fwd.json")["results"]["b2_10s"]
    assert res["eager"] == exp
    assert res["graphed"] == exp
    assert res["blocks"] == exp


def test_bench_launcher_one_gpu():
    """bench.py --gpus 1 goes through torch.distributed.run (child process), joins an RCCL
    group, runs the resident and the scatter/gather legs and prints one JSON line."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
                        "--roofline-steps", "1", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                       timeout=400, cwd=REPO)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # ONE JSON line, no banners
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert "RCCL" in d["config"]["parallelism"]
    assert d["graph_tokens_match_eager"] is True
    assert d["rank0_tokens_match_reference"] is True
    assert d["with_scatter"]["rank0_tokens_match"] is True and d["with_scatter"]["value"] > 0
    for k in ("valu_frac", "hbm_ceiling_frac", "gemm_frac", "gemm_f32eq_frac"):
        assert k in d["roofline"], k


CHILD2 = r"""
import json, os, sys
sys.path[:0] = [{pkg!r}, {repo!r}]
import torch, torch.distributed as dist
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)  # both ranks share the one GPU
torch.cuda.set_device(dev)
import velocity_asr as va
from velocity_asr import synthetic as S
from velocity_asr.distributed import hip_step, shard_range, transcribe_sharded
from velocity_asr.pipeline import audio_to_token_ids, token_lists
res = {{}}
for dtype in ("f32", "bf16"):
    m = va.VELOCITYASR()
    m.load_state_dict({{k: torch.from_numpy(v) for k, v in S.make_weights(None, seed=0).items()}}, strict=True)
    m = m.to(dev).eval()
    if dtype == "bf16":
        m = m.to(torch.bfloat16)  # BASELINE C3: the bf16 model, 32 clips per GPU
    step = hip_step(m)

    def host_step(shard):  # gloo moves host tensors: shard to the GPU, tokens back
        t, n = step(shard.to(dev))
        return t.cpu(), n.cpu()

    audio = torch.from_numpy(S.make_audio(4, 160000, seed=1234)) if rank == 0 else None
    lists = transcribe_sharded(host_step, audio, 4, 160000, torch.device("cpu"))
    if rank == 0:
        # the same 4 clips in one unsharded batch on this process
        whole = token_lists(*audio_to_token_ids(m, audio.to(dev)))
        res[dtype] = dict(sharded=lists, whole=whole)
    lo, hi = shard_range(4, world, rank)
    res.setdefault("ranges", {{}})[dtype] = [lo, hi]
if rank == 0:
    print("RESULT " + json.dumps(res), flush=True)
dist.destroy_process_group()
"""


def test_two_rank_sharded_transcription_one_gpu(tmp_path):
    """World size 2 with both ranks on the one GPU (gloo transport): each rank runs the real
    HIP step on its half of the batch; rank 0's gathered token lists equal the reference's for
    the fp32 model (the bench's first 4 clips, tests/golden/fwd_fullbatch.npz) and, for the
    bf16 model (C3), the unsharded batch on the same device."""
    from conftest import golden
    script = tmp_path / "child2.py"
    script.write_text(CHILD2.format(pkg=PKG_ROOT, repo=REPO))
    env = _env()
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", env["MASTER_PORT"], str(script)],
                       env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    exp = json.loads(str(golden("fwd_fullbatch.npz")["greedy"]))["c2"][:4]
    assert res["f32"]["sharded"] == exp
    assert res["f32"]["whole"] == exp
    assert res["bf16"]["sharded"] == res["bf16"]["whole"]
    assert res["ranges"]["f32"] == [0, 2]
