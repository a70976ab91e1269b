"""Multi-process plumbing of utterance sharding (gloo, world_size 2 and 8, CPU).

The HIP step is replaced by a CPU stand-in that reproduces the reference's greedy decode
through the oracle on a deterministic fake "logit" function, so the test checks scatter
order, shard boundaries and the token gather, not the kernels (those are -m gpu tests)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from velocity_asr.distributed import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_step(shard):
    """Deterministic per-utterance tokens from audio: argmax over 5 'classes' of frame sums."""
    B, S = shard.shape
    frames = shard[:, : (S // 160) * 160].reshape(B, -1, 160)
    scores = torch.stack([frames[..., k::5].sum(-1) for k in range(5)], -1)  # (B, F, 5)
    pred = scores.argmax(-1)
    toks = torch.zeros_like(pred, dtype=torch.int32)
    lens = torch.zeros(B, dtype=torch.int32)
    for b in range(B):
        out, prev = [], None
        for t in pred[b].tolist():
            if t == 0:
                prev = None
                continue
            if t == prev:
                continue
            out.append(t)
            prev = t
        toks[b, : len(out)] = torch.tensor(out, dtype=torch.int32)
        lens[b] = len(out)
    return toks, lens


def _worker(rank, world, port, audio, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from velocity_asr.distributed import transcribe_sharded
    res = transcribe_sharded(fake_step, audio if rank == 0 else None, audio.shape[0], audio.shape[1],
                             torch.device("cpu"))
    # device-tensor form (the bench's serving leg) into a caller-provided shard buffer
    shard = torch.empty((audio.shape[0] // world, audio.shape[1]))
    blocks = transcribe_sharded(fake_step, audio if rank == 0 else None, audio.shape[0], audio.shape[1],
                                torch.device("cpu"), shard=shard, as_lists=False)
    if rank == 0:
        t, n = blocks
        q.put((res, [t[i, : int(n[i])].tolist() for i in range(t.shape[0])]))
    else:
        assert blocks is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,clips", [(2, 6), (8, 16)])
def test_sharded_transcription_matches_single_process(world, clips):
    """world 8 rehearses C3's layout (an equal utterance shard per rank of one 8-GPU node)."""
    rng = np.random.default_rng(0)
    audio = torch.from_numpy(rng.standard_normal((clips, 3200)).astype(np.float32))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, audio, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, res_blocks = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    toks, lens = fake_step(audio)
    expect = [toks[b, : lens[b]].tolist() for b in range(audio.shape[0])]
    assert res == expect
    assert res_blocks == expect


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N with fewer visible GPUs exits non-zero with a clear message (the
    launcher checks before starting torch.distributed.run)."""
    import subprocess
    import sys
    from conftest import REPO
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "--gpus 4 requested but only 0 GPU(s) are visible" in r.stderr


def test_shard_range_partitions():
    for n in (1, 7, 32, 256):
        for w in (1, 2, 3, 8):
            cover = []
            for r in range(w):
                s, e = shard_range(n, w, r)
                cover.extend(range(s, e))
            assert cover == list(range(n))
    assert shard_range(256, 8, 3) == (96, 128)
