"""Multi-process plumbing of utterance sharding (gloo, world_size 2, CPU).

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
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_transcription_matches_single_process(world):
    rng = np.random.default_rng(0)
    audio = torch.from_numpy(rng.standard_normal((6, 3200)).astype(np.float32))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, audio, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    toks, lens = fake_step(audio)
    expect = [toks[b, : lens[b]].tolist() for b in range(audio.shape[0])]
    assert res == expect


def test_shard_range_partitions():
    for n in (1, 7, 32, 256):
        for w in (1, 2, 3, 8):
            cover = []
            for r in range(w):
                s, e = shard_range(n, w, r)
                cover.extend(range(s, e))
            assert cover == list(range(n))
    assert shard_range(256, 8, 3) == (96, 128)
