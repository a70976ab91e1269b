#!/usr/bin/env python3
"""Throughput of mixed-length clips (diagnostic): the reference's one-file-at-a-time loop
(scripts/evaluate.py:91-98) vs length-sorted zero-padded batches with per-clip lengths
(pipeline.audio_to_token_ids(..., lengths=)), both eager, audio resident on the device.
Clip lengths follow a LibriSpeech-test-clean-like spread (log-normal, mean ~7.5 s, clipped to
1.3-35 s).  Checks that both give the same tokens for every clip.

Usage: python tools/ragged_bench.py [n_clips] [batch]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import velocity_asr as va  # noqa: E402
from velocity_asr import synthetic as S  # noqa: E402
from velocity_asr.pipeline import audio_to_token_ids, token_lists  # noqa: E402

SR = 16000


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    dev = torch.device("cuda:0")
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(dev).eval()
    rng = np.random.default_rng(2024)
    secs = np.clip(rng.lognormal(np.log(6.0), 0.6, n), 1.3, 35.0)
    lens = [int(s * SR) for s in secs]
    clips = [torch.from_numpy(S.make_audio(1, L, seed=i)[0]).to(dev) for i, L in enumerate(lens)]
    total_s = sum(lens) / SR

    def per_file():
        return [token_lists(*audio_to_token_ids(m, c[None]))[0] for c in clips]

    order = sorted(range(n), key=lambda i: lens[i])

    def ragged():
        out = [None] * n
        for k in range(0, n, batch):
            idx = order[k:k + batch]
            S_ = max(lens[i] for i in idx)
            a = torch.zeros((len(idx), S_), device=dev)
            for j, i in enumerate(idx):
                a[j, :lens[i]] = clips[i]
            res = token_lists(*audio_to_token_ids(m, a, lengths=[lens[i] for i in idx]))
            for j, i in enumerate(idx):
                out[i] = res[j]
        return out

    res = {}
    toks = {}
    for name, fn in (("per_file", per_file), ("ragged", ragged)):
        fn()  # warm-up: caches, kernels
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        toks[name] = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[name] = {"wall_s": round(dt, 4), "rtfx": round(total_s / dt, 1)}
    pad = sum(max(lens[i] for i in order[k:k + batch]) * len(order[k:k + batch]) for k in range(0, n, batch))
    print(json.dumps({"clips": n, "batch": batch, "audio_s": round(total_s, 1),
                      "mean_s": round(float(np.mean(secs)), 2), "padded_fraction": round(1 - sum(lens) / pad, 3),
                      "tokens_equal": toks["per_file"] == toks["ragged"], **res}))


if __name__ == "__main__":
    main()
