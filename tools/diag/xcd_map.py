#!/usr/bin/env python3
"""Which XCD (XCC_ID register) each workgroup of a launch runs on (vasr_probe_clock), for a few
launch sizes: the scan's and the tile GEMM's XCD-aware block maps assume workgroup i runs on
XCD i % 8 (round-robin dispatch)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()
for blocks, iters in ((64, 1000), (768, 1000), (768, 20000), (2048, 20000), (6144, 2000)):
    for rep in range(2):
        out = torch.zeros(3 * blocks, device=dev, dtype=torch.int64)
        _lib.check(lib.vasr_probe_clock(out.data_ptr(), blocks, iters, torch.cuda.current_stream(dev).cuda_stream),
                   "vasr_probe_clock")
        x = out.view(blocks, 3)[:, 0].cpu()
        rr = [(x == (torch.arange(blocks) + k) % 8).double().mean().item() for k in range(8)]
        perm = {}
        for i in range(min(blocks, 64)):
            perm.setdefault(i % 8, set()).add(int(x[i]))
        print(f"blocks {blocks:5d} iters {iters:6d} rep {rep}: first 32 xcc {x[:32].tolist()}")
        print(f"    fraction with xcc == (i + k) % 8 for k = 0..7: {[round(v, 3) for v in rr]}; "
              f"i % 8 -> xcc over the first 64: {dict(sorted((k, sorted(v)) for k, v in perm.items()))}")
