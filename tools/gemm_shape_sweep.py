#!/usr/bin/env python3
"""Time the split-bf16 GEMM over K (fixed M, N) to separate per-tile overheads from the main loop."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import ops  # noqa: E402


def t(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    M = 16032
    for mode in ("x3", "f32"):
        ops.set_gemm_mode(mode)
        for N in (768, 192):
            for K in (192, 384, 768, 1536, 3072):
                a = torch.randn(M, K, device="cuda")
                w = torch.randn(N, K, device="cuda") * 0.05
                out = torch.empty(M, N, device="cuda")
                us = t(lambda: ops.gemm(a, w, out=out))
                tf = 2 * M * N * K / us / 1e6
                print(f"{mode} M={M} N={N:4d} K={K:5d}: {us:8.1f} us {tf:7.1f} TF/s  "
                      f"({tf * 6 / 2500 * 100 if mode == 'x3' else tf / 157.3 * 100:5.1f}% of MFMA peak)")


if __name__ == "__main__":
    main()
