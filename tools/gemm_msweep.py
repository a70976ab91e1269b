#!/usr/bin/env python3
"""Diagnostic: the composed SSM-head GEMM (N = 1280, K = 192, softplus on the dt columns) timed
alone over M, to separate tile-count quantisation (tiles vs 2 blocks x 256 CUs) from per-tile cost.
Usage: gemm_msweep.py [M ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import _lib, ops  # noqa: E402


def main():
    Ms = [int(v) for v in sys.argv[1:]] or [2048, 4096, 6528, 8016, 8192, 9856, 12288, 13056, 16032]
    K, N = 192, 1280
    w = torch.randn(N, K, device="cuda") * 0.05
    b = torch.zeros(N, device="cuda")
    for M in Ms:
        a = torch.randn(M, K, device="cuda")
        f = lambda: ops.gemm(a, w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=896)
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 50 * 1e3
        tiles = ((M + 127) // 128) * (N // 128)
        print(f"M={M:6d} tiles128={tiles:5d} ({tiles / 512:.2f} rounds) {us:7.1f} us  {us / tiles * 512:6.2f} us per 512 tiles",
              flush=True)


if __name__ == "__main__":
    main()
