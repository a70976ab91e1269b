#!/usr/bin/env python3
"""Time the GEMM engines (split-bf16 "x3" and f32-input MFMA) on the model's GEMM shapes
(C2: B=32 x 10 s -> M = 16032 tokens).  Usage: gemm_bench.py [x3|f32 ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import _lib, ops  # noqa: E402

M = 16032
SHAPES = [  # name, M, N, K, lda, epilogue, n_out
    ("in_proj", M, 768, 192, 192, _lib.EPI_NONE, 0),
    ("x_dt_proj", M, 512, 384, 768, _lib.EPI_SOFTPLUS_FROM, 128),
    ("out_proj+res", M, 192, 384, 384, _lib.EPI_RESIDUAL, 0),
    ("ffn1+gelu", M, 384, 192, 192, _lib.EPI_GELU, 0),
    ("ffn2+res", M, 192, 384, 384, _lib.EPI_RESIDUAL, 0),
    ("ctc_head", M, 1000, 192, 192, _lib.EPI_NONE, 0),
    ("fusion_t1", M, 384, 192, 192, _lib.EPI_NONE, 0),
]


def main():
    for mode in (sys.argv[1:] or ["x3", "f32", "bf16"]):
        if mode != "bf16":
            ops.set_gemm_mode(mode)
        print(f"--- {mode}")
        run(bf16=mode == "bf16")


def run(bf16=False):
    reps = int(os.environ.get("GEMM_REPS", "30"))
    only = os.environ.get("GEMM_SHAPES")
    tot = 0.0
    for name, m, n, k, lda, epi, n_out in SHAPES:
        if only and name not in only.split(","):
            continue
        a = torch.randn(m, lda, device="cuda")[:, :k]
        w = torch.randn(n, k, device="cuda") * 0.05
        if bf16:
            w = w.to(torch.bfloat16)
        b = torch.randn(n, device="cuda")
        aux = torch.randn(m, n, device="cuda") if epi == _lib.EPI_RESIDUAL else None
        out = torch.empty(m, n, device="cuda")
        f = lambda: ops.gemm(a, w, b, epilogue=epi, aux=aux, n_out=n_out, out=out)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        tf = 2 * m * n * k / us / 1e6
        nbytes = 4 * (m * k + m * n * (2 if aux is not None else 1) + n * k)
        tot += us
        print(f"{name:14s} M={m} N={n:4d} K={k}: {us:7.1f} us  {tf:6.1f} TFLOP/s ({tf / 157.3 * 100:4.1f}% of f32 peak)"
              f"  {nbytes / us / 1e3:6.0f} GB/s")
    print(f"sum {tot:.1f} us")


if __name__ == "__main__":
    main()
