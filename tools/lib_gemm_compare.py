"""The split-bf16 fp32 GEMM (vasr_linear_x3_f32) against the vendor libraries on the model's
shapes, isolated (torch.matmul -> hipBLASLt / rocBLAS): bf16 inputs (one product, not
fp32-accurate) and fp32 inputs.  Usage (GPU box): python tools/lib_gemm_compare.py"""
import os, sys, torch
sys.path.insert(0, "velocity-asr_amd")
from velocity_asr import _lib, ops
_lib.require_device()
def timed(fn, iters=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters
g = torch.Generator(device="cuda").manual_seed(0)
for M, N, K in [(8016, 1280, 192), (16032, 1280, 192), (8016, 768, 192), (8016, 512, 384), (8016, 1000, 192)]:
    a = torch.randn(M, K, device="cuda", generator=g); w = torch.randn(N, K, device="cuda", generator=g)
    ab, wb = a.bfloat16(), w.bfloat16()
    t_bf = timed(lambda: ab @ wb.t())
    t_f32 = timed(lambda: a @ w.t())
    t_x3 = timed(lambda: ops.gemm(a, w))
    fl = 2 * M * N * K
    print(f"M={M} N={N} K={K}: torch bf16 {t_bf:.1f}us ({fl/t_bf/1e6:.0f} TF/s)  torch fp32 {t_f32:.1f}us ({fl/t_f32/1e6:.0f} TF/s)  "
          f"vasr x3 {t_x3:.1f}us ({fl/t_x3/1e6:.0f} fp32-TF/s, {6*fl/t_x3/1e6:.0f} bf16-TF/s)", flush=True)
