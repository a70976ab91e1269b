"""Isolated timings of the HBM-bound row kernels at the bench's shapes (C = 192 token rows):
LayerNorm, LN + causal depthwise conv, the log-mel normalisation.  Usage: python tools/rowops_bench.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402


def timed(fn, iters=20, reps=5):
    """Per-call device time from a HIP graph of `iters` calls (no host launch overhead)."""
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (iters * reps)


def digest(t):
    """Order-independent bit digest of a float tensor (variants compared bitwise)."""
    return int(t.contiguous().view(torch.int32).to(torch.int64).sum().item()) & 0xFFFFFFFF


def main():
    _lib.require_device()
    C, L = 192, 501
    g = torch.Generator(device="cuda").manual_seed(7)
    w, bb = torch.randn(C, device="cuda", generator=g), torch.randn(C, device="cuda", generator=g)
    cw, cb = torch.randn(C, 4, device="cuda", generator=g), torch.randn(C, device="cuda", generator=g)
    for B in (1, 16, 32):
        x = torch.randn(B, L, C, device="cuda", generator=g)
        byt = 2 * x.numel() * 4
        t_ln = timed(lambda: ops.layer_norm(x, w, bb))
        t_dw = timed(lambda: ops.ln_dwconv(x, w, bb, cw, cb))
        d_ln, d_dw = digest(ops.layer_norm(x, w, bb)), digest(ops.ln_dwconv(x, w, bb, cw, cb))
        print(f"B={B}: layer_norm {t_ln:.2f} us ({byt / t_ln / 1e3:.0f} GB/s), ln_dwconv {t_dw:.2f} us "
              f"({byt / t_dw / 1e3:.0f} GB/s) digests {d_ln:08x} {d_dw:08x}", flush=True)


if __name__ == "__main__":
    main()
