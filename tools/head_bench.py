"""Fused SSMBlock head vs the three launches it replaces, isolated, at the bench's launch shape
(16 clips x 501 tokens).  Usage (GPU box): python tools/head_bench.py [B]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    _lib.require_device()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    L = 501
    g0 = torch.Generator(device="cuda").manual_seed(0)
    rn = lambda *s, sc=1.0: torch.randn(*s, device="cuda", generator=g0) * sc  # noqa: E731
    x = rn(B * L, 192)
    lw, lb, cw, cb = 1 + rn(192, sc=0.1), rn(192, sc=0.1), rn(192, 4, sc=0.3), rn(192, sc=0.1)
    win, wxd = rn(768, 192, sc=0.07), rn(512, 384, sc=0.05)
    bxd = torch.cat([torch.zeros(128, device="cuda"), rn(384, sc=0.1)])

    def fused():
        return ops.ssm_block_head(x, B, L, lw, lb, 1e-5, cw, cb, win, wxd, bxd, 128)

    def ln_conv():
        return ops.ln_dwconv(x.view(B, L, 192), lw, lb, cw, cb, 1e-5)

    u = ln_conv().view(B * L, 192)

    def inproj():
        return ops.gemm(u, win)
    xz = inproj()

    def xdt():
        return ops.gemm(xz[:, :384], wxd, bxd, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=128)
    tf, t1, t2, t3 = timed(fused), timed(ln_conv), timed(inproj), timed(xdt)
    print(f"B={B}: fused head {tf:.1f} us; ln_dwconv {t1:.1f} + in_proj {t2:.1f} + x_dt {t3:.1f} = {t1 + t2 + t3:.1f} us",
          flush=True)


if __name__ == "__main__":
    main()
