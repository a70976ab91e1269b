"""Fused SSMBlock tail vs the unfused launches it replaces, isolated, at the bench's launch
shapes (M = 8016 and 16032 token rows), and its workgroup forms (VASR_OPT_TAIL_ROWS x
VASR_OPT_TAIL_WAVES).  Usage (GPU box): python tools/tail_bench.py [M ...]"""
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
    g0 = torch.Generator(device="cuda").manual_seed(0)
    rn = lambda *s, sc=1.0: torch.randn(*s, device="cuda", generator=g0) * sc  # noqa: E731
    wo, w1, w2 = rn(192, 384, sc=0.05), rn(384, 192, sc=0.07), rn(192, 384, sc=0.05)
    lw, lb, b1, b2 = 1 + rn(192, sc=0.1), rn(192, sc=0.1), rn(384, sc=0.1), rn(192, sc=0.1)
    for M in [int(a) for a in sys.argv[1:]] or (8016, 16032):
        g, x = rn(M, 384), rn(M, 192)

        def fused():
            return ops.ssm_block_tail(g, x, wo, lw, lb, 1e-5, w1, b1, w2, b2)

        def plain():
            x1 = ops.gemm(g, wo, epilogue=_lib.EPI_RESIDUAL, aux=x)
            f = ops.gemm(x1, w1, b1, epilogue=_lib.EPI_GELU, ln=(lw, lb, 1e-5))
            return ops.gemm(f, w2, b2, epilogue=_lib.EPI_RESIDUAL, aux=x1)
        tf, tp = timed(fused), timed(plain)
        ref = fused()
        err = (ref - plain()).abs().max().item()
        print(f"M={M}: fused tail {tf:.1f} us, unfused (3 GEMMs + LN) {tp:.1f} us, max |diff| {err:.2e}", flush=True)
        # workgroup forms (rows x waves): same arithmetic per output, bitwise equal
        for rows in (16, 32):
            for waves in (4, 6, 12):
                with ops.option(_lib.OPT_TAIL_ROWS, rows), ops.option(_lib.OPT_TAIL_WAVES, waves):
                    t = timed(fused)
                    same = torch.equal(fused(), ref)
                print(f"M={M}: rows {rows} waves {waves:2d}: {t:6.1f} us{'' if same else '  MISMATCH'}", flush=True)


if __name__ == "__main__":
    main()
