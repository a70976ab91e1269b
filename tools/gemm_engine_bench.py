"""Split-bf16 GEMM main loops on the model's shapes: LDS-ring tiles vs LDS-resident panels
(isolated launches, torch events).  Usage (GPU box): python tools/gemm_engine_bench.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

# (name, M, N, K, epilogue, lda) per 16-clip half step (M = 16 x 501) and the full 32 clips
SHAPES = [("in_proj", 768, 192, "none", None), ("x_dt", 512, 384, "softplus", 768), ("out_proj", 192, 384, "residual", None),
          ("ffn1", 384, 192, "gelu", None), ("ffn2", 192, 384, "residual", None), ("head_argmax", 1000, 192, "argmax", None)]


def timed(fn, iters=30):
    for _ in range(3):
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
    engines = ("tiles",) if sys.argv[1:] == ["tiles"] else ("tiles", "panel", "panel2")
    E = {"none": _lib.EPI_NONE, "softplus": _lib.EPI_SOFTPLUS_FROM, "residual": _lib.EPI_RESIDUAL, "gelu": _lib.EPI_GELU}
    for M in (8016, 16032):
        tot = {"tiles": 0.0, "panel": 0.0, "panel2": 0.0}
        for name, N, K, epi, lda in SHAPES:
            a_full = torch.randn(M, lda or K, device="cuda")
            a = a_full[:, :K]
            w = torch.randn(N, K, device="cuda") / K ** 0.5
            b = torch.randn(N, device="cuda")
            kw = {}
            if epi == "softplus":
                kw["n_out"] = 128
            if epi == "residual":
                kw["aux"] = torch.randn(M, N, device="cuda")
            if epi == "argmax":
                fn = lambda: ops.gemm_argmax(a, w, b)  # noqa: E731
            else:
                fn = lambda: ops.gemm(a, w, b, epilogue=E[epi], **kw)  # noqa: E731
            res = {}
            for eng in engines:
                prev = ops.set_x3_engine(eng)
                res[eng] = timed(fn)
                ops.set_x3_engine(prev)
                tot[eng] += res[eng]
            fl = 2.0 * M * N * K * 6
            print(f"M={M:5d} {name:12s} N={N:4d} K={K}: " + "  ".join(f"{e} {res[e]:6.1f} us" for e in engines)
                  + f"  ({fl / res['tiles'] / 1e6:.0f} bf16-TF/s tiles)", flush=True)
        print(f"M={M:5d} per-SSM-block set (+head): " + "  ".join(f"{e} {tot[e]:.1f} us" for e in engines))


if __name__ == "__main__":
    main()
