"""Time the split-bf16 GEMM engines (VASR_OPT_GEMM_ENGINE 1 = LDS-ring tiles, 2 = A-rows
stationary) on the model's K = 192 shapes, isolated launches (HIP events, median of 5 x 20).
Usage (GPU box): python tools/gemm_engines.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

SHAPES = [("head_comp", 8016, 1280, "softplus"), ("head_comp_32", 16032, 1280, "softplus"),
          ("head_comp_b1", 501, 1280, "softplus"), ("ctc_argmax", 8016, 1000, "argmax"),
          ("ctc_argmax_b1", 501, 1000, "argmax"), ("in_proj", 8016, 768, "none"), ("pool_proj", 1024, 192, "none"),
          ("ffn1_192", 8016, 384, "gelu")]


def main():
    _lib.require_device()
    only = os.environ.get("GEMM_SHAPES")
    engines = tuple(int(e) for e in os.environ.get("GEMM_ENGINES", "1,2").split(","))
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, epi in SHAPES:
        if only and name not in only.split(","):
            continue
        a = torch.randn(M, 192, device="cuda", generator=g)
        w = torch.randn(N, 192, device="cuda", generator=g) / 192 ** 0.5
        b = torch.randn(N, device="cuda", generator=g)
        if epi == "argmax":
            fn = lambda: ops.gemm_argmax(a, w, b)  # noqa: E731
        else:
            e = {"none": _lib.EPI_NONE, "softplus": _lib.EPI_SOFTPLUS_FROM, "gelu": _lib.EPI_GELU}[epi]
            kw = dict(n_out=896) if epi == "softplus" else {}
            fn = lambda: ops.gemm(a, w, b, epilogue=e, **kw)  # noqa: E731
        res, eq = {}, {}
        with ops.option(_lib.OPT_GEMM_ENGINE, 1):
            want = fn()
        for eng in engines:
            with ops.option(_lib.OPT_GEMM_ENGINE, eng):
                got = fn()
                eq[eng] = all(torch.equal(x, y) for x, y in zip(got, want)) if isinstance(got, tuple) else torch.equal(got, want)
                torch.cuda.synchronize()
                ts = []
                for _ in range(5):
                    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(20):
                        fn()
                    t.record()
                    torch.cuda.synchronize()
                    ts.append(s.elapsed_time(t) / 20 * 1e3)
                res[eng] = sorted(ts)[2]
        fl = 6 * 2.0 * M * N * 192
        lib = os.path.basename(os.environ.get("VASR_LIB", "default"))
        print(f"{lib:24s} {name:14s} M={M:6d} N={N:5d}: " + "  ".join(
            f"{'tiles' if e == 1 else 'rows'} {res[e]:7.1f} us ({fl / res[e] / 1e6:.0f} TF/s){'' if eq[e] else ' MISMATCH'}" for e in engines), flush=True)


if __name__ == "__main__":
    main()
