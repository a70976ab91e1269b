#!/usr/bin/env python3
"""Time GEMM variant libraries (tools/_variants/, built by kernel_variants.sh from gemm_x3.hip) on
the model's GEMM shapes, for the split-bf16 fp32 engine (x3) and the bf16 engine (diagnostic)."""
import ctypes
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import _lib  # noqa: E402

SHAPES = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("SHAPES", "16032x768x192,16032x512x384,16032x192x384,16032x384x192,16032x1000x192").split(",")]


def main():
    engines = sys.argv[1:] or ["x3", "bf16"]
    libs = sorted(glob.glob(os.path.join(REPO, "tools", "_variants", "lib_*.so")),
                  key=lambda p: int(os.path.basename(p).split("_")[1]))
    st = torch.cuda.current_stream().cuda_stream
    for eng in engines:
        for M, N, K in SHAPES:
            a = torch.randn(M, K, device="cuda")
            w = torch.randn(N, K, device="cuda") * 0.05
            wb = w.to(torch.bfloat16)
            out = torch.empty(M, N, device="cuda")
            args = _lib.GemmArgs()
            args.A, args.lda, args.stride_a = a.data_ptr(), K, 0
            args.W, args.ldw, args.bias = w.data_ptr(), K, None
            args.C, args.ldc, args.stride_c = out.data_ptr(), N, 0
            args.batch, args.M, args.N, args.K = 1, M, N, K
            args.epilogue, args.n_out = 0, 0
            for p in libs:
                lib = ctypes.CDLL(p)
                for fn in ("vasr_linear_x3_f32", "vasr_linear_bf16"):
                    getattr(lib, fn).argtypes = [ctypes.POINTER(_lib.GemmArgs), ctypes.c_void_p, ctypes.c_void_p]
                for fn in ("vasr_split_weights_bf16x3", "vasr_pack_weights_bf16"):
                    getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_void_p, ctypes.c_void_p]
                for fn in ("vasr_split_weights_elems", "vasr_pack_weights_bf16_elems"):
                    getattr(lib, fn).argtypes = [ctypes.c_int, ctypes.c_int]
                    getattr(lib, fn).restype = ctypes.c_int64
                if eng == "x3":
                    buf = torch.empty(lib.vasr_split_weights_elems(N, K), dtype=torch.int16, device="cuda")
                    assert lib.vasr_split_weights_bf16x3(w.data_ptr(), K, N, K, buf.data_ptr(), st) == 0
                    f = lambda: lib.vasr_linear_x3_f32(args, buf.data_ptr(), st)
                    ref = a.double() @ w.double().T
                else:
                    buf = torch.empty(lib.vasr_pack_weights_bf16_elems(N, K), dtype=torch.int16, device="cuda")
                    assert lib.vasr_pack_weights_bf16(wb.data_ptr(), K, N, K, buf.data_ptr(), st) == 0
                    f = lambda: lib.vasr_linear_bf16(args, buf.data_ptr(), st)
                    ref = a.to(torch.bfloat16).double() @ wb.double().T
                for _ in range(3):
                    assert f() == 0
                torch.cuda.synchronize()
                err = (out.double() - ref).abs().max().item()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    f()
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) / 20 * 1e3
                gbs = 4 * (M * K + M * N) / us / 1e3
                print(f"{eng:4s} M={M} N={N:4d} K={K:4d} {os.path.basename(p)[4:-3]:14s} {us:7.1f} us "
                      f"{2 * M * N * K / us / 1e6:6.1f} TF/s {gbs:6.0f} GB/s err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
