"""Time the panel-GEMM ablation libraries (tools/_variants/, built by kernel_variants.sh from
gemm_x3.hip + gemm_panel.hip with VASR_PANEL_ABLATE) on the model's K = 192 / 384 shapes."""
import ctypes
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import _lib  # noqa: E402

SHAPES = [(16032, 768, 192), (16032, 512, 384), (16032, 192, 384), (8016, 768, 192)]


def main():
    libs = sorted(glob.glob(os.path.join(REPO, "tools", "_variants", "lib_*.so")),
                  key=lambda p: int(os.path.basename(p).split("_")[1]))
    st = torch.cuda.current_stream().cuda_stream
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") * 0.05
        out = torch.empty(M, N, device="cuda")
        args = _lib.GemmArgs()
        args.A, args.lda, args.stride_a = a.data_ptr(), K, 0
        args.W, args.ldw, args.bias = w.data_ptr(), K, None
        args.C, args.ldc, args.stride_c = out.data_ptr(), N, 0
        args.batch, args.M, args.N, args.K = 1, M, N, K
        args.epilogue, args.n_out = 0, 0
        for p in libs:
            lib = ctypes.CDLL(p)
            lib.vasr_linear_x3_f32.argtypes = [ctypes.POINTER(_lib.GemmArgs), ctypes.c_void_p, ctypes.c_void_p]
            lib.vasr_split_weights_bf16x3.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.c_void_p]
            lib.vasr_split_weights_elems.argtypes = [ctypes.c_int, ctypes.c_int]
            lib.vasr_split_weights_elems.restype = ctypes.c_int64
            buf = torch.empty(lib.vasr_split_weights_elems(N, K), dtype=torch.int16, device="cuda")
            assert lib.vasr_split_weights_bf16x3(w.data_ptr(), K, N, K, buf.data_ptr(), st) == 0
            f = lambda: lib.vasr_linear_x3_f32(args, buf.data_ptr(), st)  # noqa: E731
            for _ in range(3):
                assert f() == 0
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                f()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / 20 * 1e3
            print(f"M={M} N={N:4d} K={K:4d} {os.path.basename(p)[4:-3]:14s} {us:7.1f} us "
                  f"{12 * M * N * K / us / 1e6:6.0f} bf16-TF/s", flush=True)


if __name__ == "__main__":
    main()
