#!/usr/bin/env python3
"""Time GEMM variant libraries (tools/_variants/) on the model shapes, interleaved rounds."""
import ctypes
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import _lib  # noqa: E402
from gemm_bench import SHAPES  # noqa: E402


def main():
    libs = sorted(glob.glob(os.path.join(REPO, "tools", "_variants", "lib_*.so")),
                  key=lambda p: int(os.path.basename(p).split("_")[1]))
    fns = []
    split_cache = {}
    check = os.environ.get("VARIANT_CHECK", "1") == "1"
    for p in libs:
        lib = ctypes.CDLL(p)
        if hasattr(lib, "vasr_linear_x3_f32"):  # split-bf16 engine: pre-split W with this library
            lib.vasr_linear_x3_f32.argtypes = [ctypes.POINTER(_lib.GemmArgs), ctypes.c_void_p, ctypes.c_void_p]
            lib.vasr_split_weights_bf16x3.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.c_void_p]
            lib.vasr_split_weights_elems.argtypes = [ctypes.c_int, ctypes.c_int]
            lib.vasr_split_weights_elems.restype = ctypes.c_int64

            def f(args, st, lib=lib):
                key = (args.W, args.N, args.K)
                if key not in split_cache:
                    buf = torch.empty(lib.vasr_split_weights_elems(args.N, args.K), dtype=torch.int16, device="cuda")
                    assert lib.vasr_split_weights_bf16x3(args.W, args.ldw, args.N, args.K, buf.data_ptr(), st) == 0
                    split_cache[key] = buf
                return lib.vasr_linear_x3_f32(args, split_cache[key].data_ptr(), st)
        else:
            f = lib.vasr_linear_f32
            f.argtypes = [ctypes.POINTER(_lib.GemmArgs), ctypes.c_void_p]
        fns.append((os.path.basename(p)[4:-3], f))
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for name, m, n, k, lda, epi, n_out in SHAPES:
        a = torch.randn(m, lda, device="cuda")
        w = torch.randn(n, k, device="cuda") * 0.05
        b = torch.randn(n, device="cuda")
        aux = torch.randn(m, n, device="cuda")
        out = torch.empty(m, n, device="cuda")
        args = _lib.GemmArgs()
        args.A, args.lda, args.stride_a = a.data_ptr(), lda, 0
        args.W, args.ldw, args.bias = w.data_ptr(), k, b.data_ptr()
        args.C, args.ldc, args.stride_c = out.data_ptr(), n, 0
        args.batch, args.M, args.N, args.K = 1, m, n, k
        args.epilogue, args.n_out = epi, n_out
        args.aux, args.ld_aux = aux.data_ptr(), n
        ref = None
        for rnd in range(4):
            for vn, f in fns:
                assert f(args, st) == 0
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                elif rnd == 0 and check:
                    assert torch.allclose(out, ref, atol=1e-3, rtol=1e-4), (vn, name)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    f(args, st)
                e.record()
                torch.cuda.synchronize()
                res.setdefault((name, vn), []).append(s.elapsed_time(e) / 20 * 1e3)
    tot = {}
    for (name, vn), v in res.items():
        med = sorted(v)[len(v) // 2]
        tot[vn] = tot.get(vn, 0) + med
        print(f"{name:14s} {vn:18s} {med:7.1f} us")
    for vn, t in tot.items():
        print(f"TOTAL {vn:18s} {t:7.1f} us")


if __name__ == "__main__":
    main()
