#!/usr/bin/env python3
"""Time the ablated scan libraries built by tools/scan_ablate.sh (diagnostic only)."""
import ctypes
import glob
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    B, L, Di, N = int(os.environ.get("SCAN_B", 32)), int(os.environ.get("SCAN_L", 501)), 384, 64
    modes = tuple(int(m) for m in os.environ.get("SCAN_MODES", "0").split(","))
    M = B * L
    g = torch.Generator(device="cuda").manual_seed(0)
    xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
    dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
    bc = torch.randn(M, 2 * N, device="cuda", generator=g)
    A2 = -torch.arange(1, N + 1, device="cuda", dtype=torch.float32) * 1.4426950408889634
    D = torch.ones(Di, device="cuda")
    out = torch.empty(M, Di, device="cuda")
    libs = sorted(glob.glob(os.path.join(HERE, os.environ.get("VARIANT_DIR", "_variants"), "lib_*.so")), key=lambda p: int(os.path.basename(p).split("_")[1]))
    fns = []
    chunked = os.environ.get("SCAN_FORM", "streaming") == "chunked"  # the chunk-parallel form (3 launches)
    wsf = 4 * B * ((L + 15) // 16) * Di * N
    ws = torch.empty(wsf, device="cuda")
    for p in libs:
        lib = ctypes.CDLL(p)
        c_p, c_i64 = ctypes.c_void_p, ctypes.c_int64
        if chunked:
            f = lib.vasr_ssm_scan_chunked_f32
            f.argtypes = [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5 + [c_p, c_i64, c_p]
        else:
            f = lib.vasr_ssm_scan_f32
            f.argtypes = [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5 + [c_p]
        fns.append((os.path.basename(p), f))
    st = torch.cuda.current_stream().cuda_stream
    args = lambda mode: (xz.data_ptr(), 2 * Di, dt.data_ptr(), Di, bc.data_ptr(), 2 * N, A2.data_ptr(), D.data_ptr(),
                         out.data_ptr(), Di, B, L, Di, N, mode) + ((ws.data_ptr(), wsf, st) if chunked else (st,))
    res = {}
    for rnd in range(5):
        for n, f in fns:
            for mode in modes:
                f(*args(mode))
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    assert f(*args(mode)) == 0
                e.record()
                torch.cuda.synchronize()
                res[f"{n} m{mode}"] = res.get(f"{n} m{mode}", []) + [s.elapsed_time(e) / 20 * 1e3]
    for n, v in res.items():
        print(f"{n:20s} median {sorted(v)[len(v)//2]:8.1f} us  min {min(v):8.1f}")


if __name__ == "__main__":
    main()
