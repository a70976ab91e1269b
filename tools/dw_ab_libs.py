#!/usr/bin/env python3
"""Interleaved launch-time A/B of vasr_ln_dwconv_f32 (SSMBlock LN1 + causal depthwise conv) between library
builds of the same ABI (ctypes only), at B x L token rows, C = 192, Kc = 4: `reps` back-to-back launches between
one HIP event pair per library and round, order rotated after a warm-up, outputs compared bitwise.
    python tools/dw_ab_libs.py <rounds> <B:L,...> lib.so[@rows] ...   (@rows: VASR_OPT_DW_ROWS 4 / 8 / 16)
DW_PRENORM=1: vasr_ln_dwconv_prenorm_f32 instead (a LayerNorm in front, its rows stored too; both compared)."""
import ctypes
import os
import sys
import time

import torch

c_p, c_int, c_f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
OPT_DW_ROWS = 6
PRE = os.environ.get("DW_PRENORM", "0") == "1"


def main():
    rounds = int(sys.argv[1])
    shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[2].split(",")]
    C, Kc, reps = 192, 4, 20
    g = torch.Generator(device="cuda").manual_seed(0)
    lw, lb = 1 + 0.1 * torch.randn(C, device="cuda", generator=g), 0.1 * torch.randn(C, device="cuda", generator=g)
    cw, cb = torch.randn(C, Kc, device="cuda", generator=g) * 0.3, 0.1 * torch.randn(C, device="cuda", generator=g)
    entries = []
    for spec in sys.argv[3:]:
        path, _, rows = spec.partition("@")
        lib = ctypes.CDLL(path)
        lib.vasr_ln_dwconv_f32.argtypes = [c_p] * 6 + [c_int] * 4 + [c_f32, c_p]
        if PRE:
            lib.vasr_ln_dwconv_prenorm_f32.argtypes = [c_p, c_p, c_p, c_f32] + [c_p] * 6 + [c_int] * 4 + [c_f32, c_p]
        lib.vasr_set_option.argtypes = [c_int, c_int]
        entries.append((os.path.basename(path) + (f"@{rows}" if rows else ""), lib, int(rows or 0)))
    pw, pb = 1 + 0.1 * torch.randn(C, device="cuda", generator=g), 0.1 * torch.randn(C, device="cuda", generator=g)
    data = {(B, L): (torch.randn(B, L, C, device="cuda", generator=g), torch.empty(B, L, C, device="cuda"),
                     torch.empty(B, L, C, device="cuda")) for B, L in shapes}

    def launch(e, key):
        _, lib, rows = e
        x, y, xo = data[key]
        lib.vasr_set_option(OPT_DW_ROWS, rows)
        if PRE:
            return lib.vasr_ln_dwconv_prenorm_f32(x.data_ptr(), pw.data_ptr(), pb.data_ptr(), 1e-5, xo.data_ptr(),
                                                  lw.data_ptr(), lb.data_ptr(), cw.data_ptr(), cb.data_ptr(),
                                                  y.data_ptr(), key[0], key[1], C, Kc, 1e-5, None)
        return lib.vasr_ln_dwconv_f32(x.data_ptr(), lw.data_ptr(), lb.data_ptr(), cw.data_ptr(), cb.data_ptr(),
                                      y.data_ptr(), key[0], key[1], C, Kc, 1e-5, None)
    for key in data:
        ref = None
        for e in entries:
            assert launch(e, key) == 0
            torch.cuda.synchronize()
            o = torch.cat([data[key][1], data[key][2]]) if PRE else data[key][1].clone()
            if ref is None:
                ref = o
            elif not torch.equal(o, ref):
                print(f"MISMATCH {e[0]} {key}", flush=True)
    t_end = time.time() + float(os.environ.get("AB_WARM_S", "3"))
    k0 = next(iter(data))
    while time.time() < t_end:
        for _ in range(20):
            launch(entries[0], k0)
        torch.cuda.synchronize()
    res = {}
    for r in range(rounds):
        for key in data:
            for e in entries[r % len(entries):] + entries[:r % len(entries)]:
                for _ in range(3):
                    launch(e, key)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(reps):
                    launch(e, key)
                b.record()
                torch.cuda.synchronize()
                res.setdefault((e[0], key), []).append(a.elapsed_time(b) * 1e3 / reps)
    for key in data:
        for e in entries:
            v = sorted(res[(e[0], key)])
            print(f"B={key[0]} L={key[1]} {e[0]:24s} median {v[len(v) // 2]:6.2f} us  best {v[0]:6.2f}", flush=True)


if __name__ == "__main__":
    main()
