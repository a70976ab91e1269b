#!/usr/bin/env python3
"""Interleaved launch-time A/B of the gated streaming scan between library builds (ctypes only, any
ABI >= 12): `reps` back-to-back launches between one HIP event pair per library and round, at
(B, L) shapes given as B:L, mode 2, Di 384, N 64.
    python tools/scan_ab_libs.py <rounds> <B:L,B:L,...> lib_a.so lib_b.so ..."""
import ctypes
import os
import sys

import torch


def main():
    rounds = int(sys.argv[1])
    shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[2].split(",")]
    libs = sys.argv[3:]
    Di, N, reps = 384, int(os.environ.get("SCAN_N", "64")), 20
    fns = []
    # every option key any entry sets is set by every entry (0 = the launcher's default where the entry
    # names none): the same library loaded twice is one handle, so an option would otherwise carry over
    keys = sorted({int(s.partition("@")[2].split("=")[0]) for s in libs if "@" in s})
    for spec in libs:  # path[@key=value]: vasr_set_option(key, value) before each of this entry's launches
        p, _, opt = spec.partition("@")
        lib = ctypes.CDLL(p)
        # SCAN_UNGATED=1: the z-in-tail blocks' ungated scan (same arguments; reads only x of xz)
        f = lib.vasr_ssm_scan_ungated_f32 if os.environ.get("SCAN_UNGATED") == "1" else lib.vasr_ssm_scan_f32
        c_p, c_i64 = ctypes.c_void_p, ctypes.c_int64
        f.argtypes = [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5 + [c_p]
        if keys:
            mine = dict([tuple(int(v) for v in opt.split("="))]) if opt else {}
            lib.vasr_set_option.argtypes = [ctypes.c_int, ctypes.c_int]

            def f(*a, _f=f, _lib=lib, _kv=tuple((k, mine.get(k, 0)) for k in keys)):
                for k, v in _kv:
                    assert _lib.vasr_set_option(k, v) >= 0
                return _f(*a)
        fns.append((spec.split("/")[-1], f))
    data = {}
    for B, L in shapes:
        g = torch.Generator(device="cuda").manual_seed(B * L)
        M = B * L
        xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
        dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
        bc = torch.randn(M, 2 * N, device="cuda", generator=g)
        A2 = -torch.arange(1, N + 1, device="cuda", dtype=torch.float32) * 1.4426950408889634
        D = torch.ones(Di, device="cuda")
        data[(B, L)] = (xz, dt, bc, A2, D, torch.empty(M, Di, device="cuda"))
    res = {}
    st = torch.cuda.current_stream().cuda_stream
    # warm the chip up first (the clock ramps over the first ~2 s of load, profiles/r06d/l_clock.txt),
    # then rotate the library order every round so no library always runs first or last
    import time
    (B0, L0), (xz, dt, bc, A2, D, out) = next(iter(data.items()))
    t_end = time.time() + float(__import__("os").environ.get("AB_WARM_S", "3"))
    while time.time() < t_end:
        for _ in range(20):
            fns[0][1](xz.data_ptr(), 2 * Di, dt.data_ptr(), Di, bc.data_ptr(), 2 * N, A2.data_ptr(), D.data_ptr(),
                      out.data_ptr(), Di, B0, L0, Di, N, 2, st)
        torch.cuda.synchronize()
    for r in range(rounds):
        for (B, L), (xz, dt, bc, A2, D, out) in data.items():
            for name, f in fns[r % len(fns):] + fns[:r % len(fns)]:
                args = (xz.data_ptr(), 2 * Di, dt.data_ptr(), Di, bc.data_ptr(), 2 * N, A2.data_ptr(), D.data_ptr(),
                        out.data_ptr(), Di, B, L, Di, N, 2, st)
                for _ in range(3):
                    assert f(*args) == 0
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(reps):
                    f(*args)
                e.record()
                torch.cuda.synchronize()
                res.setdefault((B, L, name), []).append(s.elapsed_time(e) / reps * 1e3)
                res.setdefault((B, L, name, "digest"), set()).add(int(out.view(torch.int32).double().sum().item()))
    for k, v in res.items():
        if k[-1] == "digest":
            continue
        v = sorted(v)
        print(f"B={k[0]:3d} L={k[1]:5d} {k[2]:28s} median {v[len(v) // 2]:8.2f} us  min {v[0]:8.2f}  "
              f"all {[round(x, 1) for x in res[k]]}  digest {sorted(res[k + ('digest',)])}")


if __name__ == "__main__":
    main()
