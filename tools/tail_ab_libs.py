#!/usr/bin/env python3
"""Interleaved launch-time A/B of the z-in-tail gated tail (vasr_ssm_block_tail_gated_f32 / _bf16)
between library builds of the same ABI (ctypes only): `reps` back-to-back launches between one HIP
event pair per library and round, library order rotated every round after a warm-up, and every
library's output checked bitwise against the first's.
    python tools/tail_ab_libs.py <rounds> <M,M,...> [f32|bf16] lib_a.so lib_b.so ..."""
import ctypes
import os
import sys
import time

import torch

c_p, c_i64, c_f32, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_int


def bind(path, bf16):
    lib = ctypes.CDLL(path)
    fn = lib.vasr_ssm_block_tail_gated_bf16 if bf16 else lib.vasr_ssm_block_tail_gated_f32
    fn.argtypes = [c_p, c_i64, c_p, c_i64, c_p, c_int, c_p, c_i64, c_p, c_p, c_p, c_f32, c_p, c_p, c_p, c_p, c_p,
                   c_i64] + [c_int] * 3 + [c_p]
    for n in ("vasr_split_weights_bf16x3", "vasr_split_weights16_bf16x3", "vasr_pack_weights_bf16",
              "vasr_pack_weights16_bf16"):
        getattr(lib, n).argtypes = [c_p, c_i64, c_int, c_int, c_p, c_p]
    for n in ("vasr_split_weights_elems", "vasr_split_weights16_elems", "vasr_pack_weights_bf16_elems",
              "vasr_pack_weights16_bf16_elems"):
        getattr(lib, n).argtypes = [c_int, c_int]
        getattr(lib, n).restype = c_i64
    return lib, fn


def planes(lib, w, kind):
    N, K = w.shape
    elems = {"split_weights_bf16x3": "split_weights_elems", "split_weights16_bf16x3": "split_weights16_elems"}.get(
        kind, kind + "_elems")
    out = torch.empty(int(getattr(lib, "vasr_" + elems)(N, K)), device="cuda", dtype=torch.int16)
    assert getattr(lib, f"vasr_{kind}")(w.data_ptr(), K, N, K, out.data_ptr(), None) == 0
    return out


def main():
    rounds = int(sys.argv[1])
    Ms = [int(v) for v in sys.argv[2].split(",")]
    bf16 = sys.argv[3] == "bf16"
    libs = sys.argv[4:]
    D, E, reps = 192, 384, 20
    g0 = torch.Generator(device="cuda").manual_seed(0)
    rn = lambda *s, sc=1.0: torch.randn(*s, device="cuda", generator=g0) * sc  # noqa: E731
    wz, wo, w1, w2 = rn(E, D, sc=0.07), rn(D, E, sc=0.05), rn(E, D, sc=0.07), rn(D, E, sc=0.05)
    lw, lb, b1, b2 = 1 + rn(D, sc=0.1), rn(D, sc=0.1), rn(E, sc=0.1), rn(D, sc=0.1)
    if bf16:
        wz, wo, w1, w2 = (w.to(torch.bfloat16) for w in (wz, wo, w1, w2))
    entries = []
    for path in libs:
        lib, fn = bind(path, bf16)
        if bf16:
            pz = planes(lib, wz, "pack_weights_bf16")
            pw = [planes(lib, w, "pack_weights16_bf16") for w in (wo, w1, w2)]
        else:
            pz = planes(lib, wz, "split_weights_bf16x3")
            pw = [planes(lib, w, "split_weights16_bf16x3") for w in (wo, w1, w2)]
        entries.append((os.path.basename(path), fn, pz, pw))
    data = {M: (rn(M, E), rn(M, D), rn(M, D), torch.empty(M, D, device="cuda")) for M in Ms}

    def launch(e, M):
        _, fn, pz, (po, p1, p2) = e
        yd, u, x, out = data[M]
        return fn(yd.data_ptr(), E, u.data_ptr(), D, pz.data_ptr(), 2, x.data_ptr(), D, po.data_ptr(), lw.data_ptr(),
                  lb.data_ptr(), 1e-5, p1.data_ptr(), b1.data_ptr(), p2.data_ptr(), b2.data_ptr(), out.data_ptr(), D, M,
                  D, E, None)
    ref = {}
    for i, e in enumerate(entries):
        for M in Ms:
            assert launch(e, M) == 0
            torch.cuda.synchronize()
            o = data[M][3].clone()
            if i == 0:
                ref[M] = o
            elif not torch.equal(o, ref[M]):
                print(f"MISMATCH {e[0]} M={M}: max |diff| {(o - ref[M]).abs().max().item():.3e}", flush=True)
    t_end = time.time() + float(os.environ.get("AB_WARM_S", "3"))
    while time.time() < t_end:
        for _ in range(20):
            launch(entries[0], Ms[0])
        torch.cuda.synchronize()
    res = {}
    for r in range(rounds):
        for M in Ms:
            for e in entries[r % len(entries):] + entries[:r % len(entries)]:
                for _ in range(3):
                    launch(e, M)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(reps):
                    launch(e, M)
                b.record()
                torch.cuda.synchronize()
                res.setdefault((e[0], M), []).append(a.elapsed_time(b) * 1e3 / reps)
    for M in Ms:
        for e in entries:
            v = sorted(res[(e[0], M)])
            print(f"M={M} {e[0]:28s} median {v[len(v) // 2]:7.2f} us  best {v[0]:7.2f}  all {' '.join(f'{t:.1f}' for t in res[(e[0], M)])}",
                  flush=True)


if __name__ == "__main__":
    main()
