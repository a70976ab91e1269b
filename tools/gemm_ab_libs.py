#!/usr/bin/env python3
"""Interleaved launch-time A/B of vasr_linear_x3_f32 between library builds of the same ABI (ctypes
only): the model's K = 192 projection shapes, `reps` back-to-back launches between one HIP event pair
per library and round, library order rotated every round after a warm-up, every library's C checked
bitwise against the first's.
    python tools/gemm_ab_libs.py <rounds> <M:N:n_out[:K],...> lib_a.so lib_b.so ...  (K default 192)
(n_out > 0: softplus from column n_out, the composed projection's epilogue; 0: none; -1: the argmax
head's keys, VASR_EPI_ARGMAX)"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr._lib import GemmArgs, EPI_ARGMAX, EPI_NONE, EPI_SOFTPLUS_FROM  # noqa: E402  (struct layout only)

c_p, c_i64, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int


def main():
    rounds = int(sys.argv[1])
    shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[2].split(",")]
    libs = sys.argv[3:]
    reps = 20
    g0 = torch.Generator(device="cuda").manual_seed(0)
    entries = []
    # every option key any entry sets is set by every entry (0 = default where the entry names none): the
    # same library loaded twice is one handle, so an option would otherwise carry over to the next entry
    keys = sorted({int(s.partition("@")[2].split("=")[0]) for s in libs if "@" in s})
    for spec in libs:  # path[@key=value]: vasr_set_option(key, value) before each of this entry's launches
        path, _, opt = spec.partition("@")
        lib = ctypes.CDLL(path)
        lib.vasr_set_option.argtypes = [c_int, c_int]
        lib.vasr_linear_x3_f32.argtypes = [ctypes.POINTER(GemmArgs), c_p, c_p]
        lib.vasr_split_weights_bf16x3.argtypes = [c_p, c_i64, c_int, c_int, c_p, c_p]
        lib.vasr_split_weights_elems.argtypes = [c_int, c_int]
        lib.vasr_split_weights_elems.restype = c_i64
        mine = dict([tuple(int(v) for v in opt.split("="))]) if opt else {}
        entries.append([os.path.basename(path) + (f"@{opt}" if opt else ""), lib, {},
                        tuple((k, mine.get(k, 0)) for k in keys)])
    data = {}
    for shp in shapes:
        M, N, n_out = shp[:3]
        K = shp[3] if len(shp) > 3 else 192
        w = torch.randn(N, K, device="cuda", generator=g0) * 0.07
        b = torch.randn(N, device="cuda", generator=g0) * 0.1
        a = torch.randn(M, K, device="cuda", generator=g0)
        slots = (N + 31) // 32
        c = torch.empty(M, slots, device="cuda", dtype=torch.int64) if n_out < 0 else torch.empty(M, N, device="cuda")
        data[shp] = (w, b, a, c)
        for e in entries:
            planes = torch.empty(int(e[1].vasr_split_weights_elems(N, K)), device="cuda", dtype=torch.int16)
            assert e[1].vasr_split_weights_bf16x3(w.data_ptr(), K, N, K, planes.data_ptr(), None) == 0
            args = GemmArgs()
            args.A, args.lda, args.stride_a = a.data_ptr(), K, 0
            args.W, args.ldw = w.data_ptr(), K
            args.bias = b.data_ptr()
            args.C, args.ldc, args.stride_c = c.data_ptr(), slots if n_out < 0 else N, 0
            args.batch, args.M, args.N, args.K = 1, M, N, K
            args.epilogue = EPI_ARGMAX if n_out < 0 else EPI_SOFTPLUS_FROM if n_out else EPI_NONE
            args.n_out = max(n_out, 0)
            e[2][shp] = (args, planes)

    def launch(e, key):
        args, planes = e[2][key]
        for k, v in e[3]:
            assert e[1].vasr_set_option(k, v) >= 0
        return e[1].vasr_linear_x3_f32(ctypes.byref(args), ctypes.c_void_p(planes.data_ptr()), None)
    for key in data:
        ref = None
        for e in entries:
            assert launch(e, key) == 0
            torch.cuda.synchronize()
            o = data[key][3].clone()
            if key[2] < 0:  # argmax keys: engines may spread a row's key over its slots differently
                o = o.max(dim=1).values
            if ref is None:
                ref = o
            elif not torch.equal(o, ref):
                print(f"MISMATCH {e[0]} {key}: {(o != ref).sum().item()} elements differ", flush=True)
    k0 = next(iter(data))
    t_end = time.time() + float(os.environ.get("AB_WARM_S", "3"))
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
            print(f"M={key[0]} N={key[1]} n_out={key[2]} K={key[3] if len(key) > 3 else 192} {e[0]:24s} median {v[len(v) // 2]:7.2f} us  best {v[0]:7.2f}  "
                  f"all {' '.join(f'{t:.1f}' for t in res[(e[0], key)])}", flush=True)


if __name__ == "__main__":
    main()
