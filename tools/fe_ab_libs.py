#!/usr/bin/env python3
"""Interleaved launch-time A/B of the front end (vasr_stft_power_400_f32 then vasr_mel_log_norm_f32,
the pair the model runs back to back) between library builds of the same ABI (ctypes only): `reps`
pairs between one HIP event pair per library and round, library order rotated every round after a
warm-up, every library's mel output checked bitwise against the first's.
    python tools/fe_ab_libs.py <rounds> <B:S,...> lib_a.so lib_b.so ..."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import audio as A  # noqa: E402  (window + CSR filterbank tables only)

c_p, c_i64, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int


def main():
    rounds = int(sys.argv[1])
    shapes = [tuple(int(v) for v in s.split(":")) for s in sys.argv[2].split(",")]
    libs = sys.argv[3:]
    reps, n_mels = 10, 80
    dev = torch.device("cuda")
    tb = A._tables(dev, 400, n_mels, 16000)
    rowptr, col, val = tb.fb_csr
    entries = []
    for path in libs:
        lib = ctypes.CDLL(path)
        lib.vasr_stft_power_400_f32.argtypes = [c_p, c_i64, c_int, c_int, c_p, c_p, c_i64, c_i64, c_p]
        lib.vasr_mel_log_norm_f32.argtypes = [c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64] + [c_int] * 5 + [c_p, c_p]
        lib.vasr_mel_workspace_floats.argtypes = [c_int] * 3
        lib.vasr_mel_workspace_floats.restype = c_i64
        entries.append((os.path.basename(path), lib))
    g0 = torch.Generator(device="cuda").manual_seed(0)
    data = {}
    for B, S in shapes:
        F = S // 160 + 1
        x = torch.randn(B, S, device=dev, generator=g0) * 0.1
        power = torch.empty(B, F, 201, device=dev)
        ws = torch.empty(int(entries[0][1].vasr_mel_workspace_floats(B, F, n_mels)), device=dev)
        out = torch.empty(B, F + 2, n_mels, device=dev)  # the model's padded layout: one zero frame each side
        data[(B, S)] = (F, x, power, ws, out)

    def launch(e, key):
        B, S = key
        F, x, power, ws, out = data[key]
        lib = e[1]
        rc = lib.vasr_stft_power_400_f32(x.data_ptr(), S, B, S, tb.window.data_ptr(), power.data_ptr(), 201,
                                          F * 201, None)
        return rc or lib.vasr_mel_log_norm_f32(power.data_ptr(), 201, F * 201, rowptr.data_ptr(), col.data_ptr(),
                                               val.data_ptr(), out.data_ptr(), (F + 2) * n_mels, 1, B, F, n_mels, 1,
                                               ws.data_ptr(), None)
    for key in data:
        ref = None
        for e in entries:
            assert launch(e, key) == 0
            torch.cuda.synchronize()
            o = data[key][4].clone()
            if ref is None:
                ref = o
            elif not torch.equal(o, ref):
                print(f"MISMATCH {e[0]} {key}: {(o != ref).sum().item()} elements differ", flush=True)
    k0 = next(iter(data))
    t_end = time.time() + float(os.environ.get("AB_WARM_S", "3"))
    while time.time() < t_end:
        for _ in range(10):
            launch(entries[0], k0)
        torch.cuda.synchronize()
    res = {}
    for r in range(rounds):
        for key in data:
            for e in entries[r % len(entries):] + entries[:r % len(entries)]:
                for _ in range(2):
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
            print(f"B={key[0]} S={key[1]} {e[0]:24s} median {v[len(v) // 2]:7.2f} us  best {v[0]:7.2f}  "
                  f"all {' '.join(f'{t:.1f}' for t in res[(e[0], key)])}", flush=True)


if __name__ == "__main__":
    main()
