#!/usr/bin/env python3
"""Where the z-in-tail gated tail's time goes: with a -DVASR_TAIL_STAMPS library (VASR_LIB=...), launch
vasr_ssm_block_tail_gated_f32 (or _bf16) at M token rows `reps` times back to back and read wave 0's
s_memtime at the phase boundaries of every workgroup of the last launch:
  0 entry | 1 u planes staged | 2 z product done | 3 gate + tail constants issued | 4 barrier passed
  | 5 out_proj + LN done (step 11) | 6 FFN1 done (step 23) | 7 FFN2 done | 8 output stored
Prints the median cycles of each phase, the workgroups' start / end spread (first vs second round of
workgroups on a CU), and the clock (s_memtime cycles per s_memrealtime tick at 100 MHz).
    python tools/diag/tail_stamps.py [M] [f32|bf16] [reps]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "velocity-asr_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16032
    bf16 = len(sys.argv) > 2 and sys.argv[2] == "bf16"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    from velocity_asr import _lib, ops
    lib = _lib.lib()
    nblk = (M + 31) // 32
    stamps = torch.zeros(16 * nblk, device="cuda", dtype=torch.int64)
    f = lib.vasr_diag_tail_stamps
    f.argtypes = [ctypes.c_void_p]
    assert f(ctypes.c_void_p(stamps.data_ptr())) == 0
    g0 = torch.Generator(device="cuda").manual_seed(0)
    rn = lambda *s, sc=1.0: torch.randn(*s, device="cuda", generator=g0) * sc  # noqa: E731
    D, E = 192, 384
    wz, wo, w1, w2 = rn(E, D, sc=0.07), rn(D, E, sc=0.05), rn(E, D, sc=0.07), rn(D, E, sc=0.05)
    lw, lb, b1, b2 = 1 + rn(D, sc=0.1), rn(D, sc=0.1), rn(E, sc=0.1), rn(D, sc=0.1)
    if bf16:
        wz, wo, w1, w2 = (w.to(torch.bfloat16) for w in (wz, wo, w1, w2))
    yd, u, x = rn(M, E), rn(M, D), rn(M, D)
    out = torch.empty(M, D, device="cuda")

    def run():
        ops.ssm_block_tail_gated(yd, u, wz, 2, x, wo, lw, lb, 1e-5, w1, b1, w2, b2, out=out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(3):
        for _ in range(3):
            run()
        s.record()
        for _ in range(reps):
            run()
        e.record()
        torch.cuda.synchronize()
        print(f"round {rnd}: {s.elapsed_time(e) / reps * 1e3:.2f} us per launch", flush=True)
    st = stamps.view(nblk, 16).cpu().numpy()
    order = [0, 1, 2, 3, 4, 9, 10, 5, 11, 6, 7, 8]  # slots in time order
    t = st[:, 3:15].astype(np.float64)[:, order]
    clock = (t[:, -1] - t[:, 0]) / ((st[:, 2] - st[:, 1]) / 100.0) / 1e3  # GHz (realtime: 100 MHz)
    names = ["u staged", "z product", "gate+consts", "barrier", "out_proj", "x1 scratch", "LayerNorm",
             "FFN1 half 0", "FFN1 half 1", "FFN2", "store"]
    print(f"M={M} {'bf16' if bf16 else 'f32'}: {nblk} workgroups, clock median {np.median(clock):.3f} GHz")
    dur = np.diff(t, axis=1)
    tot = t[:, -1] - t[:, 0]
    print("phase            median cycles   share")
    for i, n in enumerate(names):
        print(f"{n:16s} {np.median(dur[:, i]):10.0f}   {np.median(dur[:, i]) / np.median(tot):6.3f}")
    print(f"{'workgroup':16s} {np.median(tot):10.0f}   (us at the median clock: {np.median(tot) / np.median(clock) / 1e3:.2f})")
    # launch-relative start / end per workgroup (s_memtime is per-XCD: use realtime for the spread)
    r0 = st[:, 1] - st[:, 1].min()
    r1 = st[:, 2] - st[:, 1].min()
    order = np.argsort(r0)
    first, second = order[: min(256, nblk)], order[min(256, nblk):]
    for nm, idx in (("first 256 to start", first), ("the rest", second)):
        if len(idx):
            print(f"{nm:20s} start {np.median(r0[idx]) / 100:.2f} us (max {r0[idx].max() / 100:.2f}), "
                  f"end {np.median(r1[idx]) / 100:.2f} us (max {r1[idx].max() / 100:.2f})")
    print(f"last workgroup ends at {r1.max() / 100:.2f} us after the first starts")


if __name__ == "__main__":
    main()
