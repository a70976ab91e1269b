#!/usr/bin/env python3
"""Phase timings of the one-launch time-split scan (ssm_scan_split_kernel) from inside the kernel.

Needs a library built with -DVASR_SCAN_STAMPS (tools/scan_variants_build.sh), passed as VASR_LIB:
every wave records s_memrealtime (100 MHz) at entry, phase-1 data landed, phase 1 done, levels
done, phase-3 chunk 0 landed, loop done and stores drained.  Prints, over the waves of one launch
at the model's B = 1 shape, the median and max of each phase and the launch's first-entry to
last-exit span.

    VASR_LIB=tools/_variants/lib_0_stamps.so python tools/diag/split_stamps.py [L] [reps]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 501
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    from velocity_asr import _lib, ops
    lib = _lib.lib()
    B, Di, N = 1, 384, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    M = B * L
    xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
    dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
    bc = torch.randn(M, 2 * N, device="cuda", generator=g)
    A2 = -torch.arange(1, N + 1, device="cuda", dtype=torch.float32) * 1.4426950408889634
    D = torch.ones(Di, device="cuda")
    out = torch.empty(M, Di, device="cuda")
    nblk = B * Di // 2
    stamps = torch.zeros(8 * 16 * nblk, device="cuda", dtype=torch.int64)
    f = lib.vasr_diag_scan_stamps
    f.argtypes = [ctypes.c_void_p]
    assert f(ctypes.c_void_p(stamps.data_ptr())) == 0
    prev = ops.scan_form("chunked")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with ops.option(_lib.OPT_SCAN_SPLIT, 2), ops.option(_lib.OPT_SCAN_LANES, 2):
        for _ in range(3):
            ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
        s.record()
        for _ in range(reps):
            ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
        e.record()
        torch.cuda.synchronize()
    ops.scan_form(prev)
    print(f"L={L}: {s.elapsed_time(e) / reps * 1e3:.2f} us per launch (events, back to back)")
    st = stamps.view(nblk * 16, 8).cpu()
    valid = st[:, 1] > 0
    st = st[valid].double()
    t0 = st[:, 1].min()
    names = ["entry", "p1 landed", "p1 done", "levels done", "p3 c0 landed", "p3 loop done", "stores drained"]
    print(f"{len(st)} waves; span first entry -> last drain {(st[:, 7].max() - t0).item() * 10:.0f} ns")
    print("stamp            median_ns_from_first_entry   max_ns")
    for i, nme in enumerate(names):
        v = (st[:, 1 + i] - t0) * 10
        print(f"{nme:16s} {v.median().item():10.0f} {v.max().item():10.0f}")
    print("phase            median_ns   max_ns")
    for i in range(1, 7):
        v = (st[:, 1 + i] - st[:, i]) * 10
        print(f"{names[i - 1] + ' -> ' + names[i]:34s} {v.median().item():8.0f} {v.max().item():8.0f}")


if __name__ == "__main__":
    main()
