#!/usr/bin/env python3
"""Is the 32 x 30 s scan launch slower per element than the 32 x 10 s one (VERDICT r05 weak 3 /
next 5) in cycles or in clock?  With a -DVASR_SCAN_STAMPS library (VASR_LIB=...): rounds of `reps`
back-to-back launches at L = 501 and at L = 1501 (B = 32, Di = 384, N = 64, mode 2), alternating;
per round: us per launch, the median workgroup's cycles (s_memtime) and clock (cycles / s_memrealtime),
and cycles per chunk.  Equal cycles per chunk at a lower clock = the clock the chip holds."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "velocity-asr_amd"), REPO]
import torch  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    from velocity_asr import _lib, ops
    lib = _lib.lib()
    B, Di, N = 32, 384, 64
    nblk = B * (Di // 16)
    stamps = torch.zeros(5 * nblk, device="cuda", dtype=torch.int64)
    f = lib.vasr_diag_scan_stamps
    f.argtypes = [ctypes.c_void_p]
    assert f(ctypes.c_void_p(stamps.data_ptr())) == 0
    ops_ = {}
    for L in (501, 1501):
        g = torch.Generator(device="cuda").manual_seed(L)
        M = B * L
        xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
        dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
        bc = torch.randn(M, 2 * N, device="cuda", generator=g)
        A2 = -torch.arange(1, N + 1, device="cuda", dtype=torch.float32) * 1.4426950408889634
        D = torch.ones(Di, device="cuda")
        out = torch.empty(M, Di, device="cuda")
        ops_[L] = (xz, dt, bc, A2, D, out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print("round     L  us/launch  clock_GHz  cycles_k(med wg)  cycles/chunk  us/chunk-equiv(x 501/L)")
    for r in range(rounds):
        for L in (501, 1501):
            xz, dt, bc, A2, D, out = ops_[L]
            for _ in range(3):
                ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
            s.record()
            for _ in range(reps):
                ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / reps * 1e3
            st = stamps.view(nblk, 5).cpu().double()
            cyc = st[:, 3] - st[:, 1]
            real = st[:, 4] - st[:, 2]
            ghz = (cyc / real.clamp(min=1) * 0.1).median().item()
            nch = (L + 15) // 16
            print(f"{r:5d} {L:5d} {us:10.2f} {ghz:10.3f} {cyc.median().item() / 1e3:17.1f} {cyc.median().item() / nch:13.0f} "
                  f"{us * 501 / L:10.2f}", flush=True)


if __name__ == "__main__":
    main()
