#!/usr/bin/env python3
"""Isolated scan launches over time, to separate the scan's two observed launch times (96 vs 108 us
per 32-clip launch) into clock and placement.

Every `period` seconds for `secs` seconds: `reps` back-to-back launches of vasr_ssm_scan_f32 at the
bench's C2 shape (B=32, L=501, Di=384, N=64, mode 2) between one HIP event pair; prints one line
per burst (elapsed s, us per launch).  Between bursts the GPU runs a `load` of other launches
(the same scan) so the chip stays under load as in the bench.  Run under
`rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES ...` for per-launch counters.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import ops  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 30.0
    period = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    B, L, Di, N = 32, 501, 384, 64
    g = torch.Generator(device="cuda").manual_seed(0)
    M = B * L
    xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
    dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
    bc = torch.randn(M, 2 * N, device="cuda", generator=g)
    A2 = -torch.arange(1, N + 1, device="cuda", dtype=torch.float32) * 1.4426950408889634
    D = torch.ones(Di, device="cuda")
    out = torch.empty(M, Di, device="cuda")
    for _ in range(3):
        ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
    torch.cuda.synchronize()
    t_start = time.time()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    while time.time() - t_start < secs:
        s.record()
        for _ in range(reps):
            ops.ssm_scan(xz, dt, bc, A2, D, B, L, 2, out=out)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / reps * 1e3
        print(f"t {time.time() - t_start:7.2f} s  scan {us:7.2f} us/launch", flush=True)
        t_next = time.time() + period
        while time.time() < t_next:
            time.sleep(0.05)
    print("done", flush=True)


if __name__ == "__main__":
    main()
