#!/usr/bin/env python3
"""Micro-benchmark of vasr_ssm_scan_f32 alone at the C2 shape (B=32, L=501, Di=384, N=64): `reps`
launches captured in one HIP graph and replayed (per-launch kernel time, no host cost)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "velocity-asr_amd"))
import torch  # noqa: E402
from velocity_asr import ops  # noqa: E402


def main():
    B, L, Di, N = [int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (32, 501, 384, 64))]
    mode = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 50
    if len(sys.argv) > 7:  # "streaming" | "chunked": force the form (default: by launch size)
        ops.scan_form(sys.argv[7])
    g = torch.Generator(device="cuda").manual_seed(0)
    M = B * L
    xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
    dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
    bc = torch.randn(M, 2 * N, device="cuda", generator=g)
    A2 = -torch.arange(1, N + 1, device="cuda", dtype=torch.float32) * 1.4426950408889634
    D = torch.ones(Di, device="cuda")
    out = torch.empty(M, Di, device="cuda")
    ungated = os.environ.get("SCAN_UNGATED", "0") == "1"  # the z-in-tail block's scan (no z, no gate)

    def run():
        if ungated:
            ops.ssm_scan_ungated(xz[:, :Di], dt, bc, A2, D, B, L, mode, out=out)
        else:
            ops.ssm_scan(xz, dt, bc, A2, D, B, L, mode, out=out)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    # the launches replayed from a HIP graph: kernel time without the host wrapper's per-call cost
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for _ in range(reps):
            run()
    gr.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    gr.replay()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    byts = B * L * ((3 if ungated else 4) * Di + 2 * N) * 4
    form = sys.argv[7] if len(sys.argv) > 7 else "auto"
    print(f"scan B={B} L={L} Di={Di} N={N} mode={mode} {form}{' ungated' if ungated else ''}: {us:.1f} us/launch, {byts / us / 1e3:.1f} GB/s, "
          f"{B * L * Di * N / us / 1e3:.1f} Gelem/s")


if __name__ == "__main__":
    main()
