"""Diagnostic (GPU box): the fused SSMBlock tail's launch time per M -- 20 back-to-back launches
captured in one HIP graph, its replay between one HIP event pair, best of 3 (r04an timed the
Python calls instead: at M <= 1024 that measured the host path, ~16 us per call) -- for A/B of diagnostic builds
(VASR_LIB=tools/_variants/<name>.so; e.g. -DVASR_TAIL_ABLATE=<bits>, csrc/ssm_tail.hip).
The output digest (a position-weighted sum of the output bits) tells bitwise-equal builds apart.
usage: tail_time.py [M ...]   (default 501 1024 8016 16032)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

_lib.require_device()
dev = torch.device("cuda", 0)
g0 = torch.Generator(device=dev).manual_seed(0)
D, E = 192, 384
wo = torch.randn(D, E, device=dev, generator=g0) * 0.05
w1 = torch.randn(E, D, device=dev, generator=g0) * 0.07
w2 = torch.randn(D, E, device=dev, generator=g0) * 0.05
lnw = 1 + 0.1 * torch.randn(D, device=dev, generator=g0)
lnb = 0.1 * torch.randn(D, device=dev, generator=g0)
b1 = 0.1 * torch.randn(E, device=dev, generator=g0)
b2 = 0.1 * torch.randn(D, device=dev, generator=g0)
tag = os.path.basename(os.environ.get("VASR_LIB", "default"))
for M in [int(v) for v in sys.argv[1:]] or [501, 1024, 8016, 16032]:
    g = torch.randn(M, E, device=dev, generator=g0)
    x = torch.randn(M, D, device=dev, generator=g0)
    out = torch.empty(M, D, device=dev)
    for _ in range(3):
        ops.ssm_block_tail(g, x, wo, lnw, lnb, 1e-5, w1, b1, w2, b2, out=out)
    # 20 launches captured in one graph: the replay times the device, not the Python call path
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for _ in range(20):
            ops.ssm_block_tail(g, x, wo, lnw, lnb, 1e-5, w1, b1, w2, b2, out=out)
    ts = []
    for _ in range(3):
        gr.replay()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 20 * 1e3)
    bits = out.view(torch.int32).to(torch.int64).flatten()
    digest = int((bits * torch.arange(1, bits.numel() + 1, device=dev, dtype=torch.int64)).sum().item()) & 0xffffffffffff
    print(f"{tag:14s} M={M:6d}: {min(ts):7.2f} us (runs {', '.join(f'{t:.2f}' for t in ts)})  output digest {digest:012x}",
          flush=True)
