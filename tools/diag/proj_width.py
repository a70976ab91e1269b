"""Diagnostic (GPU box): what moving the gate's z product out of the composed projection would buy
(VERDICT r04 next 4).  Graph-timed launches (20 per graph, best of 3) of the rows-engine projection
at M = 16032, K = 192 with the softplus-from-column epilogue for N = 1280 (x | z | B | C | dt, the
shipped layout) and N = 896 (without z), and of a 16x16x32-MFMA fused tail at M = 16032 for the
per-stage cost the z product would add there (12 more 32-k stages on top of 36).
usage: proj_width.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

_lib.require_device()
dev = torch.device("cuda", 0)
g0 = torch.Generator(device=dev).manual_seed(0)


def graph_time(fn, n=20):
    for _ in range(3):
        fn()
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        for _ in range(n):
            fn()
    ts = []
    for _ in range(3):
        gr.replay()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / n * 1e3)
    return min(ts)


M, K, Di = 16032, 192, 384
u = torch.randn(M, K, device=dev, generator=g0)
for N in (1280, 896):
    w = torch.randn(N, K, device=dev, generator=g0) / K ** 0.5
    b = torch.randn(N, device=dev, generator=g0) * 0.1
    out = torch.empty(M, N, device=dev)
    t = graph_time(lambda: ops.gemm(u, w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=N - Di, out=out))
    print(f"projection M={M} N={N} K={K} (softplus on the last {Di} columns): {t:7.2f} us, "
          f"{M * N * 4 / t / 1e3:.0f} GB/s of C", flush=True)
D, E = 192, 384
wo = torch.randn(D, E, device=dev, generator=g0) * 0.05
w1 = torch.randn(E, D, device=dev, generator=g0) * 0.07
w2 = torch.randn(D, E, device=dev, generator=g0) * 0.05
lnw = 1 + 0.1 * torch.randn(D, device=dev, generator=g0)
lnb = 0.1 * torch.randn(D, device=dev, generator=g0)
b1 = 0.1 * torch.randn(E, device=dev, generator=g0)
b2 = 0.1 * torch.randn(D, device=dev, generator=g0)
g = torch.randn(M, E, device=dev, generator=g0)
x = torch.randn(M, D, device=dev, generator=g0)
out = torch.empty(M, D, device=dev)
t = graph_time(lambda: ops.ssm_block_tail(g, x, wo, lnw, lnb, 1e-5, w1, b1, w2, b2, out=out))
print(f"fused tail M={M}: {t:7.2f} us for 36 stages = {t / 36:.3f} us per stage; a z product adds 12 stages "
      f"(~{12 * t / 36:.1f} us if the time per stage holds)", flush=True)
