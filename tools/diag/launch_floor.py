"""Diagnostic (GPU box): device time per kernel node of a HIP graph of tiny kernels (the launch
floor one-utterance latency pays ~80 times), printed as us per node."""
import time
import torch
x = torch.zeros(64, device="cuda")
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    for _ in range(3):
        x.add_(1.0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for _ in range(200):
            x.add_(1.0)
torch.cuda.synchronize()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t) / 20 / 200 * 1e6:.2f} us per graph kernel node")
