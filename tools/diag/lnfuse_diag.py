"""Diagnostic (GPU box): where the conv-prologue GEMM departs from ln_dwconv + GEMM."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import numpy as np, torch
from velocity_asr import _lib, ops
DEV = "cuda"
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
rng = np.random.default_rng(16501)
B, L, D, Di, N = 16, 501, 192, 384, 64
x = t(rng.standard_normal((B, L, D)).astype(np.float32) * 1.7 + 0.3)
lw = t(1.0 + 0.1 * rng.standard_normal(D).astype(np.float32)); lb = t(0.1 * rng.standard_normal(D).astype(np.float32))
cw = t(0.5 * rng.standard_normal((D, 4)).astype(np.float32)); cb = t(0.1 * rng.standard_normal(D).astype(np.float32))
w = t((rng.standard_normal((2 * Di, D)) / np.sqrt(D)).astype(np.float32))
M = B * L
u = ops.ln_dwconv(x, lw, lb, cw, cb, 1e-5).view(M, D)
xn = ops.layer_norm(x.view(M, D), lw, lb, 1e-5)
# emulate the conv on xn: fma chain in float64, rounded to float32 each step
xd = xn.view(B, L, D).double().cpu().numpy(); wd = cw.double().cpu().numpy(); bd = cb.double().cpu().numpy()
acc = np.zeros((B, L, D), np.float32)
for j in range(4):
    back = 3 - j
    sh = np.zeros_like(xd); sh[:, back:] = xd[:, :L - back]
    acc = (acc.astype(np.float64) + sh * wd[:, j]).astype(np.float32)
emu = (acc.astype(np.float64) + bd).astype(np.float32).reshape(M, D)
un = u.cpu().numpy()
print("ln_dwconv vs emulated conv(layer_norm): mismatches", int((un != emu).sum()), "max", float(np.abs(un - emu).max()))
want = ops.gemm(u, w)
got = ops.gemm(xn, w, conv=(cw, cb, L))
emu_g = ops.gemm(t(emu), w)
torch.cuda.synchronize()
print("got vs want mismatches", int((got != want).sum().item()), "of", got.numel(), "max", float((got - want).abs().max()))
print("got vs gemm(emu) mismatches", int((got != emu_g).sum().item()))
d = (got != want).any(1).nonzero().flatten().cpu().numpy()
print("rows differing (first 20, as t):", (d % L)[:20], "count", len(d))
