"""Diagnostic (GPU box): where the rows engine's waves spend their cycles, from a build with
-DVASR_ROWS_STAMPS (tools/build_variant_lib.sh rowstamps -DVASR_ROWS_STAMPS; VASR_LIB=<that .so>).

Each wave sums s_memtime cycles per phase of its chunk steps -- the counted vmcnt wait, the block
barrier, the previous chunk's epilogue (split, bias / softplus, 16 buffer stores issued), the DMA
issue (loader waves) and the chunk's 72 MFMAs + fragment reads -- and writes the sums once at the
end.  Printed: per phase the mean over loader and over store-only waves, in cycles and as a share
of the wave's whole kernel time.  Usage: rows_stamps.py [M ...] (composed head GEMM, K = 192).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

_lib.require_device()
lib = _lib.lib()
if not hasattr(lib, "vasr_diag_rows_stamps"):
    sys.exit("rows_stamps.py: the loaded library was not built with -DVASR_ROWS_STAMPS")
lib.vasr_diag_rows_stamps.argtypes = [ctypes.c_void_p]
Ms = [int(v) for v in sys.argv[1:]] or [8016, 16032]
g0 = torch.Generator(device="cuda").manual_seed(0)
# ROWS_N=896: the z-in-tail projection (x | B | C | dt, softplus from 512); default the 1280-column form
NC = int(os.environ.get("ROWS_N", "1280"))
NOUT = NC - 384
w = torch.randn(NC, 192, device="cuda", generator=g0) * 0.07
b = torch.cat([torch.zeros(NOUT, device="cuda"), torch.randn(384, device="cuda", generator=g0) * 0.1])
buf = torch.zeros(256 * 8 * 8, device="cuda", dtype=torch.int64)
NAMES = ("wait", "barrier", "epilogue", "dma", "mfma")
for M in Ms:
    u = torch.randn(M, 192, device="cuda", generator=g0)
    out = torch.empty(M, NC, device="cuda")
    for _ in range(5):
        ops.gemm(u, w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=NOUT, out=out)
    torch.cuda.synchronize()
    buf.zero_()
    assert lib.vasr_diag_rows_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    ops.gemm(u, w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=NOUT, out=out)
    torch.cuda.synchronize()
    assert lib.vasr_diag_rows_stamps(ctypes.c_void_p(0)) == 0
    st = buf.view(-1, 8).cpu()
    st = st[st[:, 5] > 0]
    for kind, sel in (("loader", st[:, 7] == 1), ("store-only", st[:, 7] == 0)):
        x = st[sel].double()
        tot = x[:, 5].mean().item()
        parts = ", ".join(f"{n} {x[:, i].mean().item():.0f} ({x[:, i].mean().item() / tot:.0%})" for i, n in enumerate(NAMES))
        print(f"M={M} {kind:10s} waves {int(sel.sum())}, chunks/wave {x[:, 6].mean().item():.1f}: total {tot:.0f} cyc; "
              f"{parts}; max total {x[:, 5].max().item():.0f}", flush=True)
