"""Diagnostic (GPU box): the fused CTC-head GEMM + argmax (gemm_argmax, N = 1000, K = 192) on the
tile engine vs the rows engine (VASR_OPT_GEMM_ENGINE 1 / 2) at the bench's M: time per launch
(HIP events over back-to-back launches) and bitwise-equal tokens.  usage: argmax_engines.py [M ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import _lib, ops  # noqa: E402

_lib.require_device()
g = torch.Generator(device="cuda").manual_seed(0)
w = torch.randn(1000, 192, device="cuda", generator=g) * 0.07
b = torch.randn(1000, device="cuda", generator=g) * 0.1
for M in [int(v) for v in sys.argv[1:]] or [8016, 16032]:
    a = torch.randn(M, 192, device="cuda", generator=g)
    res = {}
    for eng in (1, 2):
        with ops.option(_lib.OPT_GEMM_ENGINE, eng):
            for _ in range(5):
                ops.gemm_argmax(a, w, b)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                out = ops.gemm_argmax(a, w, b)
            e1.record()
            torch.cuda.synchronize()
            res[eng] = (e0.elapsed_time(e1) * 1e3 / 50, out.clone())
    print(f"M={M}: tiles {res[1][0]:.2f} us, rows {res[2][0]:.2f} us (incl. the key reduction), "
          f"tokens equal {torch.equal(res[1][1], res[2][1])}", flush=True)
