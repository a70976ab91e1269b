"""Diagnostic (GPU box): the fused SSMBlock tail with its weights as pre-split bf16 planes
(vasr_ssm_block_tail_f32, 6 B per weight) against fp32 fragments split in registers
(vasr_ssm_block_tail_f32_frag, 4 B per weight): per M, 20 back-to-back launches of each between
one HIP event pair (3 warm-up launches), and whether the outputs are bitwise equal.
usage: tail_weights.py [M ...]   (default 501 1024 8016 16032)
Needs profiles/r04am/tail_frag_weights.patch applied (the fp32-fragment form was measured slower
and removed)."""
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


def run(fmt, g, x, out, n):
    ops.TAIL_WEIGHTS = fmt
    for _ in range(n):
        ops.ssm_block_tail(g, x, wo, lnw, lnb, 1e-5, w1, b1, w2, b2, out=out)


for M in [int(v) for v in sys.argv[1:]] or [501, 1024, 8016, 16032]:
    g = torch.randn(M, E, device=dev, generator=g0)
    x = torch.randn(M, D, device=dev, generator=g0)
    res = {}
    for rep in range(2):
        for fmt in ("planes", "frag"):
            out = torch.empty(M, D, device=dev)
            run(fmt, g, x, out, 3)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(fmt, g, x, out, 20)
            b.record()
            torch.cuda.synchronize()
            res.setdefault(fmt, []).append(a.elapsed_time(b) / 20 * 1e3)
            res[fmt + "_out"] = out
    same = torch.equal(res["planes_out"].view(torch.int32), res["frag_out"].view(torch.int32))
    print(f"M={M}: planes {min(res['planes']):.2f} us, frag {min(res['frag']):.2f} us "
          f"(runs {', '.join(f'{v:.2f}' for v in res['planes'])} / {', '.join(f'{v:.2f}' for v in res['frag'])}); "
          f"bitwise equal {same}", flush=True)
