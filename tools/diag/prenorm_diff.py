"""Where vasr_ln_dwconv_prenorm_f32's xo differs from vasr_layer_norm_f32 (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "velocity-asr_amd"))
import torch  # noqa: E402

from velocity_asr import ops  # noqa: E402

DEV = "cuda"
for B, L in ((1, 37), (2, 5), (2, 37), (1, 129), (3, 129)):
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + L)
    C = 192
    x = torch.randn(B, L, C, device=DEV, generator=g) * 2 + 0.3
    rn = lambda *s, sc=0.2: torch.randn(*s, device=DEV, generator=g) * sc  # noqa: E731
    pw, pb, lw, lb, cw, cb = 1 + rn(C), rn(C), 1 + rn(C), rn(C), rn(C, 4, sc=0.5), rn(C)
    ref_x = ops.layer_norm(x, pw, pb, 1e-5)
    y, xo = ops.ln_dwconv_prenorm(x, pw, pb, 1e-5, lw, lb, cw, cb, 1e-6)
    d = (xo != ref_x)
    rows = d.any(-1).nonzero().tolist()
    ulp = (xo.view(torch.int32) - ref_x.view(torch.int32)).abs().max().item()
    print(B, L, "rows differing", rows[:20], "n", len(rows), "max ulp", ulp,
          "cols in first", d[rows[0][0], rows[0][1]].nonzero().flatten().tolist()[:10] if rows else None, flush=True)
