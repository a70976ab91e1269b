#!/usr/bin/env python3
"""z-in-tail diagnostics on the GPU: which intermediate of the z-in-tail block differs from the
three-launch block (projection columns, ungated scan y, tail), and the isolated launch times of
both forms' kernels at the C2 shape (32 x 10 s)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "velocity-asr_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import velocity_asr as va  # noqa: E402
from velocity_asr import _lib, ops, synthetic as S  # noqa: E402
from velocity_asr.ssm import _tree_mode  # noqa: E402

DEV = "cuda"


def per_launch(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    B, L = int(sys.argv[1]) if len(sys.argv) > 1 else 9, int(sys.argv[2]) if len(sys.argv) > 2 else 501
    blk = m.local_ssm.layers[2]
    ssm = blk.ssm
    Di, N, D = ssm.d_inner, ssm.state_dim, 192
    x = torch.from_numpy(np.random.default_rng(B * L).standard_normal((B, L, D)).astype(np.float32)).to(DEV)
    p = ssm._prepared()
    mode = _tree_mode()
    with torch.no_grad():
        x2 = x.view(B * L, D)
        u = ops.ln_dwconv(x, blk.norm1.weight, blk.norm1.bias, ops.f32(blk.conv.weight).view(D, -1), blk.conv.bias,
                          blk.norm1.eps).view(B * L, D)
        xz, xdt = ssm.project(u)
        xbd = ops.gemm(u, p["w_noz"], p["b_noz"], epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=Di + 2 * N)
        print("x  equal", torch.equal(xz[:, :Di], xbd[:, :Di]))
        print("bc equal", torch.equal(xdt[:, :2 * N], xbd[:, Di:Di + 2 * N]))
        print("dt equal", torch.equal(xdt[:, 2 * N:], xbd[:, Di + 2 * N:]))
        yd = ops.ssm_scan_ungated(xbd[:, :Di], xbd[:, Di + 2 * N:], xbd[:, Di:Di + 2 * N], p["A2"], ssm.D, B, L, mode)
        # the gated scan with z = 256: silu(256) = 256 exactly (exp2 underflows to 0), so g / 256 = y exactly
        xz256 = xz.clone()
        xz256[:, Di:] = 256.0
        g256 = ops.ssm_scan(xz256, xdt[:, 2 * N:], xdt[:, :2 * N], p["A2"], ssm.D, B, L, mode)
        print("y  equal", torch.equal(g256 / 256.0, yd), (g256 / 256.0 - yd).abs().max().item())
        g = ssm.scan(xz, xdt, B, L)
        ref = blk.tail(g, x2, B, L).view(B * L, D)
        new = ops.ssm_block_tail_gated(yd, u, p["w_z"], mode, x2, ssm.out_proj.weight, blk.norm2.weight,
                                       blk.norm2.bias, blk.norm2.eps, blk.ffn[0].weight, blk.ffn[0].bias,
                                       blk.ffn[3].weight, blk.ffn[3].bias)
        d = (ref - new).abs()
        print("tail equal", torch.equal(ref, new), d.max().item(), "rows differing", int((d.amax(1) > 0).sum()))
        # z alone: the 1280 projection's z columns vs a z-only GEMM through the same engine
        z_only = ops.gemm(u, p["w_z"])
        print("z(gemm w_z) equal z(1280)", torch.equal(z_only, xz[:, Di:]), (z_only - xz[:, Di:]).abs().max().item())
        # gated tail fed yd = y: with z = 256 handled on the tail side we cannot read z; instead feed
        # the original tail g = the gated scan's own output and the gated tail yd = g256 / 256
        t = dict(
            proj1280=per_launch(lambda: ssm.project(u)),
            proj896=per_launch(lambda: ops.gemm(u, p["w_noz"], p["b_noz"], epilogue=_lib.EPI_SOFTPLUS_FROM,
                                                n_out=Di + 2 * N)),
            scan_gated=per_launch(lambda: ssm.scan(xz, xdt, B, L)),
            scan_ungated=per_launch(lambda: ops.ssm_scan_ungated(xbd[:, :Di], xbd[:, Di + 2 * N:],
                                                                 xbd[:, Di:Di + 2 * N], p["A2"], ssm.D, B, L, mode)),
            tail=per_launch(lambda: blk.tail(g, x2, B, L)),
            tail_gated=per_launch(lambda: ops.ssm_block_tail_gated(
                yd, u, p["w_z"], mode, x2, ssm.out_proj.weight, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps,
                blk.ffn[0].weight, blk.ffn[0].bias, blk.ffn[3].weight, blk.ffn[3].bias)),
            block_old=per_launch(lambda: blk.tail(ssm.scan(*ssm.project(u), B, L), x2, B, L)),
        )
        os.environ["VASR_Z_IN_TAIL"] = "1"
        t["block_z_in_tail"] = per_launch(lambda: blk(x))
        os.environ["VASR_Z_IN_TAIL"] = "0"
        t["block_gated"] = per_launch(lambda: blk(x))
        print(f"B={B} L={L} isolated us:", {k: round(v, 2) for k, v in t.items()})


if __name__ == "__main__":
    main()
