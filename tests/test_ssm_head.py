"""Fused SSMBlock head (vasr_ssm_block_head_f32): LayerNorm_1 + causal depthwise conv ->
in_proj -> [x_proj; dt_proj] + softplus in one kernel (reference ssm.py:404-414, :105-113).

Compared with the three launches it replaces (fp32 split-bf16 products: equal to fp32
accumulation-order rounding), including row tiles that straddle utterance boundaries (the
conv's causal window must not reach into the previous utterance).  The head is opt-in
(VASR_FUSED_HEAD=1; measured slower end to end)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _block(seed=0, bf16=False):
    import velocity_asr as va
    from velocity_asr import synthetic as S
    W = S.make_weights(None, seed=seed)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    if bf16:
        m = m.to(torch.bfloat16)
    return m.local_ssm.layers[1]


def _heads(blk, x):
    """(xz, xdt) from the fused kernel and from the unfused launches."""
    from velocity_asr import ops
    B, L, D = x.shape
    s = blk.ssm
    p = s._prepared()
    x2 = x.reshape(B * L, D).contiguous()
    fz, fd = ops.ssm_block_head(x2, B, L, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps,
                                ops.f32(blk.conv.weight).view(D, -1), blk.conv.bias, s.in_proj.weight,
                                p["w_xdt"], p["b_xdt"], 2 * s.state_dim)
    u = ops.ln_dwconv(x.contiguous(), blk.norm1.weight, blk.norm1.bias, ops.f32(blk.conv.weight).view(D, -1),
                      blk.conv.bias, blk.norm1.eps)
    from velocity_asr import _lib
    uz = ops.gemm(u.view(B * L, D), s.in_proj.weight)
    ud = ops.gemm(uz[:, :s.d_inner], p["w_xdt"], p["b_xdt"], epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=2 * s.state_dim)
    return fz, fd, uz, ud


@pytest.mark.parametrize("B,L", [(1, 1), (1, 2), (2, 3), (3, 50), (1, 501), (16, 501), (2, 1501)])
def test_head_matches_unfused(B, L):
    blk = _block()
    x = torch.from_numpy(np.random.default_rng(B * 1000 + L).standard_normal((B, L, 192)).astype(np.float32)).to(DEV)
    fz, fd, uz, ud = _heads(blk, x)
    torch.testing.assert_close(fz, uz, atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(fd, ud, atol=2e-5, rtol=1e-5)


def test_head_bf16_model():
    blk = _block(bf16=True)
    x = torch.from_numpy(np.random.default_rng(9).standard_normal((3, 300, 192)).astype(np.float32)).to(DEV)
    fz, fd, uz, ud = _heads(blk, x)
    assert (fz - uz).abs().max().item() < 2e-2 and (fz - uz).abs().mean().item() < 1e-3
    assert (fd - ud).abs().max().item() < 2e-2 and (fd - ud).abs().mean().item() < 1e-3


def test_block_fused_head_vs_unfused(monkeypatch):
    blk = _block(seed=1)
    x = torch.from_numpy(np.random.default_rng(4).standard_normal((2, 257, 192)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("VASR_FUSED_HEAD", "1")
    a = blk(x)
    monkeypatch.setenv("VASR_FUSED_HEAD", "0")
    b = blk(x)
    torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)
