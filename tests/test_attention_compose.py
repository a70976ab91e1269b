"""The cross-attention's out_proj folded into the gated fusion's global-branch product
(GatedFusion.forward_attention, the default; VASR_ATTN_COMPOSE=0 keeps the separate GEMM).
global_context = o Wo^T + bo is read only by that product (reference attention.py:303-319, :190-220),
so the composite [gate_g | global_proj] Wo is formed in float64 and rounded once: the result differs
from the two GEMMs only by global_context's fp32 rounding (as the SSM's composed projection skips
x_p's).  Tolerance: 1e-5 relative to the output's scale."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(dtype=torch.float32):
    import velocity_asr as va
    from velocity_asr import synthetic as S
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    return m.to(DEV).to(dtype).eval()


@pytest.mark.parametrize("B,L", [(1, 501), (3, 250), (32, 501)])
def test_composed_fusion_matches_separate(monkeypatch, B, L):
    m = _model()
    ctx = m.global_context
    assert ctx.fusion.composable(ctx.cross_attention)
    x = torch.from_numpy(np.random.default_rng(B * L).standard_normal((B, L, 192)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("VASR_ATTN_COMPOSE", "1")
    a = ctx(x)
    monkeypatch.setenv("VASR_ATTN_COMPOSE", "0")
    assert not ctx.fusion.composable(ctx.cross_attention)
    b = ctx(x)
    scale = b.abs().max().item()
    err = (a - b).abs().max().item()
    assert err <= 1e-5 * scale, (err, scale)


def test_composed_fusion_bf16_and_logits(monkeypatch):
    """bf16 model: composite rounded to bf16 (bf16 tolerance); fp32 model: logits within the headline
    tolerance of the separate form."""
    m = _model()
    from velocity_asr import synthetic as S
    import velocity_asr as va
    mel = va.compute_mel_spectrogram(torch.from_numpy(S.make_audio(2, 160000, seed=7)).to(DEV))
    monkeypatch.setenv("VASR_ATTN_COMPOSE", "1")
    a = m(mel)
    monkeypatch.setenv("VASR_ATTN_COMPOSE", "0")
    b = m(mel)
    torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-5)
    mb = _model(torch.bfloat16)
    monkeypatch.setenv("VASR_ATTN_COMPOSE", "1")
    a16 = mb(mel)
    monkeypatch.setenv("VASR_ATTN_COMPOSE", "0")
    b16 = mb(mel)
    assert (a16 - b16).abs().max().item() < 0.1


def test_quantized_fusion_keeps_separate_out_proj():
    """QAT layers (fake-quant on global_context or the fusion inputs) are not folded."""
    from velocity_asr import quantize as Q
    qm = Q.prepare_model_for_qat(_model())
    assert not qm.global_context.fusion.composable(qm.global_context.cross_attention)
