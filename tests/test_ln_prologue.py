"""Row-LayerNorm prologue of the split GEMM (vasr_gemm_args.ln_w / ln_b / ln_eps): the
LayerNorm is computed inside the GEMM's A read with the float operations of
vasr_layer_norm_f32, so LN-in-GEMM equals LayerNorm-then-GEMM bit for bit (x3 and bf16
engines, every supported epilogue, ragged M, strided rows), and it matches the oracle's
LayerNorm + fp64 product to the GEMM tolerance.  Used by SSMBlock norm2 -> FFN-in and the
CTC head (reference ssm.py:394-427, model.py:218-227)."""

import numpy as np
import pytest
import torch

from oracle import velocity_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture()
def ops(monkeypatch):
    from velocity_asr import _lib, ops
    _lib.require_device()
    _lib.load()
    monkeypatch.setenv("VASR_LN_PROLOGUE", "1")  # the fused form is opt-in (see ops._ln_prologue)
    return ops


def _inputs(M, K, N, seed):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(M, K, generator=g) * 2 + 0.5
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    lw = 1 + 0.1 * torch.randn(K, generator=g)
    lb = 0.1 * torch.randn(K, generator=g)
    aux = torch.randn(M, N, generator=g)
    return [t.to(DEV) for t in (a, w, b, lw, lb, aux)]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("M,K,N", [(8016, 192, 384), (501, 192, 1000), (33, 384, 192), (1, 192, 64), (130, 192, 768)])
@pytest.mark.parametrize("epi", ["none", "gelu", "residual", "argmax"])
def test_ln_prologue_equals_ln_then_gemm(ops, dtype, M, K, N, epi):
    from velocity_asr import _lib
    a, w, b, lw, lb, aux = _inputs(M, K, N, M + K + N)
    if dtype == "bf16":
        w = w.to(torch.bfloat16)
    ln = (lw, lb, 1e-5)
    h = ops.layer_norm(a, lw, lb, 1e-5)
    if epi == "argmax":
        fused = ops.gemm_argmax(a, w, b, ln=ln)
        ref = ops.gemm_argmax(h, w, b)
    else:
        e = {"none": _lib.EPI_NONE, "gelu": _lib.EPI_GELU, "residual": _lib.EPI_RESIDUAL}[epi]
        kw = {"aux": aux} if epi == "residual" else {}
        fused = ops.gemm(a, w, b, epilogue=e, ln=ln, **kw)
        ref = ops.gemm(h, w, b, epilogue=e, **kw)
    assert torch.equal(fused, ref)


def test_ln_prologue_vs_oracle_and_strided_rows(ops):
    """Strided A rows (a column slice of a wider buffer) and the oracle's LayerNorm in fp64."""
    g = torch.Generator().manual_seed(3)
    big = (torch.randn(700, 256, generator=g) * 3).to(DEV)
    a = big[:, 32:224]
    w = (torch.randn(384, 192, generator=g) / 14).to(DEV)
    b = torch.randn(384, generator=g).to(DEV)
    lw = (1 + 0.1 * torch.randn(192, generator=g)).to(DEV)
    lb = (0.1 * torch.randn(192, generator=g)).to(DEV)
    out = ops.gemm(a, w, b, ln=(lw, lb, 1e-5)).cpu().double()
    h = R.layer_norm(a.cpu().numpy(), lw.cpu().numpy(), lb.cpu().numpy())
    ref = torch.from_numpy(h).double() @ w.cpu().double().T + b.cpu().double()
    assert (out - ref).abs().max().item() < 2e-5 * ref.abs().max().item()
    assert torch.equal(ops.gemm(a, w, b, ln=(lw, lb, 1e-5)), ops.gemm(ops.layer_norm(a, lw, lb), w, b))


def test_ln_prologue_falls_back_off_the_fused_path(ops, monkeypatch):
    """The f32 engine and unsupported K / epilogues run vasr_layer_norm_f32 first: same result."""
    from velocity_asr import _lib
    a, w, b, lw, lb, _ = _inputs(300, 192, 128, 9)
    ln = (lw, lb, 1e-5)
    fused = ops.gemm(a, w, b, ln=ln)
    prev = ops.set_gemm_mode("f32")
    try:
        f32 = ops.gemm(a, w, b, ln=ln)
        f32_ref = ops.gemm(ops.layer_norm(a, lw, lb), w, b)
    finally:
        ops.set_gemm_mode(prev)
    assert torch.equal(f32, f32_ref)
    assert (f32 - fused).abs().max().item() < 2e-5 * fused.abs().max().item()
    monkeypatch.setenv("VASR_LN_PROLOGUE", "0")
    assert torch.equal(ops.gemm(a, w, b, ln=ln), fused)
    sp = ops.gemm(a, w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=64, ln=ln)  # not fused: LN kernel first
    assert torch.equal(sp, ops.gemm(ops.layer_norm(a, lw, lb), w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=64))
