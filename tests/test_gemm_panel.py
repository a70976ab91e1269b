"""The LDS-resident-panel main loop of the split-bf16 GEMM (csrc/gemm_panel.hip) against the
LDS-ring tile main loop on the same inputs: both run the same MFMA sequence per output
element, so every output (and every fused-argmax key) is bit-identical.  Shapes: the model's
K = 192 / 384 GEMMs at ragged M, N not a multiple of the 64-column panel, strided A rows,
batched A/C/aux, every unpaired epilogue, per-column fake-quant parameters."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from velocity_asr import _lib, ops
    _lib.require_device()
    _lib.load()
    return ops


def both(ops, fn):
    """(tiles, panel) outputs; the 2-waves-per-SIMD panel variant must equal the default one."""
    outs = {}
    for eng in ("tiles", "panel", "panel2"):
        prev = ops.set_x3_engine(eng)
        try:
            outs[eng] = fn().cpu()
        finally:
            ops.set_x3_engine(prev)
    assert torch.equal(outs["panel"], outs["panel2"])
    return outs["tiles"], outs["panel"]


@pytest.mark.parametrize("M,N,K", [(16032, 768, 192), (8016, 512, 384), (8016, 192, 384), (8016, 384, 192),
                                   (8016, 1000, 192), (1, 64, 192), (33, 100, 384), (250, 40, 192)])
@pytest.mark.parametrize("epi", ["none", "gelu", "softplus", "residual", "gelu_pe"])
def test_gemm_panel_matches_tiles(ops, M, N, K, epi):
    from velocity_asr import _lib
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    kw = {}
    e = {"none": _lib.EPI_NONE, "gelu": _lib.EPI_GELU, "softplus": _lib.EPI_SOFTPLUS_FROM,
         "residual": _lib.EPI_RESIDUAL, "gelu_pe": _lib.EPI_GELU_PE}[epi]
    if epi == "softplus":
        kw["n_out"] = N // 3
    if epi in ("residual", "gelu_pe"):
        kw["aux"] = torch.randn(M, N, generator=g).to(DEV)
    t, p = both(ops, lambda: ops.gemm(a, w, b, epilogue=e, **kw))
    assert torch.equal(t, p)
    ref = a.double() @ w.double().T + b.double()
    if epi == "none":
        assert (p.double() - ref.cpu()).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())


def test_gemm_panel_strided_batched_qparams(ops):
    """xz[:, :Di] (row stride 2 Di) as A; a 3-utterance batched GEMM with aux; fake-quant
    columns (scale 0 = passthrough) in the epilogue."""
    g = torch.Generator().manual_seed(9)
    xz = torch.randn(5000, 768, generator=g).to(DEV)
    w = (torch.randn(512, 384, generator=g) / 20).to(DEV)
    b = torch.randn(512, generator=g).to(DEV)
    from velocity_asr import _lib
    t, p = both(ops, lambda: ops.gemm(xz[:, :384], w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=128))
    assert torch.equal(t, p)
    qp = torch.zeros(512, 4)
    qp[::2, 0] = 0.05
    qp[:, 2], qp[:, 3] = -128, 127
    qp = qp.to(DEV)
    t, p = both(ops, lambda: ops.gemm(xz[:, :384], w, b, qparams=qp))
    assert torch.equal(t, p)
    base = torch.randn(3, 700 * 192, generator=g).to(DEV)
    w2 = (torch.randn(192, 192, generator=g) / 14).to(DEV)
    aux = torch.randn(3, 650, 192, generator=g).to(DEV)

    def run():
        out = torch.empty(3, 650, 192, device=DEV)
        ops.gemm_batched(base, 192, 700 * 192, 650, 3, 192, w2, None, out, 192, 650 * 192,
                         epilogue=_lib.EPI_RESIDUAL, aux=aux, ld_aux=192, stride_aux=650 * 192)
        return out
    t, p = both(ops, run)
    assert torch.equal(t, p)


@pytest.mark.parametrize("M", [1, 501, 16032])
def test_gemm_panel_argmax_matches_tiles(ops, M):
    g = torch.Generator().manual_seed(M)
    a = torch.randn(M, 192, generator=g).to(DEV)
    w = (torch.randn(1000, 192, generator=g) / 14).to(DEV)
    b = torch.randn(1000, generator=g).to(DEV)
    a[: M // 2, :] = 0  # ties: every logit = bias -> first max index
    t, p = both(ops, lambda: ops.gemm_argmax(a, w, b))
    assert torch.equal(t, p)
    logits = ops.gemm(a, w, b)
    assert torch.equal(p.long(), logits.argmax(1).cpu())
