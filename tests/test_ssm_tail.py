"""Fused SSMBlock tail (vasr_ssm_block_tail_f32): out_proj + residual -> LayerNorm_2 -> FFN1 +
GELU -> FFN2 + residual in one kernel (reference ssm.py:415-425).

Checked against an fp64 numpy restatement of the same four steps (fp32 parity bar: the
split-bf16 products are fp32-accurate), against the unfused launches, and at model level by
the golden-pinned parity suite (tests/test_gpu_parity.py), which runs with the fused tail (the
default)."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gelu(x):
    from scipy.special import erf
    return 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))


def _params(seed, D=192, E=384):
    rng = np.random.default_rng(seed)
    f = lambda *s, sc=1.0: (rng.standard_normal(s) * sc).astype(np.float32)  # noqa: E731
    return dict(wo=f(D, E, sc=1 / math.sqrt(E)), ln_w=(1 + 0.1 * rng.standard_normal(D)).astype(np.float32),
                ln_b=f(D, sc=0.1), w1=f(E, D, sc=1 / math.sqrt(D)), b1=f(E, sc=0.1),
                w2=f(D, E, sc=1 / math.sqrt(E)), b2=f(D, sc=0.1))


def _ref(g, x, P, eps=1e-5):
    g, x = g.astype(np.float64), x.astype(np.float64)
    x1 = g @ P["wo"].astype(np.float64).T + x
    mu = x1.mean(-1, keepdims=True)
    var = ((x1 - mu) ** 2).mean(-1, keepdims=True)
    h = (x1 - mu) / np.sqrt(var + eps) * P["ln_w"] + P["ln_b"]
    f = _gelu(h @ P["w1"].astype(np.float64).T + P["b1"])
    return f @ P["w2"].astype(np.float64).T + P["b2"] + x1


def _run(g, x, P, ldg=None):
    from velocity_asr import ops
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    gt = t(g)
    if ldg is not None:
        big = torch.zeros((g.shape[0], ldg), device=DEV)
        big[:, :g.shape[1]] = gt
        gt = big[:, :g.shape[1]]
    return ops.ssm_block_tail(gt, t(x), t(P["wo"]), t(P["ln_w"]), t(P["ln_b"]), 1e-5, t(P["w1"]), t(P["b1"]),
                              t(P["w2"]), t(P["b2"])).cpu().numpy()


@pytest.mark.parametrize("M", [1, 16, 31, 32, 33, 100, 501, 8016])
def test_tail_matches_fp64(M):
    rng = np.random.default_rng(M)
    P = _params(7)
    g = rng.standard_normal((M, 384)).astype(np.float32)
    x = rng.standard_normal((M, 192)).astype(np.float32)
    got = _run(g, x, P)
    ref = _ref(g, x, P)
    np.testing.assert_allclose(got, ref, atol=2e-5 * max(1.0, np.abs(ref).max()), rtol=2e-5)


@pytest.mark.parametrize("M", [17, 501, 4097])
def test_tail_row_forms_bitwise_equal(M):
    """16- and 32-row workgroups (VASR_OPT_TAIL_ROWS; the default takes 16 up to M = 4096) of 4, 6
    or 12 waves (VASR_OPT_TAIL_WAVES: 3, 2 or 1 output column tiles per wave) perform the same
    float operations per element: outputs are bitwise equal."""
    from velocity_asr import _lib, ops
    rng = np.random.default_rng(M + 1)
    P = _params(9)
    g = rng.standard_normal((M, 384)).astype(np.float32)
    x = rng.standard_normal((M, 192)).astype(np.float32)
    with ops.option(_lib.OPT_TAIL_ROWS, 16), ops.option(_lib.OPT_TAIL_WAVES, 4):
        a = _run(g, x, P)
    for rows in (16, 32):
        for waves in (4, 6, 12):
            with ops.option(_lib.OPT_TAIL_ROWS, rows), ops.option(_lib.OPT_TAIL_WAVES, waves):
                np.testing.assert_array_equal(_run(g, x, P), a, err_msg=f"rows {rows} waves {waves}")


def test_tail_strided_input():
    rng = np.random.default_rng(3)
    P = _params(8)
    g = rng.standard_normal((77, 384)).astype(np.float32)
    x = rng.standard_normal((77, 192)).astype(np.float32)
    np.testing.assert_allclose(_run(g, x, P, ldg=768), _ref(g, x, P), atol=1e-4, rtol=2e-5)


def test_fused_block_equals_unfused_launches(monkeypatch):
    """SSMBlock.forward with the fused tail vs the four launches it replaces (same model
    weights): equal to the fp32 rounding of the two accumulation groupings."""
    import velocity_asr as va
    from velocity_asr import synthetic as S
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    blk = m.to(DEV).eval().local_ssm.layers[3]
    x = torch.from_numpy(np.random.default_rng(5).standard_normal((3, 250, 192)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("VASR_FUSED_TAIL", "1")
    fused = blk(x)
    monkeypatch.setenv("VASR_FUSED_TAIL", "0")
    plain = blk(x)
    torch.testing.assert_close(fused, plain, atol=3e-5, rtol=1e-5)


def test_fused_block_bf16_model(monkeypatch):
    """The bf16 model's fused tail (vasr_ssm_block_tail_bf16: one bf16 plane, activations
    rounded to bf16 at the MFMA input as vasr_linear_bf16 does) vs the bf16 launches it
    replaces; both round h and f to bf16, so they agree to bf16 rounding of rare boundary
    cases."""
    import velocity_asr as va
    from velocity_asr import synthetic as S
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    blk = m.to(DEV).eval().to(torch.bfloat16).local_ssm.layers[2]
    x = torch.from_numpy(np.random.default_rng(6).standard_normal((2, 300, 192)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("VASR_FUSED_TAIL", "1")
    fused = blk(x)
    monkeypatch.setenv("VASR_FUSED_TAIL", "0")
    plain = blk(x)
    err = (fused - plain).abs()
    assert err.max().item() < 2e-2 and err.mean().item() < 1e-3, (err.max().item(), err.mean().item())


def _block(i):
    import velocity_asr as va
    from velocity_asr import synthetic as S
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    return m, m.local_ssm.layers[i]


@pytest.mark.parametrize("fma", ["1", "0"], ids=["mode2", "mode0"])
@pytest.mark.parametrize("B,L", [(9, 501), (32, 501), (11, 1501), (17, 257), (5, 1000)])
def test_z_in_tail_block_bitwise(monkeypatch, B, L, fma):
    """The z-in-tail block (projection without the z columns, ungated scan, tail that forms z
    with the split GEMM's exact product and applies the scan's gate) vs the three-launch block:
    bitwise equal, both scan modes, 4- and 2-states-per-lane scan layouts ((5, 1000): 480 waves)."""
    _, blk = _block(2)
    x = torch.from_numpy(np.random.default_rng(B * L).standard_normal((B, L, 192)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("VASR_SCAN_FMA", fma)
    monkeypatch.setenv("VASR_Z_IN_TAIL", "1")
    assert blk._z_in_tail(B, L, 192)
    a = blk(x)
    monkeypatch.setenv("VASR_Z_IN_TAIL", "0")
    assert not blk._z_in_tail(B, L, 192)
    b = blk(x)
    assert torch.equal(a, b), (a - b).abs().max().item()


def test_z_in_tail_model_logits_bitwise(monkeypatch):
    """C2's shape (32 x 10 s, one forward): the model's logits with and without z-in-tail are
    bitwise equal; small launches (one utterance) keep the gated scan."""
    import velocity_asr as va
    from velocity_asr import synthetic as S
    m, blk = _block(0)
    assert not blk._z_in_tail(1, 501, 192)
    mel = va.compute_mel_spectrogram(torch.from_numpy(S.make_audio(32, 160000, seed=1234)).to(DEV))
    monkeypatch.setenv("VASR_Z_IN_TAIL", "1")
    a = m(mel)
    monkeypatch.setenv("VASR_Z_IN_TAIL", "0")
    b = m(mel)
    assert torch.equal(a, b)


@pytest.mark.parametrize("fma", ["1", "0"], ids=["mode2", "mode0"])
@pytest.mark.parametrize("B,L", [(9, 501), (11, 1501), (5, 1000)])
def test_z_in_tail_block_bitwise_bf16(monkeypatch, B, L, fma):
    """The bf16 model's z-in-tail block (in_proj's x rows alone, ungated scan, tail that forms z
    with vasr_linear_bf16's one bf16 product per k-step and stages g rounded to bf16) vs the
    three-launch bf16 block: bitwise equal."""
    m, _ = _block(2)
    blk = m.to(torch.bfloat16).local_ssm.layers[2]
    x = torch.from_numpy(np.random.default_rng(B + L).standard_normal((B, L, 192)).astype(np.float32)).to(DEV)
    monkeypatch.setenv("VASR_SCAN_FMA", fma)
    monkeypatch.setenv("VASR_Z_IN_TAIL", "1")
    assert blk._z_in_tail(B, L, 192)
    a = blk(x)
    monkeypatch.setenv("VASR_Z_IN_TAIL", "0")
    assert not blk._z_in_tail(B, L, 192)
    b = blk(x)
    assert torch.equal(a, b), (a - b).abs().max().item()


def test_z_in_tail_model_logits_bitwise_bf16(monkeypatch):
    """C3's model (bf16 weights) on 32 x 10 s: logits with and without z-in-tail bitwise equal;
    a mixed-dtype block keeps the gated scan."""
    import velocity_asr as va
    from velocity_asr import synthetic as S
    m, _ = _block(0)
    m = m.to(torch.bfloat16)
    blk = m.local_ssm.layers[0]
    assert blk._z_in_tail(32, 501, 192)
    mel = va.compute_mel_spectrogram(torch.from_numpy(S.make_audio(32, 160000, seed=4321)).to(DEV))
    monkeypatch.setenv("VASR_Z_IN_TAIL", "1")
    a = m(mel)
    monkeypatch.setenv("VASR_Z_IN_TAIL", "0")
    b = m(mel)
    assert torch.equal(a, b)
    monkeypatch.setenv("VASR_Z_IN_TAIL", "1")
    blk.ffn[0].float()
    assert not blk._z_in_tail(32, 501, 192)


def test_z_in_tail_argument_checks():
    from velocity_asr import _lib
    lib = _lib.lib()
    x = torch.zeros(64, device=DEV)
    p = x.data_ptr()
    # mode 1 (recurrence) has no ungated form; a null u / wz is refused
    assert lib.vasr_ssm_scan_ungated_f32(p, 384, p, 384, p, 128, p, p, p, 384, 1, 1, 384, 64, 1, None) == -1
    assert lib.vasr_ssm_block_tail_gated_f32(p, 384, None, 192, p, 2, p, 192, p, p, p, 1e-5, p, p, p, p, p, 192,
                                             1, 192, 384, None) == -1
    assert b"u" in lib.vasr_last_error()
    assert lib.vasr_ssm_block_tail_gated_bf16(p, 384, p, 192, None, 2, p, 192, p, p, p, 1e-5, p, p, p, p, p, 192,
                                              1, 192, 384, None) == -1
    assert lib.vasr_ssm_block_tail_gated_bf16(p, 384, p, 192, p, 1, p, 192, p, p, p, 1e-5, p, p, p, p, p, 192,
                                              1, 192, 384, None) == -1
    assert b"mode" in lib.vasr_last_error()
