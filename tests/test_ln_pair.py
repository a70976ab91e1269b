"""The paired LayerNorm (vasr_layer_norm_pair_f32): the local stack's final norm and the global
context's query norm in one launch.  Both outputs bitwise equal to two vasr_layer_norm_f32 calls,
and the model's logits / tokens bitwise equal with the pair on (VASR_LN_PAIR=1, default) and off."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("rows,C,ld", [(1, 192, 192), (7, 192, 192), (16032, 192, 192), (1001, 192, 256),
                                       (33, 384, 384), (5, 80, 80), (9, 1000, 1000), (3, 1024, 1030)])
def test_layer_norm_pair_bitwise(rows, C, ld):
    from velocity_asr import ops
    g = torch.Generator(device=DEV).manual_seed(rows * 7 + C)
    xs = torch.randn(rows, ld, device=DEV, generator=g) * 3 + 0.5
    x = xs[:, :C]  # row stride ld
    w1, b1 = 1 + 0.2 * torch.randn(C, device=DEV, generator=g), 0.1 * torch.randn(C, device=DEV, generator=g)
    w2, b2 = 1 + 0.2 * torch.randn(C, device=DEV, generator=g), 0.1 * torch.randn(C, device=DEV, generator=g)
    y1, y2 = ops.layer_norm_pair(x, w1, b1, 1e-5, w2, b2, 1e-6)
    r1 = ops.layer_norm(x, w1, b1, 1e-5)
    r2 = ops.layer_norm(r1, w2, b2, 1e-6)
    assert torch.equal(y1, r1)
    assert torch.equal(y2, r2)
    ref = torch.nn.functional.layer_norm(x.double(), (C,), w1.double(), b1.double(), 1e-5)
    assert (y1.double() - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


def test_layer_norm_pair_argument_checks():
    from velocity_asr import _lib
    lib = _lib.lib()
    x = torch.zeros(192, device=DEV)
    p = x.data_ptr()
    assert lib.vasr_layer_norm_pair_f32(p, 192, p, p, 1e-5, p, 192, None, p, 1e-5, x[1:].data_ptr(), 192, 1, 192,
                                        None) == -1
    assert b"null" in lib.vasr_last_error()
    assert lib.vasr_layer_norm_pair_f32(p, 192, p, p, 1e-5, p, 192, p, p, 1e-5, p, 192, 1, 192, None) == -1
    assert b"differ" in lib.vasr_last_error()
    assert lib.vasr_layer_norm_pair_f32(p, 192, p, p, 1e-5, p, 192, p, p, 1e-5, x[1:].data_ptr(), 192, 1, 1025,
                                        None) == -1


@pytest.mark.parametrize("B,S", [(2, 48000), (32, 160000)])
def test_model_ln_pair_bitwise(monkeypatch, B, S):
    import velocity_asr as va
    from velocity_asr import synthetic as S_
    W = S_.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    mel = va.compute_mel_spectrogram(torch.from_numpy(S_.make_audio(B, S, seed=99)).to(DEV))
    monkeypatch.setenv("VASR_LN_PAIR", "1")
    a, fa = m(mel, return_features=True)
    ta = m.greedy_token_ids(mel)
    monkeypatch.setenv("VASR_LN_PAIR", "0")
    b, fb = m(mel, return_features=True)
    tb = m.greedy_token_ids(mel)
    assert torch.equal(fa["local_features"], fb["local_features"])
    assert torch.equal(a, b)
    assert torch.equal(ta[1], tb[1])  # collapsed lengths; tokens past them are unwritten
    assert all(torch.equal(ta[0][i, :n], tb[0][i, :n]) for i, n in enumerate(ta[1].tolist()))
