"""LayerNorms folded into neighbouring launches, each bitwise the separate launches:
* the paired LayerNorm (vasr_layer_norm_pair_f32): the local stack's final norm and the global
  context's query norm in one launch (VASR_LN_PAIR);
* the temporal binding's LayerNorm inside the first SSM block's norm1 + conv launch
  (vasr_ln_dwconv_prenorm_f32, VASR_TB_PRENORM);
* the global SSM stack's final LayerNorm inside the second pooling launch
  (vasr_ln_adaptive_pool_f32, VASR_POOL_PRENORM).
The model's logits / tokens are compared with each fold on and off against every LayerNorm as its
own launch."""
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


@pytest.mark.parametrize("B,L", [(1, 1), (1, 5), (2, 37), (3, 129), (32, 501)])
def test_ln_dwconv_prenorm_bitwise(B, L):
    from velocity_asr import _lib, ops
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + L)
    C = 192
    x = torch.randn(B, L, C, device=DEV, generator=g) * 2 + 0.3
    rn = lambda *s, sc=0.2: torch.randn(*s, device=DEV, generator=g) * sc  # noqa: E731
    pw, pb, lw, lb, cw, cb = 1 + rn(C), rn(C), 1 + rn(C), rn(C), rn(C, 4, sc=0.5), rn(C)
    ref_x = ops.layer_norm(x, pw, pb, 1e-5)
    for rows in (0, 4, 8, 16):
        with ops.option(_lib.OPT_DW_ROWS, rows):
            y, xo = ops.ln_dwconv_prenorm(x, pw, pb, 1e-5, lw, lb, cw, cb, 1e-6)
            ref_y = ops.ln_dwconv(ref_x, lw, lb, cw, cb, 1e-6)
        assert torch.equal(xo, ref_x), rows
        assert torch.equal(y, ref_y), rows


def test_ln_dwconv_prenorm_argument_checks():
    from velocity_asr import _lib
    lib = _lib.lib()
    x = torch.zeros(4 * 192, device=DEV)
    p, q, r = x.data_ptr(), x[192:].data_ptr(), x[384:].data_ptr()
    assert lib.vasr_ln_dwconv_prenorm_f32(p, p, p, 1e-5, q, p, p, p, p, None, 1, 1, 192, 4, 1e-5, None) == -1
    assert b"null" in lib.vasr_last_error()
    assert lib.vasr_ln_dwconv_prenorm_f32(p, p, p, 1e-5, p, p, p, p, p, r, 1, 1, 192, 4, 1e-5, None) == -1
    assert b"distinct" in lib.vasr_last_error()
    assert lib.vasr_ln_dwconv_prenorm_f32(p, p, p, 1e-5, q, p, p, p, p, r, 1, 1, 128, 4, 1e-5, None) == -1
    assert lib.vasr_ln_dwconv_prenorm_f32(p, p, p, 1e-5, q, p, p, p, p, r, 1, 1, 192, 3, 1e-5, None) == -1


@pytest.mark.parametrize("B,L,K,C", [(32, 64, 16, 192), (2, 37, 9, 192), (1, 5, 5, 192), (3, 63, 16, 80),
                                     (2, 200, 64, 192), (1, 64, 1, 192)])
def test_ln_adaptive_pool_bitwise(B, L, K, C):
    from velocity_asr import ops
    g = torch.Generator(device=DEV).manual_seed(B * 100 + L + K)
    x = torch.randn(B, L, C, device=DEV, generator=g) * 2 - 0.4
    w, b = 1 + 0.2 * torch.randn(C, device=DEV, generator=g), 0.1 * torch.randn(C, device=DEV, generator=g)
    ref = ops.adaptive_pool(ops.layer_norm(x, w, b, 1e-5), K)
    assert torch.equal(ops.ln_adaptive_pool(x, w, b, 1e-5, K), ref)
    if B > 1:  # per-utterance sizes: utterance 1 pools its first rows into fewer bins, the rest 0
        lens = torch.tensor([L] + [max(K // 2, L // 2)] * (B - 1), dtype=torch.int32, device=DEV)
        ks = torch.tensor([K] + [max(1, K // 2)] * (B - 1), dtype=torch.int32, device=DEV)
        ref = ops.adaptive_pool(ops.layer_norm(x, w, b, 1e-5), K, lens=lens, ks=ks)
        assert torch.equal(ops.ln_adaptive_pool(x, w, b, 1e-5, K, lens=lens, ks=ks), ref)


def test_ln_adaptive_pool_argument_checks():
    from velocity_asr import _lib
    lib = _lib.lib()
    x = torch.zeros(192 * 4, device=DEV)
    p = x.data_ptr()
    assert lib.vasr_ln_adaptive_pool_f32(p, p, None, 1e-5, p, 1, 4, 192, 2, None, None, None) == -1
    assert b"null" in lib.vasr_last_error()
    assert lib.vasr_ln_adaptive_pool_f32(p, p, p, 1e-5, p, 1, 4, 192, 5, None, None, None) == -1
    assert lib.vasr_ln_adaptive_pool_f32(p, p, p, 1e-5, p, 1, 4, 192, 2, p, None, None) == -1
    assert b"together" in lib.vasr_last_error()


FOLDS = ("VASR_LN_PAIR", "VASR_TB_PRENORM", "VASR_POOL_PRENORM")


@pytest.mark.parametrize("B,S", [(1, 16000), (2, 48000), (32, 160000)])
def test_model_ln_folds_bitwise(monkeypatch, B, S):
    import velocity_asr as va
    from velocity_asr import synthetic as S_
    W = S_.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    mel = va.compute_mel_spectrogram(torch.from_numpy(S_.make_audio(B, S, seed=99)).to(DEV))
    for k in FOLDS:  # every LayerNorm its own launch
        monkeypatch.setenv(k, "0")
    ref = m(mel)
    ref_f, _ = m(mel, return_features=True)
    assert torch.equal(ref_f, ref)
    runs = []
    for on in ((1, 1, 1), (0, 1, 1), (1, 0, 1), (1, 1, 0), (0, 0, 0)):
        for k, v in zip(FOLDS, on):
            monkeypatch.setenv(k, str(v))
        runs.append((m(mel), m.greedy_token_ids(mel), m.token_ids(mel)))
    for logits, (tok, n), ids in runs:
        assert torch.equal(logits, ref)
        assert torch.equal(ids, runs[0][2])
        assert torch.equal(n, runs[0][1][1])  # collapsed lengths; tokens past them are unwritten
        assert all(torch.equal(tok[i, :k], runs[0][1][0][i, :k]) for i, k in enumerate(n.tolist()))


def test_model_ln_folds_ragged_bitwise(monkeypatch):
    """A zero-padded batch of clips of different lengths (per-utterance pooling sizes)."""
    import velocity_asr as va
    from velocity_asr import synthetic as S_
    W = S_.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    ns = [48000, 20800, 33600]
    audio = torch.from_numpy(S_.make_audio(3, 48000, seed=7)).to(DEV)
    for i, n in enumerate(ns):
        audio[i, n:] = 0
    mel = va.compute_mel_spectrogram(audio, lengths=ns)
    frames = [n // 160 + 1 for n in ns]
    outs = []
    for on in ("0", "1"):
        for k in FOLDS:
            monkeypatch.setenv(k, on)
        outs.append(m(mel, frames=frames))
    for i, f in enumerate(frames):
        r = m.get_output_length(f)
        assert torch.equal(outs[0][i, :r], outs[1][i, :r])
