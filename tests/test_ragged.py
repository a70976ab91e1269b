"""Batches of clips with different lengths (zero-padded, per-utterance sizes on the device).

The reference runs one file at a time (scripts/transcribe.py:69-78, scripts/evaluate.py:91-98);
here clips of different lengths share one batch and every clip must get exactly what it gets
alone: its own reflect padding and mel statistics (audio.py:97-135), its own pooling sizes
(attention.py:37-44, :64-73) and attention keys, and its own collapse length.  Pinned against
the reference's golden tokens of each clip (tests/golden/fwd_*.npz, generated from the
reference by tests/golden/gen_goldens.py) and against the oracle.
"""
import json

import numpy as np
import pytest
import torch

from conftest import golden, record_error
from oracle import velocity_ref as R
from velocity_asr import synthetic as S

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOGIT_TOL = dict(atol=1e-4, rtol=1e-5)  # SURVEY §8(d); measured max |diff| 8.2e-6


@pytest.fixture(scope="module")
def va():
    import velocity_asr
    from velocity_asr import _lib
    _lib.load()
    return velocity_asr


@pytest.fixture(scope="module")
def model(va):
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    return m.to(DEV).eval()


def _pad(clips):
    ns = [len(c) for c in clips]
    a = np.zeros((len(clips), max(ns)), np.float32)
    for i, c in enumerate(clips):
        a[i, :len(c)] = c
    return torch.from_numpy(a).to(DEV), ns


def _golden_clips():
    """(audio, reference tokens (L,), name) for clips whose reference outputs are committed."""
    out = []
    b2 = golden("fwd_b2_3s.npz")
    a3 = S.make_audio(2, 48000, seed=21)
    out += [(a3[i], b2["tokens"][i], f"3s[{i}]") for i in range(2)]
    full = golden("fwd_fullbatch.npz")
    a10 = S.make_audio(32, 160000, seed=1234)
    out += [(a10[i], full["c2_tokens"][i].astype(np.int32), f"10s[{i}]") for i in (0, 7, 31)]
    out.append((S.make_audio(1, 480000, seed=4321)[0], golden("fwd_b1_30s.npz")["tokens"][0], "30s"))
    edge = golden("fwd_edge.npz")
    for S_, seed in ((201, 31), (400, 32), (8000, 34), (16333, 35)):
        out.append((S.make_audio(1, S_, seed=seed)[0], edge[f"S{S_}__tokens"][0], f"edge{S_}"))
    return out


def test_mel_of_a_padded_batch_is_each_clips_own(va):
    """Frames f < F_b are bitwise those of the clip alone (its own reflect end and statistics),
    later frames are 0."""
    from velocity_asr.audio import mel_on_device
    clips = [S.make_audio(1, n, seed=n)[0] for n in (16000, 48000, 24037, 201, 3333)]
    audio, ns = _pad(clips)
    mel = mel_on_device(audio, lengths=ns).cpu().numpy()
    for b, c in enumerate(clips):
        alone = va.compute_mel_spectrogram(torch.from_numpy(c).to(DEV)).cpu().numpy()
        F = len(c) // 160 + 1
        np.testing.assert_array_equal(mel[b, :F], alone, err_msg=f"clip {b}")
        assert not mel[b, F:].any()


def test_padded_batch_tokens_equal_reference_goldens(va, model):
    """One zero-padded batch of 3 s, 10 s, 30 s and edge-length clips: every clip's argmax
    tokens and greedy token list equal the reference's for that clip alone."""
    from velocity_asr.pipeline import audio_to_token_ids, token_lists
    items = _golden_clips()
    rng = np.random.default_rng(3)
    order = rng.permutation(len(items))  # lengths interleaved, not sorted
    items = [items[i] for i in order]
    audio, ns = _pad([c for c, _, _ in items])
    mel = va.compute_mel_spectrogram(audio, lengths=ns)
    frames = [n // 160 + 1 for n in ns]
    am = model.token_ids(mel, frames=frames).cpu().numpy()
    toks, lens = audio_to_token_ids(model, audio, lengths=ns)
    lists = token_lists(toks, lens)
    for b, (_, ref, name) in enumerate(items):
        L = model.get_output_length(frames[b])
        assert L == ref.shape[0], name
        np.testing.assert_array_equal(am[b, :L], ref, err_msg=name)
        assert lists[b] == R.ctc_greedy_decode(np.eye(1000, dtype=np.float32)[ref][None])[0], name


def test_padded_batch_logits_vs_oracle(va, model):
    """Logits of each clip's own rows against the oracle run on that clip alone; a uniform
    batch gives the same as before (lengths all equal to S)."""
    W = S.make_weights(None, seed=0)
    clips = [S.make_audio(1, n, seed=100 + n)[0] for n in (17600, 9000, 30011, 4000)]
    audio, ns = _pad(clips)
    mel = va.compute_mel_spectrogram(audio, lengths=ns)
    logits = model(mel, frames=[n // 160 + 1 for n in ns]).cpu().numpy()
    for b, c in enumerate(clips):
        ref = R.forward(W, R.compute_mel_spectrogram(c[None]), dict(S.DEFAULT_CONFIG))
        L = ref.shape[1]
        record_error(logits[b:b + 1, :L], ref, LOGIT_TOL)
        np.testing.assert_allclose(logits[b:b + 1, :L], ref, **LOGIT_TOL, err_msg=f"clip {b}")
        np.testing.assert_array_equal(logits[b, :L].argmax(-1), ref[0].argmax(-1))
    same = _pad([c[:4000] for c in clips])[0]
    a = model(va.compute_mel_spectrogram(same, lengths=[4000] * 4), frames=[26] * 4)
    b = model(va.compute_mel_spectrogram(same))
    assert torch.equal(a, b)


def test_var_kernels_against_numpy(va):
    """adaptive_pool / pooled_attention / ctc_collapse with per-utterance sizes."""
    from velocity_asr import ops
    rng = np.random.default_rng(0)
    B, L, C = 3, 40, 16
    x = rng.standard_normal((B, L, C)).astype(np.float32)
    lens, ks = [40, 17, 5], [9, 6, 5]
    out = ops.adaptive_pool(torch.from_numpy(x).to(DEV), 9, lens=torch.tensor(lens, dtype=torch.int32, device=DEV),
                            ks=torch.tensor(ks, dtype=torch.int32, device=DEV)).cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(out[b, :ks[b]], R.adaptive_avg_pool(x[b:b + 1, :lens[b]], ks[b])[0], atol=1e-6)
        assert not out[b, ks[b]:].any()
    # attention over each utterance's own keys = the uniform kernel on its own key set
    heads, hd, Kp, Lq = 4, 12, 20, 7
    A = heads * hd
    q = torch.from_numpy(rng.standard_normal((B * Lq, A)).astype(np.float32)).to(DEV)
    kv = torch.from_numpy(rng.standard_normal((B * Kp, 2 * A)).astype(np.float32)).to(DEV)
    kps = [20, 3, 11]
    o = ops.pooled_attention(q, kv, B, Lq, Kp, heads, kps=torch.tensor(kps, dtype=torch.int32, device=DEV))
    for b in range(B):
        ob = ops.pooled_attention(q[b * Lq:(b + 1) * Lq], kv[b * Kp:b * Kp + kps[b]].contiguous(), 1, Lq, kps[b],
                                  heads)
        assert torch.equal(o[b * Lq:(b + 1) * Lq], ob)
    pred = torch.from_numpy(rng.integers(0, 4, (B, 30)).astype(np.int32)).to(DEV)
    fr = [30, 12, 0]
    toks, n, st, en = ops.ctc_collapse(pred, 0, True, True, frames=torch.tensor(fr, dtype=torch.int32, device=DEV))
    for b in range(B):
        t1, n1, s1, e1 = ops.ctc_collapse(pred[b:b + 1, :fr[b]].contiguous(), 0, True, True) if fr[b] else (None,) * 4
        k = int(n[b])
        if fr[b] == 0:
            assert k == 0
            continue
        assert k == int(n1[0])
        assert torch.equal(toks[b, :k], t1[0, :k]) and torch.equal(st[b, :k], s1[0, :k]) and torch.equal(en[b, :k], e1[0, :k])


def test_length_checks(va, model):
    from velocity_asr.audio import mel_on_device
    audio = torch.zeros((2, 1000), device=DEV)
    with pytest.raises(RuntimeError, match="lengths"):
        mel_on_device(audio, lengths=[1000, 150])
    with pytest.raises(RuntimeError, match="lengths"):
        mel_on_device(audio, lengths=[1001, 500])
    mel = mel_on_device(audio, lengths=[1000, 500])
    with pytest.raises(ValueError, match="frames"):
        model(mel, frames=[7, 0])


@pytest.mark.parametrize("lengths", [None, [16000, 9000, 12345]])
def test_zero_framed_mel_feeds_the_conv_in_place(va, model, lengths):
    """the pipeline's mel is written into a zero-framed (B, F + 2, 80) buffer
    by the normalisation pass (no padding kernel); the view equals compute_mel_spectrogram bit
    for bit, the outer frames are 0, and the model's outputs on it equal those on the plain mel."""
    from velocity_asr import ops
    from velocity_asr.audio import mel_on_device
    audio = torch.from_numpy(S.make_audio(3, 16000, seed=77)).to(DEV)
    if lengths is not None:
        for b, n in enumerate(lengths):
            audio[b, n:] = 0
    plain = mel_on_device(audio, lengths=lengths)
    framed = mel_on_device(audio, lengths=lengths, frame_pad=1)
    assert torch.equal(framed, plain)
    buf = ops.zero_framed(framed, 1)
    assert buf is not None and tuple(buf.shape) == (3, plain.shape[1] + 2, 80)
    assert not buf[:, 0].any() and not buf[:, -1].any()
    frames = None if lengths is None else [n // 160 + 1 for n in lengths]
    assert torch.equal(model(framed, frames=frames), model(plain.clone(), frames=frames))
    assert ops.zero_framed(plain, 1) is None and ops.zero_framed(framed.clone(), 1) is None
