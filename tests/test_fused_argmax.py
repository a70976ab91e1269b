"""CTC head with the row argmax fused into the GEMM epilogue (SURVEY §8 f rank 1): the
(B, L, V) logits are never written.  Integer output, so the bar is bit-exact: the fused
argmax must equal torch's argmax (first index on ties, decode.py:46) of the logits the same
GEMM engine writes, and the reference goldens' tokens."""

import numpy as np
import pytest
import torch

from conftest import golden, golden_json
from oracle import velocity_ref as R
from velocity_asr import synthetic as S

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def va():
    import velocity_asr
    from velocity_asr import _lib
    _lib.require_device()
    _lib.load()
    return velocity_asr


@pytest.mark.parametrize("engine", ["x3", "bf16"])
@pytest.mark.parametrize("M,N,K", [(1, 64, 32), (77, 1000, 192), (16032, 1000, 192), (300, 50, 96), (129, 257, 192)])
def test_gemm_argmax_matches_logits(va, engine, M, N, K):
    from velocity_asr import ops
    g = torch.Generator().manual_seed(M + N)
    a = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    w[N // 2] = w[N // 3]             # duplicate rows -> exact ties between two columns
    w[N - 1] = w[N // 3]
    b = torch.randn(N, generator=g) * 0.1
    b[N // 2] = b[N // 3]
    b[N - 1] = b[N // 3]
    a[: M // 2] *= 0.0                # rows whose logits are the bias alone (ties on bias)
    if engine == "bf16":
        w = w.to(torch.bfloat16)
    A, W, Bv = a.to(DEV), w.to(DEV), b.to(DEV)
    logits = ops.gemm(A, W, Bv)
    want = torch.argmax(logits, dim=-1).to(torch.int32).cpu()
    got = ops.gemm_argmax(A, W, Bv).cpu()
    assert torch.equal(got, want)


def test_model_token_ids(va):
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    for fname, (B, S_, seed) in (("fwd_b2_10s.npz", (2, 160000, 1234)), ("fwd_b2_3s.npz", (2, 48000, 21))):
        audio = torch.from_numpy(S.make_audio(B, S_, seed=seed)).to(DEV)
        mel = va.compute_mel_spectrogram(audio)
        ids = m.token_ids(mel).cpu().numpy()
        logits = m(mel)
        assert np.array_equal(ids, logits.argmax(-1).cpu().numpy())
        assert np.array_equal(ids, golden(fname)["tokens"])


def test_pipeline_tokens_equal_golden_greedy(va):
    from velocity_asr.pipeline import audio_to_token_ids, token_lists
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    audio = torch.from_numpy(S.make_audio(2, 160000, seed=1234)).to(DEV)
    toks, lens = audio_to_token_ids(m, audio)
    assert token_lists(toks, lens) == golden_json("decode_fwd.json")["results"]["b2_10s"]


def test_int8_token_ids(va):
    from velocity_asr import quantize as Q
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = Q.prepare_model_for_qat(m).to(DEV).eval()
    audio = torch.from_numpy(S.make_audio(2, 48000, seed=21)).to(DEV)
    mel = va.compute_mel_spectrogram(audio)
    Q.calibrate_from_activations(m, mel)
    assert np.array_equal(m.token_ids(mel).cpu().numpy(), m(mel).argmax(-1).cpu().numpy())


@pytest.mark.parametrize("streams", [1, 2])
def test_graphed_streams_match_eager(va, streams):
    """The bench's timed path: utterance groups as HIP graphs on concurrent streams."""
    from velocity_asr.pipeline import GraphedTranscriber, audio_to_token_ids, token_lists
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    audio = torch.from_numpy(S.make_audio(4, 48000, seed=8)).to(DEV)
    te, le = audio_to_token_ids(m, audio)
    gt = GraphedTranscriber(m, 4, 48000, streams=streams)
    gt.audio.copy_(audio)
    gt.step()
    gt.step()
    torch.cuda.synchronize()
    assert token_lists(*gt.collect()) == token_lists(te, le)
    # the static outputs are refreshed by every replay (all stream groups write their rows)
    assert token_lists(gt.tokens, gt.lengths) == token_lists(te, le)
    gt.audio.copy_(torch.flip(audio, [0]))
    gt.step()
    torch.cuda.synchronize()
    assert token_lists(gt.tokens, gt.lengths) == token_lists(te, le)[::-1]


def test_graphed_transcriber_refuses_changed_weights(va):
    """Replaying graphs whose weights were modified (or whose derived layouts were rebuilt)
    would read stale pointers: step() must raise instead."""
    from velocity_asr.pipeline import GraphedTranscriber
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    gt = GraphedTranscriber(m, 2, 16000, streams=2)
    gt.step()
    with torch.no_grad():
        m.ctc_head.proj[2].bias.add_(1.0)
    with pytest.raises(RuntimeError, match="changed after capture"):
        gt.step()
    # the replay that ran on the old weights is not handed out
    with pytest.raises(RuntimeError, match="changed after capture"):
        gt.collect()
    torch.cuda.synchronize()
    # its static outputs are cleared: a caller holding the buffers sees empty transcripts
    assert (gt.lengths == 0).all() and (gt.tokens == 0).all()
    from velocity_asr.distributed import graphed_step
    with pytest.raises(RuntimeError, match="changed after capture"):
        graphed_step(gt)(gt.audio)


@pytest.mark.parametrize("N", [5, 1000])
@pytest.mark.parametrize("B,Lq", [(1, 1), (1, 63), (1, 64), (1, 65), (1, 501), (3, 130)])
@pytest.mark.parametrize("collapse,timestamps,ragged", [(True, False, False), (False, False, False),
                                                       (True, True, False), (True, False, True),
                                                       (True, True, True)])
def test_ctc_greedy_one_launch_matches_argmax_then_collapse(va, N, B, Lq, collapse, timestamps, ragged):
    """vasr_ctc_collapse_keys (argmax keys + collapse in one launch) equals vasr_argmax_keys then
    vasr_ctc_collapse[_var] exactly: tokens, lengths, timestamps, per-frame argmax; a 5-token
    vocabulary gives long runs, repeats across blanks and empty outputs."""
    from velocity_asr import _lib, ops
    g = torch.Generator().manual_seed(B * 1000 + Lq + N)
    K = 32
    a = torch.randn(B * Lq, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.5).to(DEV)
    bias[0] += 0.7  # blank frequent
    frames = None
    if ragged:
        frames = torch.tensor([max(0, Lq - 17 * i) for i in range(B)], dtype=torch.int32).to(DEV)
    pred = ops.gemm_argmax(a, w, bias).view(B, Lq)
    want = ops.ctc_collapse(pred, 0, collapse, timestamps, frames=frames)
    got = ops.gemm_ctc_greedy(a, w, bias, B, 0, collapse=collapse, timestamps=timestamps, frames=frames)
    lens = want[1].cpu()
    assert torch.equal(got[1].cpu(), lens)
    for i in range(B):
        n = int(lens[i])
        assert torch.equal(got[0][i, :n].cpu(), want[0][i, :n].cpu())
        if timestamps:
            assert torch.equal(got[2][i, :n].cpu(), want[2][i, :n].cpu())
            assert torch.equal(got[3][i, :n].cpu(), want[3][i, :n].cpu())
    # the per-frame argmax output of the same launch
    keys, slots, M = ops._gemm_argmax_keys(a, w, bias, None, None, "t")
    p2 = torch.empty(M, dtype=torch.int32, device=DEV)
    t2 = torch.empty((B, Lq), dtype=torch.int32, device=DEV)
    l2 = torch.empty(B, dtype=torch.int32, device=DEV)
    L = _lib.lib()
    assert L.vasr_ctc_collapse_keys(keys.data_ptr(), slots, slots, B, Lq, None, 0, 1, p2.data_ptr(), t2.data_ptr(),
                                    l2.data_ptr(), None, None, None) == 0
    torch.cuda.synchronize()
    assert torch.equal(p2.view(B, Lq).cpu(), pred.cpu())


def test_collapse_clamps_frames_to_the_row(va):
    """frames[b] outside [0, L] is clamped: past L both collapse kernels read and
    write only the utterance's own L rows (as frames = L); negative counts give no tokens.
    Canary rows after the batch's outputs must stay untouched."""
    from velocity_asr import _lib, ops
    B, Lq, N, K = 3, 70, 7, 32
    g = torch.Generator().manual_seed(5)
    a = torch.randn(B * Lq, K, generator=g).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.3).to(DEV)
    pred = ops.gemm_argmax(a, w, bias).view(B, Lq)
    full = ops.ctc_collapse(pred, 0, True, True)
    frames = torch.tensor([Lq + 1000, -5, Lq], dtype=torch.int32, device=DEV)
    L = _lib.lib()
    for one_launch in (False, True):
        canary = -7
        toks = torch.full((B + 1, Lq), canary, dtype=torch.int32, device=DEV)
        st = torch.full((B + 1, Lq), canary, dtype=torch.int32, device=DEV)
        en = torch.full((B + 1, Lq), canary, dtype=torch.int32, device=DEV)
        lens = torch.full((B,), canary, dtype=torch.int32, device=DEV)
        if one_launch:
            keys, slots, M = ops._gemm_argmax_keys(a, w, bias, None, None, "t")
            rc = L.vasr_ctc_collapse_keys(keys.data_ptr(), slots, slots, B, Lq, frames.data_ptr(), 0, 1, None,
                                          toks.data_ptr(), lens.data_ptr(), st.data_ptr(), en.data_ptr(), None)
        else:
            rc = L.vasr_ctc_collapse_var(pred.data_ptr(), B, Lq, frames.data_ptr(), 0, 1, toks.data_ptr(),
                                         lens.data_ptr(), st.data_ptr(), en.data_ptr(), None)
        assert rc == 0
        torch.cuda.synchronize()
        assert int(lens[1]) == 0
        for b in (0, 2):  # past L -> the whole row, as frames = L
            n = int(full[1][b])
            assert int(lens[b]) == n
            assert torch.equal(toks[b, :n].cpu(), full[0][b, :n].cpu())
            assert torch.equal(st[b, :n].cpu(), full[2][b, :n].cpu()) and torch.equal(en[b, :n].cpu(), full[3][b, :n].cpu())
        for t in (toks, st, en):
            assert bool((t[B] == canary).all()), "wrote past the batch's rows"


def test_ctc_greedy_one_launch_argument_checks(va):
    from velocity_asr import _lib
    L = _lib.lib()
    x = torch.zeros(16, dtype=torch.int64, device=DEV)
    o = torch.zeros(16, dtype=torch.int32, device=DEV)
    assert L.vasr_ctc_collapse_keys(x.data_ptr(), 1, 1, 1, 9000, None, 0, 1, None, o.data_ptr(), o.data_ptr(), None,
                                    None, None) == -1
    assert b"L <= 8192" in L.vasr_last_error()
    assert L.vasr_ctc_collapse_keys(x.data_ptr(), 1, 2, 1, 4, None, 0, 1, None, o.data_ptr(), o.data_ptr(), None,
                                    None, None) == -1


def test_model_greedy_token_ids_match_reference(va):
    """The pipeline's default decode (greedy_token_ids: head GEMM, then argmax + collapse in one
    launch) gives the reference goldens' collapsed tokens."""
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    from velocity_asr import ops
    for fname, (B, S_, seed) in (("fwd_b2_10s.npz", (2, 160000, 1234)), ("fwd_b2_3s.npz", (2, 48000, 21))):
        mel = va.compute_mel_spectrogram(torch.from_numpy(S.make_audio(B, S_, seed=seed)).to(DEV))
        toks, lens = m.greedy_token_ids(mel)
        t2, l2, _, _ = ops.ctc_collapse(torch.from_numpy(golden(fname)["tokens"].astype(np.int32)).to(DEV))
        assert torch.equal(lens.cpu(), l2.cpu())
        for i in range(B):
            assert torch.equal(toks[i, : int(lens[i])].cpu(), t2[i, : int(l2[i])].cpu())
