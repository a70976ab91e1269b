"""Chunk-parallel tree scan (vasr_ssm_scan_chunked_f32) for small launches.

The chunked form performs the streaming kernel's float operations in the same order (chunk
composites, the chunk-level stack per state lane, each chunk's tree from its carried prefix),
so with the same lane layout its outputs must be BITWISE equal to the streaming kernel's; and
both within the fp32 tolerance of the oracle's restatement of the reference tree
(ssm.py:216-295).  Reference behaviour pinned: L = 1 gives h = 0 (y = x D gated)."""

import numpy as np
import pytest
import torch

from oracle import velocity_ref as R

DEV = "cuda"


def _inputs(seed, B, L, Di, N):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, L, Di)).astype(np.float32)
    dt = np.log1p(np.exp(rng.standard_normal((B, L, Di)) * 0.7 - 1.0)).astype(np.float32)
    Bm = rng.standard_normal((B, L, N)).astype(np.float32)
    Cm = rng.standard_normal((B, L, N)).astype(np.float32)
    A_log = (np.log(np.arange(1, N + 1)) + 0.01 * rng.standard_normal(N)).astype(np.float32)
    D = (1.0 + 0.1 * rng.standard_normal(Di)).astype(np.float32)
    z = (rng.standard_normal((B, L, Di)) * 2.0).astype(np.float32)
    return x, dt, Bm, Cm, A_log, D, z


def _run(x, dt, Bm, Cm, A_log, D, z, mode):
    from velocity_asr import ops
    B, L, Di = x.shape
    N = Bm.shape[-1]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    xz = np.concatenate([x.reshape(B * L, Di), z.reshape(B * L, Di)], 1)
    bc = np.concatenate([Bm.reshape(B * L, N), Cm.reshape(B * L, N)], 1)
    A2 = ((-np.exp(A_log)).astype(np.float32) * np.float32(1.4426950408889634)).astype(np.float32)
    return ops.ssm_scan(t(xz), t(dt.reshape(B * L, Di)), t(bc), t(A2), t(D), B, L, mode).cpu().numpy().reshape(B, L, Di)


def _silu(z):
    return z / (1.0 + np.exp(-z.astype(np.float64)))


def _form(form, fn, *a):
    from velocity_asr import ops
    prev = ops.scan_form(form)
    try:
        return fn(*a)
    finally:
        ops.scan_form(prev)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("npl", [2, 4])
@pytest.mark.parametrize("tc", [16, 32])
@pytest.mark.parametrize("B,L", [(1, 1), (1, 17), (2, 17), (1, 257), (1, 501), (2, 501), (1, 512), (1, 513), (1, 1501),
                                 (2, 2049), (1, 4100), (1, 8192)])
def test_chunked_bitwise_equals_streaming(mode, npl, tc, B, L):
    """The chunk-parallel form equals the streaming kernel bit for bit, with either streaming
    chunk length (16 / 32 steps: the same float operations) and either lane layout."""
    from velocity_asr import _lib, ops
    args = _inputs(31 * L + B, B, L, 64, 64)
    with ops.option(_lib.OPT_SCAN_LANES, npl), ops.option(_lib.OPT_SCAN_CHUNK, tc):
        stream = _form("streaming", _run, *args, mode)
        chunk = _form("chunked", _run, *args, mode)
    np.testing.assert_array_equal(chunk, stream)
    if L <= 2049:
        x, dt, Bm, Cm, A_log, D, z = args
        ref = R.parallel_scan(x, dt, (-np.exp(A_log)).astype(np.float32), Bm, Cm, D) * _silu(z)
        np.testing.assert_allclose(chunk, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("tc", [16, 32])
@pytest.mark.parametrize("N,Di", [(16, 64), (32, 384), (64, 384)])
def test_chunked_state_dims_and_model_width(tc, N, Di):
    from velocity_asr import _lib, ops
    args = _inputs(7 * N, 1, 300, Di, N)
    with ops.option(_lib.OPT_SCAN_LANES, 4), ops.option(_lib.OPT_SCAN_CHUNK, tc):
        stream = _form("streaming", _run, *args, 2)
        np.testing.assert_array_equal(_form("chunked", _run, *args, 2), stream)


@pytest.mark.gpu
def test_chunked_is_the_default_for_one_utterance():
    """The model shape at B = 1 takes the chunked form; at the bench's 16-clip launches, at
    B = 4 (384 waves) and for the global blocks' short L the streaming kernel (profiles/r03ae)."""
    from velocity_asr import ops
    assert ops._use_chunked(1, 501, 384, 64, 2) and ops._use_chunked(2, 1501, 384, 64, 0)
    assert ops._use_chunked(1, 187, 384, 32, 2)
    assert not ops._use_chunked(16, 501, 384, 64, 2)
    assert not ops._use_chunked(4, 501, 384, 64, 2)
    assert not ops._use_chunked(1, 64, 384, 32, 2)   # the global blocks at 10 s
    assert not ops._use_chunked(1, 501, 384, 64, 1)  # the recurrence keeps its own kernel
    assert not ops._use_chunked(1, 16, 384, 64, 2)   # one chunk: nothing to parallelise


@pytest.mark.gpu
def test_one_utterance_30s_tokens_match_reference():
    """B = 1 x 30 s through the chunked scan: argmax tokens equal the reference golden
    (fwd_b1_30s.npz) and the streaming form's logits bit for bit."""
    import velocity_asr as va
    from conftest import golden
    from velocity_asr import synthetic as S
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    mel = va.compute_mel_spectrogram(torch.from_numpy(S.make_audio(1, 480000, seed=4321)).to(DEV))
    from velocity_asr import _lib, ops
    with ops.option(_lib.OPT_SCAN_LANES, 4):  # the same lane layout for both forms: bitwise comparable
        lc = _form("chunked", m, mel)
        ls = _form("streaming", m, mel)
    assert torch.equal(lc, ls)
    np.testing.assert_array_equal(lc.argmax(-1).cpu().numpy(), golden("fwd_b1_30s.npz")["tokens"])


def test_chunked_workspace_size():
    """Host-only: the workspace is two [B][2 * ceil(L/16)][Di][N] float arrays (chunk and
    block composites)."""
    from velocity_asr import _lib
    lib = _lib.load()
    assert lib.vasr_ssm_scan_workspace_floats(1, 501, 384, 64) == 4 * 32 * 384 * 64
    assert lib.vasr_ssm_scan_workspace_floats(2, 16, 8, 16) == 4 * 2 * 1 * 8 * 16
    assert lib.vasr_ssm_scan_workspace_floats(0, 16, 8, 16) == 0
