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
    """The model shape at B = 1 takes the chunked form, and so do the global blocks' short L
    at B = 1 (one launch: the time-split form, profiles/r05aq); at the bench's 16-clip launches
    and at B = 4 (384 waves) the streaming kernel (profiles/r03ae)."""
    from velocity_asr import _lib, ops
    assert ops._use_chunked(1, 501, 384, 64, 2) and ops._use_chunked(2, 1501, 384, 64, 0)
    assert ops._use_chunked(1, 187, 384, 32, 2)
    assert not ops._use_chunked(16, 501, 384, 64, 2)
    assert not ops._use_chunked(4, 501, 384, 64, 2)
    assert ops._use_chunked(1, 64, 384, 32, 2)   # the global blocks at 10 s: one launch
    with ops.option(_lib.OPT_SCAN_SPLIT, 1):
        assert not ops._use_chunked(1, 64, 384, 32, 2)   # three launches: streaming wins at L = 64
    assert not ops._use_chunked(32, 64, 384, 32, 2)
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


def _run_split(x, dt, Bm, Cm, A_log, D, z, mode, split):
    """vasr_ssm_scan_chunked_f32 through the C ABI with VASR_OPT_SCAN_SPLIT = split (1: three
    launches, 2: one launch) at 2 state indices per lane (any L, also L <= 16)."""
    from velocity_asr import _lib, ops
    B, L, Di = x.shape
    N = Bm.shape[-1]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    xz = t(np.concatenate([x.reshape(B * L, Di), z.reshape(B * L, Di)], 1))
    bc = t(np.concatenate([Bm.reshape(B * L, N), Cm.reshape(B * L, N)], 1))
    dtt = t(dt.reshape(B * L, Di))
    A2 = t(((-np.exp(A_log)).astype(np.float32) * np.float32(1.4426950408889634)).astype(np.float32))
    Dt = t(D)
    out = torch.full((B * L, Di), float("nan"), device=DEV)
    lib = _lib.load()
    ws = torch.empty(max(1, int(lib.vasr_ssm_scan_workspace_floats(B, L, Di, N))), device=DEV)
    with ops.option(_lib.OPT_SCAN_LANES, 2), ops.option(_lib.OPT_SCAN_SPLIT, split):
        rc = lib.vasr_ssm_scan_chunked_f32(xz.data_ptr(), 2 * Di, dtt.data_ptr(), Di, bc.data_ptr(), 2 * N,
                                           A2.data_ptr(), Dt.data_ptr(), out.data_ptr(), Di, B, L, Di, N, mode,
                                           ws.data_ptr(), ws.numel(), None)
        assert rc == 0, lib.vasr_last_error()
        torch.cuda.synchronize()
    return out.cpu().numpy().reshape(B, L, Di)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("B,L", [(1, 1), (1, 7), (1, 8), (1, 9), (1, 16), (1, 17), (3, 100), (1, 128), (1, 129),
                                 (1, 257), (1, 501), (2, 501), (1, 1024), (1, 1025), (1, 1501), (1, 4100), (1, 8192)])
def test_split_bitwise_equals_streaming(mode, B, L):
    """The one-launch time-split form (phase-1 range composites, the segment tree over the
    waves, each range's streaming tree from its folded prefix) equals the streaming kernel of
    the same lane layout and the three-launch form bit for bit: ranges of 1 .. 64 chunks of 8
    steps (L up to 8192), a ragged last chunk, one-chunk launches, several utterances."""
    from velocity_asr import _lib, ops
    args = _inputs(17 * L + B, B, L, 64, 64)
    with ops.option(_lib.OPT_SCAN_LANES, 2):
        stream = _form("streaming", _run, *args, mode)
    one = _run_split(*args, mode, 2)
    np.testing.assert_array_equal(one, stream)
    if L > 16:
        np.testing.assert_array_equal(_run_split(*args, mode, 1), stream)


@pytest.mark.gpu
@pytest.mark.parametrize("N,Di,L", [(16, 64, 300), (32, 384, 187), (32, 384, 501), (64, 384, 501), (64, 384, 1501)])
def test_split_state_dims_and_model_width(N, Di, L):
    """The model's shapes (local blocks N = 64, Di = 384; global blocks N = 32) and N = 16."""
    from velocity_asr import _lib, ops
    args = _inputs(5 * N + L, 1, L, Di, N)
    with ops.option(_lib.OPT_SCAN_LANES, 2):
        stream = _form("streaming", _run, *args, 2)
    np.testing.assert_array_equal(_run_split(*args, 2, 2), stream)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["b1_30s", "b2_10s_first"])
def test_one_utterance_split_form_tokens_match_reference(case):
    """One utterance through the one-launch scan (the default at B = 1): argmax tokens equal the
    reference goldens (30 s; the first 10-s clip of fwd_b2_10s on its own) and the logits equal
    the streaming form's (2 states per lane) bit for bit."""
    import velocity_asr as va
    from conftest import golden
    from velocity_asr import synthetic as S
    from velocity_asr import _lib, ops
    W = S.make_weights(None, seed=0)
    m = va.VELOCITYASR()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in W.items()}, strict=True)
    m = m.to(DEV).eval()
    if case == "b1_30s":
        audio, tokens = S.make_audio(1, 480000, seed=4321), golden("fwd_b1_30s.npz")["tokens"]
    else:
        audio, tokens = S.make_audio(2, 160000, seed=1234)[:1], golden("fwd_b2_10s.npz")["tokens"][:1]
    mel = va.compute_mel_spectrogram(torch.from_numpy(np.ascontiguousarray(audio)).to(DEV))
    with ops.option(_lib.OPT_SCAN_LANES, 2):
        lc = _form("chunked", m, mel)
        ls = _form("streaming", m, mel)
    assert torch.equal(lc, ls)
    np.testing.assert_array_equal(lc.argmax(-1).cpu().numpy(), tokens)


def test_chunked_workspace_size():
    """Host-only: the workspace is two [B][2 * ceil(L/16)][Di][N] float arrays (chunk and
    block composites)."""
    from velocity_asr import _lib
    lib = _lib.load()
    assert lib.vasr_ssm_scan_workspace_floats(1, 501, 384, 64) == 4 * 32 * 384 * 64
    assert lib.vasr_ssm_scan_workspace_floats(2, 16, 8, 16) == 4 * 2 * 1 * 8 * 16
    assert lib.vasr_ssm_scan_workspace_floats(0, 16, 8, 16) == 0


# ----------------------------------------------------------------------------- ungated form (round 6)
@pytest.mark.gpu
@pytest.mark.parametrize("N,Di", [(16, 64), (32, 384), (64, 384), (128, 256)])
@pytest.mark.parametrize("B,L", [(1, 17), (3, 501), (16, 501), (2, 1501), (1, 4100)])
@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("npl,tc", [(4, 16), (2, 16), (4, 32)])
def test_ungated_scan_is_the_gated_scan_at_unit_gate(N, Di, B, L, mode, npl, tc):
    """vasr_ssm_scan_ungated_f32 (the z-in-tail block's scan: no z staged, out = y + x D) against the
    gated streaming kernel with z = 256, where silu(z) is exactly 256 (exp2 underflows to 0, so the
    reciprocal is of 1): gated = 256 y, a power-of-two scaling, so the two must agree bit for bit --
    every lane layout, chunk length and upper-stack depth (L up to 4100: levels in LDS)."""
    import torch
    from velocity_asr import _lib, ops
    if N == 128 and npl == 2:
        pytest.skip("N = 128 runs 4 states per lane only")
    g = torch.Generator(device="cuda").manual_seed(N * 7 + B * L + mode)
    M = B * L
    xz = torch.randn(M, 2 * Di, device="cuda", generator=g)
    xz[:, Di:] = 256.0
    dt = torch.nn.functional.softplus(torch.randn(M, Di, device="cuda", generator=g) - 1)
    bc = torch.randn(M, 2 * N, device="cuda", generator=g)
    A2 = -(torch.arange(1, N + 1, device="cuda", dtype=torch.float32)
           + 0.1 * torch.rand(N, device="cuda", generator=g)) * 1.4426950408889634
    D = 1 + 0.1 * torch.randn(Di, device="cuda", generator=g)
    prev = ops.scan_form("streaming")
    try:
        with ops.option(_lib.OPT_SCAN_LANES, npl), ops.option(_lib.OPT_SCAN_CHUNK, tc):
            gated = ops.ssm_scan(xz, dt, bc, A2, D, B, L, mode)
            ungated = ops.ssm_scan_ungated(xz[:, :Di], dt, bc, A2, D, B, L, mode)
    finally:
        ops.scan_form(prev)
    torch.cuda.synchronize()
    assert torch.equal(gated, ungated * 256.0), (gated - ungated * 256.0).abs().max().item()
