"""load_audio without torchaudio (reference audio.py:22-62): the library's host FLAC decoder
and torchaudio-Resample-style resampler (csrc/audio_io.cpp).

Parity is UNPINNED against torchaudio (not installed in this image, no reference fixture
holds decoded FLAC): the decoder is checked by exact round trips through tests/flac_writer.py,
an independent encoder written from the format specification that covers every subframe type,
residual coding, stereo mode and header code the decoder handles; the resampler against a
float64 numpy restatement of torchaudio's kernel formula and by signal properties.  Host-only:
these run on the CPU (no device work)."""

import math
import os

import numpy as np
import pytest
import torch

import flac_writer as FW


def _decode_bytes(tmp_path, data, name="a.flac"):
    from velocity_asr.audio import _read_flac
    p = tmp_path / name
    p.write_bytes(data)
    return _read_flac(str(p))


def _sig(n, bps, seed, chans=1):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    amp = (1 << (bps - 1)) - 1
    out = []
    for c in range(chans):
        x = 0.5 * np.sin(2 * math.pi * (220 + 110 * c) * t / 16000) + 0.05 * rng.standard_normal(n)
        out.append(np.clip(np.round(x * amp * 0.8), -amp - 1, amp).astype(np.int64))
    return out


def _expect(chans, bps):
    return np.stack([c.astype(np.float64) / (1 << (bps - 1)) for c in chans]).astype(np.float32)


@pytest.mark.parametrize("kind,order", [("fixed", 0), ("fixed", 1), ("fixed", 2), ("fixed", 3), ("fixed", 4),
                                        ("lpc", 1), ("lpc", 8), ("lpc", 12), ("lpc", 32), ("verbatim", 0)])
def test_flac_subframe_types_16bit_mono(tmp_path, kind, order):
    x = _sig(5000, 16, order)
    data = FW.encode(x, 16000, 16, block=1152, frame_kw=lambda i, s, n: dict(sub=[dict(kind=kind, order=order)]))
    wav, sr = _decode_bytes(tmp_path, data)
    assert sr == 16000 and wav.shape == (1, 5000)
    np.testing.assert_array_equal(wav.numpy(), _expect(x, 16))


@pytest.mark.parametrize("mode", ["independent", "left_side", "side_right", "mid_side"])
def test_flac_stereo_decorrelation(tmp_path, mode):
    x = _sig(3000, 16, 5, chans=2)
    data = FW.encode(x, 44100, 16, block=1024, frame_kw=lambda i, s, n: dict(mode=mode, sub=[dict(order=2)] * 2))
    wav, sr = _decode_bytes(tmp_path, data)
    assert sr == 44100
    np.testing.assert_array_equal(wav.numpy(), _expect(x, 16))


@pytest.mark.parametrize("bps", [8, 12, 20, 24])
def test_flac_sample_sizes(tmp_path, bps):
    x = _sig(2000, bps, bps)
    data = FW.encode(x, 16000, bps, block=512, frame_kw=lambda i, s, n: dict(sub=[dict(kind="lpc", order=6,
                                                                                  precision=14)]))
    wav, _ = _decode_bytes(tmp_path, data)
    np.testing.assert_array_equal(wav.numpy(), _expect(x, bps))


def test_flac_residual_codings_and_partitions(tmp_path):
    """Rice (4-bit parameters) and Rice2 (5-bit), partition orders 0-4, escape partitions,
    per-partition parameters, a constant frame and wasted bits."""
    x = _sig(4096 * 5, 16, 9)[0]
    x[4096:8192] = 1234                      # frame 1: CONSTANT
    x[8192:12288] &= ~np.int64(7)            # frame 2: 3 wasted bits
    kws = [dict(sub=[dict(order=2, porder=4, k=[3, 4, 5, 6] * 4)]),
           dict(sub=[dict(kind="constant")]),
           dict(sub=[dict(order=1, wasted=3, porder=2)]),
           dict(sub=[dict(kind="lpc", order=4, method=1, porder=3, escape=(0, 5))]),
           dict(sub=[dict(order=3, porder=1, escape=(1,), method=1)])]
    data = FW.encode([x], 16000, 16, block=4096, frame_kw=lambda i, s, n: kws[i])
    wav, _ = _decode_bytes(tmp_path, data)
    np.testing.assert_array_equal(wav.numpy(), _expect([x], 16))


def test_flac_variable_blocking_explicit_codes_id3(tmp_path):
    """Variable block sizes (sample-number headers), 8/16-bit explicit block-size codes,
    explicit sample-rate codes, a ragged last block, an ID3v2 tag and extra metadata."""
    x = _sig(7001, 16, 3, chans=2)
    sizes = [100, 257, 4096, 1000, 1548]

    def kw(i, s, n):
        return dict(block=sizes[i % len(sizes)], variable=True, bs_explicit=True, sr_explicit=(i % 2 == 0),
                    mode="mid_side", sub=[dict(order=2), dict(order=1)])
    data = FW.encode(x, 22050, 16, frame_kw=kw, id3=True)
    wav, sr = _decode_bytes(tmp_path, data)
    assert sr == 22050
    np.testing.assert_array_equal(wav.numpy(), _expect(x, 16))


def test_flac_crc_and_format_errors(tmp_path):
    x = _sig(2000, 16, 4)
    data = bytearray(FW.encode(x, 16000, 16, block=1024))
    bad = bytearray(data)
    bad[-5] ^= 0x10  # inside the last frame: CRC-16 mismatch
    with pytest.raises(ValueError, match="CRC"):
        _decode_bytes(tmp_path, bytes(bad))
    with pytest.raises(ValueError, match="fLaC"):
        _decode_bytes(tmp_path, b"RIFF0000WAVE")
    with pytest.raises(ValueError):
        _decode_bytes(tmp_path, bytes(data[:60]))


def _stream(frames, bps, n, sr=16000):
    """fLaC + a lone STREAMINFO block (bps, n samples) + the given frames."""
    info = FW.streaminfo(sr, 1, bps, n)
    return b"fLaC" + bytes([0x80]) + len(info).to_bytes(3, "big") + info + b"".join(frames)


def test_flac_rejects_corrupt_streams(tmp_path):
    """Frames whose sample size differs from STREAMINFO, and predictors whose decoded samples
    leave the sample size (a corrupt residual), end the decode with an error."""
    x = _sig(1024, 16, 6)[0]
    ok = _stream([FW.frame(0, [x], 16, 16000)], 16, 1024)
    wav, _ = _decode_bytes(tmp_path, ok)
    np.testing.assert_array_equal(wav.numpy()[0], _expect([x], 16)[0])
    with pytest.raises(ValueError, match="sample size differs"):
        _decode_bytes(tmp_path, _stream([FW.frame(0, [x], 24, 16000)], 16, 1024))
    ramp = 30000 + 500 * np.arange(64, dtype=np.int64)  # leaves int16 after 6 samples
    for kind in ("fixed", "lpc"):
        bad = _stream([FW.frame(0, [ramp], 16, 16000, sub=[dict(kind=kind, order=2)])], 16, 64)
        with pytest.raises(ValueError, match="exceeds the sample size"):
            _decode_bytes(tmp_path, bad)


def test_resample_rejects_huge_kernels():
    """Coprime rates (44101 -> 16000 Hz) would need a 16000 x 44135-tap kernel: refused."""
    from velocity_asr.audio import resample
    with pytest.raises(Exception, match="tap kernel"):
        resample(torch.zeros(100), 44101, 16000)


def _resample_ref(x, orig, new):
    """float64 numpy restatement of torchaudio.functional.resample (sinc_interp_hann,
    lowpass_filter_width 6, rolloff 0.99): kernel in float64 rounded to float32, stride-orig
    convolution over the (width, width + orig)-padded signal."""
    g = math.gcd(orig, new)
    o, nw = orig // g, new // g
    base = min(o, nw) * 0.99
    width = math.ceil(6 * o / base)
    idx = np.arange(-width, width + o, dtype=np.float64)[None] / o
    t = (np.arange(0, -nw, -1, dtype=np.float64)[:, None] / nw + idx) * base
    t = np.clip(t, -6, 6)
    win = np.cos(t * math.pi / 6 / 2) ** 2
    t = t * math.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    k = (k * (win * (base / o))).astype(np.float32).astype(np.float64)
    xp = np.pad(x.astype(np.float64), (width, width + o))
    frames = (len(xp) - k.shape[1]) // o + 1
    y = np.stack([xp[f * o:f * o + k.shape[1]] @ k.T for f in range(frames)]).reshape(-1)
    return y[: math.ceil(nw * len(x) / o)].astype(np.float32)


@pytest.mark.parametrize("orig,new", [(48000, 16000), (44100, 16000), (8000, 16000), (22050, 16000), (16000, 16000)])
def test_resample_matches_kernel_restatement(orig, new):
    from velocity_asr.audio import resample
    rng = np.random.default_rng(orig)
    x = (rng.standard_normal(3000) * 0.3).astype(np.float32)
    y = resample(torch.from_numpy(np.stack([x, -x])), orig, new).numpy()
    assert y.shape == (2, math.ceil(new * 3000 / orig) if orig != new else 3000)
    if orig == new:
        np.testing.assert_array_equal(y[0], x)
        return
    ref = _resample_ref(x, orig, new)
    np.testing.assert_allclose(y[0], ref, atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(y[1], -ref, atol=2e-6, rtol=1e-5)


def test_resample_passes_band_and_removes_alias():
    """A 1 kHz tone survives 48 -> 16 kHz at unit gain; a 10 kHz tone (above the new 8 kHz
    Nyquist) is removed."""
    from velocity_asr.audio import resample
    t = np.arange(48000) / 48000.0
    lo = np.sin(2 * math.pi * 1000 * t).astype(np.float32)
    hi = np.sin(2 * math.pi * 10000 * t).astype(np.float32)
    y_lo = resample(torch.from_numpy(lo), 48000, 16000).numpy()
    y_hi = resample(torch.from_numpy(hi), 48000, 16000).numpy()
    t16 = np.arange(len(y_lo)) / 16000.0
    mid = slice(200, -200)
    np.testing.assert_allclose(y_lo[mid], np.sin(2 * math.pi * 1000 * t16)[mid], atol=3e-3)
    assert np.abs(y_hi[mid]).max() < 1e-2


def test_load_audio_flac_end_to_end(tmp_path):
    """load_audio on a 44.1 kHz stereo FLAC: decode, mono mix, resample to 16 kHz, as the
    reference's load_audio does with torchaudio (audio.py:47-60)."""
    import velocity_asr as v
    from velocity_asr.audio import resample
    x = _sig(44100, 16, 12, chans=2)
    p = tmp_path / "clip.FLAC"
    p.write_bytes(FW.encode(x, 44100, 16, block=4096, frame_kw=lambda i, s, n: dict(mode="left_side")))
    got = v.load_audio(str(p))
    stereo = torch.from_numpy(_expect(x, 16))
    want = resample(stereo.mean(dim=0, keepdim=True), 44100, 16000).squeeze(0)
    assert got.shape == (16000,)
    torch.testing.assert_close(got, want, atol=0, rtol=0)
    both = v.load_audio(str(p), sample_rate=44100, mono=False)
    torch.testing.assert_close(both, stereo, atol=0, rtol=0)
