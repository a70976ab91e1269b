"""Audio loading and the log-mel front end (drop-in for reference velocity_asr/audio.py).

compute_mel_spectrogram runs on the MI355X: |STFT|^2 (HIP real FFT for the default n_fft 400 /
hop 160 with reflect padding on the fly; otherwise reflect pad + a windowed-DFT GEMM with an
in-register |X|^2 epilogue) -> sparse mel + log + per-bin normalisation (HIP).  Input on the CPU is moved to the current HIP device and the result moved back,
so callers that compute mel on the host (scripts/transcribe.py:73) keep working; there is
no CPU execution path.

Constant tables (Hann window, mel filterbank) are built once per device with the
reference's own float32 formulas (audio.py:97, :146-199), so they are bit-identical to
what the reference uses.
"""

from __future__ import annotations

import math
import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import ops

# Default audio parameters (reference audio.py:15-19)
SAMPLE_RATE = 16000
N_FFT = 400
HOP_LENGTH = 160
N_MELS = 80
WINDOW_FN = torch.hann_window


_WAVE_PCM, _WAVE_FLOAT, _WAVE_EXTENSIBLE = 1, 3, 0xFFFE


def _read_wav(path: str) -> Tuple[torch.Tensor, int]:
    """RIFF/WAVE reader: (channels, samples) float32, like torchaudio.load.

    Integer PCM (8/16/24/32-bit) is scaled to [-1, 1); IEEE float (32/64-bit, format 3, or
    WAVE_FORMAT_EXTENSIBLE with either sub-format) is returned as stored, so float32 clips
    round-trip bit-exactly.
    """
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    fmt = body = None
    pos = 12
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], int.from_bytes(data[pos + 4:pos + 8], "little")
        chunk = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = chunk
        elif cid == b"data":
            body = chunk
        pos += 8 + size + (size & 1)
    if fmt is None or body is None or len(fmt) < 16:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, nch, sr = int.from_bytes(fmt[0:2], "little"), int.from_bytes(fmt[2:4], "little"), int.from_bytes(fmt[4:8], "little")
    bits = int.from_bytes(fmt[14:16], "little")
    if tag == _WAVE_EXTENSIBLE and len(fmt) >= 26:
        tag = int.from_bytes(fmt[24:26], "little")
    width = bits // 8
    if nch < 1 or width < 1:
        raise ValueError(f"{path}: bad format ({nch} channels, {bits} bits)")
    body = body[: len(body) // (width * nch) * width * nch]
    if tag == _WAVE_FLOAT and width in (4, 8):
        x = np.frombuffer(body, "<f4" if width == 4 else "<f8").astype(np.float32)
    elif tag != _WAVE_PCM:
        raise ValueError(f"{path}: unsupported WAV format tag {tag}")
    elif width == 1:
        x = (np.frombuffer(body, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif width == 2:
        x = np.frombuffer(body, "<i2").astype(np.float32) / 32768.0
    elif width == 3:
        b = np.frombuffer(body, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif width == 4:
        x = np.frombuffer(body, "<i4").astype(np.float32) / float(1 << 31)
    else:
        raise ValueError(f"{path}: unsupported PCM sample width {width}")
    return torch.from_numpy(np.ascontiguousarray(x.reshape(-1, nch).T)), sr


def write_wav(path: str, audio, sample_rate: int = SAMPLE_RATE) -> None:
    """Write (samples,) or (channels, samples) audio as 32-bit IEEE-float WAV (lossless for float32)."""
    x = np.asarray(audio.cpu().numpy() if isinstance(audio, torch.Tensor) else audio, dtype="<f4")
    if x.ndim == 1:
        x = x[None]
    nch = x.shape[0]
    body = np.ascontiguousarray(x.T).tobytes()
    fmt = (_WAVE_FLOAT.to_bytes(2, "little") + nch.to_bytes(2, "little") + sample_rate.to_bytes(4, "little")
           + (sample_rate * 4 * nch).to_bytes(4, "little") + (4 * nch).to_bytes(2, "little") + (32).to_bytes(2, "little"))
    riff = b"WAVE" + b"fmt " + len(fmt).to_bytes(4, "little") + fmt + b"data" + len(body).to_bytes(4, "little") + body
    with open(path, "wb") as f:
        f.write(b"RIFF" + len(riff).to_bytes(4, "little") + riff)


def _read_flac(path: str) -> Tuple[torch.Tensor, int]:
    """FLAC file -> ((channels, samples) float32 scaled by 2^(bits-1), sample rate), decoded by
    the library's host decoder (vasr_flac_decode; frame CRCs checked)."""
    import ctypes
    with open(path, "rb") as f:
        data = f.read()
    lib = _lib.lib()
    ch, sr, bits, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    buf = ctypes.create_string_buffer(data, len(data))
    args = (ctypes.byref(ch), ctypes.byref(sr), ctypes.byref(bits), ctypes.byref(ns))
    rc = lib.vasr_flac_decode(ctypes.addressof(buf), len(data), None, 0, *args)
    if rc != 0:
        raise ValueError(f"{path}: {lib.vasr_last_error().decode(errors='replace')}")
    out = np.empty((ch.value, ns.value), np.float32)
    _lib.check(lib.vasr_flac_decode(ctypes.addressof(buf), len(data), out.ctypes.data, out.size, *args),
               "vasr_flac_decode")
    return torch.from_numpy(out), sr.value


def resample(waveform: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.transforms.Resample(orig_freq, new_freq) with its defaults (sinc_interp_hann,
    lowpass_filter_width 6, rolloff 0.99) on a host (..., samples) float32 waveform, by the
    library's host resampler (vasr_resample_f32).  Equality with torchaudio is unpinned
    (torchaudio is not installed here): same kernel formula, float64 accumulation."""
    x = np.ascontiguousarray(waveform.detach().cpu().numpy(), dtype=np.float32)
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    n = x2.shape[1]
    lib = _lib.lib()
    m = int(lib.vasr_resample_length(n, int(orig_freq), int(new_freq)))
    y = np.empty((x2.shape[0], m), np.float32)
    if n and x2.shape[0]:
        _lib.check(lib.vasr_resample_f32(x2.ctypes.data, x2.shape[0], n, n, int(orig_freq), int(new_freq), y.ctypes.data,
                                         m), "vasr_resample_f32")
    return torch.from_numpy(y.reshape(*lead, m))


def load_audio(path: str, sample_rate: int = SAMPLE_RATE, mono: bool = True) -> torch.Tensor:
    """Load audio and resample (reference audio.py:22-62).

    Uses torchaudio when it is installed (same as the reference); otherwise reads WAV with the
    standard library and FLAC (LibriSpeech's format) with the library's host decoder, and
    resamples with the host resampler that follows torchaudio's Resample defaults.  Returns
    (samples,) for mono or (channels, samples), float32 on the host like the reference.
    """
    try:
        import torchaudio
        waveform, sr = torchaudio.load(path)
        resampler = lambda w, a, b: torchaudio.transforms.Resample(a, b)(w)  # noqa: E731
    except ImportError:
        low = path.lower()
        if low.endswith(".wav"):
            waveform, sr = _read_wav(path)
        elif low.endswith(".flac"):
            waveform, sr = _read_flac(path)
        else:
            raise ImportError("torchaudio is required for audio formats other than WAV and FLAC. "
                              "Install with: pip install torchaudio")
        resampler = resample
    if mono and waveform.size(0) > 1:
        waveform = waveform.mean(dim=0, keepdim=True)
    if sr != sample_rate:
        waveform = resampler(waveform, sr, sample_rate)
    if mono:
        waveform = waveform.squeeze(0)
    return waveform


def _create_mel_filterbank(n_fft: int, n_mels: int, sample_rate: int, device: torch.device) -> torch.Tensor:
    """HTK triangular filterbank, float32 torch ops in the reference's order (audio.py:146-199).
    Built once per configuration on the host; it is a constant table of the front end."""
    n_freqs = n_fft // 2 + 1
    freqs = torch.linspace(0, sample_rate / 2, n_freqs)

    def hz_to_mel(hz):
        return 2595 * torch.log10(1 + hz / 700)

    def mel_to_hz(mel):
        return 700 * (10 ** (mel / 2595) - 1)

    mel_min = hz_to_mel(torch.tensor(0.0))
    mel_max = hz_to_mel(torch.tensor(sample_rate / 2.0))
    mel_points = torch.linspace(mel_min, mel_max, n_mels + 2)
    hz_points = mel_to_hz(mel_points)
    fb = torch.zeros(n_mels, n_freqs)
    for i in range(n_mels):
        lower, center, upper = hz_points[i], hz_points[i + 1], hz_points[i + 2]
        lower_slope = (freqs - lower) / (center - lower + 1e-10)
        upper_slope = (upper - freqs) / (upper - center + 1e-10)
        fb[i] = torch.maximum(torch.zeros_like(freqs), torch.minimum(lower_slope, upper_slope))
    return fb.to(device)


class _FrontEndTables:
    """Per (device, n_fft, n_mels, sample_rate) constants: paired DFT matrix and CSR filterbank."""

    def __init__(self, device: torch.device, n_fft: int, n_mels: int, sample_rate: int):
        n_bins = n_fft // 2 + 1
        pairs = (n_bins + 31) // 32
        win = WINDOW_FN(n_fft).double().numpy()          # reference window, float32 values
        n = np.arange(n_fft, dtype=np.float64)
        W = np.zeros((pairs * 64, n_fft), dtype=np.float64)
        for k in range(n_bins):
            p, j = divmod(k, 32)
            ang = 2.0 * math.pi * ((k * n) % n_fft) / n_fft
            W[64 * p + j] = win * np.cos(ang)
            W[64 * p + 32 + j] = -win * np.sin(ang)
        self.n_bins = n_bins
        self.window = WINDOW_FN(n_fft).to(device)
        self.dft = torch.from_numpy(W.astype(np.float32)).to(device)
        fb = _create_mel_filterbank(n_fft, n_mels, sample_rate, torch.device("cpu"))
        nz = fb.nonzero(as_tuple=False)
        rowptr = torch.zeros(n_mels + 1, dtype=torch.int32)
        counts = torch.bincount(nz[:, 0], minlength=n_mels)
        rowptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        self.fb_csr = (rowptr.to(device), nz[:, 1].to(torch.int32).contiguous().to(device),
                       fb[nz[:, 0], nz[:, 1]].contiguous().to(device))


_TABLES: Dict[tuple, _FrontEndTables] = {}


def _tables(device: torch.device, n_fft: int, n_mels: int, sample_rate: int) -> _FrontEndTables:
    key = (str(device), n_fft, n_mels, sample_rate)
    t = _TABLES.get(key)
    if t is None:
        t = _TABLES[key] = _FrontEndTables(device, n_fft, n_mels, sample_rate)
    return t


def _target_device(t: torch.Tensor) -> torch.device:
    if t.device.type == "cuda":
        return t.device
    _lib.require_device()
    return torch.device("cuda", torch.cuda.current_device())


def compute_mel_spectrogram(audio: torch.Tensor, sample_rate: int = SAMPLE_RATE, n_fft: int = N_FFT,
                            hop_length: int = HOP_LENGTH, n_mels: int = N_MELS,
                            normalize: bool = True, lengths=None) -> torch.Tensor:
    """Log-mel spectrogram (reference audio.py:65-143) on the MI355X.

    audio (samples,) or (batch, samples) -> (frames, n_mels) or (batch, frames, n_mels),
    frames = samples // hop_length + 1, on the input's device.  lengths (extension): the
    per-clip sample counts of a batch of clips of different lengths zero-padded to a common
    length (see mel_on_device).
    """
    squeeze = audio.dim() == 1
    if squeeze:
        audio = audio.unsqueeze(0)
    if audio.dim() != 2:
        raise ValueError(f"compute_mel_spectrogram: expected (samples,) or (batch, samples), got {tuple(audio.shape)}")
    dev = _target_device(audio)
    x = audio.to(device=dev, dtype=torch.float32).contiguous()
    mel = mel_on_device(x, sample_rate, n_fft, hop_length, n_mels, normalize, lengths=lengths)
    if audio.device.type != "cuda":
        mel = mel.to(audio.device)
    return mel.squeeze(0) if squeeze else mel


# Default geometry (n_fft 400, hop 160): the real-FFT launch writing |X|^2 rows (6 frames per
# workgroup), then the chunked log-mel passes.  VASR_STFT=gemm or other geometries: reflect pad
# + windowed-DFT GEMM with the |X|^2 epilogue.
_STFT_MODE = os.environ.get("VASR_STFT", "fft")
_STFT_FFT = _STFT_MODE != "gemm"


def ragged_supported(n_mels: int = N_MELS, n_fft: int = N_FFT, hop_length: int = HOP_LENGTH) -> bool:
    """Whether mel_on_device(..., lengths=) can run a zero-padded batch of clips of different
    lengths: the per-length (_var) kernels exist for the FFT front end of the default geometry
    with at most 85 mel bins (VASR_STFT=gemm or other geometries raise NotImplementedError)."""
    return n_fft == 400 and hop_length == 160 and _STFT_FFT and n_mels <= 85


def mel_on_device(x: torch.Tensor, sample_rate: int = SAMPLE_RATE, n_fft: int = N_FFT,
                  hop_length: int = HOP_LENGTH, n_mels: int = N_MELS, normalize: bool = True,
                  lengths=None, frame_pad: int = 0) -> torch.Tensor:
    """(B, S) float32 HIP tensor -> (B, F, n_mels) on the same device.

    lengths (extension): per-utterance sample counts of a batch of clips of different lengths,
    zero-padded to S.  Utterance b's first audio_to_frames(lengths[b]) frames are then those of
    the clip alone (its reflect padding and its normalisation statistics are its own) and its
    later frames are 0; pass the frame counts on as VELOCITYASR(..., frames=).

    frame_pad (extension): write the mel into a buffer with frame_pad zero frames before and
    after each utterance (the normalisation pass writes them) and return the (B, F, n_mels)
    view into it: the temporal conv (padding 1) then reads it in place, with no padding pass."""
    B, S = x.shape
    pad = n_fft // 2
    if S <= pad:
        raise RuntimeError(f"compute_mel_spectrogram: reflect padding of {pad} needs more than {pad} samples, got {S}")
    if n_fft % 4 or hop_length % 4:
        raise NotImplementedError("HIP front end needs n_fft and hop_length to be multiples of 4")
    n_frames = (S + 2 * pad - n_fft) // hop_length + 1
    tb = _tables(x.device, n_fft, n_mels, sample_rate)
    if lengths is not None:
        lengths = [int(v) for v in lengths]
        if len(lengths) != B or not all(pad < v <= S for v in lengths):
            raise RuntimeError(f"compute_mel_spectrogram: lengths must be {B} sample counts in ({pad}, {S}], "
                               f"got {lengths}")
        if not ragged_supported(n_mels, n_fft, hop_length):
            raise NotImplementedError("per-utterance lengths need the FFT front end (n_fft 400, hop 160, n_mels <= 85)")
        samples = torch.tensor(lengths, dtype=torch.int32).to(x.device)
        frames = torch.tensor([(v + 2 * pad - n_fft) // hop_length + 1 for v in lengths], dtype=torch.int32).to(x.device)
        power = ops.stft_power_400(x, tb.window, samples=samples)
        return ops.mel_log_norm(power, tb.n_bins, n_frames * tb.n_bins, tb.fb_csr, B, n_frames, n_mels, normalize,
                                frames=frames, frame_pad=frame_pad)
    if n_fft == 400 and hop_length == 160 and _STFT_FFT:
        power = ops.stft_power_400(x, tb.window)
        return ops.mel_log_norm(power, tb.n_bins, n_frames * tb.n_bins, tb.fb_csr, B, n_frames, n_mels, normalize,
                                frame_pad=frame_pad)
    ld = (S + 2 * pad + 3) // 4 * 4
    xp = ops.reflect_pad(x, pad, ld)
    power = torch.empty((B, n_frames, tb.n_bins), device=x.device, dtype=torch.float32)
    ops.gemm_batched(xp, hop_length, ld, n_frames, B, n_fft, tb.dft, None, power, tb.n_bins, n_frames * tb.n_bins,
                     epilogue=_lib.EPI_PAIR_POWER, n_out=tb.n_bins)
    return ops.mel_log_norm(power, tb.n_bins, n_frames * tb.n_bins, tb.fb_csr, B, n_frames, n_mels, normalize,
                            frame_pad=frame_pad)


class MelSpectrogramTransform(nn.Module):
    """nn.Module wrapper of compute_mel_spectrogram (reference audio.py:202-261); same buffers."""

    def __init__(self, sample_rate: int = SAMPLE_RATE, n_fft: int = N_FFT, hop_length: int = HOP_LENGTH,
                 n_mels: int = N_MELS, normalize: bool = True):
        super().__init__()
        self.sample_rate = sample_rate
        self.n_fft = n_fft
        self.hop_length = hop_length
        self.n_mels = n_mels
        self.normalize = normalize
        self.register_buffer("window", WINDOW_FN(n_fft))
        self.register_buffer("mel_filters", _create_mel_filterbank(n_fft, n_mels, sample_rate, torch.device("cpu")))

    def forward(self, audio: torch.Tensor) -> torch.Tensor:
        return compute_mel_spectrogram(audio, sample_rate=self.sample_rate, n_fft=self.n_fft,
                                       hop_length=self.hop_length, n_mels=self.n_mels, normalize=self.normalize)


def audio_to_frames(audio_length: int, hop_length: int = HOP_LENGTH, n_fft: int = N_FFT) -> int:
    """Same formula as the reference (audio.py:264-280), including its off-by-one:
    compute_mel_spectrogram produces audio_length // hop_length + 1 frames."""
    return (audio_length + n_fft) // hop_length


def frames_to_audio(num_frames: int, hop_length: int = HOP_LENGTH) -> int:
    return num_frames * hop_length


def pad_or_trim(audio: torch.Tensor, target_length: int) -> torch.Tensor:
    """Zero-pad or trim the last dim to target_length (reference audio.py:300-324)."""
    current = audio.shape[-1]
    if current > target_length:
        return audio[..., :target_length]
    if current < target_length:
        return F.pad(audio, (0, target_length - current))
    return audio
