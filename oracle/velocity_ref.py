"""CPU oracle: a numpy restatement of the reference VELOCITY-ASR inference path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (``velocity-asr_amd/``)
imports, links or executes this file; only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg use it, as the checker / CPU baseline.

Parity pin: this restatement is checked against the golden fixtures in
``tests/golden/`` that ``tests/golden/gen_goldens.py`` produced by running the
real reference (``/root/reference``, torch CPU) on the same seeded inputs and
weights (``tests/test_oracle.py``).  Every function cites the reference
``file:line`` it restates (paths relative to the reference root).

Numerics: float32 throughout, elementwise ops in the reference's order, the
selective scan in the reference's exact (non-standard) Blelloch tree order.  Two
forms of that tree scan are provided: the literal materialised sweep
(``associative_scan_tree``, a line-by-line restatement of ``ssm.py:216-295``) and
an O(log L)-state streaming form (``associative_scan_stream``) that performs the
identical float operations in the identical order, so the two are bitwise equal
(``tests/test_oracle.py::test_stream_equals_tree``).  The streaming form is what
the HIP kernel implements.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
from scipy.special import erf as _erf

f32 = np.float32

SAMPLE_RATE = 16000
N_FFT = 400
HOP_LENGTH = 160
N_MELS = 80


# --------------------------------------------------------------------------- audio
def hann_window(n: int = N_FFT) -> np.ndarray:
    """torch.hann_window(n) periodic (audio.py:19, :97)."""
    k = np.arange(n, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2.0 * math.pi * k / n)).astype(f32)


def _torch_linspace_f32(start: float, end: float, steps: int) -> np.ndarray:
    """torch.linspace in float32 (ATen RangeFactories): start + i*step for the first half,
    end - (steps-1-i)*step for the second half, each a fused multiply-add (one rounding);
    this is what audio.py:166 and :176 evaluate."""
    start = f32(start)
    end = f32(end)
    step = f32((end - start) / f32(steps - 1))
    i = np.arange(steps)
    half = steps // 2
    lo = (np.float64(start) + np.float64(step) * i).astype(f32)
    hi = (np.float64(end) - np.float64(step) * (steps - 1 - i)).astype(f32)
    return np.where(i < half, lo, hi).astype(f32)


def mel_filterbank(n_fft: int = N_FFT, n_mels: int = N_MELS, sample_rate: int = SAMPLE_RATE) -> np.ndarray:
    """_create_mel_filterbank (audio.py:146-199): HTK mel, float32 ops."""
    n_freqs = n_fft // 2 + 1
    freqs = _torch_linspace_f32(0.0, sample_rate / 2, n_freqs)

    def hz_to_mel(hz):  # audio.py:169-170
        return f32(2595) * np.log10(f32(1) + hz / f32(700)).astype(f32)

    def mel_to_hz(mel):  # audio.py:172-173
        # torch evaluates the float32 power as a correctly rounded pow
        return f32(700) * (np.power(10.0, (mel / f32(2595)).astype(np.float64)).astype(f32) - f32(1))

    mel_min = hz_to_mel(np.array(0.0, f32))
    mel_max = hz_to_mel(np.array(sample_rate / 2.0, f32))
    mel_points = _torch_linspace_f32(float(mel_min), float(mel_max), n_mels + 2)
    hz_points = mel_to_hz(mel_points).astype(f32)
    fb = np.zeros((n_mels, n_freqs), f32)
    for i in range(n_mels):  # audio.py:184-197
        lower, center, upper = hz_points[i], hz_points[i + 1], hz_points[i + 2]
        lower_slope = (freqs - lower) / (center - lower + f32(1e-10))
        upper_slope = (upper - freqs) / (upper - center + f32(1e-10))
        fb[i] = np.maximum(f32(0), np.minimum(lower_slope, upper_slope))
    return fb


def power_spectrogram(audio: np.ndarray) -> np.ndarray:
    """Reflect pad n_fft//2, framed STFT (center=False), |X|^2 (audio.py:96-115).
    audio (B, S) -> (B, n_fft//2+1, F)."""
    pad = N_FFT // 2
    xp = np.pad(audio, ((0, 0), (pad, pad)), mode="reflect")
    F = (xp.shape[1] - N_FFT) // HOP_LENGTH + 1
    idx = np.arange(F)[:, None] * HOP_LENGTH + np.arange(N_FFT)[None, :]
    frames = xp[:, idx] * hann_window()[None, None, :]
    X = np.fft.rfft(frames.astype(f32), axis=-1)
    mag = np.abs(X).astype(f32)
    return np.transpose(mag * mag, (0, 2, 1)).astype(f32)


def compute_mel_spectrogram(audio: np.ndarray, normalize: bool = True) -> np.ndarray:
    """compute_mel_spectrogram (audio.py:65-143): (S,)|(B,S) -> (F,80)|(B,F,80)."""
    audio = np.asarray(audio, f32)
    squeeze = audio.ndim == 1
    if squeeze:
        audio = audio[None]
    P = power_spectrogram(audio)
    mel = np.matmul(mel_filterbank()[None], P).astype(f32)           # audio.py:126
    mel = np.log(mel + f32(1e-10)).astype(f32)                       # audio.py:129
    if normalize:                                                    # audio.py:132-135
        mean = mel.astype(np.float64).mean(axis=-1, keepdims=True).astype(f32)
        std = mel.astype(np.float64).std(axis=-1, ddof=1, keepdims=True).astype(f32)
        mel = ((mel - mean) / (std + f32(1e-10))).astype(f32)
    mel = np.transpose(mel, (0, 2, 1))
    return np.ascontiguousarray(mel[0] if squeeze else mel)


# --------------------------------------------------------------------------- layers
def layer_norm(x: np.ndarray, w: np.ndarray, b: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    """nn.LayerNorm (biased variance, eps 1e-5)."""
    mean = x.mean(axis=-1, keepdims=True, dtype=np.float64)
    var = ((x.astype(np.float64) - mean) ** 2).mean(axis=-1, keepdims=True)
    y = ((x - mean.astype(f32)) * (1.0 / np.sqrt(var + eps)).astype(f32)).astype(f32)
    return (y * w + b).astype(f32)


def gelu(x: np.ndarray) -> np.ndarray:
    """nn.GELU() exact erf form."""
    x = x.astype(f32)
    return (f32(0.5) * x * (f32(1) + _erf(x / f32(math.sqrt(2.0))).astype(f32))).astype(f32)


def softplus(x: np.ndarray) -> np.ndarray:
    """F.softplus(beta=1, threshold=20) (ssm.py:113)."""
    x = x.astype(f32)
    return np.where(x > 20, x, np.log1p(np.exp(np.minimum(x, 20)))).astype(f32)


def silu(x: np.ndarray) -> np.ndarray:
    x = x.astype(f32)
    return (x / (f32(1) + np.exp(-x))).astype(f32)


def sigmoid(x: np.ndarray) -> np.ndarray:
    x = x.astype(f32)
    return (f32(1) / (f32(1) + np.exp(-x))).astype(f32)


def linear(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray] = None) -> np.ndarray:
    y = np.matmul(x, w.T).astype(f32)
    if b is not None:
        y = (y + b).astype(f32)
    return y


# --------------------------------------------------------------------------- INT8 fake quant (C5)
def fake_quantize(x: np.ndarray, scale, zero_point, qmin: float, qmax: float) -> np.ndarray:
    """FakeQuantize.forward in eval with calibrated buffers (quantize.py:79-97): q =
    clamp(round_half_even(x / scale + zp), qmin, qmax) (:118-124), x_dq = (q - zp) * scale
    (:126-128), returned as x + (x_dq - x) (:97).  scale / zp broadcast (per-tensor or
    per-output-channel)."""
    x = np.asarray(x, f32)
    s = np.asarray(scale, f32)
    zp = np.asarray(zero_point, f32)
    q = np.clip(np.rint((x / s).astype(f32) + zp), f32(qmin), f32(qmax)).astype(f32)
    xdq = ((q - zp).astype(f32) * s).astype(f32)
    return (x + (xdq - x).astype(f32)).astype(f32)


def observe_scale_zp(x: np.ndarray, symmetric: bool, per_channel: bool, qmin: int, qmax: int):
    """FakeQuantize._update_scale_zp (quantize.py:99-116), channel_dim 0."""
    x = np.asarray(x, f32)
    if per_channel:
        axes = tuple(range(1, x.ndim))
        lo, hi = x.min(axis=axes, keepdims=True), x.max(axis=axes, keepdims=True)
    else:
        lo, hi = x.min(), x.max()
    lo, hi = np.asarray(lo, f32), np.asarray(hi, f32)
    if symmetric:
        scale = (np.maximum(np.abs(lo), np.abs(hi)) / f32(qmax)).astype(f32)
        zp = np.zeros_like(scale)
    else:
        scale = ((hi - lo) / f32(qmax - qmin)).astype(f32)
        zp = (f32(qmin) - (lo / scale).astype(f32)).astype(f32)
    return np.maximum(scale, f32(1e-10)).astype(f32), zp


def qat_params(state: Dict[str, np.ndarray], weight_bits: int = 8, activation_bits: int = 8,
               symmetric_activations: bool = False) -> Dict[str, dict]:
    """Quantizer buffers of a prepare_model_for_qat state_dict (quantize.py:269-322) ->
    {module path: {"w": (scale, zp, qmin, qmax) or None, "a": ... or None}}; an
    uncalibrated quantizer passes through in eval (quantize.py:82-84) and maps to None."""
    wq = (-(2 ** (weight_bits - 1)), 2 ** (weight_bits - 1) - 1)
    aq = ((-(2 ** (activation_bits - 1)), 2 ** (activation_bits - 1) - 1) if symmetric_activations
          else (0, 2 ** activation_bits - 1))
    out: Dict[str, dict] = {}
    for k in state:
        if not k.endswith(".weight_quantizer.scale"):
            continue
        path = k[: -len(".weight_quantizer.scale")]
        ent = {}
        for kind, qr, key in (("w", wq, "weight_quantizer"), ("a", aq, "activation_quantizer")):
            pre = f"{path}.{key}."
            cal = bool(np.asarray(state[pre + "calibrated"]))
            ent[kind] = (np.asarray(state[pre + "scale"], f32), np.asarray(state[pre + "zero_point"], f32),
                         qr[0], qr[1]) if cal else None
        out[path] = ent
    return out


def qlinear(W, Q, path: str, x: np.ndarray) -> np.ndarray:
    """nn.Linear, or QuantizedLinear.forward (quantize.py:177-191) when Q has `path`."""
    w, b = W[path + ".weight"], W.get(path + ".bias")
    q = Q.get(path) if Q else None
    if q is None:
        return linear(x, w, b)
    if q["w"] is not None:
        w = fake_quantize(w, *q["w"])
    y = linear(x, w, b)
    return fake_quantize(y, *q["a"]) if q["a"] is not None else y


def conv1d_k3s2(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    """TemporalBindingLayer.conv (model.py:156-162): Conv1d(80->D, k3, s2, p1) on
    (B, F, C) input, returned as (B, L, D)."""
    B, F, C = x.shape
    L = (F + 2 - 3) // 2 + 1
    xp = np.zeros((B, F + 2, C), f32)
    xp[:, 1:F + 1] = x
    cols = np.concatenate([xp[:, k:k + 2 * L:2][:, :L] for k in range(3)], axis=-1)  # (B,L,3C) [k-major]
    wm = np.transpose(w, (0, 2, 1)).reshape(w.shape[0], -1)                           # (D, 3C) [k-major]
    return (np.matmul(cols, wm.T) + b).astype(f32)


def causal_dwconv(x: np.ndarray, w: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Depthwise Conv1d(k, padding=k-1) keeping the first L outputs (ssm.py:377-383,
    :411-414): y[t,c] = b[c] + sum_j w[c,0,j] * x[t-(k-1)+j, c]."""
    B, L, C = x.shape
    k = w.shape[-1]
    xp = np.concatenate([np.zeros((B, k - 1, C), f32), x], axis=1)
    y = np.zeros((B, L, C), f32)
    for j in range(k):
        y = (y + xp[:, j:j + L] * w[:, 0, j]).astype(f32)
    return (y + b).astype(f32)


# --------------------------------------------------------------------------- scans
def sequential_scan(x, dt, A, Bm, Cm, D):
    """_sequential_scan (ssm.py:134-171): true recurrence h_t = dA_t h_{t-1} + x_t dB_t,
    y_t = <h_t, C_t> + x_t D."""
    Bsz, L, Di = x.shape
    N = A.shape[0]
    h = np.zeros((Bsz, Di, N), f32)
    y = np.empty_like(x)
    for t in range(L):
        dA = np.exp(dt[:, t, :, None] * A[None, None, :]).astype(f32)
        dB = (dt[:, t, :, None] * Bm[:, t, None, :]).astype(f32)
        h = (dA * h + x[:, t, :, None] * dB).astype(f32)
        y[:, t] = np.einsum("bdn,bn->bd", h, Cm[:, t]).astype(f32)
    return (y + x * D).astype(f32)


def selective_scan_ref(u, delta, A, Bv, Cv, D=None, z=None, delta_bias=None, delta_softplus=False):
    """Restatement of mamba_ssm's published reference algorithm, ``selective_scan_ref``
    (state-spaces/mamba, ``mamba_ssm/ops/selective_scan_interface.py``; the function its CUDA
    ``selective_scan_fn`` is tested against).  mamba-ssm is absent here and unpinned by the
    reference (not in ``requirements.txt``); the algorithm is the same in every 1.x/2.x release:
    u, delta (B, D, L); A (D, N); variable Bv, Cv (B, G, N, L) with D % G == 0;
    deltaA = exp(delta A), deltaB_u = delta B u, x_t = deltaA_t x_{t-1} + deltaB_u_t,
    y_t = <x_t, C_t>, out = y + u D, then out * silu(z) if z is given."""
    u = u.astype(f32)
    delta = delta.astype(f32)
    if delta_bias is not None:
        delta = (delta + delta_bias[None, :, None]).astype(f32)
    if delta_softplus:
        delta = softplus(delta)
    Bsz, Dd, L = u.shape
    N = A.shape[1]
    G = Bv.shape[1]
    Bx = np.repeat(Bv, Dd // G, axis=1).astype(f32)  # (B, D, N, L), "b g n l -> b (g h) n l"
    Cx = np.repeat(Cv, Dd // G, axis=1).astype(f32)
    deltaA = np.exp(delta[:, :, :, None] * A[None, :, None, :]).astype(f32)           # b d l n
    deltaB_u = (delta[:, :, :, None] * Bx.transpose(0, 1, 3, 2) * u[:, :, :, None]).astype(f32)
    x = np.zeros((Bsz, Dd, N), f32)
    ys = np.empty((Bsz, Dd, L), f32)
    for i in range(L):
        x = (deltaA[:, :, i] * x + deltaB_u[:, :, i]).astype(f32)
        ys[:, :, i] = np.einsum("bdn,bdn->bd", x, Cx[:, :, :, i]).astype(f32)
    out = ys if D is None else (ys + u * D[None, :, None]).astype(f32)
    if z is not None:
        out = (out * silu(z.astype(f32))).astype(f32)
    return out


def mamba_scan(x, dt, A, Bm, Cm, D):
    """_mamba_scan (ssm.py:297-337) in the layout selective_scan_fn documents: u = x^T,
    delta = dt^T (B, D, L), A expanded to (D, N), B and C as (B, 1, N, L) with no delta bias
    or softplus (applied before, ssm.py:113), z = None; the result transposed back to
    (B, L, D).  The reference itself passes B and C as (B, 1, L, N) (ssm.py:318-321), which
    the package's shape check rejects unless L == N: this restates the call as
    the package defines it."""
    Di = x.shape[2]
    u = x.transpose(0, 2, 1)
    delta = dt.transpose(0, 2, 1)
    Ad = np.broadcast_to(A[None, :], (Di, A.shape[0]))
    Bv = Bm.transpose(0, 2, 1)[:, None]
    Cv = Cm.transpose(0, 2, 1)[:, None]
    return selective_scan_ref(u, delta, Ad, Bv, Cv, D).transpose(0, 2, 1)


def discretize(x, dt, A, Bm):
    """_parallel_scan discretisation (ssm.py:196-202): dA = exp(dt*A), x_dB = x*(dt*B)."""
    dA = np.exp(dt[..., None] * A).astype(f32)
    dB = (dt[..., None] * Bm[:, :, None, :]).astype(f32)
    return dA, (x[..., None] * dB).astype(f32)


def associative_scan_tree(dA: np.ndarray, xdB: np.ndarray) -> np.ndarray:
    """Literal restatement of _associative_scan (ssm.py:216-295) over axis 1.

    Up-sweep (a_r, b_r) <- (a_r*a_l, a_r*b_l + b_r); root <- (1, 0); down-sweep
    left <- right, a_r <- a_r*a_l_old, b_r <- a_r(new)*b_l_old + b_r.  Returns b[:, :L]:
    the reference's exclusive, mis-combined prefix."""
    L = dA.shape[1]
    log_len = int(math.ceil(math.log2(max(L, 1))))
    P = 2 ** log_len
    a = np.ones((dA.shape[0], P) + dA.shape[2:], f32)
    b = np.zeros_like(a)
    a[:, :L] = dA
    b[:, :L] = xdB
    stride = 1
    for _ in range(log_len):                       # ssm.py:244-261
        s2 = stride * 2
        r = np.arange(s2 - 1, P, s2)
        l = r - stride
        al, bl, ar, br = a[:, l], b[:, l], a[:, r], b[:, r]
        a[:, r] = ar * al
        b[:, r] = ar * bl + br
        stride = s2
    a[:, -1] = 1.0                                 # ssm.py:264-265
    b[:, -1] = 0.0
    stride = P // 2
    for _ in range(log_len):                       # ssm.py:267-286
        s2 = stride * 2
        r = np.arange(s2 - 1, P, s2)
        l = r - stride
        al_old = a[:, l].copy()
        bl_old = b[:, l].copy()
        a[:, l] = a[:, r]
        b[:, l] = b[:, r]
        a[:, r] = a[:, r] * al_old
        b[:, r] = a[:, r] * bl_old + b[:, r]
        stride //= 2
    return b[:, :L]


def associative_scan_stream(dA: np.ndarray, xdB: np.ndarray) -> np.ndarray:
    """Streaming form of associative_scan_tree with a binary-counter stack of aligned
    blocks (la, lb: up-sweep composite; ca, cb: down-sweep prefix after the block).
    Same float operations in the same order, so bitwise equal to the tree."""
    L = dA.shape[1]
    out = np.empty_like(xdB)
    stack: List[list] = []  # entries [lvl, la, lb, ca, cb]
    zero = np.zeros_like(xdB[:, 0])
    for t in range(L):
        out[:, t] = stack[-1][4] if stack else zero
        la, lb, lvl = dA[:, t], xdB[:, t], 0
        while stack and stack[-1][0] == lvl:          # up-sweep merge with left sibling
            _, pla, plb, _, _ = stack.pop()
            lb = la * plb + lb
            la = la * pla
            lvl += 1
        if stack:                                     # down-sweep prefix through this block
            pa, pb = stack[-1][3], stack[-1][4]
            ca = pa * la
            cb = ca * lb + pb
        else:
            ca = la * np.float32(1.0)
            cb = ca * lb
        stack.append([lvl, la, lb, ca, cb])
    return out


# Form of the tree scan used by forward(): "stream" (O(log L) state, bitwise equal) or "tree"
# (the reference's materialised (B, P, Di, N) up/down-sweep, its CPU cost profile; bench.py's
# cpu_baseline times this form).
SCAN_FORM = "stream"


def parallel_scan(x, dt, A, Bm, Cm, D, stream: Optional[bool] = None):
    """_parallel_scan (ssm.py:173-214): y = einsum(h, C) + x*D with the tree scan."""
    if stream is None:
        stream = SCAN_FORM == "stream"
    dA, xdB = discretize(x, dt, A, Bm)
    h = associative_scan_stream(dA, xdB) if stream else associative_scan_tree(dA, xdB)
    y = np.einsum("bldn,bln->bld", h, Cm).astype(f32)
    return (y + x * D).astype(f32)


# --------------------------------------------------------------------------- blocks
def selective_ssm(W: Dict[str, np.ndarray], p: str, x: np.ndarray, mode: str) -> np.ndarray:
    """SelectiveSSM.forward (ssm.py:92-132)."""
    Di = W[p + "D"].shape[0]
    xz = linear(x, W[p + "in_proj.weight"])
    xp, z = xz[..., :Di], xz[..., Di:]
    xdbl = linear(xp, W[p + "x_proj.weight"])
    N = xdbl.shape[-1] // 2
    Bm, Cm = xdbl[..., :N], xdbl[..., N:]
    dt = softplus(linear(xp, W[p + "dt_proj.weight"], W[p + "dt_proj.bias"]))
    A = (-np.exp(W[p + "A_log"])).astype(f32)
    if mode == "sequential":
        y = sequential_scan(xp, dt, A, Bm, Cm, W[p + "D"])
    elif mode == "parallel":
        y = parallel_scan(xp, dt, A, Bm, Cm, W[p + "D"])
    else:
        raise ValueError(f"Unknown scan_mode: {mode}")
    y = (y * silu(z)).astype(f32)
    return linear(y, W[p + "out_proj.weight"])


def ssm_block(W, p: str, x: np.ndarray, mode: str) -> np.ndarray:
    """SSMBlock._forward_impl (ssm.py:404-427); dropout is identity in eval."""
    r = x
    h = layer_norm(x, W[p + "norm1.weight"], W[p + "norm1.bias"])
    h = causal_dwconv(h, W[p + "conv.weight"], W[p + "conv.bias"])
    x = (selective_ssm(W, p + "ssm.", h, mode) + r).astype(f32)
    r = x
    h = layer_norm(x, W[p + "norm2.weight"], W[p + "norm2.bias"])
    h = gelu(linear(h, W[p + "ffn.0.weight"], W[p + "ffn.0.bias"]))
    h = linear(h, W[p + "ffn.3.weight"], W[p + "ffn.3.bias"])
    return (h + r).astype(f32)


def temporal_binding(W, mel: np.ndarray, Q=None) -> np.ndarray:
    """TemporalBindingLayer.forward (model.py:176-202) + PositionalEncoding2D (:106-127);
    with Q the conv is QuantizedConv1d (quantize.py:252-266)."""
    w = W["temporal_binding.conv.weight"]
    q = Q.get("temporal_binding.conv") if Q else None
    if q is not None and q["w"] is not None:
        w = fake_quantize(w, *q["w"])
    x = conv1d_k3s2(mel, w, W["temporal_binding.conv.bias"])
    if q is not None and q["a"] is not None:
        x = fake_quantize(x, *q["a"])
    x = gelu(x)
    L = x.shape[1]
    pe_t = W["temporal_binding.pos_encoding.pe_time"][:L]
    pe_f = np.broadcast_to(W["temporal_binding.pos_encoding.pe_freq"][0], (L, pe_t.shape[1]))
    x = (x + np.concatenate([pe_t, pe_f], axis=-1)[None]).astype(f32)
    return layer_norm(x, W["temporal_binding.norm.weight"], W["temporal_binding.norm.bias"])


def pool_sizes(L: int) -> Tuple[int, int]:
    """AdaptivePool._compute_pool_size + clamp to seq_len (attention.py:37-44, :67)."""
    k1 = min(max(64, L // 8), L)
    k2 = min(min(64, max(16, k1 // 4)), k1)
    return k1, k2


def adaptive_avg_pool(x: np.ndarray, K: int) -> np.ndarray:
    """F.adaptive_avg_pool1d over time: bin i = [floor(iL/K), ceil((i+1)L/K))."""
    B, L, C = x.shape
    out = np.empty((B, K, C), f32)
    for i in range(K):
        s = (i * L) // K
        e = -((-(i + 1) * L) // K)
        out[:, i] = (x[:, s:e].sum(axis=1, dtype=f32) / f32(e - s)).astype(f32)
    return out


def multi_head_attention(W, p: str, q_in, kv_in, heads: int, Q=None) -> np.ndarray:
    """MultiHeadAttention.forward (attention.py:116-164), mask=None."""
    q = qlinear(W, Q, p + "q_proj", q_in)
    k = qlinear(W, Q, p + "k_proj", kv_in)
    v = qlinear(W, Q, p + "v_proj", kv_in)
    B, Lq, A = q.shape
    hd = A // heads
    qh = q.reshape(B, Lq, heads, hd).transpose(0, 2, 1, 3)
    kh = k.reshape(B, -1, heads, hd).transpose(0, 2, 1, 3)
    vh = v.reshape(B, -1, heads, hd).transpose(0, 2, 1, 3)
    s = (np.matmul(qh, kh.transpose(0, 1, 3, 2)) / f32(math.sqrt(hd))).astype(f32)
    s = s - s.max(axis=-1, keepdims=True)
    e = np.exp(s).astype(f32)
    attn = (e / e.sum(axis=-1, keepdims=True)).astype(f32)
    o = np.matmul(attn, vh).astype(f32).transpose(0, 2, 1, 3).reshape(B, Lq, A)
    return qlinear(W, Q, p + "out_proj", o)


def gated_fusion(W, p: str, local, glob, Q=None) -> np.ndarray:
    """GatedFusion.forward (attention.py:191-220)."""
    g = sigmoid(qlinear(W, Q, p + "gate_proj.0", np.concatenate([local, glob], axis=-1)))
    lt = qlinear(W, Q, p + "local_proj", local)
    gt = qlinear(W, Q, p + "global_proj", glob)
    fused = (g * lt + (f32(1) - g) * gt).astype(f32)
    return qlinear(W, Q, p + "out_proj", fused)


def global_context(W, local: np.ndarray, cfg: dict, Q=None) -> np.ndarray:
    """HierarchicalGlobalContext.forward (attention.py:283-319)."""
    g = "global_context."
    L = local.shape[1]
    k1, _ = pool_sizes(L)
    x = qlinear(W, Q, g + "pool1.pool_proj", adaptive_avg_pool(local, k1))
    for i in range(cfg["global_ssm_layers"]):
        x = ssm_block(W, f"{g}global_ssm.layers.{i}.", x, "parallel")   # GlobalSSM: always parallel
    x = layer_norm(x, W[g + "global_ssm.norm.weight"], W[g + "global_ssm.norm.bias"])
    k2 = min(min(64, max(16, k1 // 4)), x.shape[1])
    x2 = qlinear(W, Q, g + "pool2.pool_proj", adaptive_avg_pool(x, k2))
    x2 = layer_norm(x2, W[g + "norm1.weight"], W[g + "norm1.bias"])
    q = layer_norm(local, W[g + "norm2.weight"], W[g + "norm2.bias"])
    ctx = multi_head_attention(W, g + "cross_attention.", q, x2, cfg["attention_heads"], Q)
    return gated_fusion(W, g + "fusion.", local, ctx, Q)


def forward(W: Dict[str, np.ndarray], mel: np.ndarray, cfg: dict, return_features: bool = False, Q=None):
    """VELOCITYASR.forward (model.py:333-368): (B, F, mel_bins) -> (B, L, V).  Q (from
    qat_params) runs the prepare_model_for_qat form of the model (C5)."""
    x = temporal_binding(W, np.asarray(mel, f32), Q)
    tb = x
    for i in range(cfg["ssm_layers"]):
        x = ssm_block(W, f"local_ssm.layers.{i}.", x, cfg["scan_mode"])
    local = layer_norm(x, W["local_ssm.norm.weight"], W["local_ssm.norm.bias"])
    fused = global_context(W, local, cfg, Q)
    h = layer_norm(fused, W["ctc_head.proj.0.weight"], W["ctc_head.proj.0.bias"])
    logits = qlinear(W, Q, "ctc_head.proj.2", h)
    if return_features:
        return logits, dict(temporal_binding=tb, local_features=local, fused_features=fused)
    return logits


# --------------------------------------------------------------------------- decode
def ctc_greedy_decode(logits: np.ndarray, blank: int = 0, collapse_repeated: bool = True) -> List[List[int]]:
    """ctc_greedy_decode (decode.py:27-71); argmax ties resolve to the first index."""
    pred = np.argmax(logits, axis=-1)
    out = []
    for row in pred.tolist():
        toks, prev = [], None
        for tok in row:
            if tok == blank:
                prev = None
                continue
            if collapse_repeated and tok == prev:
                continue
            toks.append(tok)
            prev = tok
        out.append(toks)
    return out


def ctc_greedy_decode_with_timestamps(logits: np.ndarray, blank: int = 0):
    """ctc_greedy_decode_with_timestamps (decode.py:74-125)."""
    pred = np.argmax(logits, axis=-1)
    results = []
    for row in pred.tolist():
        toks, ts, prev, start = [], [], None, 0
        for i, tok in enumerate(row):
            if tok == blank:
                if prev is not None and prev != blank:
                    ts.append((start, i))
                prev = tok
                continue
            if tok != prev:
                if prev is not None and prev != blank:
                    ts.append((start, i))
                toks.append(tok)
                start = i
            prev = tok
        if prev is not None and prev != blank:
            ts.append((start, len(row)))
        results.append((toks, ts))
    return results


def log_softmax(x: np.ndarray) -> np.ndarray:
    """F.log_softmax over the last dim in float32: (x - max) - log(sum(exp(x - max)))."""
    x = np.asarray(x, f32)
    m = x.max(axis=-1, keepdims=True)
    d = (x - m).astype(f32)
    return (d - np.log(np.exp(d).sum(axis=-1, keepdims=True, dtype=f32))).astype(f32)


def ctc_beam_search(logits: np.ndarray, beam_width: int = 10, blank: int = 0):
    """ctc_beam_search (decode.py:128-217), lm_scorer None: prefix beams keyed by the collapsed
    prefix, strict-greater updates in insertion order, stable sort by score, float64 scores.
    Returns per utterance a list of (tokens, score)."""
    lp_all = log_softmax(logits)
    out = []
    for b in range(lp_all.shape[0]):
        beams = {(): (0.0, None)}
        for t in range(lp_all.shape[1]):
            lp = lp_all[b, t]
            new = {}
            for prefix, (score, last) in beams.items():
                s = score + float(lp[blank])
                if prefix not in new or new[prefix][0] < s:
                    new[prefix] = (s, blank)
                for tok in range(lp.shape[0]):
                    if tok == blank:
                        continue
                    s = score + float(lp[tok])
                    key = prefix if last == tok else prefix + (tok,)
                    if key not in new or new[key][0] < s:
                        new[key] = (s, tok)
            beams = dict(sorted(new.items(), key=lambda kv: kv[1][0], reverse=True)[:beam_width])
        out.append([(list(p), sc) for p, (sc, _) in sorted(beams.items(), key=lambda kv: kv[1][0], reverse=True)])
    return out
