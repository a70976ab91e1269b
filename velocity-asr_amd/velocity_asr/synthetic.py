"""Portable, seeded synthetic weights and audio for VELOCITY-ASR.

There are no trained checkpoints and no speech data available offline, so every
test, golden fixture and benchmark in this repository runs on weights drawn from
this recipe.  It depends on numpy only (PCG64 streams are bit-identical across
machines), so the GPU box regenerates exactly the weights the golden fixtures
were produced with, without shipping a 26.7 MB checkpoint.

The key set and shapes follow the reference ``VELOCITYASR().state_dict()``
(reference ``velocity_asr/model.py:242-303``, ``ssm.py:32-90``, ``ssm.py:340-400``,
``attention.py:17-319``).  The draw statistics follow the reference initialiser
``VELOCITYASR._init_weights`` (``model.py:305-318``: xavier-uniform Linear,
kaiming-normal fan_out Conv1d, LayerNorm 1/0) plus small noise on biases,
LayerNorm affine parameters, ``A_log`` and ``D`` so that every term of every
kernel is exercised by the parity tests (the reference initialiser leaves them
at exact constants, which would hide a dropped bias or a mis-indexed D).

This module must stay importable on its own (``tests/golden/gen_goldens.py``
loads it by file path next to the reference package of the same name).
"""

from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np

# Defaults mirror reference VelocityASRConfig (model.py:23-68).
DEFAULT_CONFIG = dict(
    mel_bins=80,
    d_model=192,
    ssm_layers=8,
    ssm_state_dim=64,
    ssm_expand_ratio=2,
    ssm_kernel_size=4,
    global_ssm_layers=2,
    global_ssm_state_dim=32,
    attention_heads=4,
    attention_dim=48,
    vocab_size=1000,
    dropout=0.1,
    gradient_checkpointing=False,
    scan_mode="parallel",
    use_compile=False,
)

PE_MAX_LEN = 5000  # PositionalEncoding2D max_len (model.py:87)


def _cfg(config) -> dict:
    if config is None:
        return dict(DEFAULT_CONFIG)
    if isinstance(config, dict):
        out = dict(DEFAULT_CONFIG)
        out.update({k: v for k, v in config.items() if k in DEFAULT_CONFIG})
        return out
    return {k: getattr(config, k) for k in DEFAULT_CONFIG}


def state_dict_spec(config=None) -> List[Tuple[str, Tuple[int, ...], str]]:
    """Ordered (key, shape, kind) triples of the reference state_dict."""
    c = _cfg(config)
    D = c["d_model"]
    E = c["ssm_expand_ratio"]
    Di = D * E
    spec: List[Tuple[str, Tuple[int, ...], str]] = []

    def lin(prefix, out_f, in_f, bias=True):
        spec.append((prefix + ".weight", (out_f, in_f), "linear_w"))
        if bias:
            spec.append((prefix + ".bias", (out_f,), "bias"))

    def ln(prefix):
        spec.append((prefix + ".weight", (D,), "ln_w"))
        spec.append((prefix + ".bias", (D,), "ln_b"))

    def block(prefix, n_state, ksize):
        ln(prefix + ".norm1")
        ln(prefix + ".norm2")
        spec.append((prefix + ".conv.weight", (D, 1, ksize), "conv_w"))
        spec.append((prefix + ".conv.bias", (D,), "bias"))
        spec.append((prefix + ".ssm.A_log", (n_state,), "A_log"))
        spec.append((prefix + ".ssm.D", (Di,), "D"))
        lin(prefix + ".ssm.in_proj", 2 * Di, D, bias=False)
        lin(prefix + ".ssm.x_proj", 2 * n_state, Di, bias=False)
        lin(prefix + ".ssm.dt_proj", Di, Di)
        lin(prefix + ".ssm.out_proj", D, Di, bias=False)
        lin(prefix + ".ffn.0", D * E, D)
        lin(prefix + ".ffn.3", D, D * E)

    # TemporalBindingLayer (model.py:150-174)
    spec.append(("temporal_binding.conv.weight", (D, c["mel_bins"], 3), "conv_w"))
    spec.append(("temporal_binding.conv.bias", (D,), "bias"))
    spec.append(("temporal_binding.pos_encoding.pe_freq", (1, 1, D // 2), "pe_freq"))
    spec.append(("temporal_binding.pos_encoding.pe_time", (PE_MAX_LEN, D // 2), "pe_time"))
    ln("temporal_binding.norm")
    # LocalSSMProcessor (ssm.py:444-489)
    for i in range(c["ssm_layers"]):
        block(f"local_ssm.layers.{i}", c["ssm_state_dim"], c["ssm_kernel_size"])
    ln("local_ssm.norm")
    # HierarchicalGlobalContext (attention.py:246-281)
    g = "global_context"
    lin(g + ".pool1.pool_proj", D, D)
    for i in range(c["global_ssm_layers"]):
        # GlobalSSM hard-codes expand 2, kernel 4 (ssm.py:530-537)
        block(f"{g}.global_ssm.layers.{i}", c["global_ssm_state_dim"], 4)
    ln(g + ".global_ssm.norm")
    lin(g + ".pool2.pool_proj", D, D)
    A = c["attention_dim"]
    lin(g + ".cross_attention.q_proj", A, D)
    lin(g + ".cross_attention.k_proj", A, D)
    lin(g + ".cross_attention.v_proj", A, D)
    lin(g + ".cross_attention.out_proj", D, A)
    ln(g + ".norm1")
    ln(g + ".norm2")
    lin(g + ".fusion.gate_proj.0", D, 2 * D)
    lin(g + ".fusion.local_proj", D, D)
    lin(g + ".fusion.global_proj", D, D)
    lin(g + ".fusion.out_proj", D, D)
    # CTCOutputHead (model.py:218-222)
    ln("ctc_head.proj.0")
    lin("ctc_head.proj.2", c["vocab_size"], D)
    if E != 2:
        # GlobalSSM blocks always use expand 2; fix up their shapes.
        fixed = []
        for k, s, kind in spec:
            if ".global_ssm.layers." in k:
                gi = 2 * D
                if k.endswith(".ssm.D"):
                    s = (gi,)
                elif k.endswith(".ssm.in_proj.weight"):
                    s = (2 * gi, D)
                elif k.endswith(".ssm.x_proj.weight"):
                    s = (s[0], gi)
                elif k.endswith(".ssm.dt_proj.weight"):
                    s = (gi, gi)
                elif k.endswith(".ssm.dt_proj.bias"):
                    s = (gi,)
                elif k.endswith(".ssm.out_proj.weight"):
                    s = (D, gi)
                elif k.endswith(".ffn.0.weight"):
                    s = (gi, D)
                elif k.endswith(".ffn.0.bias"):
                    s = (gi,)
                elif k.endswith(".ffn.3.weight"):
                    s = (D, gi)
            fixed.append((k, s, kind))
        spec = fixed
    return spec


def pe_time_table(d_model: int, max_len: int = PE_MAX_LEN) -> np.ndarray:
    """Sinusoidal temporal encoding (model.py:90-98), computed in float64 then
    rounded once to float32 so it is identical on every host."""
    half = d_model // 2
    pos = np.arange(max_len, dtype=np.float64)[:, None]
    div = np.exp(np.arange(0, half, 2, dtype=np.float64) * (-math.log(10000.0) / half))
    pe = np.zeros((max_len, half), dtype=np.float64)
    pe[:, 0::2] = np.sin(pos * div)
    pe[:, 1::2] = np.cos(pos * div)[:, : pe[:, 1::2].shape[1]]
    return pe.astype(np.float32)


def make_weights(config=None, seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """Draw every state_dict entry in key order from one PCG64 stream."""
    c = _cfg(config)
    rng = np.random.default_rng(seed)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, shape, kind in state_dict_spec(c):
        if kind == "linear_w":
            fan_out, fan_in = shape
            bound = math.sqrt(6.0 / (fan_in + fan_out))
            w = rng.uniform(-bound, bound, size=shape)
        elif kind == "conv_w":
            fan_out = shape[0] * shape[2]
            w = rng.standard_normal(shape) * math.sqrt(2.0 / fan_out)
        elif kind == "bias":
            w = rng.uniform(-0.05, 0.05, size=shape)
        elif kind == "ln_w":
            w = 1.0 + 0.05 * rng.standard_normal(shape)
        elif kind == "ln_b":
            w = 0.05 * rng.standard_normal(shape)
        elif kind == "A_log":
            n = shape[0]
            w = np.log(np.arange(1, n + 1, dtype=np.float64)) + 0.01 * rng.standard_normal(shape)
        elif kind == "D":
            w = 1.0 + 0.1 * rng.standard_normal(shape)
        elif kind == "pe_freq":
            w = 0.02 * rng.standard_normal(shape)
        elif kind == "pe_time":
            w = pe_time_table(2 * shape[1], shape[0])
        else:  # pragma: no cover
            raise ValueError(kind)
        out[key] = np.ascontiguousarray(w, dtype=np.float32)
    return out


def make_audio(batch: int, samples: int, seed: int = 1234) -> np.ndarray:
    """Synthetic 16 kHz clips: rng.standard_normal((B, S)) * 0.1 (SURVEY §8 d)."""
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((batch, samples), dtype=np.float32) * np.float32(0.1)).astype(np.float32)


def make_chirp(samples: int, seed: int = 7, sample_rate: int = 16000) -> np.ndarray:
    """A speech-like clip: a rising chirp with a 4 Hz envelope plus noise."""
    t = np.arange(samples, dtype=np.float64) / sample_rate
    f0, f1 = 120.0, 3000.0
    dur = max(t[-1], 1e-3)
    phase = 2 * math.pi * (f0 * t + (f1 - f0) * t * t / (2 * dur))
    env = 0.5 + 0.5 * np.sin(2 * math.pi * 4.0 * t)
    rng = np.random.default_rng(seed)
    x = 0.3 * env * np.sin(phase) + 0.01 * rng.standard_normal(samples)
    return x.astype(np.float32)


def frames_for(samples: int, hop: int = 160) -> int:
    """Mel frames produced by compute_mel_spectrogram: S // hop + 1."""
    return samples // hop + 1


def tokens_for(frames: int) -> int:
    """Sequence length after the stride-2 temporal conv: (F - 1) // 2 + 1."""
    return (frames - 1) // 2 + 1
