"""VELOCITY-ASR model (drop-in for reference velocity_asr/model.py) on MI355X kernels.

Module tree, parameter/buffer names, config dataclass and checkpoint format are the
reference's (model.py:23-467), so reference checkpoints load with strict=True and
scripts/transcribe.py / scripts/evaluate.py work unchanged.  The forward pass runs
entirely in libvasr_hip.so; CPU tensors are rejected with a clear error.
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Any, Dict, Optional

import torch
import torch.nn as nn

from . import _lib, ops
from . import quantize as Q
from ._prep import cached
from .attention import HierarchicalGlobalContext
from .ssm import LocalSSMProcessor, ScanMode


@dataclass
class VelocityASRConfig:
    """Configuration for VELOCITY-ASR (reference model.py:23-68)."""

    mel_bins: int = 80
    d_model: int = 192
    ssm_layers: int = 8
    ssm_state_dim: int = 64
    ssm_expand_ratio: int = 2
    ssm_kernel_size: int = 4
    global_ssm_layers: int = 2
    global_ssm_state_dim: int = 32
    attention_heads: int = 4
    attention_dim: int = 48
    vocab_size: int = 1000
    dropout: float = 0.1
    gradient_checkpointing: bool = False
    scan_mode: ScanMode = "parallel"
    use_compile: bool = False

    @classmethod
    def from_dict(cls, config_dict: Dict[str, Any]) -> "VelocityASRConfig":
        return cls(**{k: v for k, v in config_dict.items() if k in cls.__dataclass_fields__})


class PositionalEncoding2D(nn.Module):
    """[sinusoidal time (D/2) | learned frequency (D/2)] encoding (reference model.py:71-127)."""

    def __init__(self, d_model: int = 192, max_len: int = 5000, mel_bins: int = 80):
        super().__init__()
        self.d_model = d_model
        pe_time = torch.zeros(max_len, d_model // 2)
        position = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
        div_term = torch.exp(torch.arange(0, d_model // 2, 2).float() * (-math.log(10000.0) / (d_model // 2)))
        pe_time[:, 0::2] = torch.sin(position * div_term)
        pe_time[:, 1::2] = torch.cos(position * div_term)
        self.register_buffer("pe_time", pe_time)
        self.pe_freq = nn.Parameter(torch.randn(1, 1, d_model // 2) * 0.02)

    def table(self, seq_len: int) -> torch.Tensor:
        """(seq_len, d_model) rows [pe_time[t] | pe_freq] on the parameters' device."""
        if seq_len > self.pe_time.shape[0]:
            raise RuntimeError(f"sequence of {seq_len} tokens exceeds the positional table ({self.pe_time.shape[0]}); "
                               "the reference fails the same way (model.py:125)")

        def build():
            half = self.pe_time.shape[1]
            return torch.cat([self.pe_time[:seq_len], self.pe_freq.reshape(1, half).expand(seq_len, half)],
                             -1).float().contiguous()
        return cached(self, f"pe{seq_len}", (self.pe_time, self.pe_freq), build)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, L, D = x.shape
        return ops.add_table(x, self.table(L))


class TemporalBindingLayer(nn.Module):
    """Conv1d(k3, s2) -> GELU -> +2-D PE -> LayerNorm (reference model.py:130-202).

    One batched fp32-MFMA GEMM: the mel frames are zero-padded once so every conv output
    row is a plain strided row (stride 2 frames, K = 3 frames) of the padded buffer; bias,
    exact GELU and the positional table are fused in the epilogue.
    """

    def __init__(self, mel_bins: int = 80, d_model: int = 192, kernel_size: int = 3, stride: int = 2):
        super().__init__()
        self.conv = nn.Conv1d(in_channels=mel_bins, out_channels=d_model, kernel_size=kernel_size, stride=stride,
                              padding=kernel_size // 2)
        self.pos_encoding = PositionalEncoding2D(d_model=d_model, mel_bins=mel_bins)
        self.norm = nn.LayerNorm(d_model)
        self.activation = nn.GELU()

    def conv_padding(self) -> int:
        return Q.inner(self.conv).padding[0]

    def output_length(self, frames: int) -> int:
        c = Q.inner(self.conv)
        k, s, p = c.kernel_size[0], c.stride[0], c.padding[0]
        return (frames + 2 * p - k) // s + 1

    def forward(self, mel_spectrogram: torch.Tensor, raw: bool = False) -> torch.Tensor:
        """raw (extension): the rows before the final LayerNorm (the first SSM block applies it
        inside its own first launch, VELOCITYASR._local_global)."""
        D = Q.inner(self.conv).out_channels
        L = self.output_length(mel_spectrogram.shape[1])
        if Q.observing(self.conv):
            Q.record(self.conv, Q.conv1d_rows(self.conv, mel_spectrogram))
        # conv (+ activation fake-quant for QuantizedConv1d) -> GELU -> + PE, one GEMM
        x = Q.conv1d_rows(self.conv, mel_spectrogram, epilogue=_lib.EPI_GELU_PE, aux=self.pos_encoding.table(L),
                          ld_aux=D)
        if raw:
            return x
        return ops.layer_norm(x, self.norm.weight, self.norm.bias, self.norm.eps)


class CTCOutputHead(nn.Module):
    """LayerNorm -> Dropout -> Linear(d_model, vocab) (reference model.py:205-239)."""

    def __init__(self, d_model: int = 192, vocab_size: int = 50000, dropout: float = 0.1):
        super().__init__()
        self.proj = nn.Sequential(nn.LayerNorm(d_model), nn.Dropout(dropout), nn.Linear(d_model, vocab_size))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, L, D = x.shape
        ln = self.proj[0]
        w, b, qp = Q.linear_parts(self.proj[2])
        # the LayerNorm runs inside the GEMM's A read (identical float operations)
        logits = ops.gemm(x.reshape(B * L, D), w, b, qparams=qp, ln=(ln.weight, ln.bias, ln.eps))
        Q.record(self.proj[2], logits)
        return logits.view(B, L, w.shape[0])

    def argmax(self, x: torch.Tensor) -> torch.Tensor:
        """argmax over the vocabulary of forward(x), (B, L) int32, fused into the head GEMM: the
        (B, L, V) logits are never written (SURVEY §8 f, rank 1)."""
        B, L, D = x.shape
        ln = self.proj[0]
        w, b, qp = Q.linear_parts(self.proj[2])
        return ops.gemm_argmax(x.reshape(B * L, D), w, b, qparams=qp, ln=(ln.weight, ln.bias, ln.eps)).view(B, L)

    def greedy(self, x: torch.Tensor, blank: int = 0, out=None, rows=None):
        """Greedy CTC decode of forward(x) -- argmax(x) then the collapse of decode.py:46-69 --
        with the argmax and the collapse in one launch after the head GEMM: (tokens (B, L),
        lengths (B,)) int32.  rows: per-utterance row counts (int32 (B,)) of a padded batch."""
        B, L, D = x.shape
        ln = self.proj[0]
        w, b, qp = Q.linear_parts(self.proj[2])
        toks, lens, _, _ = ops.gemm_ctc_greedy(x.reshape(B * L, D), w, b, B, blank, qparams=qp,
                                               ln=(ln.weight, ln.bias, ln.eps), out=out, frames=rows)
        return toks, lens


class VELOCITYASR(nn.Module):
    """VELOCITY-ASR v2 (reference model.py:242-471)."""

    def __init__(self, config: Optional[VelocityASRConfig] = None):
        super().__init__()
        if config is None:
            config = VelocityASRConfig()
        self.config = config
        self.temporal_binding = TemporalBindingLayer(mel_bins=config.mel_bins, d_model=config.d_model)
        self.local_ssm = LocalSSMProcessor(d_model=config.d_model, num_layers=config.ssm_layers,
                                           state_dim=config.ssm_state_dim, expand_ratio=config.ssm_expand_ratio,
                                           kernel_size=config.ssm_kernel_size, dropout=config.dropout,
                                           use_checkpoint=config.gradient_checkpointing, scan_mode=config.scan_mode)
        self.global_context = HierarchicalGlobalContext(d_model=config.d_model, num_heads=config.attention_heads,
                                                        attention_dim=config.attention_dim,
                                                        global_ssm_layers=config.global_ssm_layers,
                                                        global_ssm_state_dim=config.global_ssm_state_dim,
                                                        dropout=config.dropout)
        self.ctc_head = CTCOutputHead(d_model=config.d_model, vocab_size=config.vocab_size, dropout=config.dropout)
        self._init_weights()
        # config.use_compile: the reference wraps submodules in torch.compile
        # (model.py:320-331); here the whole forward is already native HIP and can be
        # captured in a HIP graph (velocity_asr.pipeline.GraphedTranscriber) instead.

    def _init_weights(self):
        """Same initialisers, same order as the reference (model.py:305-318)."""
        for module in self.modules():
            if isinstance(module, nn.Linear):
                nn.init.xavier_uniform_(module.weight)
                if module.bias is not None:
                    nn.init.zeros_(module.bias)
            elif isinstance(module, nn.Conv1d):
                nn.init.kaiming_normal_(module.weight, mode="fan_out", nonlinearity="relu")
                if module.bias is not None:
                    nn.init.zeros_(module.bias)
            elif isinstance(module, nn.LayerNorm):
                nn.init.ones_(module.weight)
                nn.init.zeros_(module.bias)

    def _token_lengths(self, frames, n_frames: int):
        """Per-utterance token counts of a zero-padded batch (frames: its per-utterance mel frame
        counts, each <= n_frames, frames past them zero), or None for a uniform batch."""
        if frames is None:
            return None
        frames = [int(f) for f in frames]
        if not all(1 <= f <= n_frames for f in frames):
            raise ValueError(f"frames: each utterance needs 1..{n_frames} frames, got {frames}")
        return [self.temporal_binding.output_length(f) for f in frames]

    def _local_global(self, mel: torch.Tensor, lengths):
        """mel -> (local features, fused features): the temporal binding, the local stack, then the
        global context.  The stack's final LayerNorm and the context's query LayerNorm run as one
        launch (VASR_LN_PAIR=0: two), and the temporal binding's LayerNorm inside the first block's
        norm1 + conv launch (VASR_TB_PRENORM=0: its own launch); bitwise the same either way."""
        gc, tb = self.global_context, self.temporal_binding
        pre = None
        if os.environ.get("VASR_TB_PRENORM", "1") != "0" and type(tb.norm) is nn.LayerNorm:
            x, pre = tb(mel, raw=True), tb.norm
        else:
            x = tb(mel)
        if os.environ.get("VASR_LN_PAIR", "1") != "0" and type(gc.norm2) is nn.LayerNorm \
                and type(self.local_ssm.norm) is nn.LayerNorm:
            local, query = self.local_ssm.forward_pair(x, gc.norm2, pre_norm=pre)
            return local, gc(local, lengths=lengths, query=query)
        local = self.local_ssm(x, pre_norm=pre)
        return local, gc(local, lengths=lengths)

    def forward(self, mel_spectrogram: torch.Tensor, return_features: bool = False, frames=None):
        """(B, frames, mel_bins) -> CTC logits (B, (frames + 1) // 2, vocab_size).

        frames (extension): per-utterance frame counts of a batch of utterances of different
        lengths, zero-padded to a common length (velocity_asr.audio.mel_on_device(...,
        lengths=) writes such a batch).  Every utterance's logits over its own
        get_output_length(frames[b]) rows are then those it gets alone; later rows are junk."""
        if mel_spectrogram.device.type != "cuda":
            _lib.require_device()
            raise RuntimeError("velocity_asr (MI355X build): move the model and input to the HIP device "
                               "(model.to('cuda'), mel.to('cuda')); there is no CPU execution path")
        mel = mel_spectrogram.to(torch.float32)
        lengths = self._token_lengths(frames, mel.shape[1])
        with torch.no_grad():
            if return_features:  # the temporal binding's rows are returned, so they are formed on their own
                x = self.temporal_binding(mel)
                local_features = self.local_ssm(x)
                fused_features = self.global_context(local_features, lengths=lengths)
            else:
                local_features, fused_features = self._local_global(mel, lengths)
            logits = self.ctc_head(fused_features)
        if return_features:
            return logits, {"temporal_binding": x, "local_features": local_features,
                            "fused_features": fused_features}
        return logits

    def token_ids(self, mel_spectrogram: torch.Tensor, frames=None) -> torch.Tensor:
        """argmax(forward(mel), -1) as (B, L) int32 on the device, without materialising logits
        (the CTC head's GEMM reduces each row in its epilogue).  Identical to the argmax of
        forward()'s logits: same GEMM, same accumulation order."""
        if mel_spectrogram.device.type != "cuda":
            _lib.require_device()
            raise RuntimeError("velocity_asr (MI355X build): token_ids needs HIP tensors")
        lengths = self._token_lengths(frames, mel_spectrogram.shape[1])
        with torch.no_grad():
            x = self._local_global(mel_spectrogram.to(torch.float32), lengths)[1]
            return self.ctc_head.argmax(x)

    def greedy_token_ids(self, mel_spectrogram: torch.Tensor, frames=None, blank: int = 0, out=None, rows=None):
        """Collapsed greedy CTC tokens of forward(mel) on the device, (tokens (B, L), lengths (B,))
        int32: token_ids + ops.ctc_collapse with the argmax and the collapse in one launch.
        rows: per-utterance token-row counts (int32 (B,) on the device) of a padded batch."""
        if mel_spectrogram.device.type != "cuda":
            _lib.require_device()
            raise RuntimeError("velocity_asr (MI355X build): greedy_token_ids needs HIP tensors")
        lengths = self._token_lengths(frames, mel_spectrogram.shape[1])
        with torch.no_grad():
            x = self._local_global(mel_spectrogram.to(torch.float32), lengths)[1]
            return self.ctc_head.greedy(x, blank, out=out, rows=rows)

    def get_output_length(self, input_length: int) -> int:
        return (input_length + 1) // 2

    @classmethod
    def from_pretrained(cls, model_name_or_path: str, quantized: bool = False, **kwargs) -> "VELOCITYASR":
        """Load a checkpoint written by save_pretrained or Trainer (reference model.py:385-433)."""
        if not os.path.exists(model_name_or_path):
            raise NotImplementedError("Model hub download not yet implemented. "
                                      "Please provide a local path to the checkpoint.")
        checkpoint = torch.load(model_name_or_path, map_location="cpu", weights_only=True)
        if "config" in checkpoint:
            config = VelocityASRConfig.from_dict(checkpoint["config"])
        else:
            config = VelocityASRConfig()
        model = cls(config)
        if "model_state_dict" in checkpoint:
            model.load_state_dict(checkpoint["model_state_dict"])
        else:
            model.load_state_dict(checkpoint)
        return model

    def save_pretrained(self, save_path: str):
        """Same on-disk format as the reference (model.py:435-467)."""
        d = os.path.dirname(save_path)
        if d:
            os.makedirs(d, exist_ok=True)
        c = self.config
        checkpoint = {
            "config": {
                "mel_bins": c.mel_bins, "d_model": c.d_model, "ssm_layers": c.ssm_layers,
                "ssm_state_dim": c.ssm_state_dim, "ssm_expand_ratio": c.ssm_expand_ratio,
                "ssm_kernel_size": c.ssm_kernel_size, "global_ssm_layers": c.global_ssm_layers,
                "global_ssm_state_dim": c.global_ssm_state_dim, "attention_heads": c.attention_heads,
                "attention_dim": c.attention_dim, "vocab_size": c.vocab_size, "dropout": c.dropout,
                "gradient_checkpointing": c.gradient_checkpointing, "scan_mode": c.scan_mode,
                "use_compile": c.use_compile,
            },
            "model_state_dict": {k: v.detach().cpu() for k, v in self.state_dict().items()},
        }
        torch.save(checkpoint, save_path)

    def count_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad)
