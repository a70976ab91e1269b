"""Batch transcription pipeline on the device: audio (B, S) -> tokens, no host round trip.

    mel (reflect pad + DFT GEMM + log-mel)  ->  VELOCITYASR.token_ids (forward with the CTC head's
    row argmax fused into its GEMM)  ->  CTC collapse

Everything stays in HBM; the only device->host traffic is the (B, L) int32 token block
and lengths when the caller asks for Python lists.  ``GraphedTranscriber`` captures the
whole step in a HIP graph (torch.cuda.CUDAGraph over our HIP launches), which removes
the ~150 host launches per step from the critical path.
"""

from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch

from . import ops
from .audio import HOP_LENGTH, N_FFT, N_MELS, SAMPLE_RATE, mel_on_device
from .model import VELOCITYASR


# VASR_FUSED_ARGMAX=0 selects logits + a separate argmax pass (diagnostic comparison)
FUSED_ARGMAX = os.environ.get("VASR_FUSED_ARGMAX", "1") != "0"


def audio_to_token_ids(model: VELOCITYASR, audio: torch.Tensor, blank: int = 0,
                       out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                       lengths: Optional[List[int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(B, S) float32 HIP audio -> (tokens (B, L) int32, lengths (B,) int32), all on the device.
    out = (tokens, lengths) buffers to write the collapsed result into.  lengths: per-clip
    sample counts of clips of different lengths zero-padded to S (each clip's tokens are then
    those it gets alone: mel statistics, pooling sizes, attention keys and the collapse follow
    its own length, and the SSM stacks are causal)."""
    mel = mel_on_device(audio, SAMPLE_RATE, N_FFT, HOP_LENGTH, model.config.mel_bins, lengths=lengths)
    frames = None if lengths is None else [int(v) // HOP_LENGTH + 1 for v in lengths]
    if FUSED_ARGMAX:
        pred = model.token_ids(mel, frames=frames)  # CTC head GEMM with the row argmax fused: no logits in HBM
    else:
        pred = ops.argmax(model(mel, frames=frames))
    rows = None
    if frames is not None:
        rows = torch.tensor([model.get_output_length(f) for f in frames], dtype=torch.int32).to(audio.device)
    toks, lens, _, _ = ops.ctc_collapse(pred, blank, True, False, out=out, frames=rows)
    return toks, lens


def token_lists(toks: torch.Tensor, lens: torch.Tensor) -> List[List[int]]:
    t, n = toks.cpu().numpy(), lens.cpu().numpy()
    return [t[b, : n[b]].tolist() for b in range(t.shape[0])]


def _cu_masks(n_streams: int, mode: str, n_cu: int):
    """Per-stream CU masks (lists of uint32 words): "half" = contiguous blocks of logical CU ids,
    "interleave" = CU i to stream i % n_streams."""
    words = (n_cu + 31) // 32
    masks = []
    for s in range(n_streams):
        m = [0] * words
        for cu in range(n_cu):
            own = (cu * n_streams // n_cu == s) if mode == "half" else (cu % n_streams == s)
            if own:
                m[cu // 32] |= 1 << (cu % 32)
        masks.append(m)
    return masks


class _MaskedStream:
    """A torch ExternalStream over a CU-masked HIP stream created (and destroyed) by the library."""

    def __init__(self, device: torch.device, mask):
        import ctypes
        arr = (ctypes.c_uint32 * len(mask))(*mask)
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            ops.check(ops.L.lib().vasr_stream_create_cu_mask(arr, len(mask), ctypes.byref(h)),
                      "vasr_stream_create_cu_mask")
        self.handle = h.value
        self.stream = torch.cuda.ExternalStream(self.handle, device=device)

    def close(self):
        if self.handle is not None:
            ops.L.lib().vasr_stream_destroy(self.handle)
            self.handle = None


def _model_fingerprint(model: torch.nn.Module):
    """(tensor, data_ptr, version) of every parameter and buffer: a captured graph holds raw
    pointers to them and to the derived weight layouts built from them (split-bf16 planes,
    fake-quantized copies, [x_proj; dt_proj]), which are rebuilt -- and the old ones freed --
    when a parameter changes."""
    return [(t, t.data_ptr(), t._version) for t in list(model.parameters()) + list(model.buffers())]


class GraphedTranscriber:
    """Fixed-shape (B, S) audio -> tokens step captured once in HIP graphs.

    ``audio`` is the static input buffer (write new clips into it, or use it as-is for
    resident benchmark inputs); ``step()`` replays; ``tokens`` (B, L) int32 and ``lengths``
    (B,) int32 are the static outputs, refreshed by every replay.  With ``streams > 1`` the
    batch is split into that many utterance groups, each captured in its own graph and
    replayed on its own HIP stream; every group's collapse writes its rows of the shared
    outputs.  The groups are independent (no padding masks, per-utterance statistics), so
    results are bitwise those of one graph, while the VALU-bound scan of one group overlaps
    the MFMA-bound GEMMs of another on the same CUs (separate pipes).

    The graphs are tied to the model's parameters as they were at capture: ``step()`` raises
    if any parameter or buffer was replaced or modified in place since (build a new
    transcriber), and the derived weight layouts the graphs read are pinned for the
    transcriber's lifetime so replay never reads freed memory.
    """

    def __init__(self, model: VELOCITYASR, batch: int, samples: int, device: Optional[torch.device] = None,
                 warmup: int = 2, streams: int = 1, cu_split: Optional[str] = None):
        self.model = model
        dev = device or next(model.parameters()).device
        self.device = dev
        if batch % streams:
            raise ValueError("batch must divide by the number of streams")
        self.audio = torch.zeros((batch, samples), device=dev, dtype=torch.float32)
        frames = samples // HOP_LENGTH + 1
        L = model.get_output_length(frames)
        self.tokens = torch.zeros((batch, L), device=dev, dtype=torch.int32)
        self.lengths = torch.zeros((batch,), device=dev, dtype=torch.int32)
        g = batch // streams
        # cu_split ("half" | "interleave"; VASR_CU_SPLIT): each utterance group's stream owns a
        # disjoint share of the CUs (hipExtStreamCreateWithCUMask) instead of competing for all.
        # Measured much slower (65k / 91k vs 133k RTFx, tools/ab_env.sh): the groups' kernels
        # are latency-bound and gain from every CU; kept as an option, off by default.
        cu_split = cu_split if cu_split is not None else os.environ.get("VASR_CU_SPLIT", "none")
        self._masked = []
        if streams > 1 and cu_split in ("half", "interleave"):
            n_cu = int(ops.L.lib().vasr_device_cu_count())
            self._masked = [_MaskedStream(dev, m) for m in _cu_masks(streams, cu_split, n_cu)]
            self.streams = [m.stream for m in self._masked]
        elif cu_split not in ("none", "", None):
            raise ValueError(f"cu_split {cu_split!r}: expected none, half or interleave")
        else:
            self.streams = [torch.cuda.Stream(dev) for _ in range(streams)]
        views = [self.audio[i * g:(i + 1) * g] for i in range(streams)]
        outs = [(self.tokens[i * g:(i + 1) * g], self.lengths[i * g:(i + 1) * g]) for i in range(streams)]
        main = torch.cuda.current_stream(dev)
        for st, v in zip(self.streams, views):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                for _ in range(warmup):  # builds the cached weight layouts before capture
                    audio_to_token_ids(model, v)
            main.wait_stream(st)
        self._fingerprint = _model_fingerprint(model)
        # pin every derived layout the graphs will read (they stay alive with the transcriber)
        self._pinned = [dict(m.__dict__.get("_vasr_prepared", {})) for m in model.modules()]
        self._pinned += [dict(ops._splits), dict(ops._splits16), dict(ops._f32_copies)]
        self.graphs = []
        for st, v, o in zip(self.streams, views, outs):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=st):
                audio_to_token_ids(model, v, out=o)
            self.graphs.append(gr)

    def _check_params(self) -> None:
        for t, p, v in self._fingerprint:
            if t.data_ptr() != p or t._version != v:
                raise RuntimeError("GraphedTranscriber: the model's parameters changed after capture "
                                   "(the graphs read the old weights); build a new GraphedTranscriber")

    def step(self) -> None:
        self._check_params()
        main = torch.cuda.current_stream(self.device)
        for st, gr in zip(self.streams, self.graphs):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                gr.replay()
        for st in self.streams:
            main.wait_stream(st)

    def collect(self):
        """(tokens, lengths) of the last step (the static outputs)."""
        return self.tokens, self.lengths
