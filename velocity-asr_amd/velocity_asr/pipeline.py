"""Batch transcription pipeline on the device: audio (B, S) -> tokens, no host round trip.

    mel (reflect pad + DFT GEMM + log-mel)  ->  VELOCITYASR.forward  ->  argmax  ->  CTC collapse

Everything stays in HBM; the only device->host traffic is the (B, L) int32 token block
and lengths when the caller asks for Python lists.  ``GraphedTranscriber`` captures the
whole step in a HIP graph (torch.cuda.CUDAGraph over our HIP launches), which removes
the ~150 host launches per step from the critical path.
"""

from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from . import ops
from .audio import HOP_LENGTH, N_FFT, N_MELS, SAMPLE_RATE, mel_on_device
from .model import VELOCITYASR


def audio_to_token_ids(model: VELOCITYASR, audio: torch.Tensor, blank: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """(B, S) float32 HIP audio -> (tokens (B, L) int32, lengths (B,) int32), all on the device."""
    mel = mel_on_device(audio, SAMPLE_RATE, N_FFT, HOP_LENGTH, model.config.mel_bins)
    logits = model(mel)
    pred = ops.argmax(logits)
    toks, lens, _, _ = ops.ctc_collapse(pred, blank, True, False)
    return toks, lens


def token_lists(toks: torch.Tensor, lens: torch.Tensor) -> List[List[int]]:
    t, n = toks.cpu().numpy(), lens.cpu().numpy()
    return [t[b, : n[b]].tolist() for b in range(t.shape[0])]


class GraphedTranscriber:
    """Fixed-shape (B, S) audio -> tokens step captured once in a HIP graph.

    ``audio`` is the static input buffer (write new clips into it, or use it as-is for
    resident benchmark inputs); ``step()`` replays the graph; ``tokens`` / ``lengths``
    are the static outputs.
    """

    def __init__(self, model: VELOCITYASR, batch: int, samples: int, device: Optional[torch.device] = None,
                 warmup: int = 2):
        self.model = model
        dev = device or next(model.parameters()).device
        self.audio = torch.zeros((batch, samples), device=dev, dtype=torch.float32)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):  # builds the cached weight layouts before capture
                audio_to_token_ids(model, self.audio)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.tokens, self.lengths = audio_to_token_ids(model, self.audio)

    def step(self) -> None:
        self.graph.replay()
