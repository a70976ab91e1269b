"""Batch transcription pipeline on the device: audio (B, S) -> tokens, no host round trip.

    mel (real-FFT |STFT|^2 straight from the unpadded audio + log-mel; other n_fft / hop: reflect
    pad + DFT GEMM)  ->  VELOCITYASR.greedy_token_ids (forward with the CTC head's row argmax
    fused into its GEMM, then the argmax keys and the CTC collapse in one launch)

Everything stays in HBM; the only device->host traffic is the (B, L) int32 token block
and lengths when the caller asks for Python lists.  ``GraphedTranscriber`` captures the
whole step in a HIP graph (torch.cuda.CUDAGraph over our HIP launches), which removes
the ~150 host launches per step from the critical path.
"""

from __future__ import annotations

import operator
import os
import time
from typing import Callable, Dict, List, Optional, Tuple

import torch

from . import ops
from .audio import HOP_LENGTH, N_FFT, N_MELS, SAMPLE_RATE, mel_on_device
from .model import VELOCITYASR


# VASR_FUSED_ARGMAX=0 selects logits + a separate argmax pass (diagnostic comparison)
FUSED_ARGMAX = os.environ.get("VASR_FUSED_ARGMAX", "1") != "0"
# VASR_COLLAPSE_KEYS=0: the argmax keys and the collapse as two launches (A/B comparison)
COLLAPSE_KEYS = os.environ.get("VASR_COLLAPSE_KEYS", "1") != "0"


def audio_to_token_ids(model: VELOCITYASR, audio: torch.Tensor, blank: int = 0,
                       out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                       lengths: Optional[List[int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(B, S) float32 HIP audio -> (tokens (B, L) int32, lengths (B,) int32), all on the device.
    out = (tokens, lengths) buffers to write the collapsed result into.  lengths: per-clip
    sample counts of clips of different lengths zero-padded to S (each clip's tokens are then
    those it gets alone: mel statistics, pooling sizes, attention keys and the collapse follow
    its own length, and the SSM stacks are causal)."""
    # zero-framed for the temporal conv (its padding): no separate padding pass
    mel = mel_on_device(audio, SAMPLE_RATE, N_FFT, HOP_LENGTH, model.config.mel_bins, lengths=lengths,
                        frame_pad=model.temporal_binding.conv_padding())
    frames = None if lengths is None else [int(v) // HOP_LENGTH + 1 for v in lengths]
    rows = None
    if frames is not None:
        rows = torch.tensor([model.get_output_length(f) for f in frames], dtype=torch.int32).to(audio.device)
    if FUSED_ARGMAX and COLLAPSE_KEYS:
        # CTC head GEMM with the row argmax fused (no logits in HBM), then argmax keys + collapse
        # in one launch
        return model.greedy_token_ids(mel, frames=frames, blank=blank, out=out, rows=rows)
    pred = model.token_ids(mel, frames=frames) if FUSED_ARGMAX else ops.argmax(model(mel, frames=frames))
    toks, lens, _, _ = ops.ctc_collapse(pred, blank, True, False, out=out, frames=rows)
    return toks, lens


def token_lists(toks: torch.Tensor, lens: torch.Tensor) -> List[List[int]]:
    t, n = toks.cpu().numpy(), lens.cpu().numpy()
    if (n < 0).any() or (n > t.shape[1]).any():
        raise ValueError("token_lists: lengths outside [0, L] (outputs of an invalidated step?)")
    return [t[b, : n[b]].tolist() for b in range(t.shape[0])]


def _model_tensors(model: torch.nn.Module):
    """Every parameter and buffer: a captured graph holds raw pointers to them and to the
    derived weight layouts built from them (split-bf16 planes, fake-quantized copies,
    [x_proj; dt_proj]), which are rebuilt -- and the old ones freed -- when a parameter changes."""
    return list(model.parameters()) + list(model.buffers())


_VERSION = operator.attrgetter("_version")


class GraphedTranscriber:
    """Fixed-shape (B, S) audio -> tokens step captured once in HIP graphs.

    ``audio`` is the static input buffer (write new clips into it, or use it as-is for
    resident benchmark inputs); ``step()`` replays; ``tokens`` (B, L) int32 and ``lengths``
    (B,) int32 are the static outputs, refreshed by every replay.  With ``streams > 1`` the
    batch is split into that many utterance groups, each captured in its own graph; group 0
    replays on the caller's stream, the others on their own HIP streams; every group's collapse
    writes its rows of the shared
    outputs.  The groups are independent (no padding masks, per-utterance statistics), so
    results are bitwise those of one graph, while the VALU-bound scan of one group overlaps
    the MFMA-bound GEMMs of another on the same CUs (separate pipes).  (Up to round 3 two groups
    replayed concurrently could return wrong tokens for group 1: kernels of one stream disturbed
    co-resident workgroups of the other: a scan LDS slab read back wrong, and the |STFT|^2 kernel's
    packed-fp32 complex arithmetic came back wrong in one half-wave beside tile GEMMs.  Both code
    forms are gone from the kernels; profiles/r04b-r04o.)

    The graphs are tied to the model's parameters as they were at capture: ``step()`` raises
    if any parameter or buffer was replaced or modified in place since (build a new
    transcriber); the parameters and the derived weight layouts the graphs read are held for
    the transcriber's lifetime so replay never reads freed memory.
    """

    def __init__(self, model: VELOCITYASR, batch: int, samples: int, device: Optional[torch.device] = None,
                 warmup: int = 2, streams: int = 1):
        self.model = model
        self._stale = False
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
        # the tensors are held (so a replaced parameter's old storage stays allocated for the
        # graphs) with their pointers and versions at capture
        self._tensors = _model_tensors(model)
        self._ptrs = [t.data_ptr() for t in self._tensors]
        self._versions = list(map(_VERSION, self._tensors))
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
        if (list(map(_VERSION, self._tensors)) != self._versions
                or [t.data_ptr() for t in self._tensors] != self._ptrs):
            # the replay just issued ran on the old weights: clear its outputs (zero tokens and
            # lengths, ordered after the replay on the caller's stream) and refuse to hand them out
            # (collect() raises); a caller holding the static buffers sees empty transcripts
            self._stale = True
            self.tokens.zero_()
            self.lengths.zero_()
            raise RuntimeError("GraphedTranscriber: the model's parameters changed after capture "
                               "(the graphs read the old weights); build a new GraphedTranscriber")

    def step(self) -> None:
        """Replay the graphs (group 0 on the caller's current stream, the others on their own
        streams after it), then check (while the device runs them) that no parameter or buffer
        was replaced or modified since capture: the check (~60 us of host time for the 208
        tensors) overlaps the replay instead of delaying it.  The graphs only ever read storage
        this object keeps alive, so a failed check raises after a replay on the old weights."""
        main = torch.cuda.current_stream(self.device)
        # group 0 replays on the caller's stream itself: ordered with the caller's work without
        # cross-stream events (each event wait costs the device a queue-to-queue hop: one 10-s
        # utterance 0.602 vs 0.714 ms per step, C2 +1.3 %; profiles/r03ah/); the other groups on
        # their own streams, fenced by events on the caller's stream
        for st in self.streams[1:]:
            st.wait_stream(main)
        self.graphs[0].replay()
        for st, gr in zip(self.streams[1:], self.graphs[1:]):
            with torch.cuda.stream(st):
                gr.replay()
        for st in self.streams[1:]:
            main.wait_stream(st)
        self._check_params()

    def release_candidates(self) -> None:
        """Free the other schedules autotuned_transcriber built and timed beside this one."""
        self.__dict__.pop("_candidates", None)
        torch.cuda.synchronize(self.device)

    def collect(self):
        """(tokens, lengths) of the last step (the static outputs).  Raises once a step found
        the parameters changed since capture (its outputs came from the old weights)."""
        if self._stale:
            raise RuntimeError("GraphedTranscriber: the last step ran on weights that changed after capture; "
                               "build a new GraphedTranscriber")
        return self.tokens, self.lengths


def schedule_candidates(batch: int) -> List[int]:
    """Stream counts GraphedTranscriber can use for `batch` clips: one graph of the whole batch,
    and two utterance groups when the batch splits into groups of at least 4 clips."""
    return [1, 2] if batch >= 8 and batch % 2 == 0 else [1]


def autotuned_transcriber(model: VELOCITYASR, batch: int, samples: int, device: Optional[torch.device] = None,
                          candidates: Optional[List[int]] = None, reps: int = 5, rounds: int = 3,
                          audio: Optional[torch.Tensor] = None,
                          agree: Optional[Callable[[Dict[int, float]], Dict[int, float]]] = None,
                          max_rounds: int = 12, settle: float = 0.01, keep_candidates: bool = False):
    """The GraphedTranscriber schedule that runs fastest on this device.

    One graph of the whole batch and two utterance-group graphs on concurrent streams give
    bitwise the same tokens; which is faster depends on the box (round 4, C2 on two MI355X
    boxes: 143.4k vs 140.4k RTFx for two groups on one, 146k vs 150k for one graph on another,
    profiles/r04r, r04t).  Each candidate is built, then replayed in interleaved rounds (two warm
    replays, then `reps` timed); rounds continue past `rounds` until every candidate's last round
    is within `settle` of its previous one (at most `max_rounds`): a device fresh from idle runs
    the same replays up to 25 % slower for its first few tens of milliseconds of load
    (profiles/r05h/), so early rounds would time the ramp, not the schedule.  The fastest
    candidate is returned and the others are freed before returning, unless keep_candidates:
    then they stay alive on the returned transcriber (their graphs and static buffers) until its
    release_candidates() -- bench.py's choice, since freeing a graph's memory pool stalls the
    device, which would idle it between the tuning and the timed steps.  Returns (transcriber,
    {streams: best ms per replay}); the transcriber's .autotune_rounds holds every round's times.

    audio: the (batch, samples) clips the transcriber will serve, copied into every candidate
    before timing (the step's time depends on the data: the projection's per-chunk softplus
    branch, exp arguments, clocks held on silence); without it the candidates time zeros.
    agree: maps this process's {streams: ms} to the times every rank of a job decides on (e.g.
    the max over ranks), so all ranks keep the same schedule."""
    cands = list(candidates or schedule_candidates(batch))
    trs = {s: GraphedTranscriber(model, batch, samples, device, streams=s) for s in cands}
    if audio is not None:
        for tr in trs.values():
            tr.audio.copy_(audio)
    if len(cands) == 1:
        tr = trs[cands[0]]
        tr.autotune_rounds = []
        return tr, {}
    times = {s: float("inf") for s in cands}
    hist: List[Dict[int, float]] = []
    for r in range(max_rounds):
        this = {}
        for s, tr in trs.items():
            tr.step()
            tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                tr.step()
            torch.cuda.synchronize()
            this[s] = (time.perf_counter() - t0) / reps * 1e3
            times[s] = min(times[s], this[s])
        hist.append(this)
        if r + 1 >= rounds and (len(hist) < 2 or all(abs(hist[-1][s] - hist[-2][s]) <= settle * hist[-1][s]
                                                      for s in cands)):
            break
    if agree is not None:
        times = dict(agree(times))
    best = min(cands, key=lambda s: times[s])
    keep = trs.pop(best)
    keep._candidates = list(trs.values())  # released by release_candidates()
    if not keep_candidates:
        keep.release_candidates()
    keep.autotune_rounds = [{s: round(t, 4) for s, t in h.items()} for h in hist]
    return keep, {s: round(t, 4) for s, t in times.items()}
