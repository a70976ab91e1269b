"""Utterance-sharded multi-GPU transcription (one process per GPU, torch.distributed).

VELOCITY-ASR inference has no cross-utterance dependency (per-utterance normalisation,
per-token LayerNorm, per-utterance pooling and attention; SURVEY §8 e), so a batch shards
embarrassingly: rank r transcribes utterances [r*B/W, (r+1)*B/W).  The only collectives are
at the edges of the job:

  * scatter_audio: rank 0 scatters equal (B/W, S) audio shards (RCCL over xGMI with the
    "nccl" backend on ROCm; each shard rides its own peer link),
  * gather_tokens: rank 0 gathers the per-rank (B/W, L) int32 token blocks and lengths
    (64 KB per rank at 32 x 10 s) and turns them into Python lists.

Nothing else is exchanged: weights are loaded (or broadcast once) per rank at start-up.
The step function is pluggable so the plumbing is testable with gloo on CPU.
"""

from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, end) of rank's utterances; the first n % world ranks get one more."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def scatter_audio(audio: Optional[torch.Tensor], per_rank: int, samples: int, device: torch.device,
                  src: int = 0, out: Optional[torch.Tensor] = None, group=None) -> torch.Tensor:
    """Scatter (world*per_rank, samples) audio held by `src` into (per_rank, samples) shards.
    out: the destination shard (e.g. a GraphedTranscriber's static input), else allocated.
    group: the process group to use (default: the default group; every rank a member)."""
    world = dist.get_world_size(group)
    if out is None:
        out = torch.empty((per_rank, samples), dtype=torch.float32, device=device)
    elif tuple(out.shape) != (per_rank, samples) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"scatter_audio: out must be a contiguous float32 ({per_rank}, {samples}) tensor")
    if dist.get_rank() == src:
        if audio is None or audio.shape != (world * per_rank, samples):
            raise ValueError(f"scatter_audio: src needs ({world * per_rank}, {samples}) audio")
        chunks = list(audio.to(device=device, dtype=torch.float32).contiguous().chunk(world, 0))
        dist.scatter(out, chunks, src=src, group=group)
    else:
        dist.scatter(out, None, src=src, group=group)
    return out


def gather_token_blocks(tokens: torch.Tensor, lengths: torch.Tensor, dst: int = 0,
                        group=None) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """Gather per-rank (b, L) int32 tokens + (b,) lengths into (world*b, L) / (world*b,) device
    tensors on `dst` (rank order = utterance order); None on the other ranks."""
    world = dist.get_world_size(group)
    tok = tokens.contiguous()
    ln = lengths.contiguous()
    if dist.get_rank() == dst:
        tok_all = torch.empty((world * tok.shape[0],) + tuple(tok.shape[1:]), dtype=tok.dtype, device=tok.device)
        len_all = torch.empty((world * ln.shape[0],), dtype=ln.dtype, device=ln.device)
        dist.gather(tok, list(tok_all.chunk(world, 0)), dst=dst, group=group)
        dist.gather(ln, list(len_all.chunk(world, 0)), dst=dst, group=group)
        return tok_all, len_all
    dist.gather(tok, None, dst=dst, group=group)
    dist.gather(ln, None, dst=dst, group=group)
    return None


def gather_tokens(tokens: torch.Tensor, lengths: torch.Tensor, dst: int = 0,
                  group=None) -> Optional[List[List[int]]]:
    """Gather per-rank (b, L) int32 tokens + (b,) lengths on `dst`; returns lists there, else None."""
    blocks = gather_token_blocks(tokens, lengths, dst, group)
    if blocks is None:
        return None
    t, n = blocks[0].cpu(), blocks[1].cpu()
    return [t[i, : int(n[i])].tolist() for i in range(t.shape[0])]


def transcribe_sharded(step: Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]],
                       audio: Optional[torch.Tensor], batch: int, samples: int, device: torch.device,
                       src: int = 0, shard: Optional[torch.Tensor] = None, as_lists: bool = True, group=None):
    """Scatter `batch` clips from `src`, run `step(shard) -> (tokens, lengths)` on every rank,
    gather the results on `src`: token lists, or with as_lists=False the (batch, L) / (batch,)
    device tensors.  `batch` must divide by the world size (equal shards: the model has no
    padding masks, so utterances are never padded to a common length).  shard: the buffer to
    scatter into (a GraphedTranscriber's static input; see graphed_step).  group: the process
    group of the collectives (default: the default group)."""
    world = dist.get_world_size(group)
    if batch % world:
        raise ValueError(f"batch {batch} must be a multiple of the world size {world}")
    shard = scatter_audio(audio, batch // world, samples, device, src, out=shard, group=group)
    tokens, lengths = step(shard)
    if as_lists:
        return gather_tokens(tokens, lengths, src, group)
    return gather_token_blocks(tokens, lengths, src, group)


def hip_step(model) -> Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]]:
    """The MI355X step: audio shard -> device tokens via velocity_asr.pipeline."""
    from .pipeline import audio_to_token_ids

    def step(shard: torch.Tensor):
        return audio_to_token_ids(model, shard)
    return step


def graphed_step(tr) -> Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]]:
    """The MI355X step as HIP graph replays of a GraphedTranscriber; the shard must be the
    transcriber's own input buffer (pass shard=tr.audio to transcribe_sharded)."""

    def step(shard: torch.Tensor):
        if shard.data_ptr() != tr.audio.data_ptr():
            raise ValueError("graphed_step: scatter into the transcriber's input (shard=tr.audio)")
        tr.step()
        return tr.collect()  # raises if the step ran on weights changed since capture
    return step
