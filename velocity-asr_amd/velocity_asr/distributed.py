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
                  src: int = 0) -> torch.Tensor:
    """Scatter (world*per_rank, samples) audio held by `src` into (per_rank, samples) shards."""
    world = dist.get_world_size()
    out = torch.empty((per_rank, samples), dtype=torch.float32, device=device)
    if dist.get_rank() == src:
        if audio is None or audio.shape != (world * per_rank, samples):
            raise ValueError(f"scatter_audio: src needs ({world * per_rank}, {samples}) audio")
        chunks = list(audio.to(device=device, dtype=torch.float32).contiguous().chunk(world, 0))
        dist.scatter(out, chunks, src=src)
    else:
        dist.scatter(out, None, src=src)
    return out


def gather_tokens(tokens: torch.Tensor, lengths: torch.Tensor, dst: int = 0) -> Optional[List[List[int]]]:
    """Gather per-rank (b, L) int32 tokens + (b,) lengths on `dst`; returns lists there, else None."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    tok = tokens.contiguous()
    ln = lengths.contiguous()
    if rank == dst:
        tok_all = [torch.empty_like(tok) for _ in range(world)]
        len_all = [torch.empty_like(ln) for _ in range(world)]
        dist.gather(tok, tok_all, dst=dst)
        dist.gather(ln, len_all, dst=dst)
        out = []
        for t, n in zip(tok_all, len_all):
            t, n = t.cpu(), n.cpu()
            out.extend(t[i, : int(n[i])].tolist() for i in range(t.shape[0]))
        return out
    dist.gather(tok, None, dst=dst)
    dist.gather(ln, None, dst=dst)
    return None


def transcribe_sharded(step: Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]],
                       audio: Optional[torch.Tensor], batch: int, samples: int, device: torch.device,
                       src: int = 0) -> Optional[List[List[int]]]:
    """Scatter `batch` clips from `src`, run `step(shard) -> (tokens, lengths)` on every rank,
    gather the token lists on `src`.  `batch` must divide by the world size (equal shards:
    the model has no padding masks, so utterances are never padded to a common length)."""
    world = dist.get_world_size()
    if batch % world:
        raise ValueError(f"batch {batch} must be a multiple of the world size {world}")
    shard = scatter_audio(audio, batch // world, samples, device, src)
    tokens, lengths = step(shard)
    return gather_tokens(tokens, lengths, src)


def hip_step(model) -> Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]]:
    """The MI355X step: audio shard -> device tokens via velocity_asr.pipeline."""
    from .pipeline import audio_to_token_ids

    def step(shard: torch.Tensor):
        return audio_to_token_ids(model, shard)
    return step
