"""CTC decoding (drop-in for reference velocity_asr/decode.py).

Greedy decoding runs on the device: an argmax kernel over the vocabulary and a
per-utterance collapse kernel (blank removal, repeat collapse, optional run
timestamps), so only the kept token ids cross PCIe instead of (B, L, V) logits.
Token -> text conversion is host string handling, as in the reference.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _lib, ops

BLANK_TOKEN = 0


@dataclass
class DecodingResult:
    """Result of CTC decoding (reference decode.py:18-24)."""

    text: str
    tokens: List[int]
    score: float
    timestamps: Optional[List[Tuple[int, int]]] = None


def _on_device(logits: torch.Tensor) -> torch.Tensor:
    if logits.device.type != "cuda":
        _lib.require_device()
        logits = logits.to(torch.device("cuda", torch.cuda.current_device()))
    if logits.dtype != torch.float32:
        logits = logits.float()
    return logits


def greedy_token_ids(logits: torch.Tensor, blank_token: int = BLANK_TOKEN, collapse_repeated: bool = True,
                     timestamps: bool = False):
    """Device argmax + collapse; returns (tokens (B,L) int32, lengths (B,), start, end) on the device."""
    logits = _on_device(logits)
    pred = ops.argmax(logits).view(logits.shape[0], -1)
    return ops.ctc_collapse(pred, blank_token, collapse_repeated, timestamps)


def ctc_greedy_decode(logits: torch.Tensor, blank_token: int = BLANK_TOKEN,
                      collapse_repeated: bool = True) -> List[List[int]]:
    """Greedy CTC decoding (reference decode.py:27-71)."""
    toks, lens, _, _ = greedy_token_ids(logits, blank_token, collapse_repeated)
    toks, lens = toks.cpu().numpy(), lens.cpu().numpy()
    return [toks[b, : lens[b]].tolist() for b in range(toks.shape[0])]


def ctc_greedy_decode_with_timestamps(logits: torch.Tensor,
                                      blank_token: int = BLANK_TOKEN) -> List[Tuple[List[int], List[Tuple[int, int]]]]:
    """Greedy decoding with (start_frame, end_frame) per token (reference decode.py:74-125)."""
    toks, lens, st, en = greedy_token_ids(logits, blank_token, True, timestamps=True)
    toks, lens, st, en = toks.cpu().numpy(), lens.cpu().numpy(), st.cpu().numpy(), en.cpu().numpy()
    out = []
    for b in range(toks.shape[0]):
        n = int(lens[b])
        out.append((toks[b, :n].tolist(), [(int(s), int(e)) for s, e in zip(st[b, :n], en[b, :n])]))
    return out


def ctc_beam_search(logits: torch.Tensor, beam_width: int = 10, blank_token: int = BLANK_TOKEN,
                    lm_weight: float = 0.0, lm_scorer: Optional[Any] = None) -> List[List[DecodingResult]]:
    """Prefix beam search (reference decode.py:128-217) on the HIP device.

    Without a language model the whole search runs in vasr_ctc_beam_search (one workgroup
    per utterance, prefixes as trie nodes, the reference's insertion-order tie rules).  An
    lm_scorer is a Python callable, so with one (or beam_width > 32) the search runs on the
    host with the same bookkeeping over device-computed log-probabilities.
    """
    logits = _on_device(logits)
    if (lm_scorer is None or lm_weight <= 0) and 1 <= beam_width <= 32:
        toks, lens, scores, nb = ops.ctc_beam_search(logits.float(), beam_width, blank_token)
        toks, lens, scores, nb = toks.cpu().numpy(), lens.cpu().numpy(), scores.cpu().numpy(), nb.cpu().numpy()
        return [[DecodingResult(text="", tokens=toks[b, r, :lens[b, r]].tolist(), score=float(scores[b, r]))
                 for r in range(int(nb[b]))] for b in range(toks.shape[0])]
    return _ctc_beam_search_host(logits, beam_width, blank_token, lm_weight, lm_scorer)


def _ctc_beam_search_host(logits: torch.Tensor, beam_width: int, blank_token: int, lm_weight: float,
                          lm_scorer: Optional[Any]) -> List[List[DecodingResult]]:
    """Host form of the same search (used with a Python lm_scorer)."""
    log_probs = torch.log_softmax(logits, dim=-1).cpu().numpy().astype(np.float64)
    B, L, V = log_probs.shape
    all_results = []
    for b in range(B):
        beams: Dict[Tuple[int, ...], Tuple[float, Optional[int]]] = {(): (0.0, None)}
        for t in range(L):
            lp = log_probs[b, t]
            new_beams: Dict[Tuple[int, ...], Tuple[float, Optional[int]]] = {}
            for prefix, (score, last) in beams.items():
                blank_score = score + lp[blank_token]
                cur = new_beams.get(prefix)
                if cur is None or cur[0] < blank_score:
                    new_beams[prefix] = (blank_score, blank_token)
                scores = (score + lp).tolist()
                for token in range(V):
                    if token == blank_token:
                        continue
                    key = prefix if last == token else prefix + (token,)
                    s = scores[token]
                    if lm_scorer is not None and lm_weight > 0:
                        s += lm_weight * lm_scorer.score(list(key))
                    cur = new_beams.get(key)
                    if cur is None or cur[0] < s:
                        new_beams[key] = (s, token)
            beams = dict(sorted(new_beams.items(), key=lambda x: x[1][0], reverse=True)[:beam_width])
        results = [DecodingResult(text="", tokens=list(prefix), score=score)
                   for prefix, (score, _) in sorted(beams.items(), key=lambda x: x[1][0], reverse=True)]
        all_results.append(results)
    return all_results


class CTCDecoder:
    """CTC decoder with vocabulary (reference decode.py:220-327)."""

    def __init__(self, vocabulary: List[str], blank_token: int = BLANK_TOKEN):
        self.vocabulary = vocabulary
        self.blank_token = blank_token
        self.vocab_size = len(vocabulary)
        self.token_to_idx = {token: idx for idx, token in enumerate(vocabulary)}

    def decode_greedy(self, logits: torch.Tensor, collapse_repeated: bool = True) -> List[str]:
        seqs = ctc_greedy_decode(logits, blank_token=self.blank_token, collapse_repeated=collapse_repeated)
        return [self._tokens_to_text(t) for t in seqs]

    def decode_beam_search(self, logits: torch.Tensor, beam_width: int = 10, return_all_beams: bool = False):
        beam_results = ctc_beam_search(logits, beam_width=beam_width, blank_token=self.blank_token)
        if return_all_beams:
            for batch_results in beam_results:
                for result in batch_results:
                    result.text = self._tokens_to_text(result.tokens)
            return beam_results
        return [self._tokens_to_text(results[0].tokens) if results else "" for results in beam_results]

    def _tokens_to_text(self, tokens: List[int]) -> str:
        chars = [self.vocabulary[t] if 0 <= t < self.vocab_size else "<unk>" for t in tokens]
        return "".join(chars).replace("▁", " ").strip()

    def text_to_tokens(self, text: str) -> List[int]:
        tokens = []
        for char in text:
            if char in self.token_to_idx:
                tokens.append(self.token_to_idx[char])
            elif "<unk>" in self.token_to_idx:
                tokens.append(self.token_to_idx["<unk>"])
        return tokens


def create_default_vocabulary(vocab_size: int = 50000) -> List[str]:
    """Character vocabulary + placeholders (reference decode.py:330-362)."""
    vocab = ["<blank>", "<unk>", "<pad>", " "]
    vocab.extend(list("abcdefghijklmnopqrstuvwxyz"))
    vocab.extend(list("ABCDEFGHIJKLMNOPQRSTUVWXYZ"))
    vocab.extend(list("0123456789"))
    vocab.extend(list(".,!?;:'\"()-"))
    for i in range(len(vocab), vocab_size):
        vocab.append(f"<token_{i}>")
    return vocab
