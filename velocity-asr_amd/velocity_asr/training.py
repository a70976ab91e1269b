"""Evaluation metrics used by scripts/evaluate.py (reference velocity_asr/training.py:412-501).

Training itself (CTCLoss, schedulers, Trainer) is outside this inference build's scope
(SURVEY §2 row 8); only the WER/CER helpers that evaluate.py imports are provided.
"""

from __future__ import annotations

from typing import List, Sequence


def _edit_distance(a: Sequence, b: Sequence) -> int:
    """Levenshtein distance, unit costs, two-row DP (same values as the reference's full table)."""
    prev = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        cur = [i] + [0] * len(b)
        ai = a[i - 1]
        for j in range(1, len(b) + 1):
            if ai == b[j - 1]:
                cur[j] = prev[j - 1]
            else:
                cur[j] = 1 + min(prev[j], cur[j - 1], prev[j - 1])
        prev = cur
    return prev[len(b)]


def compute_wer(predictions: List[str], references: List[str]) -> float:
    """Word error rate: total word edits / total reference words (0.0 if no words)."""
    errors = words = 0
    for pred, ref in zip(predictions, references):
        ref_words = ref.lower().split()
        errors += _edit_distance(pred.lower().split(), ref_words)
        words += len(ref_words)
    return errors / words if words > 0 else 0.0


def compute_cer(predictions: List[str], references: List[str]) -> float:
    """Character error rate: total char edits / total reference chars (0.0 if none)."""
    errors = chars = 0
    for pred, ref in zip(predictions, references):
        ref_chars = list(ref.lower())
        errors += _edit_distance(list(pred.lower()), ref_chars)
        chars += len(ref_chars)
    return errors / chars if chars > 0 else 0.0
