"""File-level transcription used by scripts/transcribe.py and scripts/evaluate.py.

The reference scripts run one file at a time: load -> mel on the host -> (1, F, 80) forward
-> greedy decode (reference scripts/transcribe.py:48-131, scripts/evaluate.py:60-107).
Here files are read on the host, sorted by length and cut into batches that go through the
device pipeline together (mel, forward, argmax, collapse all on the HIP device).  A batch of
clips of different lengths is zero-padded to its longest clip and carries each clip's own
length (pipeline.audio_to_token_ids(..., lengths=)): the mel statistics, pooling sizes,
attention keys and the collapse follow each clip's length and the SSM stacks are causal, so
the output for a file is the one the reference's per-file loop produces.  Where the front end
has no per-length kernels (VASR_STFT=gemm, n_mels > 85) batches hold clips of one length.
"""

from __future__ import annotations

import logging
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from . import ops
from .audio import HOP_LENGTH, N_FFT, SAMPLE_RATE, load_audio, mel_on_device, ragged_supported
from .decode import CTCDecoder

logger = logging.getLogger(__name__)

AUDIO_EXTENSIONS = {".wav", ".mp3", ".flac", ".ogg", ".m4a"}


def find_audio_files(directory: str) -> List[Path]:
    """Recursive listing with the reference's extension set (scripts/transcribe.py:233-238)."""
    return [p for p in Path(directory).rglob("*") if p.suffix.lower() in AUDIO_EXTENSIONS]


def frames_to_seconds(frame_idx: int, hop_length: int = HOP_LENGTH, sample_rate: int = SAMPLE_RATE) -> float:
    """Token frame -> seconds; tokens sit at stride 2 in mel frames (reference scripts/transcribe.py:42-45)."""
    return (frame_idx * 2 * hop_length) / sample_rate


def group_words(tokens: Sequence[int], spans: Sequence[Tuple[int, int]], vocabulary: Sequence[str]) -> List[Dict]:
    """Word segmentation of a timed token list (reference scripts/transcribe.py:83-117).

    A word is a run of non-separator characters (" " and "▁" separate). Its start is the
    first character's start frame; its end is the end frame of the separator that closes
    it, or of the utterance's last token for the final word — the reference's convention.
    """
    words: List[Dict] = []
    chars: List[str] = []
    first: Optional[int] = None

    def flush(end_frame: int) -> None:
        text = "".join(chars).replace("▁", "")
        if text:
            words.append({"word": text, "start": frames_to_seconds(first), "end": frames_to_seconds(end_frame)})

    for tok, (s, e) in zip(tokens, spans):
        ch = vocabulary[tok] if 0 <= tok < len(vocabulary) else "<unk>"
        if ch in (" ", "▁"):
            if chars:
                flush(e)
                chars, first = [], None
        else:
            if first is None:
                first = s
            chars.append(ch)
    if chars and spans:
        flush(spans[-1][1])
    return words


def _decode_batch(model, audio: torch.Tensor, decoder: CTCDecoder, timestamps: bool,
                  beam_width: int = 1, lengths: Optional[List[int]] = None) -> List[Tuple[str, Optional[List[Dict]]]]:
    """(b, S) device audio -> [(text, words or None)] through the device pipeline.  lengths:
    per-clip sample counts when the clips were zero-padded to S."""
    with torch.no_grad():
        mel = mel_on_device(audio, n_mels=model.config.mel_bins, lengths=lengths,
                            frame_pad=model.temporal_binding.conv_padding())
        frames = None if lengths is None else [n // HOP_LENGTH + 1 for n in lengths]
        if beam_width > 1:
            logits = model(mel, frames=frames)
            if frames is None:
                return [(t, None) for t in decoder.decode_beam_search(logits, beam_width=beam_width)]
            return [(decoder.decode_beam_search(logits[b:b + 1, :model.get_output_length(f)],
                                                beam_width=beam_width)[0], None) for b, f in enumerate(frames)]
        # greedy: the CTC head's GEMM reduces each frame to its argmax (no logits in HBM)
        rows = None
        if frames is not None:
            rows = torch.tensor([model.get_output_length(f) for f in frames], dtype=torch.int32).to(audio.device)
        toks, lens, st, en = ops.ctc_collapse(model.token_ids(mel, frames=frames), decoder.blank_token, True,
                                              timestamps, frames=rows)
    toks, lens = toks.cpu().numpy(), lens.cpu().numpy()
    if timestamps:
        st, en = st.cpu().numpy(), en.cpu().numpy()
    out = []
    for b in range(toks.shape[0]):
        n = int(lens[b])
        ids = toks[b, :n].tolist()
        if timestamps:
            words = group_words(ids, list(zip(st[b, :n].tolist(), en[b, :n].tolist())), decoder.vocabulary)
            out.append((" ".join(w["word"] for w in words), words))
        else:
            out.append((decoder._tokens_to_text(ids), None))
    return out


def _batches(items: List[Tuple[int, torch.Tensor]], batch_size: int, ragged: bool):
    """Consecutive batches of the length-sorted items: up to batch_size clips each, zero-padded
    to the longest when the front end takes per-clip lengths (ragged), else runs of clips of
    one sample count (the per-length kernels need the FFT front end with n_mels <= 85)."""
    k = 0
    while k < len(items):
        end = min(k + batch_size, len(items))
        if not ragged:
            n = items[k][1].numel()
            end = k + 1
            while end < len(items) and end - k < batch_size and items[end][1].numel() == n:
                end += 1
        yield items[k:end]
        k = end


def transcribe_files(model, paths: Iterable, decoder: CTCDecoder, device, timestamps: bool = False,
                     batch_size: int = 16, beam_width: int = 1) -> List[Dict]:
    """Transcribe audio files; returns one result dict per file in input order.

    A result is {"file", "duration", "transcription"} (+ "words" with timestamps), as the
    reference's transcribe_file returns; a file that fails gets {"file", "error"} instead,
    so callers can log it the way the reference's per-file try/except does.
    """
    paths = [str(p) for p in paths]
    results: List[Optional[Dict]] = [None] * len(paths)
    items: List[Tuple[int, torch.Tensor]] = []
    for i, p in enumerate(paths):
        try:
            a = load_audio(p)
            if a.dim() != 1 or a.numel() < 2:
                raise ValueError(f"expected a mono clip of at least 2 samples, got shape {tuple(a.shape)}")
            if a.numel() <= N_FFT // 2:  # the reference's reflect padding rejects it too
                raise RuntimeError(f"compute_mel_spectrogram: reflect padding of {N_FFT // 2} needs more than "
                                   f"{N_FFT // 2} samples, got {a.numel()}")
            items.append((i, a))
        except Exception as e:  # reported per file, like the reference's loop
            results[i] = {"file": p, "error": str(e)}
    dev = torch.device(device)
    items.sort(key=lambda it: it[1].numel())  # neighbours of similar length: little padding
    for chunk in _batches(items, max(1, batch_size), ragged_supported(model.config.mel_bins)):
        try:
            ns = [a.numel() for _, a in chunk]
            S = max(ns)
            audio = torch.zeros((len(chunk), S), dtype=torch.float32)
            for j, (_, a) in enumerate(chunk):
                audio[j, :ns[j]] = a.to(torch.float32)
            decoded = _decode_batch(model, audio.to(dev), decoder, timestamps, beam_width,
                                    lengths=None if min(ns) == S else ns)
            for (i, _), n, (text, words) in zip(chunk, ns, decoded):
                r = {"file": paths[i], "duration": n / SAMPLE_RATE, "transcription": text}
                if timestamps:
                    r["words"] = words
                results[i] = r
        except Exception as e:
            for i, _ in chunk:
                results[i] = {"file": paths[i], "error": str(e)}
    return results  # type: ignore[return-value]


def load_manifest(path: str) -> List[Tuple[str, str]]:
    """Test-set manifest: one `audio_path<TAB>reference text` per line (relative paths are
    resolved against the manifest's directory). The reference's load_test_data is a stub
    that returns [] (scripts/evaluate.py:41-57); a manifest file is the local equivalent."""
    p = Path(path)
    if not p.is_file():
        logger.warning(f"Dataset loading not implemented for '{path}'. Pass a TSV manifest file.")
        return []
    out = []
    for line in p.read_text(encoding="utf-8").splitlines():
        if not line.strip():
            continue
        audio, _, ref = line.partition("\t")
        a = Path(audio)
        out.append((str(a if a.is_absolute() else p.parent / a), ref))
    return out
