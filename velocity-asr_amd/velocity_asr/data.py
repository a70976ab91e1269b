"""Training-data loaders (reference velocity_asr/data.py) — outside this build's scope.

SURVEY §2 row 9: manifest/LibriSpeech datasets feed training, which this inference-only
MI355X build does not implement (LibriSpeech also needs network access and torchaudio).
The names are kept so ``import velocity_asr`` exposes the reference's ``__all__``; using
them raises NotImplementedError with that explanation.
"""

from __future__ import annotations

_MSG = ("velocity_asr (MI355X inference build): training data loading is out of scope; "
        "see SURVEY.md §2 row 9")


class ASRDataset:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(_MSG)


class ASRCollator:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(_MSG)


class LibriSpeechDataset:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(_MSG)


def create_dataloader(*args, **kwargs):
    raise NotImplementedError(_MSG)


def create_librispeech_dataloaders(*args, **kwargs):
    raise NotImplementedError(_MSG)
