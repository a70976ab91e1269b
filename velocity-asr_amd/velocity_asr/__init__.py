"""VELOCITY-ASR v2 inference on AMD Instinct MI355X (gfx950).

Drop-in replacement for the reference ``velocity_asr`` package (same public names as its
``__init__.py:95-145``): put ``velocity-asr_amd/`` first on ``PYTHONPATH`` and
``scripts/transcribe.py`` / ``scripts/evaluate.py`` run unchanged.  All compute on the
inference path runs in hand-written HIP kernels (``libvasr_hip.so``, C ABI in
``include/vasr.h``); there is no CPU execution path.

Example:
    >>> from velocity_asr import VELOCITYASR, compute_mel_spectrogram, ctc_greedy_decode
    >>> model = VELOCITYASR().cuda().eval()
    >>> mel = compute_mel_spectrogram(audio.cuda())
    >>> tokens = ctc_greedy_decode(model(mel.unsqueeze(0)))
"""

__version__ = "2.0.0"
__author__ = "VELOCITY Research Team"

from .model import (
    VELOCITYASR,
    VelocityASRConfig,
    TemporalBindingLayer,
    CTCOutputHead,
)

from .ssm import (
    SelectiveSSM,
    SSMBlock,
    LocalSSMProcessor,
    GlobalSSM,
    ScanMode,
    MAMBA_AVAILABLE,
)

from .attention import (
    HierarchicalGlobalContext,
    AdaptivePool,
    MultiHeadAttention,
    GatedFusion,
)

from .audio import (
    load_audio,
    compute_mel_spectrogram,
    MelSpectrogramTransform,
    audio_to_frames,
    frames_to_audio,
    pad_or_trim,
    SAMPLE_RATE,
    N_FFT,
    HOP_LENGTH,
    N_MELS,
)

from .decode import (
    ctc_greedy_decode,
    ctc_greedy_decode_with_timestamps,
    ctc_beam_search,
    CTCDecoder,
    DecodingResult,
    create_default_vocabulary,
)

from .data import (
    ASRDataset,
    ASRCollator,
    LibriSpeechDataset,
    create_dataloader,
    create_librispeech_dataloaders,
)


def from_pretrained(model_name_or_path: str, **kwargs) -> VELOCITYASR:
    """Load a VELOCITY-ASR checkpoint (reference __init__.py:81-92)."""
    return VELOCITYASR.from_pretrained(model_name_or_path, **kwargs)


__all__ = [
    "__version__",
    "__author__",
    "VELOCITYASR",
    "VelocityASRConfig",
    "from_pretrained",
    "TemporalBindingLayer",
    "CTCOutputHead",
    "SelectiveSSM",
    "SSMBlock",
    "LocalSSMProcessor",
    "GlobalSSM",
    "ScanMode",
    "MAMBA_AVAILABLE",
    "HierarchicalGlobalContext",
    "AdaptivePool",
    "MultiHeadAttention",
    "GatedFusion",
    "load_audio",
    "compute_mel_spectrogram",
    "MelSpectrogramTransform",
    "audio_to_frames",
    "frames_to_audio",
    "pad_or_trim",
    "SAMPLE_RATE",
    "N_FFT",
    "HOP_LENGTH",
    "N_MELS",
    "ctc_greedy_decode",
    "ctc_greedy_decode_with_timestamps",
    "ctc_beam_search",
    "CTCDecoder",
    "DecodingResult",
    "create_default_vocabulary",
    "ASRDataset",
    "ASRCollator",
    "LibriSpeechDataset",
    "create_dataloader",
    "create_librispeech_dataloaders",
]
