"""ctypes binding of libvasr_hip.so (the C ABI declared in include/vasr.h).

The library is loaded lazily on the first kernel call, after torch, so the HIP runtime
it links against (SONAME libamdhip64.so.7) resolves to the one torch already loaded and
both share streams and device allocations.  There is no CPU fallback: if the library is
missing or no HIP device is visible, every op raises.
"""

from __future__ import annotations

import ctypes
import os
import re
from typing import Optional

import torch

ABI_VERSION = 19
_HERE = os.path.dirname(os.path.abspath(__file__))
# VASR_LIB overrides the library path (diagnostic builds of the same sources, tools/).
LIB_PATH = os.environ.get("VASR_LIB") or os.path.join(_HERE, "lib", "libvasr_hip.so")
HEADER_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "include", "vasr.h"))

(EPI_NONE, EPI_GELU, EPI_SOFTPLUS_FROM, EPI_RESIDUAL, EPI_GELU_PE, EPI_PAIR_POWER, EPI_PAIR_FUSION,
 EPI_ARGMAX) = range(8)
OPT_SCAN_LANES, OPT_SCAN_CHUNK, OPT_TAIL_ROWS, OPT_GEMM_ENGINE, OPT_TAIL_WAVES, OPT_SCAN_SPLIT, OPT_DW_ROWS = range(7)  # enum vasr_option

c_i32, c_i64, c_f32, c_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p


class GemmArgs(ctypes.Structure):
    """Mirror of struct vasr_gemm_args (include/vasr.h)."""

    _fields_ = [
        ("A", c_p), ("lda", c_i64), ("stride_a", c_i64),
        ("W", c_p), ("ldw", c_i64),
        ("bias", c_p),
        ("C", c_p), ("ldc", c_i64), ("stride_c", c_i64),
        ("batch", c_i32), ("M", c_i32), ("N", c_i32), ("K", c_i32),
        ("epilogue", c_i32),
        ("aux", c_p), ("ld_aux", c_i64), ("stride_aux", c_i64),
        ("aux2", c_p),
        ("n_out", c_i32),
        ("qparams", c_p),
    ]


_SIGNATURES = {
    "vasr_version": ([], ctypes.c_int),
    "vasr_set_option": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "vasr_probe_clock": ([c_p, ctypes.c_int, ctypes.c_int, c_p], ctypes.c_int),
    "vasr_last_error": ([], ctypes.c_char_p),
    "vasr_linear_x3_f32": ([ctypes.POINTER(GemmArgs), c_p, c_p], ctypes.c_int),
    "vasr_split_weights_bf16x3": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p], ctypes.c_int),
    "vasr_split_weights_elems": ([ctypes.c_int, ctypes.c_int], c_i64),
    "vasr_linear_bf16": ([ctypes.POINTER(GemmArgs), c_p, c_p], ctypes.c_int),
    "vasr_pack_weights_bf16": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p], ctypes.c_int),
    "vasr_pack_weights_bf16_elems": ([ctypes.c_int, ctypes.c_int], c_i64),
    "vasr_layer_norm_f32": ([c_p, c_i64, c_p, c_p, c_p, c_i64, ctypes.c_int, ctypes.c_int, c_f32, c_p], ctypes.c_int),
    "vasr_layer_norm_pair_f32": ([c_p, c_i64, c_p, c_p, c_f32, c_p, c_i64, c_p, c_p, c_f32, c_p, c_i64, ctypes.c_int,
                                  ctypes.c_int, c_p], ctypes.c_int),
    "vasr_add_table_f32": ([c_p, c_p, c_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_p], ctypes.c_int),
    "vasr_ln_dwconv_prenorm_f32": ([c_p, c_p, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_p] + [ctypes.c_int] * 4
                                   + [c_f32, c_p], ctypes.c_int),
    "vasr_ln_dwconv_f32": ([c_p, c_p, c_p, c_p, c_p, c_p] + [ctypes.c_int] * 4 + [c_f32, c_p], ctypes.c_int),
    "vasr_ssm_scan_f32": ([c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5 + [c_p],
                          ctypes.c_int),
    "vasr_ssm_scan_chunked_f32": ([c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5
                                  + [c_p, c_i64, c_p], ctypes.c_int),
    "vasr_ssm_scan_ungated_f32": ([c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5 + [c_p],
                                  ctypes.c_int),
    "vasr_ssm_scan_workspace_floats": ([ctypes.c_int] * 4, c_i64),
    "vasr_ssm_scan_split_selected": ([ctypes.c_int] * 4, ctypes.c_int),
    "vasr_ssm_block_tail_f32": ([c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64]
                                + [ctypes.c_int] * 3 + [c_p], ctypes.c_int),
    "vasr_ssm_block_tail_gated_f32": ([c_p, c_i64, c_p, c_i64, c_p, ctypes.c_int, c_p, c_i64, c_p, c_p, c_p, c_f32, c_p,
                                       c_p, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 3 + [c_p], ctypes.c_int),
    "vasr_ssm_block_tail_gated_bf16": ([c_p, c_i64, c_p, c_i64, c_p, ctypes.c_int, c_p, c_i64, c_p, c_p, c_p, c_f32, c_p,
                                        c_p, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 3 + [c_p], ctypes.c_int),
    "vasr_ssm_block_tail_bf16": ([c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_f32, c_p, c_p, c_p, c_p, c_p, c_i64]
                                 + [ctypes.c_int] * 3 + [c_p], ctypes.c_int),
    "vasr_pack_weights16_bf16": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p], ctypes.c_int),
    "vasr_pack_weights16_bf16_elems": ([ctypes.c_int, ctypes.c_int], c_i64),
    "vasr_split_weights16_bf16x3": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p], ctypes.c_int),
    "vasr_split_weights16_elems": ([ctypes.c_int, ctypes.c_int], c_i64),
    "vasr_flac_decode": ([c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p], ctypes.c_int),
    "vasr_resample_length": ([c_i64, ctypes.c_int, ctypes.c_int], c_i64),
    "vasr_resample_f32": ([c_p, ctypes.c_int, c_i64, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_i64], ctypes.c_int),
    "vasr_reflect_pad_f32": ([c_p, c_i64, c_p, c_i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_p], ctypes.c_int),
    "vasr_mel_log_norm_f32": ([c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5 + [c_p, c_p],
                              ctypes.c_int),
    "vasr_mel_workspace_floats": ([ctypes.c_int] * 3, c_i64),
    "vasr_stft_power_400_f32": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p, c_i64, c_i64, c_p], ctypes.c_int),
    "vasr_stft_power_400_var_f32": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p, c_p, c_i64, c_i64, c_p],
                                    ctypes.c_int),
    "vasr_mel_log_norm_var_f32": ([c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_i64] + [ctypes.c_int] * 5 + [c_p, c_p, c_p],
                                  ctypes.c_int),
    "vasr_adaptive_pool_var_f32": ([c_p, c_p] + [ctypes.c_int] * 4 + [c_p, c_p, c_p], ctypes.c_int),
    "vasr_pooled_attention_var_f32": ([c_p, c_i64, c_p, c_p] + [ctypes.c_int] * 5 + [c_p, c_p], ctypes.c_int),
    "vasr_ctc_collapse_var": ([c_p, ctypes.c_int, ctypes.c_int, c_p, ctypes.c_int, ctypes.c_int, c_p, c_p, c_p, c_p,
                               c_p], ctypes.c_int),
    "vasr_pad_frames_f32": ([c_p, c_p] + [ctypes.c_int] * 5 + [c_p], ctypes.c_int),
    "vasr_ln_adaptive_pool_f32": ([c_p, c_p, c_p, c_f32, c_p] + [ctypes.c_int] * 4 + [c_p, c_p, c_p], ctypes.c_int),
    "vasr_adaptive_pool_f32": ([c_p, c_p] + [ctypes.c_int] * 4 + [c_p], ctypes.c_int),
    "vasr_pooled_attention_f32": ([c_p, c_i64, c_p, c_p] + [ctypes.c_int] * 5 + [c_p], ctypes.c_int),
    "vasr_argmax_f32": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p], ctypes.c_int),
    "vasr_fakequant_f32": ([c_p, c_i64, c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p, ctypes.c_int, c_f32, c_f32,
                            c_p], ctypes.c_int),
    "vasr_minmax_f32": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p, c_p], ctypes.c_int),
    "vasr_argmax_keys": ([c_p, c_i64, ctypes.c_int, ctypes.c_int, c_p, c_p], ctypes.c_int),
    "vasr_ctc_collapse_keys": ([c_p, c_i64] + [ctypes.c_int] * 3 + [c_p, ctypes.c_int, ctypes.c_int] + [c_p] * 6,
                               ctypes.c_int),
    "vasr_ctc_beam_search": ([c_p, c_i64, c_i64] + [ctypes.c_int] * 5 + [c_p] * 5 + [c_p], ctypes.c_int),
    "vasr_ctc_beam_workspace_elems": ([ctypes.c_int, ctypes.c_int], c_i64),
    "vasr_ctc_collapse": ([c_p] + [ctypes.c_int] * 4 + [c_p, c_p, c_p, c_p, c_p], ctypes.c_int),
}

_lib: Optional[ctypes.CDLL] = None


def header_functions(path: str = HEADER_PATH):
    """Names of every function the C ABI header declares."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vasr_\w+)\s*\(", text)))


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the library.  Raises RuntimeError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"velocity_asr: HIP kernel library not built ({path}). Build it with "
            "`make -C velocity-asr_amd` or `python -c 'import __graft_entry__ as g; g.build()'`.")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (args, res) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.vasr_version() != ABI_VERSION:
        raise RuntimeError(f"libvasr_hip.so ABI {lib.vasr_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def lib() -> ctypes.CDLL:
    return load()


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().vasr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def require_device() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError(
            "velocity_asr (MI355X build) needs a HIP device: no GPU is visible. "
            "There is no CPU execution path.")


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()
