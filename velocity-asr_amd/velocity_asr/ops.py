"""Thin tensor-level wrappers over the HIP kernels of libvasr_hip.so.

Each wrapper validates device / dtype / layout on the host (raising ValueError or
RuntimeError like torch would), allocates its output with the torch caching allocator
and enqueues the kernel on the current HIP stream.  Nothing here computes on the CPU.
"""

from __future__ import annotations

import math
import os
import weakref
from typing import Optional, Tuple

import torch

from . import _lib as L
from ._lib import GemmArgs, check, ptr, stream_of

LOG2E = 1.4426950408889634

# Optional per-launch timing (bench.py roofline): while `_timing` is a dict, every launch of
# a timed op records a (start, end, info) triple of HIP events on the launch stream.
_timing = None


class kernel_timer:
    """Context manager: record HIP events around every launch of the named ops."""

    def __init__(self, *names):
        self.names = set(names)
        self.records = {n: [] for n in names}

    def __enter__(self):
        global _timing
        _timing = self
        return self

    def __exit__(self, *exc):
        global _timing
        _timing = None
        return False

    def summary(self):
        torch.cuda.synchronize()
        return {n: [(s.elapsed_time(e) * 1e-3, info) for s, e, info in recs] for n, recs in self.records.items()}


def _t0(name):
    if _timing is not None and name in _timing.names:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev
    return None


def _t1(name, start, info):
    if start is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        _timing.records[name].append((start, ev, info))


def _cuda_f32(name: str, t: torch.Tensor) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{name}: tensor is on {t.device}; velocity_asr (MI355X build) runs on HIP devices only")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")


def _cuda_w(name: str, t: torch.Tensor) -> None:
    """GEMM weights: float32 (fp32 GEMM) or bfloat16 (bf16 model, vasr_linear_bf16)."""
    if isinstance(t, torch.Tensor) and t.dtype == torch.bfloat16 and t.device.type == "cuda":
        return
    _cuda_f32(name, t)


def _dropper(cache: dict, key: int):
    """Weakref callback that drops `key` from `cache`.  The dict is bound into the closure (not
    looked up as a module global): at interpreter exit the module's globals are cleared before
    the last tensors die, and a global lookup then raised inside the callback."""
    def drop(_ref, cache=cache, key=key):
        cache.pop(key, None)
    return drop


# fp32 copies of bf16 parameters for the kernels that take fp32 operands (norm weights, biases,
# conv taps, D, tables): built once per (tensor, version), dropped with the tensor.
_f32_copies = {}


def f32(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """t itself if float32 (or None), else a cached float32 copy (bf16 models)."""
    if t is None or t.dtype == torch.float32:
        return t
    sig = (t.data_ptr(), t._version, tuple(t.shape), tuple(t.stride()))
    ent = _f32_copies.get(id(t))
    if ent is not None and ent[0]() is t and ent[1] == sig:
        return ent[2]
    with torch.no_grad():
        c = t.detach().float().contiguous()
    key = id(t)
    _f32_copies[key] = (weakref.ref(t, _dropper(_f32_copies, key)), sig, c)
    return c


def _rows(name: str, t: torch.Tensor) -> Tuple[int, int, int]:
    """(rows, cols, row_stride) of a 2-D row-major view with unit column stride."""
    if t.dim() != 2:
        raise ValueError(f"{name}: expected a 2-D view, got shape {tuple(t.shape)}")
    if t.stride(1) != 1 and t.shape[1] > 1:
        raise ValueError(f"{name}: columns must be contiguous")
    return t.shape[0], t.shape[1], t.stride(0) if t.shape[0] > 1 else max(t.shape[1], 1)


class option:
    """Set a launcher tuning option (vasr_set_option; enum vasr_option in include/vasr.h) for the
    duration of a with-block, e.g. ``with ops.option(L.OPT_SCAN_CHUNK, 16): ...``.  Options
    change work decomposition only, never the computed values."""

    def __init__(self, key: int, value: int):
        self.key, self.value = key, value

    def __enter__(self):
        prev = L.lib().vasr_set_option(self.key, self.value)
        check(min(prev, 0), "vasr_set_option")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        L.lib().vasr_set_option(self.key, self.prev)
        return False


# Split-bf16 planes of weight matrices, built once per (tensor, version) and dropped with the
# tensor.  Keys are tensor identities: the model passes parameters or cached derived weights.
_splits = {}


def split_weights(w: torch.Tensor) -> torch.Tensor:
    """[3][N][Kp] bf16 planes (as int16 storage) of a (N, K) fp32 weight view."""
    N, K, ldw = _rows("split.w", w)
    sig = (w.data_ptr(), w._version, N, K, ldw)
    ent = _splits.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == sig:
        return ent[2]
    planes = torch.empty(int(L.lib().vasr_split_weights_elems(N, K)), device=w.device, dtype=torch.int16)
    check(L.lib().vasr_split_weights_bf16x3(w.data_ptr(), ldw, N, K, planes.data_ptr(), stream_of(w)),
          "vasr_split_weights_bf16x3")
    key = id(w)
    _splits[key] = (weakref.ref(w, _dropper(_splits, key)), sig, planes)
    return planes


_splits16 = {}


def split_weights16(w: torch.Tensor) -> torch.Tensor:
    """Split-bf16 planes of a (N, K) fp32 weight in the v_mfma_f32_16x16x32_bf16 fragment
    layout (the fused SSMBlock tail), built once per (tensor, version)."""
    N, K, ldw = _rows("split16.w", w)
    sig = (w.data_ptr(), w._version, N, K, ldw)
    ent = _splits16.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == sig:
        return ent[2]
    planes = torch.empty(int(L.lib().vasr_split_weights16_elems(N, K)), device=w.device, dtype=torch.int16)
    check(L.lib().vasr_split_weights16_bf16x3(w.data_ptr(), ldw, N, K, planes.data_ptr(), stream_of(w)),
          "vasr_split_weights16_bf16x3")
    key = id(w)
    _splits16[key] = (weakref.ref(w, _dropper(_splits16, key)), sig, planes)
    return planes


def pack_weights16(w: torch.Tensor) -> torch.Tensor:
    """One bf16 plane of a (N, K) bf16 weight in the v_mfma_f32_16x16x32_bf16 fragment layout
    (the bf16 model's fused SSMBlock tail), built once per (tensor, version)."""
    N, K, ldw = _rows("pack16.w", w)
    sig = (w.data_ptr(), w._version, N, K, ldw)
    ent = _splits16.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == sig:
        return ent[2]
    packed = torch.empty(int(L.lib().vasr_pack_weights16_bf16_elems(N, K)), device=w.device, dtype=torch.int16)
    check(L.lib().vasr_pack_weights16_bf16(w.data_ptr(), ldw, N, K, packed.data_ptr(), stream_of(w)),
          "vasr_pack_weights16_bf16")
    key = id(w)
    _splits16[key] = (weakref.ref(w, _dropper(_splits16, key)), sig, packed)
    return packed


def ssm_block_tail(g: torch.Tensor, x: torch.Tensor, wo: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor,
                   ln_eps: float, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused SSMBlock tail (vasr_ssm_block_tail_f32, or _bf16 for bf16 weights): out =
    ffn(LN2(g Wo^T + x)) + (g Wo^T + x) for g (M, 384) and x (M, 192) row views (d_model 192,
    FFN width 384)."""
    bf16 = wo.dtype == torch.bfloat16
    if bf16:
        if not (w1.dtype == w2.dtype == torch.bfloat16):
            raise TypeError("ssm_block_tail: mixed weight dtypes")
        ln_w, ln_b, b1, b2 = f32(ln_w), f32(ln_b), f32(b1), f32(b2)
    for n, t in (("g", g), ("x", x), ("ln_w", ln_w), ("ln_b", ln_b), ("b1", b1), ("b2", b2)) + (
            () if bf16 else (("wo", wo), ("w1", w1), ("w2", w2))):
        _cuda_f32(f"ssm_block_tail.{n}", t)
    M, E, ldg = _rows("ssm_block_tail.g", g)
    Mx, D, ldx = _rows("ssm_block_tail.x", x)
    if Mx != M or tuple(wo.shape) != (D, E) or tuple(w1.shape) != (E, D) or tuple(w2.shape) != (D, E):
        raise ValueError("ssm_block_tail: inconsistent shapes")
    if out is None:
        out = torch.empty((M, D), device=g.device, dtype=torch.float32)
    _, _, ldo = _rows("ssm_block_tail.out", out)
    prep = pack_weights16 if bf16 else split_weights16
    fn = "vasr_ssm_block_tail_bf16" if bf16 else "vasr_ssm_block_tail_f32"
    ev = _t0("ssm_tail")
    check(getattr(L.lib(), fn)(g.data_ptr(), ldg, x.data_ptr(), ldx, prep(wo).data_ptr(), ln_w.contiguous().data_ptr(),
                               ln_b.contiguous().data_ptr(), float(ln_eps), prep(w1).data_ptr(),
                               b1.contiguous().data_ptr(), prep(w2).data_ptr(), b2.contiguous().data_ptr(),
                               out.data_ptr(), ldo, M, D, E, stream_of(g)), fn)
    _t1("ssm_tail", ev, dict(M=M, D=D, E=E))
    return out


def pack_bf16(w: torch.Tensor) -> torch.Tensor:
    """One fragment-native bf16 plane (as int16 storage) of a (N, K) bf16 weight view."""
    N, K, ldw = _rows("pack.w", w)
    sig = (w.data_ptr(), w._version, N, K, ldw)
    ent = _splits.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == sig:
        return ent[2]
    packed = torch.empty(int(L.lib().vasr_pack_weights_bf16_elems(N, K)), device=w.device, dtype=torch.int16)
    check(L.lib().vasr_pack_weights_bf16(w.data_ptr(), ldw, N, K, packed.data_ptr(), stream_of(w)),
          "vasr_pack_weights_bf16")
    key = id(w)
    _splits[key] = (weakref.ref(w, _dropper(_splits, key)), sig, packed)
    return packed


def _linear(args: GemmArgs, w: torch.Tensor, stream) -> None:
    if w.dtype == torch.bfloat16:
        check(L.lib().vasr_linear_bf16(args, pack_bf16(w).data_ptr(), stream), "vasr_linear_bf16")
    else:
        check(L.lib().vasr_linear_x3_f32(args, split_weights(w).data_ptr(), stream), "vasr_linear_x3_f32")


def _ln_prologue(a: torch.Tensor, ln) -> torch.Tensor:
    """Row LayerNorm of `a` (vasr_layer_norm_f32) when ln = (weight, bias, eps) is given: the
    LayerNorm feeding a Linear (SSMBlock norm2 -> FFN, the CTC head).  Returns the A the GEMM
    reads.  (Fusing it into the GEMM's A read was bit-identical but slower end to end, 99.5k vs
    102.5k RTFx; removed in r03)"""
    if ln is None:
        return a
    ln_w, ln_b, eps = ln
    return layer_norm(a, f32(ln_w), f32(ln_b), eps)


def _qp(qparams: Optional[torch.Tensor], cols: int) -> Optional[int]:
    if qparams is None:
        return None
    _cuda_f32("gemm.qparams", qparams)
    if not qparams.is_contiguous() or tuple(qparams.shape) != (cols, 4):
        raise ValueError(f"gemm: qparams must be a contiguous ({cols}, 4) tensor, got {tuple(qparams.shape)}")
    return qparams.data_ptr()


def gemm(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, epilogue: int = L.EPI_NONE,
         out: Optional[torch.Tensor] = None, aux: Optional[torch.Tensor] = None,
         aux2: Optional[torch.Tensor] = None, n_out: int = 0, n_cols_out: Optional[int] = None,
         qparams: Optional[torch.Tensor] = None, ln=None) -> torch.Tensor:
    """out = epilogue(fq(a @ w.T + bias)) for a (M, K) row view and w (N, K); fq is the
    per-column activation fake-quant of `qparams` ((ncols, 4) {scale, zp, qmin, qmax}) if given.
    ln = (weight, bias, eps): LayerNorm each row of `a` first."""
    _cuda_f32("gemm.a", a)
    args = GemmArgs()
    a = _ln_prologue(a, ln)
    _cuda_w("gemm.w", w)
    bias, aux, aux2 = f32(bias), f32(aux), f32(aux2)
    M, K, lda = _rows("gemm.a", a)
    N, Kw, ldw = _rows("gemm.w", w)
    if Kw != K:
        raise ValueError(f"gemm: a has K={K} but w has K={Kw}")
    cols = n_cols_out if n_cols_out is not None else (n_out if epilogue in (L.EPI_PAIR_POWER, L.EPI_PAIR_FUSION) else N)
    if out is None:
        out = torch.empty((M, cols), device=a.device, dtype=torch.float32)
    _, _, ldc = _rows("gemm.out", out)
    args.A, args.lda, args.stride_a = a.data_ptr(), lda, 0
    args.W, args.ldw = w.data_ptr(), ldw
    args.bias = ptr(bias)
    args.C, args.ldc, args.stride_c = out.data_ptr(), ldc, 0
    args.batch, args.M, args.N, args.K = 1, M, N, K
    args.epilogue = epilogue
    if aux is not None:
        _, _, ld_aux = _rows("gemm.aux", aux)
        args.aux, args.ld_aux, args.stride_aux = aux.data_ptr(), ld_aux, 0
    args.aux2 = ptr(aux2)
    args.n_out = n_out
    args.qparams = _qp(qparams, N + (n_out if epilogue == L.EPI_PAIR_FUSION else 0))
    ev = _t0("gemm")
    _linear(args, w, stream_of(a))
    _t1("gemm", ev, dict(M=M, N=N, K=K, batch=1))
    return out


def _gemm_argmax_keys(a: torch.Tensor, w: torch.Tensor, bias, qparams, ln, who: str):
    """The VASR_EPI_ARGMAX GEMM: (M, ceil(N/32)) uint64 partial keys of a @ w.T + bias per row."""
    _cuda_f32(f"{who}.a", a)
    args = GemmArgs()
    a = _ln_prologue(a, ln)
    _cuda_w(f"{who}.w", w)
    bias = f32(bias)
    M, K, lda = _rows(f"{who}.a", a)
    N, Kw, ldw = _rows(f"{who}.w", w)
    if Kw != K:
        raise ValueError(f"{who}: a has K={K} but w has K={Kw}")
    slots = (N + 31) // 32
    keys = torch.empty((M, slots), device=a.device, dtype=torch.int64)  # every slot is written
    args.A, args.lda, args.stride_a = a.data_ptr(), lda, 0
    args.W, args.ldw = w.data_ptr(), ldw
    args.bias = ptr(bias)
    args.C, args.ldc, args.stride_c = keys.data_ptr(), slots, 0
    args.batch, args.M, args.N, args.K = 1, M, N, K
    args.epilogue = L.EPI_ARGMAX
    args.qparams = _qp(qparams, N)
    ev = _t0("gemm")
    _linear(args, w, stream_of(a))
    _t1("gemm", ev, dict(M=M, N=N, K=K, batch=1))
    return keys, slots, M


def gemm_argmax(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *,
                qparams: Optional[torch.Tensor] = None, ln=None) -> torch.Tensor:
    """int32 argmax over the N outputs of a @ w.T + bias (after qparams) per row, fused into the
    GEMM epilogue (VASR_EPI_ARGMAX): the (M, N) product is never written.  Ties -> first index.
    ln = (weight, bias, eps): LayerNorm each row of `a` first."""
    keys, slots, M = _gemm_argmax_keys(a, w, bias, qparams, ln, "gemm_argmax")
    out = torch.empty(M, device=a.device, dtype=torch.int32)
    check(L.lib().vasr_argmax_keys(keys.data_ptr(), slots, slots, M, out.data_ptr(), stream_of(keys)), "vasr_argmax_keys")
    return out


def gemm_ctc_greedy(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], B: int, blank: int = 0, *,
                    qparams: Optional[torch.Tensor] = None, ln=None, collapse: bool = True, timestamps: bool = False,
                    out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, frames: Optional[torch.Tensor] = None):
    """Greedy CTC decode of B utterances (a: B * L rows) straight from the argmax GEMM's keys:
    argmax + collapse in one launch (vasr_ctc_collapse_keys); same results as gemm_argmax then
    ctc_collapse.  Returns (tokens, lengths, start, end) as ctc_collapse."""
    keys, slots, M = _gemm_argmax_keys(a, w, bias, qparams, ln, "gemm_ctc_greedy")
    if B <= 0 or M % B:
        raise ValueError(f"gemm_ctc_greedy: {M} rows do not split into B={B} utterances")
    Lq = M // B
    toks, lens, st, en, frames = _collapse_outputs("gemm_ctc_greedy", B, Lq, keys.device, out, timestamps, frames)
    check(L.lib().vasr_ctc_collapse_keys(keys.data_ptr(), slots, slots, B, Lq, ptr(frames), int(blank), int(collapse),
                                         None, toks.data_ptr(), lens.data_ptr(), ptr(st), ptr(en), stream_of(keys)),
          "vasr_ctc_collapse_keys")
    return toks, lens, st, en


def gemm_batched(a_base: torch.Tensor, lda: int, stride_a: int, rows: int, batch: int, K: int, w: torch.Tensor,
                 bias: Optional[torch.Tensor], out: torch.Tensor, ldc: int, stride_c: int, *,
                 epilogue: int = L.EPI_NONE, aux: Optional[torch.Tensor] = None, ld_aux: int = 0,
                 stride_aux: int = 0, n_out: int = 0, qparams: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Strided batched form: A[b] rows at a_base + b*stride_a + m*lda (overlapping rows allowed)."""
    _cuda_f32("gemm_batched.a", a_base)
    _cuda_w("gemm_batched.w", w)
    bias, aux = f32(bias), f32(aux)
    need = (batch - 1) * stride_a + (rows - 1) * lda + K
    avail = a_base.untyped_storage().nbytes() // 4 - a_base.storage_offset()
    if rows > 0 and batch > 0 and need > avail:
        raise ValueError(f"gemm_batched: A view needs {need} elements, {avail} available")
    N, Kw, ldw = _rows("gemm_batched.w", w)
    if Kw != K:
        raise ValueError("gemm_batched: K mismatch")
    args = GemmArgs()
    args.A, args.lda, args.stride_a = a_base.data_ptr(), lda, stride_a
    args.W, args.ldw = w.data_ptr(), ldw
    args.bias = ptr(bias)
    args.C, args.ldc, args.stride_c = out.data_ptr(), ldc, stride_c
    args.batch, args.M, args.N, args.K = batch, rows, N, K
    args.epilogue = epilogue
    if aux is not None:
        args.aux, args.ld_aux, args.stride_aux = aux.data_ptr(), ld_aux, stride_aux
    args.n_out = n_out
    args.qparams = _qp(qparams, N)
    ev = _t0("gemm")
    _linear(args, w, stream_of(a_base))
    _t1("gemm", ev, dict(M=rows, N=N, K=K, batch=batch))
    return out


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _cuda_f32("layer_norm.x", x)
    w, b = f32(w), f32(b)
    C = x.shape[-1]
    x2 = x.reshape(-1, C)
    rows, _, ldx = _rows("layer_norm.x", x2)
    y = torch.empty((rows, C), device=x.device, dtype=torch.float32) if out is None else out.reshape(-1, C)
    _, _, ldy = _rows("layer_norm.out", y)
    check(L.lib().vasr_layer_norm_f32(x2.data_ptr(), ldx, w.data_ptr(), b.data_ptr(), y.data_ptr(), ldy, rows, C,
                                      float(eps), stream_of(x)), "vasr_layer_norm_f32")
    return y.view(*x.shape[:-1], C) if out is None else out


def layer_norm_pair(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, eps1: float, w2: torch.Tensor,
                    b2: torch.Tensor, eps2: float):
    """(LN1(x), LN2(LN1(x))) in one launch, each bitwise layer_norm's (vasr_layer_norm_pair_f32)."""
    _cuda_f32("layer_norm_pair.x", x)
    w1, b1, w2, b2 = f32(w1), f32(b1), f32(w2), f32(b2)
    C = x.shape[-1]
    x2 = x.reshape(-1, C)
    rows, _, ldx = _rows("layer_norm_pair.x", x2)
    y1 = torch.empty((rows, C), device=x.device, dtype=torch.float32)
    y2 = torch.empty((rows, C), device=x.device, dtype=torch.float32)
    check(L.lib().vasr_layer_norm_pair_f32(x2.data_ptr(), ldx, w1.data_ptr(), b1.data_ptr(), float(eps1),
                                           y1.data_ptr(), C, w2.data_ptr(), b2.data_ptr(), float(eps2),
                                           y2.data_ptr(), C, rows, C, stream_of(x)), "vasr_layer_norm_pair_f32")
    return y1.view(*x.shape[:-1], C), y2.view(*x.shape[:-1], C)


def add_table(x: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    """x (B, L, C) + table (L, C) broadcast over the batch."""
    _cuda_f32("add_table.x", x)
    table = f32(table)
    _cuda_f32("add_table.table", table)
    x = x.contiguous()
    B, Lq, C = x.shape
    if tuple(table.shape) != (Lq, C):
        raise ValueError("add_table: table must be (L, C)")
    out = torch.empty_like(x)
    check(L.lib().vasr_add_table_f32(x.data_ptr(), table.contiguous().data_ptr(), out.data_ptr(), B, Lq, C,
                                     stream_of(x)), "vasr_add_table_f32")
    return out


def ln_dwconv(x: torch.Tensor, ln_w, ln_b, conv_w, conv_b, eps: float = 1e-5) -> torch.Tensor:
    """(B, L, C) -> causal depthwise conv of LayerNorm(x)."""
    _cuda_f32("ln_dwconv.x", x)
    ln_w, ln_b, conv_w, conv_b = f32(ln_w), f32(ln_b), f32(conv_w), f32(conv_b)
    x = x.contiguous()
    B, Lq, C = x.shape
    Kc = conv_w.shape[-1]
    y = torch.empty_like(x)
    check(L.lib().vasr_ln_dwconv_f32(x.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(),
                                     conv_w.contiguous().data_ptr(), conv_b.data_ptr(), y.data_ptr(), B, Lq, C, Kc,
                                     float(eps), stream_of(x)), "vasr_ln_dwconv_f32")
    return y


def ln_dwconv_prenorm(x: torch.Tensor, pre_w, pre_b, pre_eps: float, ln_w, ln_b, conv_w, conv_b,
                      eps: float = 1e-5):
    """(B, L, 192) -> (ln_dwconv(LN0(x)), LN0(x)) without LN0's own launch (vasr_ln_dwconv_prenorm_f32):
    both bitwise layer_norm + ln_dwconv.  Kc = 4 only."""
    _cuda_f32("ln_dwconv_prenorm.x", x)
    pre_w, pre_b = f32(pre_w), f32(pre_b)
    ln_w, ln_b, conv_w, conv_b = f32(ln_w), f32(ln_b), f32(conv_w), f32(conv_b)
    x = x.contiguous()
    B, Lq, C = x.shape
    Kc = conv_w.shape[-1]
    y, xo = torch.empty_like(x), torch.empty_like(x)
    check(L.lib().vasr_ln_dwconv_prenorm_f32(x.data_ptr(), pre_w.data_ptr(), pre_b.data_ptr(), float(pre_eps),
                                             xo.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(),
                                             conv_w.contiguous().data_ptr(), conv_b.data_ptr(), y.data_ptr(), B, Lq, C,
                                             Kc, float(eps), stream_of(x)), "vasr_ln_dwconv_prenorm_f32")
    return y, xo


# Chunk-parallel tree scan (vasr_ssm_scan_chunked_f32, bitwise equal to the streaming kernel)
# for launches under CHUNKED_MAX_WAVES waves of the streaming kernel (B * Di * N / 256 at 4 states
# per lane) over more than CHUNKED_MIN_L steps: one utterance at a time, as the reference's
# scripts feed the model.  Measured (profiles/r03ae/forms.txt, graph-timed): the streaming kernel
# takes ~4.8 + 0.067 L us at these sizes whatever B; the chunked form's three launches win from
# L ~ 150 while the launch is at most 192 waves (B = 1, 10 s: 14.7 vs 37.1 us at N = 32, 18.3 vs
# 37.0 at N = 64) and lose at 384 (B = 4, N = 64: 41.9 vs 39.1) and for short L (the global
# blocks' L = 64 at 10 s: 10.2 vs 6.8 us).
# scan_form("streaming" | "chunked" | None) forces one (default from VASR_SCAN_CHUNKED=0|1).
# Below CHUNKED_MIN_L the chunked entry point still wins where it runs as ONE launch (the
# time-split form: N <= 64, B * Di * N / 128 <= 256 workgroups, L <= 512; the library reports its
# own rule, vasr_ssm_scan_split_selected), e.g. the global blocks' L = 64 at B = 1
# (VASR_SCAN_SPLIT_SHORT=0 turns this off; profiles/r05aq).
CHUNKED_MAX_WAVES = 256
CHUNKED_MIN_L = 160
_SCAN_FORM = {"0": "streaming", "1": "chunked"}.get(os.environ.get("VASR_SCAN_CHUNKED", ""))
_SPLIT_SHORT = os.environ.get("VASR_SCAN_SPLIT_SHORT", "1") != "0"


def scan_form(form: Optional[str]) -> Optional[str]:
    """Force the streaming or chunk-parallel tree scan (None = by launch size); returns the
    previous setting.  Both give bitwise equal outputs."""
    global _SCAN_FORM
    if form not in (None, "streaming", "chunked"):
        raise ValueError(f"scan form {form!r}: expected None, 'streaming' or 'chunked'")
    prev, _SCAN_FORM = _SCAN_FORM, form
    return prev


def _use_chunked(B: int, Lq: int, Di: int, N: int, mode: int) -> bool:
    if mode not in (0, 2) or Lq <= 16:
        return False
    if _SCAN_FORM is not None:
        return _SCAN_FORM == "chunked"
    if _SPLIT_SHORT and _split_form(B, Lq, Di, N):
        return True
    return B * Di * N // 256 < CHUNKED_MAX_WAVES and Lq > CHUNKED_MIN_L


def _split_form(B: int, Lq: int, Di: int, N: int) -> bool:
    """vasr_ssm_scan_chunked_f32 runs this launch as one (the time-split form) under the current
    options: the library's own rule (vasr_ssm_scan_split_selected), not a copy of it."""
    return bool(L.lib().vasr_ssm_scan_split_selected(B, Lq, Di, N))


SCAN_STATE_DIMS = (16, 32, 64, 128)  # the scan kernels' state dims (include/vasr.h)


def scan_state_dim(N: int) -> int:
    """The kernel state dim a state dim N runs as: N itself, or the next size up with the
    padded states zero (they stay 0 and add nothing to y)."""
    for n in SCAN_STATE_DIMS:
        if N <= n:
            return n
    raise NotImplementedError(f"selective scan: state dim {N} > {SCAN_STATE_DIMS[-1]} not supported")


def ssm_scan(xz: torch.Tensor, dt: torch.Tensor, bc: torch.Tensor, A2: torch.Tensor, D: torch.Tensor, B: int,
             Lq: int, mode: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Gated selective scan.  xz (B*L, 2Di) [x|z], dt (B*L, Di), bc (B*L, 2N) [B|C] (row views).
    Small launches of the tree modes take the chunk-parallel form (same results, bitwise).
    A state dim without a kernel instance (scan_state_dim) is zero-padded here, a copy of bc
    (the model avoids it: its projection GEMM writes the padded layout, SelectiveSSM._prepared)."""
    N0 = A2.numel()
    Np = scan_state_dim(N0)
    if Np != N0:
        Bm, Cm = bc[:, :N0], bc[:, N0:2 * N0]
        pad = torch.zeros((bc.shape[0], Np - N0), device=bc.device, dtype=bc.dtype)
        bc = torch.cat([Bm, pad, Cm, pad], 1)
        A2 = torch.cat([A2, torch.zeros(Np - N0, device=A2.device, dtype=A2.dtype)])
    D = f32(D)
    for n, t in (("xz", xz), ("dt", dt), ("bc", bc), ("A2", A2), ("D", D)):
        _cuda_f32(f"ssm_scan.{n}", t)
    M, two_di, ld_xz = _rows("ssm_scan.xz", xz)
    _, Di, ld_dt = _rows("ssm_scan.dt", dt)
    _, two_n, ld_bc = _rows("ssm_scan.bc", bc)
    if M != B * Lq or two_di != 2 * Di or two_n != 2 * A2.numel() or D.numel() != Di:
        raise ValueError("ssm_scan: inconsistent shapes")
    if out is None:
        out = torch.empty((M, Di), device=xz.device, dtype=torch.float32)
    _, _, ld_out = _rows("ssm_scan.out", out)
    N = A2.numel()
    chunked = _use_chunked(B, Lq, Di, N, int(mode))
    ws = None
    if chunked:
        nws = int(L.lib().vasr_ssm_scan_workspace_floats(B, Lq, Di, N))
        ws = torch.empty(nws, device=xz.device, dtype=torch.float32)
    ev = _t0("ssm_scan")
    if chunked:
        check(L.lib().vasr_ssm_scan_chunked_f32(xz.data_ptr(), ld_xz, dt.data_ptr(), ld_dt, bc.data_ptr(), ld_bc,
                                                A2.data_ptr(), D.data_ptr(), out.data_ptr(), ld_out, B, Lq, Di, N,
                                                int(mode), ws.data_ptr(), ws.numel(), stream_of(xz)),
              "vasr_ssm_scan_chunked_f32")
    else:
        check(L.lib().vasr_ssm_scan_f32(xz.data_ptr(), ld_xz, dt.data_ptr(), ld_dt, bc.data_ptr(), ld_bc, A2.data_ptr(),
                                        D.data_ptr(), out.data_ptr(), ld_out, B, Lq, Di, N, int(mode),
                                        stream_of(xz)), "vasr_ssm_scan_f32")
    _t1("ssm_scan", ev, dict(B=B, L=Lq, Di=Di, N=N, mode=int(mode), chunked=chunked))
    return out


def ssm_scan_ungated(x: torch.Tensor, dt: torch.Tensor, bc: torch.Tensor, A2: torch.Tensor, D: torch.Tensor, B: int,
                     Lq: int, mode: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The ungated tree scan (vasr_ssm_scan_ungated_f32, modes 0 / 2): y + x D for x (B*L, Di),
    dt (B*L, Di), bc (B*L, 2N) row views; no z.  The z-in-tail block's scan: the streaming
    kernels with the gated entry point's lane layout, so ssm_block_tail_gated's gate gives
    bitwise ssm_scan's output (the caller keeps to shapes where ssm_scan streams too)."""
    D = f32(D)
    for n, t in (("x", x), ("dt", dt), ("bc", bc), ("A2", A2), ("D", D)):
        _cuda_f32(f"ssm_scan_ungated.{n}", t)
    M, Di, ld_x = _rows("ssm_scan_ungated.x", x)
    _, Di2, ld_dt = _rows("ssm_scan_ungated.dt", dt)
    _, two_n, ld_bc = _rows("ssm_scan_ungated.bc", bc)
    N = A2.numel()
    if M != B * Lq or Di2 != Di or two_n != 2 * N or D.numel() != Di or N not in SCAN_STATE_DIMS:
        raise ValueError("ssm_scan_ungated: inconsistent shapes")
    if out is None:
        out = torch.empty((M, Di), device=x.device, dtype=torch.float32)
    _, _, ld_out = _rows("ssm_scan_ungated.out", out)
    ev = _t0("ssm_scan")
    check(L.lib().vasr_ssm_scan_ungated_f32(x.data_ptr(), ld_x, dt.data_ptr(), ld_dt, bc.data_ptr(), ld_bc,
                                            A2.data_ptr(), D.data_ptr(), out.data_ptr(), ld_out, B, Lq, Di, N,
                                            int(mode), stream_of(x)), "vasr_ssm_scan_ungated_f32")
    _t1("ssm_scan", ev, dict(B=B, L=Lq, Di=Di, N=N, mode=int(mode), chunked=False, ungated=True))
    return out


def ssm_block_tail_gated(yd: torch.Tensor, u: torch.Tensor, wz: torch.Tensor, mode: int, x: torch.Tensor,
                         wo: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor, ln_eps: float, w1: torch.Tensor,
                         b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
                         out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The z-in-tail block's tail (vasr_ssm_block_tail_gated_f32, or _bf16 for bf16 weights): z =
    u W_z^T (the projection GEMM's exact product: split planes for fp32 weights, the bf16 tile
    engine's one product for bf16), g = yd * silu(z) (scan mode `mode`'s gate), then
    ssm_block_tail on g -- for yd (M, 384) the ungated scan output, u (M, 192) the projection
    input, wz (384, 192) = in_proj rows Di..2Di-1 (a persistent tensor: its planes are cached by
    identity)."""
    bf16 = wo.dtype == torch.bfloat16
    if bf16:
        if not (wz.dtype == w1.dtype == w2.dtype == torch.bfloat16):
            raise TypeError("ssm_block_tail_gated: mixed weight dtypes")
        ln_w, ln_b, b1, b2 = f32(ln_w), f32(ln_b), f32(b1), f32(b2)
    for n, t in (("yd", yd), ("u", u), ("x", x), ("ln_w", ln_w), ("ln_b", ln_b), ("b1", b1), ("b2", b2)) + (
            () if bf16 else (("wz", wz), ("wo", wo), ("w1", w1), ("w2", w2))):
        _cuda_f32(f"ssm_block_tail_gated.{n}", t)
    M, E, ldy = _rows("ssm_block_tail_gated.yd", yd)
    Mu, D, ldu = _rows("ssm_block_tail_gated.u", u)
    Mx, Dx, ldx = _rows("ssm_block_tail_gated.x", x)
    if Mu != M or Mx != M or Dx != D or tuple(wz.shape) != (E, D) or tuple(wo.shape) != (D, E):
        raise ValueError("ssm_block_tail_gated: inconsistent shapes")
    if out is None:
        out = torch.empty((M, D), device=yd.device, dtype=torch.float32)
    _, _, ldo = _rows("ssm_block_tail_gated.out", out)
    zprep, prep = (pack_bf16, pack_weights16) if bf16 else (split_weights, split_weights16)
    fn = "vasr_ssm_block_tail_gated_bf16" if bf16 else "vasr_ssm_block_tail_gated_f32"
    ev = _t0("ssm_tail")
    check(getattr(L.lib(), fn)(yd.data_ptr(), ldy, u.data_ptr(), ldu, zprep(wz).data_ptr(), int(mode), x.data_ptr(),
                               ldx, prep(wo).data_ptr(), ln_w.contiguous().data_ptr(), ln_b.contiguous().data_ptr(),
                               float(ln_eps), prep(w1).data_ptr(), b1.contiguous().data_ptr(), prep(w2).data_ptr(),
                               b2.contiguous().data_ptr(), out.data_ptr(), ldo, M, D, E, stream_of(yd)), fn)
    _t1("ssm_tail", ev, dict(M=M, D=D, E=E, gated=True))
    return out


def reflect_pad(audio: torch.Tensor, pad: int, ld_out: int) -> torch.Tensor:
    _cuda_f32("reflect_pad.audio", audio)
    audio = audio.contiguous()
    B, S = audio.shape
    xp = torch.empty((B, ld_out), device=audio.device, dtype=torch.float32)
    check(L.lib().vasr_reflect_pad_f32(audio.data_ptr(), S, xp.data_ptr(), ld_out, B, S, pad, stream_of(audio)),
          "vasr_reflect_pad_f32")
    return xp


def _lens(name: str, t: Optional[torch.Tensor], B: int, device) -> Optional[torch.Tensor]:
    """Per-utterance size array of a zero-padded batch: a contiguous int32 (B,) tensor on the device."""
    if t is None:
        return None
    if t.device != device or t.dtype != torch.int32 or tuple(t.shape) != (B,) or not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous int32 ({B},) tensor on {device}")
    return t


def stft_power_400(audio: torch.Tensor, window: torch.Tensor, samples: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B, S) audio -> (B, S // 160 + 1, 201) |STFT|^2 (n_fft 400, hop 160, reflect pad, Hann).
    samples: per-utterance lengths (int32 (B,), each in (200, S]) of a zero-padded batch."""
    _cuda_f32("stft_power_400.audio", audio)
    _cuda_f32("stft_power_400.window", window)
    audio = audio.contiguous()
    B, S = audio.shape
    if window.numel() != 400:
        raise ValueError(f"stft_power_400: window must have 400 entries, got {window.numel()}")
    F = S // 160 + 1
    power = torch.empty((B, F, 201), device=audio.device, dtype=torch.float32)
    samples = _lens("stft_power_400.samples", samples, B, audio.device)
    if samples is None:
        check(L.lib().vasr_stft_power_400_f32(audio.data_ptr(), S, B, S, window.contiguous().data_ptr(),
                                              power.data_ptr(), 201, F * 201, stream_of(audio)),
              "vasr_stft_power_400_f32")
    else:
        check(L.lib().vasr_stft_power_400_var_f32(audio.data_ptr(), S, B, S, samples.data_ptr(),
                                                  window.contiguous().data_ptr(), power.data_ptr(), 201, F * 201,
                                                  stream_of(audio)), "vasr_stft_power_400_var_f32")
    return power


def mel_log_norm(power: torch.Tensor, ld_power: int, stride_power: int, fb_csr, B: int, F: int, n_mels: int,
                 normalize: bool, frames: Optional[torch.Tensor] = None, frame_pad: int = 0) -> torch.Tensor:
    """frames: per-utterance frame counts (int32 (B,), each <= F); frames past them are 0.
    frame_pad > 0: the mel is written into a (B, F + 2 frame_pad, n_mels) buffer whose outer
    frames the kernel zero-fills, and the (B, F, n_mels) view into it is returned, marked as
    zero-framed (zero_framed()) so the temporal conv reads it without a padding copy."""
    rowptr, col, val = fb_csr
    Fo = F + 2 * frame_pad
    buf = torch.empty((B, Fo, n_mels), device=power.device, dtype=torch.float32)
    ws = torch.empty(int(L.lib().vasr_mel_workspace_floats(B, F, n_mels)), device=power.device, dtype=torch.float32)
    frames = _lens("mel_log_norm.frames", frames, B, power.device)
    if frames is None:
        check(L.lib().vasr_mel_log_norm_f32(power.data_ptr(), ld_power, stride_power, rowptr.data_ptr(),
                                            col.data_ptr(), val.data_ptr(), buf.data_ptr(), Fo * n_mels, frame_pad, B,
                                            F, n_mels, int(normalize), ws.data_ptr(), stream_of(power)),
              "vasr_mel_log_norm_f32")
    else:
        check(L.lib().vasr_mel_log_norm_var_f32(power.data_ptr(), ld_power, stride_power, rowptr.data_ptr(),
                                                col.data_ptr(), val.data_ptr(), buf.data_ptr(), Fo * n_mels, frame_pad,
                                                B, F, n_mels, int(normalize), frames.data_ptr(), ws.data_ptr(),
                                                stream_of(power)), "vasr_mel_log_norm_var_f32")
    if not frame_pad:
        return buf
    out = buf[:, frame_pad:frame_pad + F]
    out._vasr_zero_framed = (buf, frame_pad)
    return out


def zero_framed(x: torch.Tensor, pad: int):
    """The (B, F + 2 q, C) buffer of a (B, F, C) view written by mel_log_norm(..., frame_pad=q)
    with q >= pad zero frames on each side, sliced to `pad` zero frames, or None."""
    ent = getattr(x, "_vasr_zero_framed", None)
    if ent is None:
        return None
    buf, q = ent
    if q < pad or buf.data_ptr() + q * buf.shape[2] * 4 != x.data_ptr() or x.shape[1] + 2 * q != buf.shape[1]:
        return None
    return buf[:, q - pad:q + x.shape[1] + pad]


def pad_frames(x: torch.Tensor, out_frames: int, off: int) -> torch.Tensor:
    _cuda_f32("pad_frames.x", x)
    x = x.contiguous()
    B, F, C = x.shape
    out = torch.empty((B, out_frames, C), device=x.device, dtype=torch.float32)
    check(L.lib().vasr_pad_frames_f32(x.data_ptr(), out.data_ptr(), out_frames, off, B, F, C, stream_of(x)),
          "vasr_pad_frames_f32")
    return out


def adaptive_pool(x: torch.Tensor, K: int, lens: Optional[torch.Tensor] = None,
                  ks: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B, L, C) -> (B, K, C) adaptive average pooling over time; with lens / ks (int32 (B,))
    utterance b pools its first lens[b] rows into ks[b] bins, later bins 0."""
    _cuda_f32("adaptive_pool.x", x)
    x = x.contiguous()
    B, Lq, C = x.shape
    out = torch.empty((B, K, C), device=x.device, dtype=torch.float32)
    if (lens is None) != (ks is None):
        raise ValueError("adaptive_pool: lens and ks go together")
    if lens is None:
        check(L.lib().vasr_adaptive_pool_f32(x.data_ptr(), out.data_ptr(), B, Lq, C, K, stream_of(x)),
              "vasr_adaptive_pool_f32")
    else:
        lens = _lens("adaptive_pool.lens", lens, B, x.device)
        ks = _lens("adaptive_pool.ks", ks, B, x.device)
        check(L.lib().vasr_adaptive_pool_var_f32(x.data_ptr(), out.data_ptr(), B, Lq, C, K, lens.data_ptr(),
                                                 ks.data_ptr(), stream_of(x)), "vasr_adaptive_pool_var_f32")
    return out


def ln_adaptive_pool(x: torch.Tensor, w, b, eps: float, K: int, lens: Optional[torch.Tensor] = None,
                     ks: Optional[torch.Tensor] = None) -> torch.Tensor:
    """adaptive_pool(layer_norm(x, w, b, eps), K, lens, ks) in one launch, bitwise the two
    (vasr_ln_adaptive_pool_f32)."""
    _cuda_f32("ln_adaptive_pool.x", x)
    w, b = f32(w), f32(b)
    x = x.contiguous()
    B, Lq, C = x.shape
    out = torch.empty((B, K, C), device=x.device, dtype=torch.float32)
    if (lens is None) != (ks is None):
        raise ValueError("ln_adaptive_pool: lens and ks go together")
    if lens is not None:
        lens = _lens("ln_adaptive_pool.lens", lens, B, x.device)
        ks = _lens("ln_adaptive_pool.ks", ks, B, x.device)
    check(L.lib().vasr_ln_adaptive_pool_f32(x.data_ptr(), w.data_ptr(), b.data_ptr(), float(eps), out.data_ptr(), B,
                                            Lq, C, K, None if lens is None else lens.data_ptr(),
                                            None if ks is None else ks.data_ptr(), stream_of(x)),
          "vasr_ln_adaptive_pool_f32")
    return out


def pooled_attention(q: torch.Tensor, kv: torch.Tensor, B: int, Lq: int, Kp: int, heads: int,
                     kps: Optional[torch.Tensor] = None) -> torch.Tensor:
    """kps: per-utterance key counts (int32 (B,), each in [1, Kp])."""
    _cuda_f32("pooled_attention.q", q)
    _cuda_f32("pooled_attention.kv", kv)
    M, A, ld_q = _rows("pooled_attention.q", q)
    kv = kv.contiguous()
    if kv.shape != (B * Kp, 2 * A) or M != B * Lq or A % heads:
        raise ValueError("pooled_attention: inconsistent shapes")
    out = torch.empty((M, A), device=q.device, dtype=torch.float32)
    kps = _lens("pooled_attention.kps", kps, B, q.device)
    if kps is None:
        check(L.lib().vasr_pooled_attention_f32(q.data_ptr(), ld_q, kv.data_ptr(), out.data_ptr(), B, Lq, Kp, heads,
                                                A // heads, stream_of(q)), "vasr_pooled_attention_f32")
    else:
        check(L.lib().vasr_pooled_attention_var_f32(q.data_ptr(), ld_q, kv.data_ptr(), out.data_ptr(), B, Lq, Kp,
                                                    heads, A // heads, kps.data_ptr(), stream_of(q)),
              "vasr_pooled_attention_var_f32")
    return out


def probe_clock(device, blocks: int = 2048, iters: int = 20000) -> dict:
    """Machine state for a benchmark record (vasr_probe_clock): the shader clock over a fixed VALU
    chain (median over workgroups, GHz) and the XCD dispatch order.  The kernels' XCD-aware block
    maps need workgroups i and i + 8 on one XCD: round-robin dispatch, from whichever XCD the
    dispatcher's pointer starts at (the previous launch's grid moves it: profiles/r05d/)."""
    out = torch.zeros(3 * blocks, device=device, dtype=torch.int64)
    check(L.lib().vasr_probe_clock(out.data_ptr(), blocks, iters, torch.cuda.current_stream(device).cuda_stream),
          "vasr_probe_clock")
    o = out.view(blocks, 3).cpu()
    ghz = (o[:, 1].double() / o[:, 2].clamp(min=1).double() * 0.1).median().item()
    xcd = o[:, 0]
    ids = torch.arange(blocks)
    fr = [(xcd == (ids + k) % 8).double().mean().item() for k in range(8)]
    k = max(range(8), key=lambda j: fr[j])
    return dict(clock_ghz=round(ghz, 3), xcd_round_robin_frac=round(fr[k], 4), xcd_start=k,
                xcds_seen=int(xcd.unique().numel()))


def argmax(logits: torch.Tensor) -> torch.Tensor:
    """int32 argmax over the last dim (ties -> first index)."""
    _cuda_f32("argmax.logits", logits)
    V = logits.shape[-1]
    x2 = logits.reshape(-1, V)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    rows = x2.shape[0]
    ld = x2.stride(0) if rows > 1 else V
    out = torch.empty(rows, device=logits.device, dtype=torch.int32)
    check(L.lib().vasr_argmax_f32(x2.data_ptr(), ld, rows, V, out.data_ptr(), stream_of(logits)), "vasr_argmax_f32")
    return out.view(logits.shape[:-1])


def _collapse_outputs(who: str, B: int, Lq: int, device, out, timestamps: bool, frames):
    """Output buffers (tokens, lengths, start, end) of a collapse and its checked frames."""
    if out is None:
        toks = torch.empty((B, Lq), device=device, dtype=torch.int32)
        lens = torch.empty((B,), device=device, dtype=torch.int32)
    else:
        toks, lens = out
        for n, t, shape in (("tokens", toks, (B, Lq)), ("lengths", lens, (B,))):
            if (t.device != device or t.dtype != torch.int32 or tuple(t.shape) != shape
                    or not t.is_contiguous()):
                raise ValueError(f"{who}: out {n} must be a contiguous int32 {shape} tensor on {device}")
    st = en = None
    if timestamps:
        st = torch.empty((B, Lq), device=device, dtype=torch.int32)
        en = torch.empty((B, Lq), device=device, dtype=torch.int32)
    return toks, lens, st, en, _lens(f"{who}.frames", frames, B, device)


def ctc_collapse(pred: torch.Tensor, blank: int = 0, collapse: bool = True, timestamps: bool = False,
                 out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, frames: Optional[torch.Tensor] = None):
    """Device-side greedy CTC collapse of (B, L) int32 predictions.  out = (tokens (B, L),
    lengths (B,)): contiguous int32 buffers to write into (e.g. row slices of a graph's
    static output).  frames: per-utterance row counts (int32 (B,)) of a padded batch."""
    if pred.device.type != "cuda" or pred.dtype != torch.int32:
        raise TypeError("ctc_collapse: expected a cuda int32 tensor")
    pred = pred.contiguous()
    B, Lq = pred.shape
    toks, lens, st, en, frames = _collapse_outputs("ctc_collapse", B, Lq, pred.device, out, timestamps, frames)
    if frames is None:
        check(L.lib().vasr_ctc_collapse(pred.data_ptr(), B, Lq, int(blank), int(collapse), toks.data_ptr(),
                                        lens.data_ptr(), ptr(st), ptr(en), stream_of(pred)), "vasr_ctc_collapse")
    else:
        check(L.lib().vasr_ctc_collapse_var(pred.data_ptr(), B, Lq, frames.data_ptr(), int(blank), int(collapse),
                                            toks.data_ptr(), lens.data_ptr(), ptr(st), ptr(en), stream_of(pred)),
              "vasr_ctc_collapse_var")
    return toks, lens, st, en


def fakequant(x: torch.Tensor, scale: torch.Tensor, zero_point: torch.Tensor, qmin: float, qmax: float,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """FakeQuantize (eval, calibrated) of x viewed as (dim0, rest): scale / zero_point hold
    dim0 entries (per-channel, channel_dim 0) or one (per-tensor)."""
    _cuda_f32("fakequant.x", x)
    _cuda_f32("fakequant.scale", scale)
    _cuda_f32("fakequant.zero_point", zero_point)
    x = x.contiguous()
    rows = x.shape[0] if x.dim() > 0 else 1
    x2 = x.reshape(rows, -1)
    cols = x2.shape[1]
    n = scale.numel()
    if zero_point.numel() != n or n not in (1, rows):
        raise ValueError(f"fakequant: scale/zero_point of {n} entries for a tensor with {rows} channels")
    y = torch.empty_like(x) if out is None else out
    check(L.lib().vasr_fakequant_f32(x2.data_ptr(), cols, y.data_ptr(), cols, rows, cols,
                                     scale.contiguous().data_ptr(), zero_point.contiguous().data_ptr(),
                                     int(n == rows and n > 1), float(qmin), float(qmax), stream_of(x)),
          "vasr_fakequant_f32")
    return y


def minmax(x: torch.Tensor, per_channel: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """(min, max) over the whole tensor, or per channel of dim 0 (shape (dim0,))."""
    _cuda_f32("minmax.x", x)
    if x.numel() == 0:
        raise RuntimeError("minmax: empty tensor")
    x = x.contiguous()
    if per_channel and x.dim() >= 1:
        x2 = x.reshape(x.shape[0], -1)
    else:
        x2 = x.reshape(-1, x.shape[-1] if x.dim() >= 1 else 1)
    rows, cols, ld = _rows("minmax.x", x2)
    lo = torch.empty(rows, device=x.device, dtype=torch.float32)
    hi = torch.empty(rows, device=x.device, dtype=torch.float32)
    check(L.lib().vasr_minmax_f32(x2.data_ptr(), ld, rows, cols, lo.data_ptr(), hi.data_ptr(), stream_of(x)),
          "vasr_minmax_f32")
    if per_channel or rows == 1:
        return lo, hi
    lo1 = torch.empty(1, device=x.device, dtype=torch.float32)
    hi1 = torch.empty(1, device=x.device, dtype=torch.float32)
    lib = L.lib()
    check(lib.vasr_minmax_f32(lo.data_ptr(), rows, 1, rows, lo1.data_ptr(), hi1.data_ptr(), stream_of(x)),
          "vasr_minmax_f32")
    scratch = torch.empty(1, device=x.device, dtype=torch.float32)
    check(lib.vasr_minmax_f32(hi.data_ptr(), rows, 1, rows, scratch.data_ptr(), hi1.data_ptr(), stream_of(x)),
          "vasr_minmax_f32")
    return lo1, hi1


def ctc_beam_search(logits: torch.Tensor, beam_width: int, blank: int = 0):
    """Device prefix beam search over (B, L, V) logits -> (tokens (B, W, L) int32, lengths (B, W),
    scores (B, W) float64, beams per utterance (B,)), all on the device."""
    _cuda_f32("ctc_beam_search.logits", logits)
    if logits.dim() != 3:
        raise ValueError("ctc_beam_search: logits must be (B, L, V)")
    x = logits if logits.stride(-1) == 1 else logits.contiguous()
    B, Lq, V = x.shape
    W = int(beam_width)
    dev = x.device
    trie = torch.empty(max(B, 1) * int(L.lib().vasr_ctc_beam_workspace_elems(Lq, W)), device=dev, dtype=torch.int32)
    toks = torch.zeros((B, W, max(Lq, 1)), device=dev, dtype=torch.int32)
    lens = torch.zeros((B, W), device=dev, dtype=torch.int32)
    scores = torch.zeros((B, W), device=dev, dtype=torch.float64)
    nbeams = torch.zeros((B,), device=dev, dtype=torch.int32)
    check(L.lib().vasr_ctc_beam_search(x.data_ptr(), x.stride(1), x.stride(0), B, Lq, V, W, int(blank), trie.data_ptr(),
                                       toks.data_ptr(), lens.data_ptr(), scores.data_ptr(), nbeams.data_ptr(),
                                       stream_of(x)), "vasr_ctc_beam_search")
    return toks, lens, scores, nbeams
