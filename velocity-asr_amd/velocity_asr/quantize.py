"""INT8 fake quantisation (drop-in for reference velocity_asr/quantize.py), BASELINE config C5.

Same classes, buffers and state_dict keys as the reference (QuantizationConfig,
FakeQuantize, QuantizedLinear, QuantizedConv1d, prepare_model_for_qat, calibrate_model),
so a QAT checkpoint written by the reference loads with strict=True.  At inference a
calibrated FakeQuantize is a fixed elementwise map; the MI355X build therefore

  * fake-quantizes each weight ONCE per parameter version (vasr_fakequant_f32, the exact
    torch evaluation order, cached like the other derived weight layouts), and
  * fuses every activation quantizer into the epilogue of the GEMM that produces it
    (vasr_gemm_args.qparams: per-column {scale, zp, qmin, qmax} applied to acc + bias
    before GELU / sigmoid / the gated blend), so C5 costs no extra pass over HBM.

Quantizer arithmetic is bit-identical to torch's CPU evaluation for identical inputs
(tests: element-level goldens of the reference FakeQuantize).  Scope: eval-mode
inference.  Training-mode fake quantisation (QAT, scale re-estimated on every call) is
out of scope and raises.  ONNX export / onnxruntime quantisation (quantize.py:372-474)
need onnx / onnxruntime, which this image does not ship; they raise ImportError like the
reference does when onnxruntime is missing.

Calibration:
  * ``calibrate_model`` keeps the reference's behaviour (quantize.py:325-369): in eval an
    uncalibrated FakeQuantize passes through, so the forwards observe nothing and every
    quantizer ends up "calibrated" with scale 1, zero_point 0 (defect ii).
  * ``calibrate_from_activations`` is the intended procedure the goldens use: weight
    quantizers observe their weights, then one forward (activations still pass-through)
    records every quantized layer's output and its activation quantizer observes it.
"""

from __future__ import annotations

import logging
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops
from ._prep import cached

logger = logging.getLogger(__name__)
_f32 = np.float32


@dataclass
class QuantizationConfig:
    """Configuration for quantization (reference quantize.py:18-37)."""

    weight_bits: int = 8
    activation_bits: int = 8
    per_channel_weights: bool = True
    ssm_state_fp32: bool = True
    num_calibration_batches: int = 100
    symmetric_weights: bool = True
    symmetric_activations: bool = False


class FakeQuantize(nn.Module):
    """Fake quantization (reference quantize.py:40-139); eval-mode forward on the HIP device."""

    def __init__(self, bits: int = 8, symmetric: bool = True, per_channel: bool = False, channel_dim: int = 0):
        super().__init__()
        self.bits = bits
        self.symmetric = symmetric
        self.per_channel = per_channel
        self.channel_dim = channel_dim
        if symmetric:
            self.qmin = -(2 ** (bits - 1))
            self.qmax = 2 ** (bits - 1) - 1
        else:
            self.qmin = 0
            self.qmax = 2 ** bits - 1
        self.register_buffer("scale", torch.tensor(1.0))
        self.register_buffer("zero_point", torch.tensor(0.0))
        self.register_buffer("calibrated", torch.tensor(False))

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        # Calibration replaces the 0-d scale / zero_point buffers by per-channel ones
        # ((out, 1[, 1]) for weights), so a calibrated checkpoint does not fit a freshly
        # prepared model; the reference's strict load_state_dict rejects it with a size
        # mismatch.  Adopt the checkpoint's shapes instead.
        for name in ("scale", "zero_point"):
            t = state_dict.get(prefix + name)
            cur = getattr(self, name)
            if isinstance(t, torch.Tensor) and t.shape != cur.shape:
                setattr(self, name, torch.empty(t.shape, dtype=cur.dtype, device=cur.device))
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    # -- host view of the calibrated flag, re-read only when the buffer changes (no per-forward
    #    device sync, so quantized forwards stay HIP-graph capturable)
    def is_calibrated(self) -> bool:
        return cached(self, "calibrated", (self.calibrated,), lambda: bool(self.calibrated.item()))

    def active(self) -> bool:
        """True if forward() quantizes (eval + calibrated); raises for training mode."""
        if self.training:
            raise NotImplementedError(
                "velocity_asr (MI355X build): training-mode fake quantization (QAT) is out of scope; "
                "call model.eval() for calibrated INT8 inference")
        return self.is_calibrated()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.active():
            return x                                   # quantize.py:82-84
        return ops.fakequant(x, self.scale, self.zero_point, self.qmin, self.qmax)

    def _update_scale_zp(self, x: torch.Tensor):
        """quantize.py:99-116: ranges observed on the device, the few scalar ops in float32 on
        the host in torch's order."""
        if x.device.type != "cuda":
            _lib.require_device()
            raise RuntimeError("FakeQuantize (MI355X build): calibrate on a HIP device tensor")
        x = x.detach().float()
        if self.per_channel:
            if self.channel_dim != 0:
                raise NotImplementedError("per-channel FakeQuantize supports channel_dim=0 (the reference's only use)")
            lo_t, hi_t = ops.minmax(x, per_channel=True)
            keep = (x.shape[0],) + (1,) * (x.dim() - 1)
        else:
            lo_t, hi_t = ops.minmax(x)
            keep = ()
        lo = lo_t.cpu().numpy().astype(_f32).reshape(keep)
        hi = hi_t.cpu().numpy().astype(_f32).reshape(keep)
        with np.errstate(all="ignore"):
            if self.symmetric:
                scale = (np.maximum(np.abs(lo), np.abs(hi)) / _f32(self.qmax)).astype(_f32)
                zp = np.zeros_like(scale)
            else:
                scale = ((hi - lo) / _f32(self.qmax - self.qmin)).astype(_f32)
                zp = (_f32(self.qmin) - (lo / scale).astype(_f32)).astype(_f32)
        scale = np.maximum(scale, _f32(1e-10)).astype(_f32)
        # (np.ascontiguousarray would promote the per-tensor 0-d buffers to 1-d)
        self.scale = torch.from_numpy(np.array(scale, dtype=_f32)).to(x.device)
        self.zero_point = torch.from_numpy(np.array(zp, dtype=_f32)).to(x.device)

    def calibrate(self, x: torch.Tensor):
        """quantize.py:135-139."""
        with torch.no_grad():
            self._update_scale_zp(x)
            self.calibrated.fill_(True)

    def qparams(self, cols: int) -> torch.Tensor:
        """(cols, 4) per-column {scale, zp, qmin, qmax} of a per-tensor quantizer (GEMM epilogue
        form); scale 0 marks pass-through columns (uncalibrated)."""
        def build():
            dev = self.scale.device
            if not self.is_calibrated():
                return torch.zeros((cols, 4), device=dev, dtype=torch.float32)
            if self.scale.numel() != 1:
                raise NotImplementedError("per-channel activation quantizers are not supported in GEMM epilogues")
            row = torch.stack([self.scale.reshape(()).float(), self.zero_point.reshape(()).float(),
                               torch.tensor(float(self.qmin), device=dev), torch.tensor(float(self.qmax), device=dev)])
            return row.reshape(1, 4).expand(cols, 4).contiguous()
        return cached(self, f"qp{cols}", (self.scale, self.zero_point, self.calibrated), build)


class QuantizedLinear(nn.Module):
    """Linear with fake-quantized weight and output (reference quantize.py:142-191)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True,
                 config: Optional[QuantizationConfig] = None):
        super().__init__()
        config = config or QuantizationConfig()
        self.linear = nn.Linear(in_features, out_features, bias=bias)
        self.weight_quantizer = FakeQuantize(bits=config.weight_bits, symmetric=config.symmetric_weights,
                                             per_channel=config.per_channel_weights, channel_dim=0)
        self.activation_quantizer = FakeQuantize(bits=config.activation_bits,
                                                 symmetric=config.symmetric_activations, per_channel=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        w, b, qp = linear_parts(self)
        shape = x.shape
        y = ops.gemm(x.reshape(-1, shape[-1]).contiguous(), w, b, qparams=qp)
        return y.view(*shape[:-1], w.shape[0])


class QuantizedConv1d(nn.Module):
    """Conv1d with fake-quantized weight and output (reference quantize.py:194-266)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, padding: int = 0,
                 groups: int = 1, bias: bool = True, config: Optional[QuantizationConfig] = None):
        super().__init__()
        config = config or QuantizationConfig()
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size, stride=stride, padding=padding, groups=groups,
                              bias=bias)
        self.weight_quantizer = FakeQuantize(bits=config.weight_bits, symmetric=config.symmetric_weights,
                                             per_channel=config.per_channel_weights, channel_dim=0)
        self.activation_quantizer = FakeQuantize(bits=config.activation_bits,
                                                 symmetric=config.symmetric_activations, per_channel=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B, C_in, L) -> (B, C_out, L_out) as one strided-row GEMM over frame-major input."""
        c = self.conv
        if c.groups != 1 or c.dilation[0] != 1 or c.padding_mode != "zeros" or isinstance(c.padding, str):
            raise NotImplementedError("QuantizedConv1d (MI355X build): groups=1, dilation 1, zero padding only")
        B, C, Lin = x.shape
        y = conv1d_rows(self, x.transpose(1, 2).contiguous())
        return y.transpose(1, 2)


# --------------------------------------------------------------------------- model-site helpers
def _is_q(mod) -> bool:
    return isinstance(mod, (QuantizedLinear, QuantizedConv1d))


def inner(mod: nn.Module) -> nn.Module:
    """The nn.Linear / nn.Conv1d holding the parameters of a (possibly quantized) layer."""
    if isinstance(mod, QuantizedLinear):
        return mod.linear
    if isinstance(mod, QuantizedConv1d):
        return mod.conv
    return mod


def effective_weight(mod: nn.Module) -> torch.Tensor:
    """The weight the layer multiplies by: fake-quantized once per version if calibrated."""
    if not _is_q(mod):
        return mod.weight
    w = inner(mod).weight
    wq = mod.weight_quantizer
    if not wq.active():
        return w
    return cached(mod, "wq", (w, wq.scale, wq.zero_point, wq.calibrated),
                  lambda: ops.fakequant(w.detach(), wq.scale, wq.zero_point, wq.qmin, wq.qmax))


def act_qparams(mod: nn.Module, cols: int) -> Optional[torch.Tensor]:
    """(cols, 4) epilogue qparams of the layer's activation quantizer, or None."""
    if not _is_q(mod) or not mod.activation_quantizer.active():
        return None
    return mod.activation_quantizer.qparams(cols)


def act_qparams_or_identity(mod: nn.Module, cols: int, device) -> torch.Tensor:
    qp = act_qparams(mod, cols)
    return qp if qp is not None else torch.zeros((cols, 4), device=device, dtype=torch.float32)


def linear_parts(mod: nn.Module) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
    """(weight, bias, activation qparams or None) of an nn.Linear or QuantizedLinear."""
    lin = inner(mod)
    return effective_weight(mod), lin.bias, act_qparams(mod, lin.out_features)


def conv1d_rows(mod: nn.Module, x_frames: torch.Tensor, epilogue: int = _lib.EPI_NONE,
                aux: Optional[torch.Tensor] = None, ld_aux: int = 0) -> torch.Tensor:
    """Conv1d (groups 1) of frame-major input (B, L_in, C_in) -> (B, L_out, C_out): the input is
    zero-padded once so every output row is a plain strided row (stride s frames, K = k
    frames) and the conv is one batched GEMM with the activation quantizer (if any) and
    `epilogue` fused."""
    c = inner(mod)
    B, Lin, C = x_frames.shape
    k, s, p = c.kernel_size[0], c.stride[0], c.padding[0]
    D = c.out_channels
    L = (Lin + 2 * p - k) // s + 1
    frames = max(Lin + 2 * p, (L - 1) * s + k)

    def wbuild():
        w = effective_weight(mod)                   # (D, C, k) -> (D, k*C), frame-major rows
        return w.permute(0, 2, 1).reshape(D, -1).contiguous()
    w = cached(mod, "wrows", (inner(mod).weight,) + _wq_deps(mod), wbuild)
    # a mel the device pipeline wrote zero-framed (ops.mel_log_norm(..., frame_pad)) is read in
    # place: its batch stride is (Lin + 2 q) frames; else one padding copy
    zf = ops.zero_framed(x_frames, p) if frames == Lin + 2 * p else None
    if zf is not None:
        buf, ld_b = zf, zf.stride(0)
    else:
        buf = ops.pad_frames(x_frames, frames, p)
        ld_b = frames * C
    out = torch.empty((B, L, D), device=buf.device, dtype=torch.float32)
    ops.gemm_batched(buf, s * C, ld_b, L, B, k * C, w, c.bias, out, D, L * D, epilogue=epilogue, aux=aux,
                     ld_aux=ld_aux, stride_aux=0, qparams=act_qparams(mod, D))
    return out


def deps(mod) -> tuple:
    """Tensors whose change invalidates a derived weight / qparams layout built from `mod`."""
    lin = inner(mod)
    d = (lin.weight,) + ((lin.bias,) if lin.bias is not None else ())
    if _is_q(mod):
        a = mod.activation_quantizer
        d += _wq_deps(mod) + (a.scale, a.zero_point, a.calibrated)
    return d


def _wq_deps(mod) -> tuple:
    if not _is_q(mod):
        return ()
    wq = mod.weight_quantizer
    return (wq.scale, wq.zero_point, wq.calibrated)


# --------------------------------------------------------------------------- observation
# While a dict, model sites record the raw output (acc + bias, before any activation
# quantizer or activation function) of every quantized layer: {module: tensor}.
_observer: Optional[Dict[nn.Module, torch.Tensor]] = None


def observing(mod: nn.Module) -> bool:
    return _observer is not None and _is_q(mod)


def record(mod: nn.Module, raw: torch.Tensor) -> None:
    if observing(mod):
        _observer[mod] = raw


# --------------------------------------------------------------------------- model preparation
def prepare_model_for_qat(model: nn.Module, config: Optional[QuantizationConfig] = None) -> nn.Module:
    """Replace Linear / Conv1d layers outside the SSMs by quantized versions (quantize.py:269-322).

    Same module selection and names as the reference (any path containing "ssm" stays fp32
    when ssm_state_fp32).  Unlike the reference, which re-initialises the new layers
    (defect i), the existing weights are carried over; a state_dict loaded
    afterwards overrides them either way.
    """
    config = config or QuantizationConfig()

    def replace_module(module: nn.Module, name: str = "") -> nn.Module:
        if config.ssm_state_fp32 and "ssm" in name.lower():
            return module
        if isinstance(module, nn.Linear):
            q = QuantizedLinear(module.in_features, module.out_features, bias=module.bias is not None, config=config)
            q.linear = module
            return q.to(module.weight.device)
        if isinstance(module, nn.Conv1d):
            q = QuantizedConv1d(module.in_channels, module.out_channels, module.kernel_size[0],
                                stride=module.stride[0], padding=module.padding[0], groups=module.groups,
                                bias=module.bias is not None, config=config)
            q.conv = module
            return q.to(module.weight.device)
        for child_name, child in module.named_children():
            full_name = f"{name}.{child_name}" if name else child_name
            setattr(module, child_name, replace_module(child, full_name))
        return module

    return replace_module(model)


def _fake_quant_modules(model: nn.Module):
    return [m for m in model.modules() if isinstance(m, FakeQuantize)]


def calibrate_model(model: nn.Module, calibration_dataloader: Iterable, num_batches: int = 100,
                    device: str = "cuda"):
    """The reference's calibrate_model (quantize.py:325-369), behaviour kept as is."""
    model.eval()
    model.to(device)
    fake_quant_modules = _fake_quant_modules(model)
    logger.info(f"Calibrating {len(fake_quant_modules)} quantization nodes...")
    with torch.no_grad():
        for batch_idx, batch in enumerate(calibration_dataloader):
            if batch_idx >= num_batches:
                break
            mel = batch["mel_spectrogram"].to(device) if isinstance(batch, dict) else batch[0].to(device)
            _ = model(mel)
            if (batch_idx + 1) % 10 == 0:
                logger.info(f"Calibration progress: {batch_idx + 1}/{num_batches}")
    for module in fake_quant_modules:
        module.calibrated.fill_(True)
    logger.info("Calibration complete.")


def calibrate_from_activations(model: nn.Module, mel_spectrogram: torch.Tensor) -> int:
    """Intended calibration: every weight quantizer observes its weight; then one forward of
    `mel_spectrogram` (activation quantizers still pass-through) records each quantized
    layer's output, which its activation quantizer observes.  Returns the number of
    calibrated activation quantizers."""
    global _observer
    model.eval()
    qmods = [m for m in model.modules() if _is_q(m)]
    with torch.no_grad():
        for m in qmods:
            m.weight_quantizer.calibrate(inner(m).weight)
            m.activation_quantizer.calibrated.fill_(False)
        _observer = {}
        try:
            model(mel_spectrogram)
            seen = _observer
        finally:
            _observer = None
        missing = [m for m in qmods if m not in seen]
        if missing:
            raise RuntimeError(f"calibrate_from_activations: {len(missing)} quantized layers were not reached "
                               "by the model's forward")
        for m in qmods:
            m.activation_quantizer.calibrate(seen[m])
    return len(qmods)


def export_quantized_onnx(model: nn.Module, output_path: str, input_shape=(1, 500, 80), opset_version: int = 17):
    """quantize.py:372-410: needs the onnx exporter, absent from this image."""
    try:
        import onnx  # noqa: F401
    except ImportError:
        raise ImportError("onnx is required for ONNX export. Install with: pip install onnx")
    raise NotImplementedError("ONNX export of the HIP model is out of scope (SURVEY §2)")


def quantize_onnx_model(onnx_path: str, output_path: str, calibration_dataloader=None):
    """quantize.py:413-474: onnxruntime INT8 (absent from this image, as in the reference's guard)."""
    try:
        import onnxruntime.quantization  # noqa: F401
    except ImportError:
        raise ImportError("onnxruntime is required for ONNX quantization. Install with: pip install onnxruntime")
    raise NotImplementedError("onnxruntime quantization is out of scope (SURVEY §2)")


def get_model_size_mb(model: nn.Module) -> float:
    """quantize.py:477-495."""
    param_size = sum(p.nelement() * p.element_size() for p in model.parameters())
    buffer_size = sum(b.nelement() * b.element_size() for b in model.buffers())
    return (param_size + buffer_size) / (1024 * 1024)
