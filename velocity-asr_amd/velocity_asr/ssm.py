"""Selective SSM blocks (drop-in for reference velocity_asr/ssm.py) on MI355X kernels.

Same module tree, parameter names and shapes as the reference, so state_dicts load
unchanged.  Forward passes run the HIP kernels of libvasr_hip.so:

  SSMBlock:  LN1 + causal depthwise conv (one kernel)
             -> in_proj GEMM (fp32 MFMA)
             -> [x_proj; dt_proj] as ONE GEMM with bias + softplus fused on the dt columns
             -> gated selective scan (tree or recurrence) with D skip and y*silu(z) fused
             -> out_proj GEMM with the residual add fused
             -> LN2 -> FFN1 GEMM + GELU -> FFN2 GEMM + bias + residual
Inference only: dropout is the identity (as in eval()), no autograd.
"""

from __future__ import annotations

import math
import os
import warnings
from typing import Literal, Optional

import torch
import torch.nn as nn

from . import _lib, ops
from ._prep import cached

ScanMode = Literal["sequential", "parallel", "mamba"]

# The reference imports mamba_ssm's selective_scan_fn for scan_mode="mamba"
# (ssm.py:20-26).  Here that operator contract is served by the HIP recurrence kernel
# (vasr_ssm_scan_f32 mode 1, the semantics selective_scan_fn computes), so the mode is
# always available.
MAMBA_AVAILABLE = True

_SCAN_MODE_ID = {"parallel": 0, "sequential": 1, "mamba": 1}


def _tree_mode() -> int:
    """Kernel mode of scan_mode="parallel": 2 (default) = the reference's tree with fused
    multiply-adds and (x*dt)*B (a third fewer state-update instructions: 97 vs 106 us per
    16-clip launch, tokens identical); 0 = the reference tree op for op (two roundings per
    a*b + c, x*(dt*B)).  VASR_SCAN_FMA=0|1 selects; read per call so tests can switch it."""
    return 0 if os.environ.get("VASR_SCAN_FMA", "1") == "0" else 2
_warned_training = False


def _bf16_compose() -> bool:
    """The bf16 model's composed projection (SelectiveSSM._prepared); VASR_BF16_COMPOSE=0 selects
    the two GEMMs (read per call so tests can compare the two)."""
    return os.environ.get("VASR_BF16_COMPOSE", "1") != "0"


def _check_eval(module: nn.Module) -> None:
    global _warned_training
    if module.training and not _warned_training:
        _warned_training = True
        warnings.warn("velocity_asr (MI355X build) is inference-only: dropout is treated as identity; "
                      "call model.eval() to silence this warning", stacklevel=3)


class SelectiveSSM(nn.Module):
    """Selective state space model (reference ssm.py:32-337)."""

    def __init__(self, d_model: int = 192, state_dim: int = 64, expand_ratio: int = 2,
                 scan_mode: ScanMode = "parallel"):
        super().__init__()
        self.d_model = d_model
        self.state_dim = state_dim
        self.d_inner = d_model * expand_ratio
        self.scan_mode = scan_mode
        if scan_mode not in _SCAN_MODE_ID:
            raise ValueError(f"Unknown scan_mode: {scan_mode}")
        self.in_proj = nn.Linear(d_model, self.d_inner * 2, bias=False)
        self.x_proj = nn.Linear(self.d_inner, state_dim * 2, bias=False)
        self.dt_proj = nn.Linear(self.d_inner, self.d_inner, bias=True)
        A = torch.arange(1, state_dim + 1, dtype=torch.float32)
        self.A_log = nn.Parameter(torch.log(A))
        self.D = nn.Parameter(torch.ones(self.d_inner))
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=False)

    def _prepared(self):
        def build():
            dev = self.x_proj.weight.device
            N, Np = self.state_dim, ops.scan_state_dim(self.state_dim)
            xw = self.x_proj.weight
            if Np != N:
                # state dims the scan kernels are not built for run as the next size up: zero rows
                # make the GEMM write B and C with Np - N zero columns each, and A2 = 0 there, so
                # the padded states stay exactly 0 and add nothing to y (include/vasr.h)
                z = torch.zeros(Np - N, xw.shape[1], device=dev, dtype=xw.dtype)
                xw = torch.cat([xw[:N], z, xw[N:], z], 0)
            w = torch.cat([xw, self.dt_proj.weight], 0).contiguous()
            b = torch.cat([torch.zeros(2 * Np, device=dev), self.dt_proj.bias.float()]).contiguous()
            # A = -exp(A_log) exactly as the reference evaluates it (float32, ssm.py:116), then
            # pre-scaled by log2(e) so the kernel's dA is one v_exp_f32.
            A = -torch.exp(self.A_log.detach().float().cpu())
            A2 = torch.zeros(Np, dtype=torch.float32)
            A2[:N] = A * torch.tensor(ops.LOG2E, dtype=torch.float32)
            out = dict(w_xdt=w, b_xdt=b, A2=A2.to(dev))
            if w.dtype == torch.float32:
                # composed projection: [x_proj; dt_proj](in_proj_x(u)) = u @ (W_xdt W_in_x)^T, the
                # product formed in float64 and rounded once (see gated_scan)
                Di = self.d_inner
                wc = (w.detach().double() @ self.in_proj.weight.detach()[:Di].double()).float()
                out["w_comb"] = torch.cat([self.in_proj.weight.detach(), wc], 0).contiguous()
                out["b_comb"] = torch.cat([torch.zeros(2 * Di, device=dev), b]).contiguous()
                # the z-in-tail block (SSMBlock._z_in_tail): [x | B | C | dt] without the z rows, and
                # W_z for the tail's own z product (the same rows, so the same split planes)
                out["w_noz"] = torch.cat([self.in_proj.weight.detach()[:Di], wc], 0).contiguous()
                out["b_noz"] = torch.cat([torch.zeros(Di, device=dev), b]).contiguous()
                out["w_z"] = self.in_proj.weight.detach()[Di:].contiguous()
            elif w.dtype == torch.bfloat16 and self.in_proj.weight.dtype == torch.bfloat16:
                # the bf16 model's z-in-tail block: in_proj split into its x rows (the projection
                # GEMM) and its z rows (the tail's product); the bf16 engine's per-column result
                # does not depend on the other columns, so both are bitwise in_proj's
                Di = self.d_inner
                out["w_x"] = self.in_proj.weight.detach()[:Di].contiguous()
                out["w_z"] = self.in_proj.weight.detach()[Di:].contiguous()
                # composed form (default; VASR_BF16_COMPOSE=0: the two GEMMs): [W_in; W_xdt W_in,x] as
                # one bf16 GEMM, the product of the bf16 weights formed in float64 and rounded to bf16
                # once -- one bf16 rounding where the two GEMMs round x_p to bf16 at the second
                # GEMM's input (C3's token edit rate vs the reference 2.28 % vs 2.31 %, profiles/r06ad/)
                wc = (w.detach().double() @ out["w_x"].double()).to(torch.bfloat16)
                out["w_comb16"] = torch.cat([self.in_proj.weight.detach(), wc], 0).contiguous()
                out["b_comb16"] = torch.cat([torch.zeros(2 * Di, device=dev), b]).contiguous()
                out["w_noz16"] = torch.cat([out["w_x"], wc], 0).contiguous()
                out["b_noz16"] = torch.cat([torch.zeros(Di, device=dev), b]).contiguous()
            return out
        return cached(self, "ssm", (self.x_proj.weight, self.dt_proj.weight, self.dt_proj.bias, self.A_log,
                                    self.in_proj.weight), build)

    def gated_scan(self, u: torch.Tensor, B: int, L: int) -> torch.Tensor:
        """u (B*L, d_model) -> y * silu(z) of shape (B*L, d_inner), before out_proj."""
        xz, xdt = self.project(u)
        return self.scan(xz, xdt, B, L)

    def project(self, u: torch.Tensor):
        """u (B*L, d_model) -> (xz, xdt): the scan's operands, [x_p | z] and [B | C | dt]
        (views into one buffer for the composed projection).

        fp32 model (default): in_proj and [x_proj; dt_proj] as ONE GEMM of u against
        [W_in; W_xdt W_in_x] (N = 2 Di + 2N + Di, K = d_model), softplus on the dt columns: the
        composition of two linear maps, with the composed matrix formed in float64 and rounded
        once.  It skips the fp32 rounding of x_p between the two products (a ~1e-7 relative
        difference, the size of GEMM accumulation-order effects) and needs 29 % fewer MACs, one
        launch instead of two and no re-read of x_p.  VASR_XDT_COMPOSE=0 selects the two
        products as the reference evaluates them (ssm.py:105-113)."""
        p = self._prepared()
        Di, N = self.d_inner, ops.scan_state_dim(self.state_dim)
        if "w_comb" in p and os.environ.get("VASR_XDT_COMPOSE", "1") != "0":
            out = ops.gemm(u, p["w_comb"], p["b_comb"], epilogue=_lib.EPI_SOFTPLUS_FROM,
                           n_out=2 * Di + 2 * N)                                 # (M, 2Di + 2N + Di)
            return out[:, :2 * Di], out[:, 2 * Di:]
        if "w_comb16" in p and _bf16_compose():  # the bf16 model's composed form (see _prepared)
            out = ops.gemm(u, p["w_comb16"], p["b_comb16"], epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=2 * Di + 2 * N)
            return out[:, :2 * Di], out[:, 2 * Di:]
        xz = ops.gemm(u, self.in_proj.weight)                                   # (M, 2Di) [x | z]
        xdt = ops.gemm(xz[:, :Di], p["w_xdt"], p["b_xdt"], epilogue=_lib.EPI_SOFTPLUS_FROM,
                       n_out=2 * N)                                              # (M, 2N + Di) [B | C | dt]
        return xz, xdt

    def scan(self, xz: torch.Tensor, xdt: torch.Tensor, B: int, L: int) -> torch.Tensor:
        """The gated scan over in_proj's [x | z] and [B | C | dt]."""
        p = self._prepared()
        N = ops.scan_state_dim(self.state_dim)
        mode = _SCAN_MODE_ID[self.scan_mode]
        return ops.ssm_scan(xz, xdt[:, 2 * N:], xdt[:, :2 * N], p["A2"], self.D, B, L,
                            _tree_mode() if mode == 0 else mode)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _check_eval(self)
        B, L, _ = x.shape
        g = self.gated_scan(x.reshape(B * L, -1), B, L)
        return ops.gemm(g, self.out_proj.weight).view(B, L, self.d_model)


class SSMBlock(nn.Module):
    """Pre-norm conv + SSM + FFN block (reference ssm.py:340-441)."""

    def __init__(self, d_model: int = 192, state_dim: int = 64, expand_ratio: int = 2, kernel_size: int = 4,
                 dropout: float = 0.1, use_checkpoint: bool = False, scan_mode: ScanMode = "parallel"):
        super().__init__()
        self.use_checkpoint = use_checkpoint
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.conv = nn.Conv1d(d_model, d_model, kernel_size=kernel_size, padding=kernel_size - 1, groups=d_model)
        self.ssm = SelectiveSSM(d_model=d_model, state_dim=state_dim, expand_ratio=expand_ratio, scan_mode=scan_mode)
        self.ffn = nn.Sequential(
            nn.Linear(d_model, d_model * expand_ratio),
            nn.GELU(),
            nn.Dropout(dropout),
            nn.Linear(d_model * expand_ratio, d_model),
            nn.Dropout(dropout),
        )
        self.dropout = nn.Dropout(dropout)

    def _fused_tail_ok(self, D: int) -> bool:
        """The one-launch tail (vasr_ssm_block_tail_f32 / _bf16) serves the fp32 and the bf16
        model at d_model 192 / FFN width 384; VASR_FUSED_TAIL=0 selects the launches below (read
        per call so tests can compare the two)."""
        w = self.ffn[0].weight
        dtype_ok = w.dtype in (torch.bfloat16, torch.float32)
        return (os.environ.get("VASR_FUSED_TAIL", "1") != "0" and dtype_ok and D == 192
                and tuple(w.shape) == (384, 192) and self.ssm.d_inner == 384
                and self.ssm.out_proj.weight.dtype == w.dtype == self.ffn[3].weight.dtype)

    def forward(self, x: torch.Tensor, pre_norm: Optional[nn.LayerNorm] = None) -> torch.Tensor:
        """pre_norm (extension): x is the temporal binding's row before its final LayerNorm, which
        this block applies inside its norm1 + conv launch (_norm_conv); the result is bitwise the
        same as for pre_norm(x)."""
        _check_eval(self)
        B, L, D = x.shape
        if self._z_in_tail(B, L, D):
            return self._forward_z_in_tail(x, pre_norm)
        x2, xz, xdt = self.head(x, pre_norm)
        g = self.ssm.scan(xz, xdt, B, L)
        return self.tail(g, x2, B, L)

    # z-in-tail: z = in_proj_z(u) feeds only the gate y * silu(z)
    # (ssm.py:106, :129).  The projection GEMM -- bound by its C stores -- then
    # skips the z columns, the scan writes the ungated y + x D, and the fused tail forms z itself
    # with the projection GEMM's exact product before applying the gate and the usual tail:
    # bitwise the three-launch block's output (tests/test_ssm_tail.py).  fp32 model: the composed
    # projection writes [x | B | C | dt] (896 of its 1280 columns).  bf16 model: in_proj writes x
    # alone (384 of 768 columns), [x_proj; dt_proj] reads it as before.  Where it runs: the tree
    # scan streamed (ops._use_chunked false) and the 32-row tail (M > 4096 token rows: the
    # bench's batches); VASR_Z_IN_TAIL=0 turns it off.
    Z_IN_TAIL_MIN_ROWS = 4097

    def _z_in_tail(self, B: int, L: int, D: int) -> bool:
        ssm = self.ssm
        if os.environ.get("VASR_Z_IN_TAIL", "1") == "0" or B * L < self.Z_IN_TAIL_MIN_ROWS:
            return False
        if _SCAN_MODE_ID[ssm.scan_mode] != 0:
            return False
        mods = (ssm.in_proj, ssm.x_proj, ssm.dt_proj, ssm.out_proj, self.ffn[0], self.ffn[3])
        dtype = ssm.in_proj.weight.dtype
        if dtype not in (torch.float32, torch.bfloat16) or not all(
                type(m) is nn.Linear and m.weight.dtype == dtype for m in mods):
            return False  # QAT (quantize.QuantizedLinear) and mixed-dtype models keep the gated scan
        if dtype == torch.float32 and os.environ.get("VASR_XDT_COMPOSE", "1") == "0":
            return False
        if not self._fused_tail_ok(D):
            return False
        N = ops.scan_state_dim(ssm.state_dim)
        if N != ssm.state_dim or ops._use_chunked(B, L, ssm.d_inner, N, _tree_mode()):
            return False
        return ("w_noz" if dtype == torch.float32 else "w_x") in ssm._prepared()

    def _norm_conv(self, x: torch.Tensor, pre_norm: Optional[nn.LayerNorm]):
        """(conv(norm1(x)), x) as (B, L, D) tensors; with pre_norm, x is first pre_norm(x), formed
        inside the same launch when the shape allows it (vasr_ln_dwconv_prenorm_f32: D = 192, 4
        taps), else by its own LayerNorm launch."""
        B, L, D = x.shape
        x = x.contiguous()
        cw = ops.f32(self.conv.weight).view(D, -1)
        if pre_norm is not None:
            if D == 192 and cw.shape[1] == 4:
                return ops.ln_dwconv_prenorm(x, pre_norm.weight, pre_norm.bias, pre_norm.eps, self.norm1.weight,
                                             self.norm1.bias, cw, self.conv.bias, self.norm1.eps)
            x = ops.layer_norm(x, pre_norm.weight, pre_norm.bias, pre_norm.eps)
        return ops.ln_dwconv(x, self.norm1.weight, self.norm1.bias, cw, self.conv.bias, self.norm1.eps), x

    def _forward_z_in_tail(self, x: torch.Tensor, pre_norm: Optional[nn.LayerNorm] = None) -> torch.Tensor:
        B, L, D = x.shape
        ssm = self.ssm
        Di, N = ssm.d_inner, ssm.state_dim
        p = ssm._prepared()
        u, x = self._norm_conv(x, pre_norm)
        x2 = x.view(B * L, D)
        u = u.view(B * L, D)
        if "w_noz" in p or ("w_noz16" in p and _bf16_compose()):
            w, b = (p["w_noz"], p["b_noz"]) if "w_noz" in p else (p["w_noz16"], p["b_noz16"])
            xbd = ops.gemm(u, w, b, epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=Di + 2 * N)  # [x|B|C|dt]
            xs, bc, dt = xbd[:, :Di], xbd[:, Di:Di + 2 * N], xbd[:, Di + 2 * N:]
        else:
            xs = ops.gemm(u, p["w_x"])                                                 # (M, Di) x
            xdt = ops.gemm(xs, p["w_xdt"], p["b_xdt"], epilogue=_lib.EPI_SOFTPLUS_FROM, n_out=2 * N)  # [B|C|dt]
            bc, dt = xdt[:, :2 * N], xdt[:, 2 * N:]
        mode = _tree_mode()
        yd = ops.ssm_scan_ungated(xs, dt, bc, p["A2"], ssm.D, B, L, mode)
        out = ops.ssm_block_tail_gated(yd, u, p["w_z"], mode, x2, ssm.out_proj.weight, self.norm2.weight,
                                       self.norm2.bias, self.norm2.eps, self.ffn[0].weight, self.ffn[0].bias,
                                       self.ffn[3].weight, self.ffn[3].bias)
        return out.view(B, L, D)

    # The block in three stages -- head (LN1, causal dwconv, projections), the scan, tail (out_proj
    # + residual, LN2, FFN + residual).  (Issuing one utterance group's scans on a stream of their
    # own beside the other group's heads and tails measured slower than independent group
    # streams: profiles/r02_paired/.)
    def head(self, x: torch.Tensor, pre_norm: Optional[nn.LayerNorm] = None):
        """x (B, L, D) -> (x2 = x as (B*L, D) rows, xz, xdt): the scan's operands (pre_norm: forward's)."""
        _check_eval(self)
        B, L, D = x.shape
        u, x = self._norm_conv(x, pre_norm)
        x2 = x.view(B * L, D)
        xz, xdt = self.ssm.project(u.view(B * L, D))
        return x2, xz, xdt

    def tail(self, g: torch.Tensor, x2: torch.Tensor, B: int, L: int) -> torch.Tensor:
        """Gated scan output g (B*L, d_inner) and the block input rows x2 -> block output (B, L, D)."""
        D = x2.shape[1]
        if self._fused_tail_ok(D):
            # out_proj + residual -> LN2 -> FFN1 + GELU -> FFN2 + residual in one kernel:
            # x1 and the FFN intermediate stay on chip
            out = ops.ssm_block_tail(g, x2, self.ssm.out_proj.weight, self.norm2.weight, self.norm2.bias,
                                     self.norm2.eps, self.ffn[0].weight, self.ffn[0].bias, self.ffn[3].weight,
                                     self.ffn[3].bias)
            return out.view(B, L, D)
        x1 = ops.gemm(g, self.ssm.out_proj.weight, epilogue=_lib.EPI_RESIDUAL, aux=x2)
        # norm2 runs inside the FFN-in GEMM's A read (identical float operations)
        f = ops.gemm(x1, self.ffn[0].weight, self.ffn[0].bias, epilogue=_lib.EPI_GELU,
                     ln=(self.norm2.weight, self.norm2.bias, self.norm2.eps))
        out = ops.gemm(f, self.ffn[3].weight, self.ffn[3].bias, epilogue=_lib.EPI_RESIDUAL, aux=x1)
        return out.view(B, L, D)


class LocalSSMProcessor(nn.Module):
    """Stack of SSM blocks + final LayerNorm (reference ssm.py:444-505)."""

    def __init__(self, d_model: int = 192, num_layers: int = 8, state_dim: int = 64, expand_ratio: int = 2,
                 kernel_size: int = 4, dropout: float = 0.1, use_checkpoint: bool = False,
                 scan_mode: ScanMode = "parallel"):
        super().__init__()
        self.layers = nn.ModuleList([
            SSMBlock(d_model=d_model, state_dim=state_dim, expand_ratio=expand_ratio, kernel_size=kernel_size,
                     dropout=dropout, use_checkpoint=use_checkpoint, scan_mode=scan_mode)
            for _ in range(num_layers)
        ])
        self.norm = nn.LayerNorm(d_model)

    def forward(self, x: torch.Tensor, pre_norm: Optional[nn.LayerNorm] = None) -> torch.Tensor:
        """pre_norm (extension): the LayerNorm still to be applied to x, folded into the first
        block's norm1 + conv launch (SSMBlock.forward)."""
        for i, layer in enumerate(self.layers):
            x = layer(x, pre_norm) if i == 0 else layer(x)
        return ops.layer_norm(x, self.norm.weight, self.norm.bias, self.norm.eps)

    def forward_pair(self, x: torch.Tensor, norm2: nn.LayerNorm, pre_norm: Optional[nn.LayerNorm] = None):
        """(forward(x), norm2(forward(x))) with both LayerNorms in one launch (the global context's
        query norm right after this stack's final one, ops.layer_norm_pair): bitwise the same."""
        for i, layer in enumerate(self.layers):
            x = layer(x, pre_norm) if i == 0 else layer(x)
        return ops.layer_norm_pair(x, self.norm.weight, self.norm.bias, self.norm.eps, norm2.weight, norm2.bias,
                                   norm2.eps)


class GlobalSSM(nn.Module):
    """SSM over pooled tokens; always the default 'parallel' scan (reference ssm.py:508-556)."""

    def __init__(self, d_model: int = 192, num_layers: int = 2, state_dim: int = 32, dropout: float = 0.1):
        super().__init__()
        self.layers = nn.ModuleList([
            SSMBlock(d_model=d_model, state_dim=state_dim, expand_ratio=2, kernel_size=4, dropout=dropout)
            for _ in range(num_layers)
        ])
        self.norm = nn.LayerNorm(d_model)

    def forward(self, x: torch.Tensor, raw: bool = False) -> torch.Tensor:
        """raw (extension): the rows before the final LayerNorm (the global context applies it
        inside its second pooling launch)."""
        for layer in self.layers:
            x = layer(x)
        if raw:
            return x
        return ops.layer_norm(x, self.norm.weight, self.norm.bias, self.norm.eps)
