"""Hierarchical pooled global context (drop-in for reference velocity_asr/attention.py).

Pooling, pooled cross-attention and the gated fusion run as HIP kernels: adaptive
average pooling, GEMMs for the projections, a per-(token, head) softmax kernel with the
pooled K/V set in LDS, and the gated fusion as two GEMMs whose second epilogue combines
gate, local and global branches in registers (no (B, L, 2D) concat, no gate tensor in HBM).
"""

from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import _lib, ops
from ._prep import cached
from .ssm import GlobalSSM


class AdaptivePool(nn.Module):
    """Adaptive average pooling + learnable projection (reference attention.py:17-78)."""

    def __init__(self, level: int = 1, d_model: int = 192):
        super().__init__()
        self.level = level
        self.d_model = d_model
        self.pool_proj = nn.Linear(d_model, d_model)

    def _compute_pool_size(self, seq_len: int, prev_pool_size: Optional[int] = None) -> int:
        if self.level == 1:
            return max(64, seq_len // 8)
        k1 = prev_pool_size if prev_pool_size else max(64, seq_len // 8)
        return min(64, max(16, k1 // 4))

    def forward(self, x: torch.Tensor, prev_pool_size: Optional[int] = None) -> Tuple[torch.Tensor, int]:
        B, L, D = x.shape
        pool_size = min(self._compute_pool_size(L, prev_pool_size), L)
        pooled = ops.adaptive_pool(x, pool_size)
        out = ops.gemm(pooled.view(B * pool_size, D), self.pool_proj.weight, self.pool_proj.bias)
        return out.view(B, pool_size, D), pool_size


class MultiHeadAttention(nn.Module):
    """Multi-head attention with a small attention dim (reference attention.py:81-164).

    The HIP core supports the pooled-key regime the model uses (kv_len <= 64, head_dim
    <= 32) and mask=None, which is the only way the reference calls it.
    """

    def __init__(self, d_model: int = 192, num_heads: int = 4, attention_dim: int = 48, dropout: float = 0.1):
        super().__init__()
        self.d_model = d_model
        self.num_heads = num_heads
        self.attention_dim = attention_dim
        self.head_dim = attention_dim // num_heads
        self.q_proj = nn.Linear(d_model, attention_dim)
        self.k_proj = nn.Linear(d_model, attention_dim)
        self.v_proj = nn.Linear(d_model, attention_dim)
        self.out_proj = nn.Linear(attention_dim, d_model)
        self.dropout = nn.Dropout(dropout)
        self.scale = math.sqrt(self.head_dim)

    def _kv_weights(self):
        def build():
            return (torch.cat([self.k_proj.weight, self.v_proj.weight], 0).contiguous(),
                    torch.cat([self.k_proj.bias, self.v_proj.bias], 0).contiguous())
        return cached(self, "kv", (self.k_proj.weight, self.v_proj.weight, self.k_proj.bias, self.v_proj.bias), build)

    def forward(self, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor,
                mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if mask is not None:
            raise NotImplementedError("velocity_asr (MI355X build): attention masks are not supported "
                                      "(the reference path never passes one)")
        B, Lq, D = query.shape
        Kp = key.shape[1]
        A = self.attention_dim
        q = ops.gemm(query.reshape(B * Lq, D), self.q_proj.weight, self.q_proj.bias)
        if key is value:
            w_kv, b_kv = self._kv_weights()
            kv = ops.gemm(key.reshape(B * Kp, D), w_kv, b_kv)
        else:
            kv = torch.empty((B * Kp, 2 * A), device=query.device, dtype=torch.float32)
            ops.gemm(key.reshape(B * Kp, D), self.k_proj.weight, self.k_proj.bias, out=kv[:, :A])
            ops.gemm(value.reshape(B * Kp, D), self.v_proj.weight, self.v_proj.bias, out=kv[:, A:])
        o = ops.pooled_attention(q, kv, B, Lq, Kp, self.num_heads)
        return ops.gemm(o, self.out_proj.weight, self.out_proj.bias).view(B, Lq, D)


class GatedFusion(nn.Module):
    """g * local_proj(local) + (1 - g) * global_proj(global) -> out_proj (reference attention.py:167-220)."""

    def __init__(self, d_model: int = 192):
        super().__init__()
        self.gate_proj = nn.Sequential(nn.Linear(d_model * 2, d_model), nn.Sigmoid())
        self.local_proj = nn.Linear(d_model, d_model)
        self.global_proj = nn.Linear(d_model, d_model)
        self.out_proj = nn.Linear(d_model, d_model)

    def _paired(self):
        """Rows interleaved in 32-row pairs so one wave holds gate and branch of the same column."""
        def build():
            D = self.local_proj.weight.shape[0]
            if D % 32:
                raise NotImplementedError("GatedFusion on HIP needs d_model % 32 == 0")
            Wg = self.gate_proj[0].weight
            bg = self.gate_proj[0].bias

            def pair(a, b):
                return torch.stack([a.reshape(D // 32, 32, *a.shape[1:]), b.reshape(D // 32, 32, *b.shape[1:])],
                                   1).reshape(2 * D, *a.shape[1:]).contiguous()
            w_local = pair(Wg[:, :D], self.local_proj.weight)      # [gate_l | local_proj]
            w_glob = pair(Wg[:, D:], self.global_proj.weight)      # [gate_g | global_proj]
            b_glob = pair(bg, self.global_proj.bias)
            return w_local, w_glob, b_glob
        deps = (self.gate_proj[0].weight, self.gate_proj[0].bias, self.local_proj.weight, self.global_proj.weight,
                self.global_proj.bias)
        return cached(self, "paired", deps, build)

    def forward(self, local_features: torch.Tensor, global_features: torch.Tensor) -> torch.Tensor:
        B, L, D = local_features.shape
        w_local, w_glob, b_glob = self._paired()
        t1 = ops.gemm(local_features.reshape(B * L, D), w_local)
        fused = ops.gemm(global_features.reshape(B * L, D), w_glob, b_glob, epilogue=_lib.EPI_PAIR_FUSION, aux=t1,
                         aux2=self.local_proj.bias, n_out=D)
        return ops.gemm(fused, self.out_proj.weight, self.out_proj.bias).view(B, L, D)


class HierarchicalGlobalContext(nn.Module):
    """pool1 -> GlobalSSM -> pool2 -> norm -> cross-attention -> gated fusion (reference attention.py:223-319)."""

    def __init__(self, d_model: int = 192, num_heads: int = 4, attention_dim: int = 48, global_ssm_layers: int = 2,
                 global_ssm_state_dim: int = 32, dropout: float = 0.1):
        super().__init__()
        self.pool1 = AdaptivePool(level=1, d_model=d_model)
        self.global_ssm = GlobalSSM(d_model=d_model, num_layers=global_ssm_layers, state_dim=global_ssm_state_dim,
                                    dropout=dropout)
        self.pool2 = AdaptivePool(level=2, d_model=d_model)
        self.cross_attention = MultiHeadAttention(d_model=d_model, num_heads=num_heads, attention_dim=attention_dim,
                                                  dropout=dropout)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.fusion = GatedFusion(d_model=d_model)

    def forward(self, local_features: torch.Tensor) -> torch.Tensor:
        x_pool1, pool_size1 = self.pool1(local_features)
        x_ssm = self.global_ssm(x_pool1)
        x_pool2, _ = self.pool2(x_ssm, prev_pool_size=pool_size1)
        x_pool2 = ops.layer_norm(x_pool2, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        query = ops.layer_norm(local_features, self.norm2.weight, self.norm2.bias, self.norm2.eps)
        global_context = self.cross_attention(query=query, key=x_pool2, value=x_pool2)
        return self.fusion(local_features, global_context)
