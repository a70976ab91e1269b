"""Hierarchical pooled global context (drop-in for reference velocity_asr/attention.py).

Pooling, pooled cross-attention and the gated fusion run as HIP kernels: adaptive
average pooling, GEMMs for the projections, a per-(token, head) softmax kernel with the
pooled K/V set in LDS, and the gated fusion as two GEMMs whose second epilogue combines
gate, local and global branches in registers (no (B, L, 2D) concat, no gate tensor in HBM).
"""

from __future__ import annotations

import math
import os
from typing import Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import _lib, ops
from . import quantize as Q
from ._prep import cached
from .ssm import GlobalSSM


def _device_ints(values: Sequence[int], device) -> torch.Tensor:
    """Host sizes -> the int32 (B,) device array the _var kernels read."""
    return torch.tensor([int(v) for v in values], dtype=torch.int32).to(device)


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

    def forward(self, x: torch.Tensor, prev_pool_size=None, lengths: Optional[Sequence[int]] = None,
                pre_norm: Optional[nn.LayerNorm] = None):
        """(B, L, D) -> ((B, K, D), K).  lengths: per-utterance valid rows of a zero-padded batch
        (prev_pool_size then per utterance too): each utterance is pooled to the size it gets
        alone, rows past it are junk nobody reads, and the sizes are returned as a list.
        pre_norm (extension): x is the row before that LayerNorm, applied inside the pooling launch
        (ops.ln_adaptive_pool), bitwise the same as pooling pre_norm(x)."""
        B, L, D = x.shape

        def pool(K, lens=None, ks=None):
            if pre_norm is None:
                return ops.adaptive_pool(x, K, lens=lens, ks=ks)
            return ops.ln_adaptive_pool(x, pre_norm.weight, pre_norm.bias, pre_norm.eps, K, lens=lens, ks=ks)
        if lengths is None:
            pool_size = min(self._compute_pool_size(L, prev_pool_size), L)
            pooled = pool(pool_size)
        else:
            prev = prev_pool_size if prev_pool_size is not None else [None] * B
            sizes = [min(self._compute_pool_size(n, p), n) for n, p in zip(lengths, prev)]
            pool_size = max(sizes)
            pooled = pool(pool_size, lens=_device_ints(lengths, x.device), ks=_device_ints(sizes, x.device))
        w, b, qp = Q.linear_parts(self.pool_proj)
        out = ops.gemm(pooled.view(B * pool_size, D), w, b, qparams=qp)
        Q.record(self.pool_proj, out)
        return out.view(B, pool_size, D), (pool_size if lengths is None else sizes)


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
        """[k_proj; v_proj] as one GEMM: weights, biases and (if either is quantized) the
        per-column activation fake-quant of both halves."""
        def build():
            A = self.attention_dim
            w = torch.cat([Q.effective_weight(self.k_proj), Q.effective_weight(self.v_proj)], 0).contiguous()
            b = torch.cat([Q.inner(self.k_proj).bias, Q.inner(self.v_proj).bias], 0).contiguous()
            qk, qv = Q.act_qparams(self.k_proj, A), Q.act_qparams(self.v_proj, A)
            qp = None
            if qk is not None or qv is not None:
                qp = torch.cat([Q.act_qparams_or_identity(self.k_proj, A, w.device),
                                Q.act_qparams_or_identity(self.v_proj, A, w.device)], 0).contiguous()
            return w, b, qp
        return cached(self, "kv", Q.deps(self.k_proj) + Q.deps(self.v_proj), build)

    def forward(self, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor,
                mask: Optional[torch.Tensor] = None, key_lengths: Optional[Sequence[int]] = None,
                project_out: bool = True) -> torch.Tensor:
        """key_lengths: per-utterance valid keys of a padded (B, Kp, D) key set.  project_out=False:
        the (B * Lq, attention_dim) head outputs before out_proj (GatedFusion.forward_attention
        folds out_proj into its global-branch product)."""
        if mask is not None:
            raise NotImplementedError("velocity_asr (MI355X build): attention masks are not supported "
                                      "(the reference path never passes one)")
        B, Lq, D = query.shape
        Kp = key.shape[1]
        A = self.attention_dim
        wq, bq, qpq = Q.linear_parts(self.q_proj)
        q = ops.gemm(query.reshape(B * Lq, D), wq, bq, qparams=qpq)
        Q.record(self.q_proj, q)
        if key is value:
            w_kv, b_kv, qp_kv = self._kv_weights()
            kv = ops.gemm(key.reshape(B * Kp, D), w_kv, b_kv, qparams=qp_kv)
        else:
            kv = torch.empty((B * Kp, 2 * A), device=query.device, dtype=torch.float32)
            for mod, src, sl in ((self.k_proj, key, slice(0, A)), (self.v_proj, value, slice(A, 2 * A))):
                w, b, qp = Q.linear_parts(mod)
                ops.gemm(src.reshape(B * Kp, D), w, b, out=kv[:, sl], qparams=qp)
        Q.record(self.k_proj, kv[:, :A])
        Q.record(self.v_proj, kv[:, A:])
        o = ops.pooled_attention(q, kv, B, Lq, Kp, self.num_heads,
                                 kps=None if key_lengths is None else _device_ints(key_lengths, q.device))
        if not project_out:
            return o
        wo, bo, qpo = Q.linear_parts(self.out_proj)
        out = ops.gemm(o, wo, bo, qparams=qpo)
        Q.record(self.out_proj, out)
        return out.view(B, Lq, D)


class GatedFusion(nn.Module):
    """g * local_proj(local) + (1 - g) * global_proj(global) -> out_proj (reference attention.py:167-220)."""

    def __init__(self, d_model: int = 192):
        super().__init__()
        self.gate_proj = nn.Sequential(nn.Linear(d_model * 2, d_model), nn.Sigmoid())
        self.local_proj = nn.Linear(d_model, d_model)
        self.global_proj = nn.Linear(d_model, d_model)
        self.out_proj = nn.Linear(d_model, d_model)

    def _paired(self):
        """Rows interleaved in 32-row pairs so one wave holds gate and branch of the same column
        (weights, biases and, for quantized layers, the epilogue's activation fake-quant)."""
        gate, loc, glob = self.gate_proj[0], self.local_proj, self.global_proj

        def build():
            D = Q.inner(loc).weight.shape[0]
            if D % 32:
                raise NotImplementedError("GatedFusion on HIP needs d_model % 32 == 0")
            Wg = Q.effective_weight(gate)
            bg = Q.inner(gate).bias

            def pair(a, b):
                return torch.stack([a.reshape(D // 32, 32, *a.shape[1:]), b.reshape(D // 32, 32, *b.shape[1:])],
                                   1).reshape(2 * D, *a.shape[1:]).contiguous()
            w_local = pair(Wg[:, :D], Q.effective_weight(loc))      # [gate_l | local_proj]
            w_glob = pair(Wg[:, D:], Q.effective_weight(glob))      # [gate_g | global_proj]
            b_glob = pair(bg, Q.inner(glob).bias)
            qp = None
            if any(Q.act_qparams(m, D) is not None for m in (gate, loc, glob)):
                dev = Wg.device
                qp = torch.cat([pair(Q.act_qparams_or_identity(gate, D, dev), Q.act_qparams_or_identity(glob, D, dev)),
                                Q.act_qparams_or_identity(loc, D, dev)], 0).contiguous()
            return w_local, w_glob, b_glob, qp
        return cached(self, "paired", Q.deps(gate) + Q.deps(loc) + Q.deps(glob), build)

    def _paired_attention(self, mha: "MultiHeadAttention"):
        """The global branch with the attention's out_proj folded in: global_context = o Wo^T + bo
        feeds only this product, so [gate_g | global_proj] (o Wo^T + bo) + b = o ([gate_g |
        global_proj] Wo)^T + ([gate_g | global_proj] bo + b), the composite formed in float64 and
        rounded once (as the SSM's composed projection): K = attention_dim (48) instead of d_model,
        and no (B * L, d_model) global_context in HBM."""
        _, w_glob, b_glob, _ = self._paired()

        def build():
            wo, bo = mha.out_proj.weight, mha.out_proj.bias
            w = (w_glob.detach().double() @ wo.detach().double()).to(w_glob.dtype).contiguous()
            b = (ops.f32(b_glob).double() + w_glob.detach().double() @ ops.f32(bo).detach().double()).float().contiguous()
            return w, b
        return cached(self, "paired_attn", (w_glob, b_glob, mha.out_proj.weight, mha.out_proj.bias), build)

    def composable(self, mha: "MultiHeadAttention") -> bool:
        """forward_attention applies: plain Linears (no QAT fake-quant on global_context or the
        fusion's inputs), one weight dtype; VASR_ATTN_COMPOSE=0 keeps the separate out_proj."""
        mods = (mha.out_proj, self.gate_proj[0], self.local_proj, self.global_proj, self.out_proj)
        return (os.environ.get("VASR_ATTN_COMPOSE", "1") != "0" and all(type(m) is nn.Linear for m in mods)
                and len({m.weight.dtype for m in mods}) == 1 and mha.out_proj.bias is not None)

    def forward_attention(self, local_features: torch.Tensor, o: torch.Tensor,
                          mha: "MultiHeadAttention") -> torch.Tensor:
        """forward(local_features, mha's output) from the attention's head outputs o (B * L, A)."""
        B, L, D = local_features.shape
        local2 = local_features.reshape(B * L, D)
        w_local, _, _, qp = self._paired()
        w_glob, b_glob = self._paired_attention(mha)
        t1 = ops.gemm(local2, w_local)
        fused = ops.gemm(o, w_glob, b_glob, epilogue=_lib.EPI_PAIR_FUSION, aux=t1,
                         aux2=self.local_proj.bias, n_out=D, qparams=qp)
        out = ops.gemm(fused, self.out_proj.weight, self.out_proj.bias)
        return out.view(B, L, D)

    def _observe(self, local2: torch.Tensor, glob2: torch.Tensor) -> None:
        """Calibration only: the raw (pre-quantizer) gate / local / global outputs, summed in
        the fused epilogue's order ((local part + global part) + bias for the gate)."""
        gate, loc, glob = self.gate_proj[0], self.local_proj, self.global_proj
        D = local2.shape[1]
        Wg = Q.effective_weight(gate)
        if Q.observing(gate):
            t = ops.gemm(local2, Wg[:, :D].contiguous())
            Q.record(gate, ops.gemm(glob2, Wg[:, D:].contiguous(), epilogue=_lib.EPI_RESIDUAL, aux=t)
                     + Q.inner(gate).bias.detach())
        for mod, src in ((loc, local2), (glob, glob2)):
            if Q.observing(mod):
                Q.record(mod, ops.gemm(src, Q.effective_weight(mod), Q.inner(mod).bias))

    def forward(self, local_features: torch.Tensor, global_features: torch.Tensor) -> torch.Tensor:
        B, L, D = local_features.shape
        local2, glob2 = local_features.reshape(B * L, D), global_features.reshape(B * L, D)
        self._observe(local2, glob2)
        w_local, w_glob, b_glob, qp = self._paired()
        t1 = ops.gemm(local2, w_local)
        fused = ops.gemm(glob2, w_glob, b_glob, epilogue=_lib.EPI_PAIR_FUSION, aux=t1,
                         aux2=Q.inner(self.local_proj).bias, n_out=D, qparams=qp)
        wo, bo, qpo = Q.linear_parts(self.out_proj)
        out = ops.gemm(fused, wo, bo, qparams=qpo)
        Q.record(self.out_proj, out)
        return out.view(B, L, D)


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

    def forward(self, local_features: torch.Tensor, lengths: Optional[Sequence[int]] = None,
                query: Optional[torch.Tensor] = None) -> torch.Tensor:
        """lengths: per-utterance token counts of a zero-padded batch (None: all L).  Pooling
        sizes and attention keys then follow each utterance's own length; the global SSM is
        causal, so the junk rows past an utterance's pooled tokens never reach them.
        query (extension): norm2(local_features) when the caller already has it
        (LocalSSMProcessor.forward_pair)."""
        x_pool1, pool_size1 = self.pool1(local_features, lengths=lengths)
        # VASR_POOL_PRENORM=1: the global stack's final LayerNorm inside the second pooling launch.
        # Bitwise the same, and 3.5 vs 5.3 us graph-timed alone at C2's 32 x 64 -> 16 rows, but C2
        # 0.3 % slower in the model's graph over three interleaved rounds (profiles/r06bh/, r06bi/):
        # off by default
        gnorm = self.global_ssm.norm
        fold = os.environ.get("VASR_POOL_PRENORM", "0") == "1" and type(gnorm) is nn.LayerNorm
        x_ssm = self.global_ssm(x_pool1, raw=fold)
        x_pool2, pool_size2 = self.pool2(x_ssm, prev_pool_size=pool_size1,
                                         lengths=None if lengths is None else pool_size1,
                                         pre_norm=gnorm if fold else None)
        x_pool2 = ops.layer_norm(x_pool2, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        if query is None:
            query = ops.layer_norm(local_features, self.norm2.weight, self.norm2.bias, self.norm2.eps)
        kl = None if lengths is None else pool_size2
        if self.fusion.composable(self.cross_attention):
            o = self.cross_attention(query=query, key=x_pool2, value=x_pool2, key_lengths=kl, project_out=False)
            return self.fusion.forward_attention(local_features, o, self.cross_attention)
        global_context = self.cross_attention(query=query, key=x_pool2, value=x_pool2, key_lengths=kl)
        return self.fusion(local_features, global_context)
