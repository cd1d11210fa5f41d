"""Paged attention layer + the per-step forward context.

A step's tokens are laid out prefill-chunks first, then one token per decoding
sequence (``AttnMetadata``).  The attention layer splits ``q`` accordingly and
runs the prefill kernel (K2) on the first part and the split-context decode
kernel (K1) on the rest, both reading the layer's paged KV cache, after the
fused RoPE + KV-write kernel (K3/K5/K6) has stored the step's new keys/values.
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import torch
import torch.nn as nn

from .. import ops


@dataclasses.dataclass
class AttnMetadata:
    slot_mapping: torch.Tensor                     # [T] int64, -1 = padding
    num_prefill_tokens: int = 0
    num_prefills: int = 0
    num_decodes: int = 0
    # prefill part (sequence i: query rows [qsl[i], qsl[i+1]) of the prefill tokens)
    prefill_block_tables: Optional[torch.Tensor] = None   # [P, max_blocks] int32
    query_start_loc: Optional[torch.Tensor] = None        # [P+1] int32
    prefill_seq_lens: Optional[torch.Tensor] = None       # [P] int32 (context incl. chunk)
    work_seq: Optional[torch.Tensor] = None
    work_mblk: Optional[torch.Tensor] = None
    # decode part
    decode_block_tables: Optional[torch.Tensor] = None    # [D, max_blocks] int32
    decode_ctx_lens: Optional[torch.Tensor] = None        # [D] int32
    decode_grid_z: int = 1
    decode_workspace: Optional[tuple] = None
    # prefill-only TP step split into two token halves for comm/compute overlap:
    # (a, meta of tokens [0, a), meta of tokens [a, T)) -- engine/model_runner.py
    split: Optional[tuple] = None


@dataclasses.dataclass
class ForwardContext:
    attn: AttnMetadata
    kv_caches: list                                    # per local layer: (k_cache, v_cache)
    cos_sin: Optional[torch.Tensor] = None
    k_scale: float = 1.0                               # fp8 KV: cache holds fp8(x / scale)
    v_scale: float = 1.0


class PagedAttention(nn.Module):
    def __init__(self, num_heads: int, num_kv_heads: int, head_dim: int, layer_idx: int,
                 scale: Optional[float] = None):
        super().__init__()
        self.nq, self.nkv, self.d = num_heads, num_kv_heads, head_dim
        self.layer_idx = layer_idx
        self.scale = head_dim ** -0.5 if scale is None else scale

    def forward(self, q: torch.Tensor, ctx: ForwardContext) -> torch.Tensor:
        """q [T, nq, d] (rotated, K/V already in cache) -> [T, nq*d]."""
        m = ctx.attn
        kc, vc = ctx.kv_caches[self.layer_idx]
        out = torch.empty_like(q)
        tp = m.num_prefill_tokens
        if tp:
            o = ops.prefill_attention(q[:tp], kc, vc, m.prefill_block_tables, m.query_start_loc,
                                      m.prefill_seq_lens, self.scale, m.work_seq, m.work_mblk,
                                      out=out[:tp], k_scale=ctx.k_scale, v_scale=ctx.v_scale)
            if o.data_ptr() != out.data_ptr():
                out[:tp].copy_(o)
        if m.num_decodes:
            dst = out[tp:tp + m.num_decodes]
            o = ops.paged_attention_decode(q[tp:tp + m.num_decodes], kc, vc,
                                           m.decode_block_tables, m.decode_ctx_lens, self.scale,
                                           m.decode_workspace, m.decode_grid_z, out=dst,
                                           k_scale=ctx.k_scale, v_scale=ctx.v_scale)
            if o.data_ptr() != dst.data_ptr():
                dst.copy_(o)
        return out.view(q.shape[0], self.nq * self.d)
