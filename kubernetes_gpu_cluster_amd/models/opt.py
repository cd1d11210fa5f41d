"""OPT (facebook/opt-125m, reference ``values-01-minimal-example.yaml:7``; BASELINE
config 1, the CPU plumbing pod).  Pre-LN decoder, learned positions with offset 2,
MHA without RoPE, biases everywhere, ReLU MLP, tied LM head.  On GPU the KV write
runs through rope_kv_write with use_rope=False and LayerNorm through the HIP
layer_norm kernel (K8)."""
from __future__ import annotations

import re
from typing import Iterable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..parallel.layers import (ColumnParallelLinear, ParallelLMHead, QKVParallelLinear,
                               RowParallelLinear, VocabParallelEmbedding)
from ..parallel.state import get_state
from .attention import ForwardContext, PagedAttention
from .configs import ModelConfig


class LayerNorm(nn.Module):
    def __init__(self, n, dtype, device):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n, dtype=dtype, device=device), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(n, dtype=dtype, device=device), requires_grad=False)

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, 1e-5)


class OPTLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, idx: int, dtype, device):
        super().__init__()
        self.cfg = cfg
        self.qkv_proj = QKVParallelLinear(cfg.hidden_size, cfg.head_dim, cfg.num_heads,
                                          cfg.num_kv_heads, bias=True, dtype=dtype, device=device)
        self.out_proj = RowParallelLinear(cfg.hidden_size, cfg.hidden_size, bias=True, dtype=dtype,
                                          device=device)
        self.attn = PagedAttention(self.qkv_proj.nq, self.qkv_proj.nkv, cfg.head_dim, idx)
        self.self_attn_layer_norm = LayerNorm(cfg.hidden_size, dtype, device)
        self.final_layer_norm = LayerNorm(cfg.hidden_size, dtype, device)
        self.fc1 = ColumnParallelLinear(cfg.hidden_size, cfg.intermediate_size, bias=True,
                                        dtype=dtype, device=device)
        self.fc2 = RowParallelLinear(cfg.intermediate_size, cfg.hidden_size, bias=True,
                                     dtype=dtype, device=device)

    def forward(self, positions, x, ctx: ForwardContext):
        h = self.self_attn_layer_norm(x)
        qkv = self.qkv_proj(h)
        kc, vc = ctx.kv_caches[self.attn.layer_idx]
        q = ops.rope_kv_write(qkv, positions, ctx.cos_sin, kc, vc, ctx.attn.slot_mapping,
                              self.qkv_proj.nq, self.qkv_proj.nkv, self.cfg.head_dim,
                              use_rope=False, k_scale=ctx.k_scale, v_scale=ctx.v_scale)
        x = x + self.out_proj(self.attn(q, ctx))
        h = self.final_layer_norm(x)
        return x + self.fc2(F.relu(self.fc1(h)))


class OPTForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=torch.float16, device=None):
        super().__init__()
        s = get_state()
        assert s.pp_size == 1, "OPT: pipeline parallel not supported"
        self.cfg, self.dtype = cfg, dtype
        self.start, self.end = 0, cfg.num_layers
        self.first = self.last = True
        self.embed_tokens = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, dtype, device)
        self.embed_positions = nn.Parameter(
            torch.empty(cfg.max_position + cfg.pos_offset, cfg.hidden_size, dtype=dtype,
                        device=device), requires_grad=False)
        self.layers = nn.ModuleList([OPTLayer(cfg, i, dtype, device) for i in range(cfg.num_layers)])
        self.final_layer_norm = LayerNorm(cfg.hidden_size, dtype, device)
        self.lm_head = ParallelLMHead(cfg.vocab_size, cfg.hidden_size, dtype, device,
                                      tied=self.embed_tokens)

    @property
    def num_local_layers(self):
        return len(self.layers)

    def local_kv_heads(self):
        return self.layers[0].qkv_proj.nkv

    def forward(self, input_ids, positions, ctx, hidden=None, residual=None):
        x = self.embed_tokens(input_ids) + self.embed_positions[positions + self.cfg.pos_offset]
        for layer in self.layers:
            x = layer(positions, x, ctx)
        return self.final_layer_norm(x)

    def compute_logits(self, hidden, gather: bool = True):
        return self.lm_head(hidden, gather)

    def load_weights(self, weights: Iterable[tuple[str, torch.Tensor]]) -> int:
        n = 0
        for name, w in weights:
            name = name.replace("model.decoder.", "decoder.")
            if name == "decoder.embed_tokens.weight":
                self.embed_tokens.weight.weight_loader(self.embed_tokens.weight, w.to(self.dtype))
            elif name == "decoder.embed_positions.weight":
                self.embed_positions.data.copy_(w[: self.embed_positions.shape[0]])
            elif name.startswith("decoder.final_layer_norm."):
                getattr(self.final_layer_norm, name.split(".")[-1]).data.copy_(w)
            else:
                m = re.match(r"decoder\.layers\.(\d+)\.(.*)", name)
                if not m:
                    continue
                L = self.layers[int(m.group(1))]
                rest = m.group(2)
                kind = rest.split(".")[-1]
                mm = re.match(r"self_attn\.([qkv])_proj\.", rest)
                if mm:
                    p = L.qkv_proj.weight if kind == "weight" else L.qkv_proj.bias
                    L.qkv_proj._load(p, w.to(self.dtype), mm.group(1))
                elif rest.startswith("self_attn.out_proj."):
                    p = getattr(L.out_proj, kind)
                    p.weight_loader(p, w.to(self.dtype)) if hasattr(p, "weight_loader") else p.data.copy_(w)
                elif rest.startswith(("fc1.", "fc2.")):
                    mod = getattr(L, rest.split(".")[0])
                    p = getattr(mod, kind)
                    p.weight_loader(p, w.to(self.dtype))
                elif rest.startswith(("self_attn_layer_norm.", "final_layer_norm.")):
                    getattr(getattr(L, rest.split(".")[0]), kind).data.copy_(w)
                else:
                    continue
            n += 1
        return n
