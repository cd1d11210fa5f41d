"""Llama-family decoder: Llama-3 (8B/70B), Mistral, Qwen2/2.5, Qwen3 (q/k norm),
Qwen v1 (fused c_attn, ``--trust-remote-code`` arch) and Mixtral (MoE).

Per layer:
  fused_add_rms_norm (K4) -> QKV GEMM -> rope_kv_write (K3/K5/K6) -> paged attention
  (K1/K2) -> O GEMM (+TP all-reduce C1) -> fused_add_rms_norm -> gate_up GEMM ->
  silu_mul (K7) -> down GEMM (+TP all-reduce C2)   |  MoE: router -> topk-softmax (K13)
  -> grouped expert MLP (K14) (+ all-reduce / all-to-all)
Pipeline stages own a contiguous slice of layers; the first stage owns the
embedding, the last the final norm and the LM head.
"""
from __future__ import annotations

import dataclasses
import os
import re
from typing import Iterable, Optional

import torch
import torch.nn as nn

from .. import ops
from ..ops import gemm
from ..parallel import comm
from ..parallel.layers import (MergedColumnParallelLinear, ParallelLMHead, QKVParallelLinear,
                               ReplicatedLinear, RowParallelLinear, VocabParallelEmbedding)
from ..parallel.state import get_state
from .attention import ForwardContext, PagedAttention
from .configs import ModelConfig
from .moe import MoEBlock


def pp_layer_range(num_layers: int, pp_size: int, pp_rank: int) -> tuple[int, int]:
    per = num_layers // pp_size
    extra = num_layers % pp_size
    start = pp_rank * per + min(pp_rank, extra)
    return start, start + per + (1 if pp_rank < extra else 0)


_tail_fusion_enabled = os.environ.get("KGC_TAIL_FUSION", "1") != "0"
# TP > 1: all-reduce fused with the residual add + RMSNorm after o / down (KGC_TP_AR_NORM=0: off)
_tp_ar_norm_enabled = os.environ.get("KGC_TP_AR_NORM", "1") != "0"
# small M on one GPU: the decoder layer without RMSNorm launches (KGC_RS_LAYER=0: off)
_rs_enabled = os.environ.get("KGC_RS_LAYER", "1") != "0"
# (Removed in round 6, measured slower and off by default: the norm-free mid-M layer --
# K9m's fan-in epilogue doing the o / down split-K combine + residual add + row norms in the
# GEMM launch, profiles/k9m_fanin_vs_tail_r5.jsonl -- and two-stream prefill,
# profiles/engine_ab_prefill_two_streams_r4.jsonl.  Last present at commit 4d8a38e.)
# decode-only steps: RoPE + KV write folded into the paged-decode kernel (KGC_DECODE_ROPE_FUSED=0: off)
_decode_rope_fused = os.environ.get("KGC_DECODE_ROPE_FUSED", "1") != "0"
# prefill-only steps of RoPE models without q/k norm: K2 rotates q as it loads it from the
# QKV row and the k / v write runs alone (8-token-group kernel, rope_cache.hip
# kv_group_kernel), so q is never written or re-read.  KGC_PREFILL_ROPE_FUSED=0: off.
# Round 3 kept it off (profiles/engine_ab_prefill_rope_fused_same_box.jsonl: K2 1.0 ms per
# 16K-token chunk slower, the per-token k / v write only 0.36 ms faster); the group kernel
# takes the k / v write from 91 to 24 us per layer (profiles/prefill_rope_kvg_r4.jsonl).
_prefill_rope_fused = os.environ.get("KGC_PREFILL_ROPE_FUSED", "1") == "1"


class RMSNorm(nn.Module):
    def __init__(self, n: int, eps: float, dtype, device):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n, dtype=dtype, device=device), requires_grad=False)
        self.eps = eps

    def forward(self, x, residual=None):
        if residual is None:
            return ops.rms_norm(x, self.weight, self.eps)
        return ops.fused_add_rms_norm(x, residual, self.weight, self.eps)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int, dtype, device):
        super().__init__()
        self.cfg = cfg
        self.qkv_proj = QKVParallelLinear(cfg.hidden_size, cfg.head_dim, cfg.num_heads,
                                          cfg.num_kv_heads, bias=cfg.qkv_bias, dtype=dtype,
                                          device=device)
        self.nq, self.nkv = self.qkv_proj.nq, self.qkv_proj.nkv
        self.o_proj = RowParallelLinear(cfg.num_heads * cfg.head_dim, cfg.hidden_size,
                                        bias=cfg.o_bias, dtype=dtype, device=device)
        if cfg.qk_norm:
            self.q_norm = RMSNorm(cfg.head_dim, cfg.rms_eps, dtype, device)
            self.k_norm = RMSNorm(cfg.head_dim, cfg.rms_eps, dtype, device)
        else:
            self.q_norm = self.k_norm = None
        self.attn = PagedAttention(self.nq, self.nkv, cfg.head_dim, layer_idx)

    def forward(self, positions, x, ctx: ForwardContext):
        return self.o_proj(self.attend(positions, self.project_qkv(x), ctx))

    @staticmethod
    def _scaled_rows(qkv, row_scale, dtype):
        """The norm-free layer's QKV where no fused decode kernel applies its row scale:
        (summed K-slices of) the projection times rsqrt(mean(x^2) + eps), rounded."""
        y = qkv.sum(0) if qkv.dim() == 3 else qkv.float()
        return (y * row_scale[:, None]).to(dtype)

    def project_qkv(self, x):
        """The QKV projection; where the decode plan runs it as K9m split-K, the fp32
        K-slices themselves (the RoPE / KV-write kernel sums them, ops/gemm.py linear_qkv)."""
        p = self.qkv_proj
        if p.bias is None and x.is_cuda:
            return gemm.linear_qkv(x, p.weight)
        return p(x)

    def attend(self, positions, qkv, ctx: ForwardContext, row_scale=None):
        """RoPE + KV-cache write + paged attention on a QKV projection -> [T, nq*d].
        ``row_scale`` [T] fp32: the norm-free layer's per-row rsqrt(mean(x^2) + eps) of a
        projection computed on the raw residual with gamma folded into the weight."""
        kc, vc = ctx.kv_caches[self.attn.layer_idx]
        m = ctx.attn
        if (_decode_rope_fused and qkv.is_cuda and not m.num_prefill_tokens and m.num_decodes
                and m.num_decodes == (qkv.shape[1] if qkv.dim() == 3 else qkv.shape[0])):
            # decode-only step: RoPE / q-k norm / KV write run inside the decode kernel
            o = ops.paged_attention_decode_rope(
                qkv, positions, ctx.cos_sin, kc, vc, m.slot_mapping, self.nq, self.nkv,
                self.cfg.head_dim, m.decode_block_tables, m.decode_ctx_lens, self.attn.scale,
                None if self.q_norm is None else self.q_norm.weight,
                None if self.k_norm is None else self.k_norm.weight, self.cfg.rms_eps,
                workspace=m.decode_workspace, grid_z=m.decode_grid_z, k_scale=ctx.k_scale,
                v_scale=ctx.v_scale, dtype=self.qkv_proj.weight.dtype, row_scale=row_scale)
            return o.view(o.shape[0], self.nq * self.cfg.head_dim)
        if row_scale is not None:
            qkv = self._scaled_rows(qkv, row_scale, self.qkv_proj.weight.dtype)
        if (_prefill_rope_fused and qkv.is_cuda and qkv.dim() == 2 and m.num_prefill_tokens
                and not m.num_decodes and self.q_norm is None and self.k_norm is None
                and m.num_prefill_tokens == qkv.shape[0]):
            ops.kv_write_rope(qkv, positions, ctx.cos_sin, kc, vc, m.slot_mapping, self.nq,
                              self.nkv, self.cfg.head_dim, k_scale=ctx.k_scale,
                              v_scale=ctx.v_scale)
            o = ops.prefill_attention_rope(
                qkv, ctx.cos_sin, kc, vc, m.prefill_block_tables, m.query_start_loc,
                m.prefill_seq_lens, self.attn.scale, self.nq, self.cfg.head_dim, m.work_seq,
                m.work_mblk, k_scale=ctx.k_scale, v_scale=ctx.v_scale)
            return o.view(o.shape[0], self.nq * self.cfg.head_dim)
        q = ops.rope_kv_write(qkv, positions, ctx.cos_sin, kc, vc, ctx.attn.slot_mapping,
                              self.nq, self.nkv, self.cfg.head_dim,
                              None if self.q_norm is None else self.q_norm.weight,
                              None if self.k_norm is None else self.k_norm.weight,
                              self.cfg.rms_eps, k_scale=ctx.k_scale, v_scale=ctx.v_scale,
                              dtype=self.qkv_proj.weight.dtype)
        return self.attn(q, ctx)


class LlamaMLP(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        self.gate_up_proj = MergedColumnParallelLinear(cfg.hidden_size, [cfg.intermediate_size] * 2,
                                                       dtype=dtype, device=device)
        self.down_proj = RowParallelLinear(cfg.intermediate_size, cfg.hidden_size, dtype=dtype,
                                           device=device)

    def forward(self, x):
        # gate_up -> silu_mul, fused into the split-K reduction where that runs (ops/gemm.py)
        gu = self.gate_up_proj
        return self.down_proj(gemm.linear_silu(x, gu.weight, gu.bias))


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int, dtype, device):
        super().__init__()
        self.self_attn = LlamaAttention(cfg, layer_idx, dtype, device)
        self.mlp = MoEBlock(cfg, dtype, device) if cfg.is_moe else LlamaMLP(cfg, dtype, device)
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_eps, dtype, device)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_eps, dtype, device)

    def forward(self, positions, x, residual, ctx):
        if residual is None:
            residual = x
            x = self.input_layernorm(x)
        else:
            x, residual = self.input_layernorm(x, residual)
        x = self.self_attn(positions, x, ctx)
        x, residual = self.post_attention_layernorm(x, residual)
        return self.mlp(x), residual


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        self.dtype = dtype
        s = get_state()
        self.start, self.end = pp_layer_range(cfg.num_layers, s.pp_size, s.pp_rank)
        self.first, self.last = s.is_first_pp, s.is_last_pp
        self.embed_tokens = (VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, dtype, device)
                             if self.first or (self.last and cfg.tie_embeddings) else None)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, i - self.start, dtype, device)
                                     for i in range(self.start, self.end)])
        if self.last:
            self.norm = RMSNorm(cfg.hidden_size, cfg.rms_eps, dtype, device)
            tied = self.embed_tokens if cfg.tie_embeddings else None
            self.lm_head = ParallelLMHead(cfg.vocab_size, cfg.hidden_size, dtype, device, tied)
        else:
            self.norm = self.lm_head = None

    @property
    def num_local_layers(self) -> int:
        return self.end - self.start

    @property
    def graph_safe(self) -> bool:
        """False when a layer synchronises with the host (MoE ep mode / uncovered dims)."""
        return all(getattr(l.mlp, "graph_safe", True) for l in self.layers)

    def local_kv_heads(self) -> int:
        return self.layers[0].self_attn.nkv if len(self.layers) else 0

    def forward(self, input_ids: Optional[torch.Tensor], positions: torch.Tensor,
                ctx: ForwardContext, hidden: Optional[torch.Tensor] = None,
                residual: Optional[torch.Tensor] = None):
        """First stage: input_ids -> ...; later stages take (hidden, residual) from the
        previous stage.  Returns the final-normed hidden on the last stage, else
        (hidden, residual) for the next stage."""
        if hidden is None and residual is None:
            rs = self._rs_cfgs(input_ids.shape[0])
            if rs is not None:
                return self._forward_rs(input_ids, positions, ctx, rs)
            cfgs = self._fused_cfgs(input_ids.shape[0])
            if cfgs is not None:
                return self._forward_fused(input_ids, positions, ctx, cfgs)
        x = self.embed_tokens(input_ids) if self.first else hidden
        if self._tail_fusable(x):
            return self._forward_tail_fused(positions, x, ctx)
        if self._tp_tail_fusable():
            if ctx.attn.split is not None:
                return self._forward_tp_overlap(positions, x, ctx)
            return self._forward_tp_fused(positions, x, ctx)
        for layer in self.layers:
            x, residual = layer(positions, x, residual, ctx)
        if not self.last:
            return x, residual
        if residual is None:
            return self.norm(x)
        x, _ = self.norm(x, residual)
        return x

    # ------------------------------------------------------------------ fused projection tails
    def _tail_fusable(self, x) -> bool:
        """One GPU, whole model, dense bias-free MLP / o_proj, and a fused-tail plan at this
        M (K9m split-K, or K9 SK_ACC_NORM at small M): the o / down projections then run
        with their reduction / residual add fused into the next norm."""
        if not (x.is_cuda and self.first and self.last and self.layers
                and get_state().tp_size == 1 and gemm.tail_plan_has_m(x.shape[0])
                and _tail_fusion_enabled):
            return False
        l0 = self.layers[0]
        if self.cfg.is_moe:
            # MoE (TP = 1): o_proj's tail is fused; the MoE block's output meets the next
            # norm through fused_add_rms_norm
            return l0.self_attn.o_proj.bias is None
        return (l0.self_attn.o_proj.bias is None and l0.mlp.down_proj.bias is None
                and l0.mlp.gate_up_proj.bias is None)

    def _forward_tail_fused(self, positions, x, ctx):
        """The regular layer loop with each row-parallel projection handed to the norm that
        consumes it (``gemm.linear_add_rms``): o_proj -> post-attention norm, down_proj ->
        the next layer's input norm (the last one -> the final norm).  Same math and
        rounding points as ``LlamaDecoderLayer.forward``."""
        residual, h, prev = x, None, None
        moe = self.cfg.is_moe
        for layer in self.layers:
            ln1 = layer.input_layernorm
            if prev is None:
                x = ln1(x)
            elif moe:
                x, residual = ln1(h, residual)
            else:
                x, residual = gemm.linear_add_rms(h, prev.mlp.down_proj.weight, residual,
                                                  ln1.weight, ln1.eps)
            at, ln2 = layer.self_attn, layer.post_attention_layernorm
            a = at.attend(positions, at.project_qkv(x), ctx)
            x, residual = gemm.linear_add_rms(a, at.o_proj.weight, residual, ln2.weight, ln2.eps)
            h = layer.mlp(x) if moe else gemm.linear_silu(x, layer.mlp.gate_up_proj.weight)
            prev = layer
        if moe:
            x, _ = self.norm(h, residual)
            return x
        x, _ = gemm.linear_add_rms(h, prev.mlp.down_proj.weight, residual, self.norm.weight,
                                   self.norm.eps)
        return x

    def _tp_tail_fusable(self) -> bool:
        """TP > 1, whole model, dense bias-free o / down projections: each row-parallel
        projection's all-reduce runs fused with the residual add + RMSNorm that consumes
        it (``comm.tp_all_reduce_add_rms``: the xGMI kernel at decode sizes)."""
        if not (get_state().tp_size > 1 and self.first and self.last and self.layers
                and not self.cfg.is_moe and _tp_ar_norm_enabled):
            return False
        l0 = self.layers[0]
        return l0.self_attn.o_proj.bias is None and l0.mlp.down_proj.bias is None

    def _forward_tp_fused(self, positions, x, ctx):
        """``LlamaDecoderLayer.forward`` at TP > 1 with the o / down all-reduces handed to
        the norms that consume them: o_proj -> post-attention norm, down_proj -> the next
        layer's input norm (the last one -> the final norm).  Same math and rounding."""
        residual, h, prev = x, None, None
        for layer in self.layers:
            ln1 = layer.input_layernorm
            if prev is None:
                x = ln1(x)
            else:
                x, residual = comm.tp_all_reduce_add_rms(
                    gemm.linear(h, prev.mlp.down_proj.weight), residual, ln1.weight, ln1.eps)
            at, ln2 = layer.self_attn, layer.post_attention_layernorm
            a = at.attend(positions, at.project_qkv(x), ctx)
            x, residual = comm.tp_all_reduce_add_rms(gemm.linear(a, at.o_proj.weight), residual,
                                                     ln2.weight, ln2.eps)
            gu = layer.mlp.gate_up_proj
            h = gemm.linear_silu(x, gu.weight, gu.bias)
            prev = layer
        x, _ = comm.tp_all_reduce_add_rms(gemm.linear(h, prev.mlp.down_proj.weight), residual,
                                          self.norm.weight, self.norm.eps)
        return x

    def _forward_tp_overlap(self, positions, x, ctx):
        """``_forward_tp_fused`` on a large prefill step split into two token halves
        (engine/model_runner.py ``_split_prefill``) so that each row-parallel all-reduce
        (RCCL at these sizes: 16K tokens x 8192 x 2 B = 256 MB per call for Llama-3-70B at
        TP = 8) runs while the OTHER half computes.  Per layer:

            attn(A)  AR_o(A) ->                 attn(B)  AR_o(B) ->
            [wait AR_o(A)] norm+MLP(A)  AR_d(A) ->   [wait AR_o(B)] norm+MLP(B)  AR_d(B) ->

        so AR_o(A) hides under attn(B), AR_o(B) under MLP(A), AR_d(A) under MLP(B) and
        AR_d(B) under the next layer's attn(A).  The first half's attention writes its
        K/V before the second half's attention reads them (one compute stream), which a
        sequence cut by the split needs.  Same math as the unsplit step; GEMM shapes
        differ (M halves), so results agree to rounding, not bit for bit."""
        a, ma, mb = ctx.attn.split
        ctxs = (dataclasses.replace(ctx, attn=ma), dataclasses.replace(ctx, attn=mb))
        pos = (positions[:a], positions[a:])
        xs = [x[:a], x[a:]]
        res = [x[:a], x[a:]]          # residual = embedding output, updated in place
        h = [None, None]
        pend = [None, None]
        prev = None
        for layer in self.layers:
            ln1, ln2 = layer.input_layernorm, layer.post_attention_layernorm
            at, gu = layer.self_attn, layer.mlp.gate_up_proj
            for i in (0, 1):
                if prev is None:
                    xi = ln1(xs[i])
                else:
                    pend[i].wait()
                    xi, res[i] = ops.fused_add_rms_norm(h[i], res[i], ln1.weight, ln1.eps)
                o = gemm.linear(at.attend(pos[i], at.project_qkv(xi), ctxs[i]), at.o_proj.weight)
                h[i], pend[i] = o, comm.tp_all_reduce_async(o)
            for i in (0, 1):
                pend[i].wait()
                xi, res[i] = ops.fused_add_rms_norm(h[i], res[i], ln2.weight, ln2.eps)
                d = gemm.linear(gemm.linear_silu(xi, gu.weight, gu.bias),
                                layer.mlp.down_proj.weight)
                h[i], pend[i] = d, comm.tp_all_reduce_async(d)
            prev = layer
        outs = []
        for i in (0, 1):
            pend[i].wait()
            xi, _ = ops.fused_add_rms_norm(h[i], res[i], self.norm.weight, self.norm.eps)
            outs.append(xi)
        return torch.cat(outs, 0)

    # ------------------------------------------------------------------ norm-free small-M layer
    def fold_rs_weights(self, budget_fraction: float = 0.08) -> int:
        """Copies of the qkv and gate_up weights with their input norm's gamma folded in
        (ops/gemm.py fold_norm_weight) for ``_forward_rs``, plus its two sum-of-squares
        partial buffers.  One GPU, dense bias-free Llama layers, KGC_RS_LAYER != 0, and the
        copies within ``budget_fraction`` of device memory (Llama-3-8B: 9.1 GB).  Call
        before the KV cache is sized.  Returns the bytes added."""
        self._rs_w = None
        if not (_rs_enabled and self._fusable and self.layers
                and self.layers[0].input_layernorm.weight.is_cuda):
            return 0
        l0 = self.layers[0]
        if any(p.bias is not None for p in (l0.self_attn.qkv_proj, l0.self_attn.o_proj,
                                            l0.mlp.gate_up_proj, l0.mlp.down_proj)):
            return 0
        dev = l0.input_layernorm.weight.device
        need = sum(l.self_attn.qkv_proj.weight.numel() + l.mlp.gate_up_proj.weight.numel()
                   for l in self.layers[1:]) * l0.mlp.gate_up_proj.weight.element_size()
        need += l0.mlp.gate_up_proj.weight.numel() * l0.mlp.gate_up_proj.weight.element_size()
        free, total = torch.cuda.mem_get_info(dev)
        if need > budget_fraction * total or need > free - (8 << 30):
            return 0
        ws = []
        for i, l in enumerate(self.layers):
            qkv = (None if i == 0 else
                   gemm.fold_norm_weight(l.self_attn.qkv_proj.weight, l.input_layernorm.weight))
            ws.append((qkv, gemm.fold_norm_weight(l.mlp.gate_up_proj.weight,
                                                  l.post_attention_layernorm.weight)))
        self._rs_w = ws
        self._rs_ssp = (torch.zeros(gemm.RS_SSP_FLOATS, dtype=torch.float32, device=dev),
                        torch.zeros(gemm.RS_SSP_FLOATS, dtype=torch.float32, device=dev))
        return need

    def _rs_shapes(self):
        l0 = self.layers[0]
        return [tuple(l0.self_attn.qkv_proj.weight.shape), tuple(l0.self_attn.o_proj.weight.shape),
                tuple(l0.mlp.gate_up_proj.weight.shape), tuple(l0.mlp.down_proj.weight.shape)]

    def _rs_cfgs(self, M: int):
        if getattr(self, "_rs_w", None) is None or not self._fusable:
            return None
        return gemm.rs_plan(M, self._rs_shapes())

    def _forward_rs(self, input_ids, positions, ctx, cfgs):
        """The decoder at small M with no RMSNorm launch inside it (K9 SK_ACC_SS /
        SK_RSCALE, gemm_skinny.hip): o_proj and down_proj add into the residual and leave
        its per-row sums of squares; qkv and gate_up run on gamma-folded weights and scale
        their rows by the rsqrt of those sums.  Per layer: qkv, attention, o, gate_up (SiLU
        pairs), down -- against two more norm launches on the regular path.  Layer 0's
        input norm (over the embedding) runs inside its qkv GEMM (SK_NORM) where tuning
        measured that cheaper; the final norm stays a kernel."""
        c_qkv, c_o, c_gu, c_dn = cfgs
        ssp_o, ssp_d = self._rs_ssp
        res = self.embed_tokens(input_ids)
        M = res.shape[0]
        nss_d = 0
        for i, layer in enumerate(self.layers):
            at, mlp = layer.self_attn, layer.mlp
            ln1, ln2 = layer.input_layernorm, layer.post_attention_layernorm
            qkv_f, gu_f = self._rs_w[i]
            if i == 0:
                # over the embedding: the input norm inside the qkv GEMM (SK_NORM) where
                # tuning measured that cheaper than the norm launch + the plain GEMM
                c0 = gemm.norm_fused_cfg(M, *at.qkv_proj.weight.shape)
                qkv = (gemm.skinny_norm(res, at.qkv_proj.weight, None, ln1.weight, ln1.eps, c0)
                       if c0 is not None else at.project_qkv(ln1(res)))
            else:
                qkv = torch.empty(M, qkv_f.shape[0], dtype=res.dtype, device=res.device)
                gemm.skinny_rscale(res, qkv_f, c_qkv, ssp_d, nss_d, ln1.eps, qkv)
            a = at.attend(positions, qkv, ctx)
            nss_o = gemm.skinny_acc_ss(res, a, at.o_proj.weight, c_o, ssp_o)
            h = torch.empty(M, gu_f.shape[0] // 2, dtype=res.dtype, device=res.device)
            gemm.skinny_rscale(res, gu_f, c_gu, ssp_o, nss_o, ln2.eps, h, silu=True)
            nss_d = gemm.skinny_acc_ss(res, h, mlp.down_proj.weight, c_dn, ssp_d)
        return self.norm(res)

    # ------------------------------------------------------------------ fused small-M decode
    def _fused_cfgs(self, M: int):
        """K9 configurations (qkv, o, gate_up, down) when this step runs the fused layer:
        one GPU (TP = PP = 1), a dense MLP, and start-up tuning measured the fused layer
        faster at this M (ops/gemm.py fused_norm_plan).  None: the regular path runs."""
        if (M > 16 or not self._fusable or not self.layers
                or not self.layers[0].input_layernorm.weight.is_cuda):
            return None
        from ..ops import gemm
        norm_ws, acc_ws = self._fused_weights()
        p = gemm.fused_norm_plan(M, [tuple(w.shape) for w in norm_ws],
                                 [tuple(w.shape) for w in acc_ws])
        if p is None:
            return None
        (c_qkv, c_gu), (c_o, c_dn) = p
        return [c_qkv, c_o, c_gu, c_dn]

    def _fused_weights(self):
        l0 = self.layers[0]
        return ((l0.self_attn.qkv_proj.weight, l0.mlp.gate_up_proj.weight),
                (l0.self_attn.o_proj.weight, l0.mlp.down_proj.weight))

    def qkv_dims(self) -> dict:
        """(N, K) of the QKV weight -> (nq, nkv, head_dim) of its RoPE / KV-write consumer
        (ops/gemm.py tunes the K9m QKV GEMM with that kernel summing its K-slices)."""
        if not self.layers or not hasattr(self.layers[0], "self_attn"):
            return {}
        at = self.layers[0].self_attn
        if at.qkv_proj.bias is not None:
            return {}
        return {tuple(at.qkv_proj.weight.shape): (at.nq, at.nkv, self.cfg.head_dim)}

    def silu_weights(self) -> list:
        """The merged gate_up weights (decode: silu_mul fused into their K9m GEMM)."""
        return [l.mlp.gate_up_proj.weight for l in self.layers
                if isinstance(getattr(l, "mlp", None), LlamaMLP)]

    def silu_shapes(self) -> set:
        """(N, K) of the merged gate_up weights (their split-K reduction carries silu_mul)."""
        return {tuple(l.mlp.gate_up_proj.weight.shape) for l in self.layers
                if isinstance(getattr(l, "mlp", None), LlamaMLP)}

    def tail_shapes(self) -> set:
        """(N, K) of the o / down projections whose split-K reduction the following
        residual add + RMSNorm absorbs (``_forward_tail_fused``), when that path can run."""
        if not (self.first and self.last and self.layers
                and get_state().tp_size == 1 and _tail_fusion_enabled):
            return set()
        l0 = self.layers[0]
        if self.cfg.is_moe:
            return {tuple(l0.self_attn.o_proj.weight.shape)}
        return {tuple(l0.self_attn.o_proj.weight.shape), tuple(l0.mlp.down_proj.weight.shape)}

    def fused_norm_shapes(self) -> set:
        """(N, K) of the GEMMs whose input RMSNorm the fused layer absorbs (tuned at start)."""
        if not self._fusable or not self.layers:
            return set()
        return {tuple(w.shape) for w in self._fused_weights()[0]}

    @property
    def _fusable(self) -> bool:
        s = get_state()
        return (self.first and self.last and s.tp_size == 1 and not self.cfg.is_moe
                and ops.fused_small_m_enabled())

    def _forward_fused(self, input_ids, positions, ctx, cfgs):
        """The decoder at small M with the residual stream kept in one buffer: every
        RMSNorm runs inside the GEMM that consumes it (K9 SK_NORM) and every residual add
        inside the GEMM that produces it (K9 SK_ACC) -- 8 launches per layer instead of
        10.  Same math as the regular path: residual += o; x = norm(residual) ..."""
        from ..ops import gemm
        c_qkv, c_o, c_gu, c_dn = cfgs
        res = self.embed_tokens(input_ids)
        for layer in self.layers:
            at, mlp = layer.self_attn, layer.mlp
            ln1, ln2 = layer.input_layernorm, layer.post_attention_layernorm
            qkv = gemm.skinny_norm(res, at.qkv_proj.weight, at.qkv_proj.bias, ln1.weight,
                                   ln1.eps, c_qkv)
            gemm.skinny_accum(res, at.attend(positions, qkv, ctx), at.o_proj.weight,
                              at.o_proj.bias, c_o)
            gu = gemm.skinny_norm(res, mlp.gate_up_proj.weight, mlp.gate_up_proj.bias,
                                  ln2.weight, ln2.eps, c_gu)
            gemm.skinny_accum(res, ops.silu_mul(gu), mlp.down_proj.weight, mlp.down_proj.bias,
                              c_dn)
        return self.norm(res)

    def compute_logits(self, hidden: torch.Tensor, gather: bool = True) -> torch.Tensor:
        """gather=False: this TP rank's vocabulary shard (vocab-parallel sampling)."""
        return self.lm_head(hidden, gather)

    # ------------------------------------------------------------------ weights
    def _hf_map(self, name: str):
        """HF checkpoint name -> (local param, shard_id) or None if not on this rank."""
        cfg = self.cfg
        if cfg.arch == "qwen":
            name = (name.replace("transformer.wte.", "model.embed_tokens.")
                    .replace("transformer.ln_f.", "model.norm.")
                    .replace("transformer.h.", "model.layers.")
                    .replace(".ln_1.", ".input_layernorm.").replace(".ln_2.", ".post_attention_layernorm.")
                    .replace(".attn.c_proj.", ".self_attn.o_proj.")
                    .replace(".mlp.c_proj.", ".mlp.down_proj."))
        m = re.match(r"model\.layers\.(\d+)\.(.*)", name)
        if m is None:
            if name.startswith("model.embed_tokens.") and self.embed_tokens is not None:
                return self.embed_tokens.weight, None
            if name.startswith("model.norm.") and self.norm is not None:
                return self.norm.weight, None
            if name.startswith("lm_head.") and self.lm_head is not None and self.lm_head.weight is not None:
                return self.lm_head.weight, None
            return None
        li = int(m.group(1))
        if not (self.start <= li < self.end):
            return None
        layer = self.layers[li - self.start]
        rest = m.group(2)
        sa = layer.self_attn
        for sid in ("q", "k", "v"):
            if rest.startswith(f"self_attn.{sid}_proj."):
                p = sa.qkv_proj.weight if rest.endswith("weight") else sa.qkv_proj.bias
                return p, sid
        if rest.startswith("attn.c_attn."):      # qwen v1 fused qkv [3H, H]
            return ("c_attn", sa.qkv_proj, rest.endswith("weight")), None
        if rest.startswith("self_attn.o_proj."):
            return (sa.o_proj.weight if rest.endswith("weight") else sa.o_proj.bias), None
        if rest.startswith("self_attn.q_norm."):
            return sa.q_norm.weight, None
        if rest.startswith("self_attn.k_norm."):
            return sa.k_norm.weight, None
        if rest.startswith("input_layernorm."):
            return layer.input_layernorm.weight, None
        if rest.startswith("post_attention_layernorm."):
            return layer.post_attention_layernorm.weight, None
        mlp = layer.mlp
        if cfg.arch == "qwen":
            if rest.startswith("mlp.w2."):
                return mlp.gate_up_proj.weight, 0
            if rest.startswith("mlp.w1."):
                return mlp.gate_up_proj.weight, 1
        if rest.startswith("mlp.gate_proj."):
            return mlp.gate_up_proj.weight, 0
        if rest.startswith("mlp.up_proj."):
            return mlp.gate_up_proj.weight, 1
        if rest.startswith("mlp.down_proj."):
            return mlp.down_proj.weight, None
        if rest.startswith("block_sparse_moe."):
            return mlp.map_weight(rest[len("block_sparse_moe."):])
        if cfg.is_moe and rest.startswith("mlp."):
            return mlp.map_weight(rest[len("mlp."):])
        return None

    def load_weights(self, weights: Iterable[tuple[str, torch.Tensor]]) -> int:
        n = 0
        for name, w in weights:
            tgt = self._hf_map(name)
            if tgt is None:
                continue
            p, sid = tgt
            if isinstance(p, tuple) and p[0] == "c_attn":
                _, qkv, is_w = p
                H = self.cfg.hidden_size
                param = qkv.weight if is_w else qkv.bias
                for i, s in enumerate(("q", "k", "v")):
                    qkv._load(param, w.narrow(0, i * H, H), s)
            elif isinstance(p, tuple) and p[0] == "moe":
                p[1](w.to(self.dtype))
            else:
                loader = getattr(p, "weight_loader", None)
                w = w.to(p.dtype)
                if loader is None:
                    p.data.copy_(w)
                else:
                    loader(p, w, sid) if sid is not None else loader(p, w)
            n += 1
        return n
