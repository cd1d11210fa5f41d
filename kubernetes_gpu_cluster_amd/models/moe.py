"""Mixtral sparse-MoE block (K13 top-k softmax routing, K14 grouped expert MLP).

Expert placement over the TP group (``--moe-parallel``):

* ``tp`` (default): every rank holds all experts, each expert's intermediate dim
  sharded like a dense MLP; the block ends with the TP all-reduce.
* ``ep``: rank r owns experts [r*E/ep, (r+1)*E/ep) whole.  Tokens are dispatched
  to the owning rank with an all-to-all (C7), processed by the local grouped
  MLP, and the weighted results are returned with a second all-to-all.

On the GPU the whole block is native and host-sync free (so decode graphs capture
it): router GEMM -> ``moe_route`` (K13) -> ``moe_align`` bucketing -> grouped MFMA
GEMM (gate/up, rows gathered) -> silu_mul (K7) -> grouped GEMM (down, rows
scattered back) -> weighted ``moe_combine`` (csrc/kernels/moe.hip).  Prefill chunks
(and shapes the grouped-GEMM tiles do not cover) sort the pairs by expert and run
one GEMM pair per non-empty expert; on the GPU the combine reads the expert-sorted rows
through the inverse permutation.  ``ep`` mode exchanges decode-size batches through
the device-side all-to-all over xGMI peer memory (``parallel/expert_a2a.py``, captured
in decode graphs); larger calls use an RCCL all_to_all with host-side counts.
"""
from __future__ import annotations

import logging

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..parallel import comm
from ..parallel.layers import ReplicatedLinear
from ..parallel.state import get_state
from .configs import ModelConfig

log = logging.getLogger("kgc.moe")
MOE_MODE = {"mode": "tp"}


def set_moe_mode(mode: str) -> None:
    assert mode in ("tp", "ep")
    MOE_MODE["mode"] = mode


def pack_moe_experts(model: nn.Module, budget_fraction: float = 0.45) -> int:
    """K14m's packed expert copies for every MoE block of ``model`` (Mixtral 8x7B bf16:
    ~93 GB more on a 288 GB GPU), skipped when they would exceed ``budget_fraction`` of the
    device or leave less than 16 GB free (KGC_MOE_PACK=0: never, for A/B runs).  Call
    before the KV cache is sized.  Returns the bytes packed."""
    import os
    blocks = [m for m in model.modules() if isinstance(m, MoEBlock) and m.native]
    if not blocks or os.environ.get("KGC_MOE_PACK", "1") == "0":
        return 0
    need = sum((b.w13.numel() + b.w2.numel()) * b.w13.element_size() for b in blocks)
    free, total = torch.cuda.mem_get_info(blocks[0].w13.device)
    if need > budget_fraction * total or need > free - (16 << 30):
        log.info("K14m: %.1f GB of packed experts exceeds the budget; register-staged "
                 "grouped GEMM", need / 1e9)
        return 0
    got = sum(b.pack_experts() for b in blocks)
    log.info("K14m: packed the experts of %d MoE blocks (%.1f GB)", len(blocks), got / 1e9)
    return got


def grouped_expert_mlp(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor,
                       topk_w: torch.Tensor, topk_ids: torch.Tensor,
                       expert_offset: int = 0) -> torch.Tensor:
    """x [T, H]; w13 [E_local, 2I, H]; w2 [E_local, H, I]; ids index global experts."""
    T, H = x.shape
    E = w13.shape[0]
    k = topk_ids.shape[1]
    flat = topk_ids.reshape(-1).long() - expert_offset
    valid = (flat >= 0) & (flat < E)
    order = torch.argsort(torch.where(valid, flat, E), stable=True)
    counts = torch.bincount(flat[valid], minlength=E).tolist()
    tok = order // k
    if x.is_cuda and ops.moe_supported(H, w2.shape[2]):
        # GPU (prefill chunks): ONE row gather, the experts' GEMMs written straight into
        # their sorted rows, and the weighted combine kernel reading those rows through the
        # inverse permutation (row_map) -- instead of a gather, an fp32 up-cast, a scaling and
        # an atomic index_add_ per expert (~40 ms of a Mixtral 16K-token chunk's 409 ms), or
        # a scatter back to pair order (index_put, 12 ms of the chunk)
        nv = sum(counts)
        xs = x[tok[:nv]]
        ys = torch.empty(nv, H, dtype=x.dtype, device=x.device)
        start = 0
        for e, c in enumerate(counts):
            if c:
                h = ops.silu_mul(F.linear(xs[start:start + c], w13[e]))
                torch.mm(h, w2[e].t(), out=ys[start:start + c])
            start += c
        rows = torch.arange(T * k, dtype=torch.int32, device=x.device)
        row_map = torch.empty_like(rows).scatter_(0, order, rows)
        row_map = torch.where(row_map < nv, row_map, -1).to(torch.int32)
        out = torch.empty(T, H, dtype=x.dtype, device=x.device)
        torch.ops.kgc.moe_combine(out, ys, topk_w.contiguous().float(), row_map)
        return out
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    start = 0
    wflat = topk_w.reshape(-1)
    for e, c in enumerate(counts):
        if c == 0:
            continue
        idx = order[start:start + c]
        t = tok[start:start + c]
        h = ops.silu_mul(F.linear(x[t], w13[e]))
        y = F.linear(h, w2[e])
        out.index_add_(0, t, y.float() * wflat[idx, None])
        start += c
    return out.to(x.dtype)


class MoEBlock(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        s = get_state()
        self.cfg = cfg
        self.E, self.k = cfg.num_experts, cfg.top_k_experts
        self.mode = MOE_MODE["mode"] if s.tp_size > 1 else "tp"
        tp, r = s.tp_size, s.tp_rank
        H, I = cfg.hidden_size, cfg.intermediate_size
        self.gate = ReplicatedLinear(H, self.E, dtype=dtype, device=device)
        if self.mode == "tp":
            assert I % tp == 0
            self.I_local, self.E_local, self.e0 = I // tp, self.E, 0
        else:
            assert self.E % tp == 0
            self.I_local, self.E_local, self.e0 = I, self.E // tp, r * (self.E // tp)
        self.w13 = nn.Parameter(torch.empty(self.E_local, 2 * self.I_local, H, dtype=dtype,
                                            device=device), requires_grad=False)
        self.w2 = nn.Parameter(torch.empty(self.E_local, H, self.I_local, dtype=dtype,
                                           device=device), requires_grad=False)
        self.native = (torch.device(device).type == "cuda" and
                       ops.moe_supported(2 * self.I_local, H) and ops.moe_supported(H, self.I_local))
        if torch.device(device).type == "cuda" and not self.native:
            log.warning("MoE dims (2I=%d, H=%d) not covered by the grouped GEMM tiles; "
                        "using the per-expert path (no decode graphs)", 2 * self.I_local, H)
        # ep mode on one node: the device-side all-to-all over xGMI peer memory
        # (parallel/expert_a2a.py), attached by the worker once the EP group exists
        self.ep_a2a = None
        # K14m packed per-expert copies (ops.moe_pack), made by the worker before the KV
        # cache is sized (pack_moe_experts); None: the register-staged grouped GEMM
        self.w13p = None
        self.w2p = None

    def pack_experts(self) -> int:
        """Packed K9m-layout copies of this block's experts for K14m (decode path).
        Returns the bytes added."""
        if not self.native or not ops.moe_packable(self.w13, self.w2) or self.w13p is not None:
            return 0
        self.w13p = ops.moe_pack(self.w13.data, True)
        self.w2p = ops.moe_pack(self.w2.data, False)
        return (self.w13p.numel() + self.w2p.numel()) * self.w13p.element_size()

    @property
    def graph_safe(self) -> bool:
        """Decode hipGraphs need a block with no host synchronisation."""
        return self.native and (self.mode == "tp" or self.ep_a2a is not None)

    def experts(self, x, topk_w, topk_ids, expert_offset: int = 0, all_local: bool = True):
        # the grouped kernel streams each expert's weights once per row block: best at
        # decode sizes; big prefill buckets run faster as one hipBLASLt GEMM per expert
        # (host sync is fine there -- prefill is never graph-captured)
        small = topk_ids.numel() <= ops.MOE_NATIVE_MAX_ROWS * self.E_local
        if self.native and x.is_cuda and (small or torch.cuda.is_current_stream_capturing()):
            return ops.fused_moe(x, self.w13, self.w2, topk_w, topk_ids, expert_offset, all_local,
                                 self.w13p, self.w2p)
        return grouped_expert_mlp(x, self.w13, self.w2, topk_w, topk_ids, expert_offset)

    def map_weight(self, rest: str):
        """Checkpoint names under ``block_sparse_moe.``: gate.weight,
        experts.{e}.w{1,2,3}.weight; or the fused transformers-v5 names under ``mlp.``:
        gate.weight, experts.gate_up_proj [E, 2I, H], experts.down_proj [E, H, I]."""
        if rest.startswith("gate."):
            return self.gate.weight, None
        if rest in ("experts.gate_up_proj", "experts.down_proj"):
            s = get_state()
            r = s.tp_rank if self.mode == "tp" else 0
            n, I = self.I_local, self.cfg.intermediate_size
            e0, e1 = self.e0, self.e0 + self.E_local

            def load_fused(w):
                if rest.endswith("gate_up_proj"):
                    self.w13.data[:, :n].copy_(w[e0:e1, r * n:(r + 1) * n])
                    self.w13.data[:, n:].copy_(w[e0:e1, I + r * n:I + (r + 1) * n])
                else:
                    self.w2.data.copy_(w[e0:e1, :, r * n:(r + 1) * n])
            return ("moe", load_fused), None
        parts = rest.split(".")
        e, which = int(parts[1]), parts[2]
        le = e - self.e0
        if not (0 <= le < self.E_local):
            return None
        s = get_state()
        r = s.tp_rank if self.mode == "tp" else 0
        n = self.I_local

        def load(w):
            if which == "w1":
                self.w13.data[le, :n].copy_(w.narrow(0, r * n, n))
            elif which == "w3":
                self.w13.data[le, n:].copy_(w.narrow(0, r * n, n))
            else:
                self.w2.data[le].copy_(w.narrow(1, r * n, n))
        return ("moe", load), None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # decode sizes: the router GEMM inside the top-k kernel (ops.moe_gate_topk); prefill
        # chunks keep the GEMM (whose 16K-row output a single wave per token would serialise)
        r = (ops.moe_gate_topk(x, self.gate.weight, self.k)
             if x.shape[0] <= ops.MOE_GATE_FUSED_MAX_T and self.gate.bias is None else None)
        if r is None:
            r = ops.moe_topk_softmax(self.gate(x), self.k)
        topk_w, topk_ids = r
        if self.mode == "tp":
            return comm.tp_all_reduce(self.experts(x, topk_w, topk_ids))
        return self._forward_ep(x, topk_w, topk_ids)

    def _forward_ep(self, x, topk_w, topk_ids):
        """All-to-all dispatch/combine (C7).  Each (token, slot) pair goes to the rank
        owning its expert; the owner computes and sends the weighted row back.  Decode
        sizes run the device-side exchange over xGMI peer memory (graph-capturable);
        larger calls an RCCL all_to_all with host-side counts."""
        a2a = self.ep_a2a
        if a2a is not None and self.native and a2a.fits(x, topk_ids):
            # the owner's receive slots hold ~T x k rows of its NR x C (this rank's own pair
            # count, on average); the down projection's split-K slices go straight to
            # ep_return, which sums them while writing the rows back
            hint = topk_ids.numel()
            return a2a.forward(x, topk_w, topk_ids,
                               lambda xs, w, ids, off: ops.fused_moe(
                                   xs, self.w13, self.w2, w, ids, off, True, self.w13p,
                                   self.w2p, rows_hint=hint, combine=False),
                               self.E_local)
        s = get_state()
        if getattr(s, "phantom", False):
            # phantom EP rank (no peers, no group): this rank's own expert work -- its local
            # experts over every pair routed to them; the other ranks' shares are zeros
            return self.experts(x, topk_w, topk_ids, expert_offset=self.e0, all_local=False)
        tp = s.tp_size
        T, H = x.shape
        flat_ids = topk_ids.reshape(-1).long()
        dest = flat_ids // self.E_local
        order = torch.argsort(dest, stable=True)
        send_counts = torch.bincount(dest, minlength=tp)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=s.tp_group)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        tok = order // self.k
        send_x = x[tok]
        send_meta = torch.stack([flat_ids[order], torch.arange(order.numel(), device=x.device)], 1)
        recv_x = torch.empty(sum(rc), H, dtype=x.dtype, device=x.device)
        dist.all_to_all_single(recv_x, send_x, rc, sc, group=s.tp_group)
        recv_ids = torch.empty(sum(rc), 2, dtype=send_meta.dtype, device=x.device)
        dist.all_to_all_single(recv_ids, send_meta, rc, sc, group=s.tp_group)
        ones = torch.ones(recv_x.shape[0], 1, dtype=torch.float32, device=x.device)
        y = self.experts(recv_x, ones, recv_ids[:, :1].to(torch.int32).contiguous(),
                         expert_offset=self.e0)
        back = torch.empty(order.numel(), H, dtype=x.dtype, device=x.device)
        dist.all_to_all_single(back, y, sc, rc, group=s.tp_group)
        out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
        w = topk_w.reshape(-1)[order]
        out.index_add_(0, tok, back.float() * w[:, None])
        return out.to(x.dtype)
