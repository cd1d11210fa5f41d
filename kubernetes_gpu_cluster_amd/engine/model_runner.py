"""Model runner: step packing, KV-cache sizing, hipGraph-captured decode, sampling.

A step is described by a ``StepPlan``: a small header of counts plus three host
blobs (int64 / int32 / fp32) at fixed offsets.  The driver builds it from the
scheduler's batch; TP/PP workers receive only the plan (never Sequence objects).
Each rank copies the blobs to static device buffers (3 H2D copies per step) and
runs the forward; views into those static buffers are what the captured decode
graphs read, so a graph replay needs no extra copies.

Decode graphs are captured per batch bucket (1, 2, 4, 8, 16, 24, 32, ..., max);
a pure-decode step pads to the next bucket (slot -1 = no KV write, ctx_len 0 =
zero output).  Mixed / prefill steps run eagerly.  Sampling uses the counter-
based HIP sampler, so every TP rank samples identical tokens from identical
(all-gathered) logits without a broadcast.
"""
from __future__ import annotations

import dataclasses
import math
import os
import time
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..models.attention import AttnMetadata, ForwardContext
from ..models.configs import ModelConfig
from ..ops import reference as ref
from ..parallel import comm
from ..parallel.state import get_state
from .logits_processor import LogitsProcessor, needs_counts
from .sequence import Sequence


def graph_buckets(max_bs: int) -> list[int]:
    b = [1, 2, 4, 8, 16, 24, 32]
    b += list(range(48, max_bs + 1, 16))
    return sorted({x for x in b if x <= max_bs} | {max_bs})


@dataclasses.dataclass
class StepPlan:
    T: int                 # tokens
    Tp: int                # prefill tokens (first Tp of T)
    P: int                 # prefill sequences
    D: int                 # decode sequences
    S: int                 # sampled rows
    W: int                 # prefill attention work items
    B: int                 # graph bucket (0 = eager)
    max_ctx: int           # longest decode context
    dev_tok: int           # 1: decode input tokens come from the device-side last_tok table
    tok_bcast: int         # 1: TP ranks take the driver's sampled ids (driver-side logits processing)
    vp: int                # 1: vocab-parallel sampling (TP > 1: no logits gather this step)
    split: int             # 1: TP prefill overlap (two token halves), decided by the driver
    i64: np.ndarray
    i32: np.ndarray
    f32: np.ndarray
    lp: Optional[list] = None   # driver only: [(sampled row, top-k)] for logprobs requests
    proc: Optional[list] = None  # driver only: [(sampled row, slot, params)] penalties/bias/min_p
    proc_init: Optional[list] = None  # driver only: [(slot, prompt ids, output ids)]

    def header(self) -> list[int]:
        return [self.T, self.Tp, self.P, self.D, self.S, self.W, self.B, self.max_ctx,
                self.dev_tok, self.tok_bcast, self.vp, self.split]


class Layout:
    """Fixed offsets of the step blobs."""

    def __init__(self, max_tokens: int, max_seqs: int, max_blocks: int, block_m: int):
        self.Tmax, self.Smax, self.mb = max_tokens, max_seqs, max_blocks
        self.Wmax = max_tokens // block_m + max_seqs + 1
        o = 0
        self.ids, o = o, o + self.Tmax
        self.pos, o = o, o + self.Tmax
        self.slots, o = o, o + self.Tmax
        self.seeds, o = o, o + self.Smax
        self.lidx, o = o, o + self.Smax
        self.dslots, o = o, o + self.Smax     # decode row -> seq slot (token gather)
        self.sslots, o = o, o + self.Smax     # sampled row -> seq slot (token scatter)
        self.n64 = o
        o = 0
        self.dbt, o = o, o + self.Smax * max_blocks
        self.ctx, o = o, o + self.Smax
        self.pbt, o = o, o + self.Smax * max_blocks
        self.qsl, o = o, o + self.Smax + 1
        self.sl, o = o, o + self.Smax
        self.ws, o = o, o + self.Wmax
        self.wm, o = o, o + self.Wmax
        self.topk, o = o, o + self.Smax
        self.n32 = o
        self.temp, self.topp = 0, self.Smax
        self.nf = 2 * self.Smax


class ModelRunner:
    def __init__(self, model, mcfg: ModelConfig, dtype: torch.dtype, device: torch.device,
                 block_size: int, max_model_len: int, max_num_seqs: int, token_budget: int,
                 enforce_eager: bool = False, graph_max_bs: int = 256,
                 kv_dtype: Optional[torch.dtype] = None, kv_scales: tuple = (1.0, 1.0)):
        self.model, self.mcfg, self.dtype, self.device = model, mcfg, dtype, device
        # KV cache element type: the activation dtype, or fp8 e4m3 (--kv-cache-dtype fp8:
        # half the bytes per cached token, twice the tokens per GB)
        self.kv_dtype = kv_dtype or dtype
        self.kv_scales = kv_scales
        self.bs = block_size
        self.max_model_len = max_model_len
        self.max_blocks = math.ceil(max_model_len / block_size)
        self.max_num_seqs = max_num_seqs
        self.token_budget = token_budget
        self.is_gpu = device.type == "cuda"
        self.use_graphs = self.is_gpu and not enforce_eager
        self.graph_max_bs = min(graph_max_bs, max_num_seqs)
        self.buckets = graph_buckets(self.graph_max_bs)
        self.ps = get_state()
        max_tokens = max(token_budget, max_num_seqs)
        self.L = Layout(max_tokens, max_num_seqs, self.max_blocks, ops.PREFILL_BLOCK_M)
        pin = self.is_gpu
        # Pinned step blobs, a ring of sets: a plan is packed into one set while the
        # non-blocking H2D copies of earlier plans (async mode: the previous step; PP: up
        # to pp_size micro-batches in flight) may still read theirs.  A set is reused only
        # after the event recorded behind its upload has completed (next_host_bufs).
        # Each set is ONE byte blob holding the int64 / int32 / fp32 arrays (256-B aligned
        # sections, as separate allocations would be), mirrored by one device blob: a step
        # uploads with one copy, not three (~4.3 us per copy node at batch 1).
        self._hsets = [self._blob_views(torch.zeros(self._blob_bytes(), dtype=torch.uint8,
                                                    pin_memory=pin))
                       for _ in range(self.ps.pp_size + 2)]
        self._hev: list = [None] * len(self._hsets)
        self._hcur = 0
        self.h64, self.h32, self.hf, self.hblob = self._hsets[0]
        self.d64, self.d32, self.df, self.dblob = self._blob_views(
            torch.zeros(self._blob_bytes(), dtype=torch.uint8, device=device))
        rope_len = max(max_model_len, mcfg.max_position if mcfg.arch != "opt" else 1)
        self.cos_sin = ref.rope_cos_sin_cache(mcfg.head_dim, rope_len + 1, mcfg.rope_theta,
                                              mcfg.rope_scaling).to(device)
        self.kv = None
        self.kv_caches: list = []
        self.workspace = None
        self.graphs: dict[int, tuple] = {}
        self.graph_pool = None
        self.sample_out = torch.zeros(max_num_seqs, dtype=torch.int64, device=device)
        self.processor = LogitsProcessor(max_num_seqs, mcfg.vocab_size, device)
        # last sampled token per sequence slot: decode steps read their input token
        # here, so the host can launch step N+1 before it has seen step N's tokens
        self.last_tok = torch.zeros(max_num_seqs, dtype=torch.int64, device=device)
        self.tok_host = [torch.zeros(max_num_seqs, dtype=torch.int64, pin_memory=self.is_gpu)
                         for _ in range(2)]
        self._tok_flip = 0
        self.stats = {"graph_steps": 0, "eager_steps": 0, "vp_steps": 0,
                      "tp_allreduce_bytes": 0, "tp_logits_bytes": 0}
        # KGC_FAKE_STAGE_MS: every step of this rank is a sleep of that many ms with the
        # real pipeline-stage traffic around it (PP scheduling / utilisation tests)
        self._fake_ms = float(os.environ.get("KGC_FAKE_STAGE_MS", "0") or 0)
        self.pp_link = None         # parallel/pp_handoff.PipelineHandoff (PP decode graphs)
        self.stage_stats = {"busy_s": 0.0, "t_first": None, "t_last": None, "steps": 0}
        # vocab-parallel sampling (TP > 1): every rank keeps its logits shard; rows
        # without top-k / top-p / processors / logprobs are sampled by an 8-byte-per-row
        # MAX all-reduce instead of an all-gather of B x V logits (ops.sample_vp_partial)
        head = getattr(model, "lm_head", None)
        self.vp = (self.ps.tp_size > 1 and getattr(model, "last", True) and head is not None
                   and hasattr(head, "start") and os.environ.get("KGC_VP_SAMPLING", "1") != "0")
        if self.vp:
            self.vp_off = head.start
            self.vp_cols = max(0, min(head.per, head.vocab - head.start))
            self.vp_packed = torch.zeros(max_num_seqs, dtype=torch.int64, device=device)

    def _blob_offsets(self):
        up = lambda n: (n + 255) // 256 * 256    # noqa: E731
        o32 = up(8 * self.L.n64)
        of = up(o32 + 4 * self.L.n32)
        return o32, of, up(of + 4 * self.L.nf)

    def _blob_bytes(self) -> int:
        return self._blob_offsets()[2]

    def _blob_views(self, blob: torch.Tensor):
        o32, of, _ = self._blob_offsets()
        L = self.L
        return (blob[:8 * L.n64].view(torch.int64), blob[o32:o32 + 4 * L.n32].view(torch.int32),
                blob[of:of + 4 * L.nf].view(torch.float32), blob)

    # ------------------------------------------------------------------ KV cache
    def kv_bytes_per_block(self) -> int:
        m = self.model
        return (2 * m.num_local_layers * m.local_kv_heads() * self.mcfg.head_dim * self.bs *
                torch.tensor([], dtype=self.kv_dtype).element_size())

    def profile_num_blocks(self, gpu_mem_util: float) -> int:
        """Run a worst-case eager prefill, measure peak activation memory, and size the
        KV pool to gpu_mem_util of total device memory (vLLM semantics)."""
        if not self.is_gpu:
            return max(64, (4 * self.max_num_seqs * self.max_blocks) // 4)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        self.init_kv_cache(16)
        seqs = []
        remaining = self.token_budget
        while remaining > 0:
            q = min(remaining, self.max_model_len)
            seqs.append(q)
            remaining -= q
        self._dummy_prefill(seqs)
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated() - base
        self.kv = None
        self.kv_caches = []
        torch.cuda.empty_cache()
        free, total = torch.cuda.mem_get_info()
        used_now = total - free
        reserve_graphs = 2 << 30 if self.use_graphs else 0
        budget = total * gpu_mem_util - used_now - peak - reserve_graphs
        nb = int(budget // self.kv_bytes_per_block())
        return max(nb, 2)

    def release(self) -> None:
        """Drop the KV arena, decode graphs and workspaces (engine shutdown): a process
        that builds a second engine must get the memory back."""
        self.graphs = {}
        self.graph_pool = None
        self.kv = None
        self.kv_caches = []
        self.workspace = None
        if self.is_gpu:
            import gc
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    def init_kv_cache(self, num_blocks: int) -> None:
        m = self.model
        L, nkv, d = m.num_local_layers, m.local_kv_heads(), self.mcfg.head_dim
        # zero-init: stale slots of partially filled blocks must hold finite values
        self.kv = torch.zeros(L, 2, num_blocks, nkv, self.bs, d, dtype=self.kv_dtype,
                              device=self.device)
        self.kv_caches = [(self.kv[l, 0], self.kv[l, 1].view(num_blocks, nkv, self.bs // 8, d, 8))
                          for l in range(L)]
        self.num_blocks = num_blocks
        nq = m.layers[0].self_attn.nq if hasattr(m.layers[0], "self_attn") else m.layers[0].qkv_proj.nq
        if self.is_gpu:
            self.workspace = ops.decode_partials(self.max_num_seqs, nq, d, self.max_blocks, self.bs,
                                                 self.device)

    def next_host_bufs(self) -> None:
        """Switch h64 / h32 / hf to the next pinned set of the ring, waiting until the
        upload that last read it has finished (normally long done: a set comes round
        again only after pp_size + 1 further plans).  Call before packing a plan into
        the blobs (driver: build_plan; other ranks: before receiving one)."""
        self._hcur = (self._hcur + 1) % len(self._hsets)
        ev = self._hev[self._hcur]
        if ev is not None:
            ev.synchronize()
            self._hev[self._hcur] = None
        self.h64, self.h32, self.hf, self.hblob = self._hsets[self._hcur]

    def _dummy_prefill(self, qlens: list[int]) -> None:
        """A prefill forward with slot -1 (no KV writes) over dummy block tables."""
        self.next_host_bufs()
        T = sum(qlens)
        P = len(qlens)
        L = self.L
        i64 = self.h64.numpy()
        i32 = self.h32.numpy()
        i64[L.ids:L.ids + T] = 0
        i64[L.pos:L.pos + T] = np.concatenate([np.arange(q) for q in qlens])
        i64[L.slots:L.slots + T] = -1
        i32[L.pbt:L.pbt + P * self.max_blocks] = 0
        qsl = np.concatenate([[0], np.cumsum(qlens)])
        i32[L.qsl:L.qsl + P + 1] = qsl
        i32[L.sl:L.sl + P] = qlens
        ws, wm = ops.prefill_work_list(qlens, qlens)
        i32[L.ws:L.ws + len(ws)] = ws
        i32[L.wm:L.wm + len(wm)] = wm
        i64[L.lidx:L.lidx + P] = qsl[1:] - 1
        self.hf.numpy()[: 2 * self.L.Smax] = 1.0
        i64[L.sslots:L.sslots + P] = 0
        # (no TP overlap split in the profiling step: every rank runs it from its own
        # copy, and the unsplit step's activations are the larger ones)
        plan = StepPlan(T, T, P, 0, P, len(ws), 0, 0, 0, 0, int(self.vp), 0, i64, i32,
                        self.hf.numpy())
        self.run(plan)

    # ------------------------------------------------------------------ packing (driver)
    def build_plan(self, prefills: list[tuple[Sequence, int]], decodes: list[Sequence],
                   table: np.ndarray, device_tokens: bool = False) -> tuple[StepPlan, list[Sequence]]:
        """Pack a scheduled batch.  Returns the plan and the sequences that sample
        (in sampled-row order).  device_tokens: decode inputs are gathered on the GPU
        from last_tok (async mode), so the host needs no sampled token values."""
        L, bs, mb = self.L, self.bs, self.max_blocks
        self.next_host_bufs()
        i64, i32, f32 = self.h64.numpy(), self.h32.numpy(), self.hf.numpy()
        P, D = len(prefills), len(decodes)
        samplers: list[Sequence] = []
        lidx: list[int] = []
        # ---- prefill chunks
        off = 0
        qlens, slens = [], []
        for i, (seq, n) in enumerate(prefills):
            a = seq.num_computed
            pos = np.arange(a, a + n, dtype=np.int64)
            i64[L.ids + off:L.ids + off + n] = seq.tokens_slice(a, a + n)
            i64[L.pos + off:L.pos + off + n] = pos
            row = table[seq.slot]
            i64[L.slots + off:L.slots + off + n] = row[pos // bs].astype(np.int64) * bs + pos % bs
            i32[L.pbt + i * mb:L.pbt + (i + 1) * mb] = row
            qlens.append(n)
            slens.append(a + n)
            off += n
            if a + n == seq.num_tokens:
                samplers.append(seq)
                lidx.append(off - 1)
        Tp = off
        W = 0
        if P:
            i32[L.qsl:L.qsl + P + 1] = np.concatenate([[0], np.cumsum(qlens)])
            i32[L.sl:L.sl + P] = slens
            ws, wm = ops.prefill_work_list(qlens, slens)
            W = len(ws)
            i32[L.ws:L.ws + W] = ws
            i32[L.wm:L.wm + W] = wm
        # ---- decodes (vectorised)
        max_ctx = 0
        B = 0
        if D:
            slots = np.fromiter((s.slot for s in decodes), dtype=np.int64, count=D)
            pos = np.fromiter((s.num_computed for s in decodes), dtype=np.int64, count=D)
            if self.use_graphs and P == 0 and D <= self.graph_max_bs:
                B = next(b for b in self.buckets if b >= D)
            n = max(D, B)
            if device_tokens:
                i64[L.dslots:L.dslots + D] = slots
                i64[L.dslots + D:L.dslots + n] = 0
            else:
                i64[L.ids + Tp:L.ids + Tp + D] = [
                    s.output_token_ids[-1] if s.output_token_ids else s.prompt_token_ids[-1]
                    for s in decodes]
            i64[L.pos + Tp:L.pos + Tp + D] = pos
            i64[L.slots + Tp:L.slots + Tp + D] = table[slots, pos // bs].astype(np.int64) * bs + pos % bs
            dbt = i32[L.dbt:L.dbt + n * mb].reshape(n, mb)
            dbt[:D] = table[slots]
            i32[L.ctx:L.ctx + D] = pos + 1
            if n > D:   # graph padding rows
                i64[L.ids + Tp + D:L.ids + Tp + n] = 0
                i64[L.pos + Tp + D:L.pos + Tp + n] = 0
                i64[L.slots + Tp + D:L.slots + Tp + n] = -1
                dbt[D:] = 0
                i32[L.ctx + D:L.ctx + n] = 0
            max_ctx = int(pos.max()) + 1
            samplers.extend(decodes)
            lidx.extend(range(Tp, Tp + D))
        S = len(samplers)
        T = Tp + D
        # ---- sampling params
        i64[L.sslots:L.sslots + S] = [s.slot for s in samplers]
        for j, s in enumerate(samplers):
            p = s.params
            f32[L.temp + j] = p.temperature
            f32[L.topp + j] = p.top_p
            i32[L.topk + j] = p.top_k
            i64[L.seeds + j] = (s.seed & 0xFFFFFFFF) | (len(s.output_token_ids) << 32)
        i64[L.lidx:L.lidx + S] = lidx
        if B:
            i64[L.lidx:L.lidx + B] = np.arange(B)   # graph rows index their own hidden row
        lp = [(j, s.params.logprobs) for j, s in enumerate(samplers)
              if s.params.logprobs is not None] or None
        proc, proc_init = None, None
        if any(s.params.needs_proc for s in samplers):
            proc = [(j, s.slot, s.params) for j, s in enumerate(samplers) if s.params.needs_proc]
            proc_init = [(s.slot, s.prompt_token_ids, list(s.output_token_ids))
                         for s in samplers if needs_counts(s.params) and s.proc_slot != s.slot] or None
            for s in samplers:
                if needs_counts(s.params):
                    s.proc_slot = s.slot
        # TP > 1: ranks adopt the driver's ids when it processes logits, and for top-k /
        # top-p rows (their float histograms are summed in a hardware-dependent order)
        thr = any((0 < s.params.top_k < self.mcfg.vocab_size) or s.params.top_p < 1.0
                  for s in samplers)
        bcast = int((proc is not None or thr) and self.ps.tp_size > 1)
        V = self.mcfg.vocab_size
        vp = int(self.vp and lp is None and proc is None
                 and all((s.params.top_k <= 0 or s.params.top_k >= V) and s.params.top_p >= 1.0
                         for s in samplers))
        # the TP prefill overlap split is decided HERE, once, and carried in the header:
        # ranks deciding it from their own environment could split differently and issue
        # all-reduces of different sizes (a hang or a corrupt step)
        split = int(P > 0 and D == 0 and self._overlap_ok(Tp))
        return StepPlan(T, Tp, P, D, S, W, B, max_ctx, int(device_tokens and D > 0), bcast, vp,
                        split, i64, i32, f32, lp, proc, proc_init), samplers

    # ------------------------------------------------------------------ execution (all ranks)
    def _upload(self, plan: StepPlan) -> None:
        if self.is_gpu:
            self.dblob.copy_(self.hblob, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._hev[self._hcur] = ev
        else:
            self.d64.copy_(torch.from_numpy(plan.i64))
            self.d32.copy_(torch.from_numpy(plan.i32))
            self.df.copy_(torch.from_numpy(plan.f32))

    def _meta(self, T, Tp, P, D, W, max_ctx, z=None, split: int = 0) -> AttnMetadata:
        L, mb = self.L, self.max_blocks
        d32 = self.d32
        m = AttnMetadata(slot_mapping=self.d64[L.slots:L.slots + T], num_prefill_tokens=Tp,
                         num_prefills=P, num_decodes=D)
        if P:
            m.prefill_block_tables = d32[L.pbt:L.pbt + P * mb].view(P, mb)
            m.query_start_loc = d32[L.qsl:L.qsl + P + 1]
            m.prefill_seq_lens = d32[L.sl:L.sl + P]
            m.work_seq = d32[L.ws:L.ws + W]
            m.work_mblk = d32[L.wm:L.wm + W]
        if D:
            m.decode_block_tables = d32[L.dbt:L.dbt + D * mb].view(D, mb)
            m.decode_ctx_lens = d32[L.ctx:L.ctx + D]
            m.decode_workspace = self.workspace
            nkv = self.model.local_kv_heads()
            m.decode_grid_z = z if z is not None else ops.decode_grid_z(D, nkv, max_ctx)
        elif P and split:
            m.split = self._split_prefill(Tp, P)
        return m

    # ------------------------------------------------------------------ TP prefill overlap
    def _overlap_ok(self, Tp: int) -> bool:
        """Large prefill-only steps at TP > 1 run as two token halves whose all-reduces
        overlap the other half's GEMMs (``LlamaForCausalLM._forward_tp_overlap``).  The
        DRIVER evaluates this (build_plan) and every rank follows the plan's ``split``.
        KGC_TP_OVERLAP=0 turns it off; KGC_TP_OVERLAP_MIN_TOKENS (default 2048) is the
        smallest step it applies to (below it the all-reduces take the xGMI kernel)."""
        if self.ps.tp_size == 1:
            return False
        if os.environ.get("KGC_TP_OVERLAP", "1") == "0":
            return False
        fn = getattr(self.model, "_tp_tail_fusable", None)
        return (fn is not None and fn()
                and Tp >= int(os.environ.get("KGC_TP_OVERLAP_MIN_TOKENS", "2048")))

    def _split_prefill(self, Tp: int, P: int):
        """Split the step's prefill tokens at row a into two AttnMetadata.  A sequence
        cut by the split becomes a chunked-prefill continuation in the second half (its
        queries [a', qlen) over seq_len keys); the first half's part of it attends over
        seq_len - (qlen - a') keys.  Within a layer the first half's attention (and its
        K/V write) runs before the second half's, so the continuation sees those keys.
        Built from this rank's host copy of the plan (identical on every TP rank)."""
        L, mb = self.L, self.max_blocks
        i32 = self.h32.numpy()
        qsl = i32[L.qsl:L.qsl + P + 1].astype(np.int64)
        sl = i32[L.sl:L.sl + P].astype(np.int64)
        pbt = i32[L.pbt:L.pbt + P * mb].reshape(P, mb)
        a = (Tp // 2) // 128 * 128 or Tp // 2
        k = int(np.searchsorted(qsl, a, side="right")) - 1      # qsl[k] <= a < qsl[k+1]
        qlens = np.diff(qsl)
        cut = a > qsl[k]
        qa = np.concatenate([qlens[:k], [a - qsl[k]] if cut else []]).astype(np.int64)
        sa = np.concatenate([sl[:k], [sl[k] - (qsl[k + 1] - a)] if cut else []]).astype(np.int64)
        qb = np.concatenate([[qsl[k + 1] - a], qlens[k + 1:]]).astype(np.int64)
        sb = sl[k:].copy()
        halves = []
        blob = []
        for q, sq, bt in ((qa, sa, pbt[:len(qa)]), (qb, sb, pbt[k:])):
            ws, wm = ops.prefill_work_list(q.tolist(), sq.tolist())
            parts = [np.concatenate([[0], np.cumsum(q)]), sq, bt.reshape(-1), ws, wm]
            halves.append([len(x) for x in parts])
            blob += parts
        flat = np.concatenate([np.asarray(x, dtype=np.int32) for x in blob])
        dev = self._split_upload(flat)
        metas, off = [], 0
        d64 = self.d64
        for h, (n0, n1) in enumerate(((0, a), (a, Tp))):
            v = []
            for n in halves[h]:
                v.append(dev[off:off + n])
                off += n
            np_ = halves[h][1]
            mh = AttnMetadata(slot_mapping=d64[L.slots + n0:L.slots + n1], num_prefill_tokens=n1 - n0,
                              num_prefills=np_, num_decodes=0)
            mh.query_start_loc, mh.prefill_seq_lens = v[0], v[1]
            mh.prefill_block_tables = v[2].view(np_, mb)
            mh.work_seq, mh.work_mblk = v[3], v[4]
            metas.append(mh)
        return a, metas[0], metas[1]

    def _split_upload(self, flat: np.ndarray) -> torch.Tensor:
        """Device copy of the split metadata through a 2-entry pinned ring (a buffer is
        refilled only after the copy that last read it has completed)."""
        if not self.is_gpu:
            return torch.from_numpy(flat.copy())
        if not hasattr(self, "_sp_bufs"):
            self._sp_bufs, self._sp_ev, self._sp_cur = [None, None], [None, None], 0
        i = self._sp_cur = 1 - self._sp_cur
        if self._sp_ev[i] is not None:
            self._sp_ev[i].synchronize()
        buf = self._sp_bufs[i]
        if buf is None or buf[0].numel() < flat.size:
            n = max(flat.size, 4096)
            buf = self._sp_bufs[i] = (torch.empty(n, dtype=torch.int32, pin_memory=True),
                                      torch.empty(n, dtype=torch.int32, device=self.device))
        buf[0].numpy()[:flat.size] = flat
        buf[1][:flat.size].copy_(buf[0][:flat.size], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._sp_ev[i] = ev
        return buf[1][:flat.size]

    def _forward(self, T, meta: AttnMetadata, hidden_in=None):
        L = self.L
        ctx = ForwardContext(meta, self.kv_caches, self.cos_sin, *self.kv_scales)
        ids = self.d64[L.ids:L.ids + T]
        pos = self.d64[L.pos:L.pos + T]
        if self.model.first:
            return self.model(ids, pos, ctx)
        h, r = hidden_in
        return self.model(None, pos, ctx, hidden=h, residual=r)

    @torch.inference_mode()
    def run(self, plan: StepPlan) -> Optional[torch.Tensor]:
        """Execute one step on this rank.  Returns sampled ids [S] (last PP stage)."""
        if ops.DEBUG and self.is_gpu:
            ops.debug_check()           # the previous step's kernels (bounds-checking build)
        if self._fake_ms:
            return self._run_fake(plan)
        self._upload(plan)
        L = self.L
        ps = self.ps
        hidden_in = None
        graph = bool(plan.B) and plan.B in self.graphs
        if not self.model.first:
            if not graph:           # a graph step receives inside its replay (pp_link)
                shp = (plan.B or plan.T, self.mcfg.hidden_size)
                hidden_in = comm.pp_recv([shp, shp], self.dtype, self.device)
        elif plan.dev_tok:
            n = max(plan.D, plan.B)
            torch.index_select(self.last_tok, 0, self.d64[L.dslots:L.dslots + n],
                               out=self.d64[L.ids + plan.Tp:L.ids + plan.Tp + n])
        if graph:
            g, logits = self.graphs[plan.B]
            link = self.pp_link
            if link is not None:
                link.pre_replay(plan.B)     # host link: this step's input rows (no-op: IPC)
            g.replay()
            if link is not None:
                link.post_replay(plan.B)    # host link: the output rows to the next stage
            self.stats["graph_steps"] += 1
            if not self.model.last:
                return None
            logits = logits[: plan.S]
            T = plan.B
        else:
            T = plan.T if not plan.B else plan.B
            D = plan.D if not plan.B else plan.B
            meta = self._meta(T, plan.Tp, plan.P, D, plan.W, plan.max_ctx, split=plan.split)
            out = self._forward(T, meta, hidden_in)
            self.stats["eager_steps"] += 1
            if not self.model.last:
                comm.pp_send(list(out))
                return None
            idx = self.d64[L.lidx:L.lidx + plan.S]
            logits = self.model.compute_logits(out.index_select(0, idx), gather=not self.vp)
        if ps.tp_size > 1:
            self._count_tp_bytes(plan, T)
        if self.vp:                 # logits are this rank's vocabulary shard
            if plan.vp:
                res = self._sample_vp(logits, plan)
                self.last_tok.index_copy_(0, self.d64[L.sslots:L.sslots + plan.S], res)
                self._last_lp = None
                return res
            logits = comm.tp_all_gather(logits, -1)[:, : self.mcfg.vocab_size]
        pre_lp = None
        if plan.proc and self.model.last:
            if plan.lp:       # logprobs report the raw distribution, before processing
                pre_lp = self._logprobs_pre(plan.lp, logits)
            if plan.proc_init:
                for slot, prompt, output in plan.proc_init:
                    self.processor.init_slot(slot, prompt, output)
            self.processor.apply(logits, plan.proc)
        out = self.sample_out[: plan.S]
        res = ops.sample(logits, self.df[L.temp:L.temp + plan.S], self.d32[L.topk:L.topk + plan.S],
                         self.df[L.topp:L.topp + plan.S], self.d64[L.seeds:L.seeds + plan.S],
                         out=out if self.is_gpu else None,
                         thresholds=self._plan_thresholds(plan))
        if plan.tok_bcast:
            comm.tp_broadcast(res, 0)          # every TP rank continues with the driver's ids
        if plan.proc and self.model.last:
            self.processor.update(plan.proc, res)
        self.last_tok.index_copy_(0, self.d64[L.sslots:L.sslots + plan.S], res)
        if plan.lp:
            self._last_lp = self._logprobs_post(pre_lp or self._logprobs_pre(plan.lp, logits), res)
        else:
            self._last_lp = None
        return res

    def _plan_thresholds(self, plan: StepPlan) -> bool:
        """Does any sampled row of this step use top-k / top-p (host-side blobs)?"""
        L, S, V = self.L, plan.S, self.mcfg.vocab_size
        k = plan.i32[L.topk:L.topk + S]
        p = plan.f32[L.topp:L.topp + S]
        return bool(((k > 0) & (k < V)).any() or (p < 1.0).any())

    def _run_fake(self, plan: StepPlan) -> Optional[torch.Tensor]:
        shp = (plan.B or plan.T, self.mcfg.hidden_size)
        if not self.model.first:
            comm.pp_recv([shp, shp], self.dtype, self.device)
        t0 = time.monotonic()
        time.sleep(self._fake_ms * 1e-3)
        t1 = time.monotonic()
        st = self.stage_stats
        st["busy_s"] += t1 - t0
        st["t_first"] = t0 if st["t_first"] is None else st["t_first"]
        st["t_last"] = t1
        st["steps"] += 1
        if not self.model.last:
            z = torch.zeros(shp, dtype=self.dtype, device=self.device)
            comm.pp_send([z, z])
            return None
        return torch.full((plan.S,), 7, dtype=torch.int64, device=self.device)

    def write_stage_stats(self) -> None:
        """KGC_STAGE_STATS_DIR: this rank's step counters (graph replays / eager steps) and,
        for fake stages, busy time and span (JSON, one file per rank)."""
        d = os.environ.get("KGC_STAGE_STATS_DIR")
        if not d or not torch.distributed.is_initialized():
            return
        import json
        with open(os.path.join(d, f"rank{torch.distributed.get_rank()}.json"), "w") as f:
            json.dump(dict(self.stage_stats, pp_rank=self.ps.pp_rank,
                           graph_steps=self.stats["graph_steps"],
                           eager_steps=self.stats["eager_steps"],
                           pp_link=type(self.pp_link).__name__ if self.pp_link else None), f)

    def _sample_vp(self, local: torch.Tensor, plan: StepPlan) -> torch.Tensor:
        S, L = plan.S, self.L
        packed = self.vp_packed[:S]
        if self.vp_cols:
            r = ops.sample_vp_partial(local, self.vp_cols, self.df[L.temp:L.temp + S],
                                      self.d64[L.seeds:L.seeds + S], self.vp_off,
                                      out=packed if self.is_gpu else None)
            if r is not packed:
                packed.copy_(r)
        else:                       # a shard of vocabulary padding only
            packed.fill_(torch.iinfo(torch.int64).min)
        comm.tp_all_reduce_max(packed)
        self.stats["vp_steps"] += 1
        return ops.sample_vp_finish(packed, out=self.sample_out[:S] if self.is_gpu else None)

    def _count_tp_bytes(self, plan: StepPlan, T: int) -> None:
        """Bytes each rank contributes to TP collectives this step (the row-parallel
        all-reduces of every layer, and the logits exchange)."""
        tp = self.ps.tp_size
        el = torch.finfo(self.dtype).bits // 8
        n_ar = 2 * self.mcfg.num_layers + 1          # o + down per layer, embedding
        self.stats["tp_allreduce_bytes"] += n_ar * T * self.mcfg.hidden_size * el
        if self.vp and plan.vp:
            self.stats["tp_logits_bytes"] += plan.S * 8
        else:
            per = self.model.lm_head.per
            self.stats["tp_logits_bytes"] += plan.S * per * (tp - 1) * el

    def _logprobs_pre(self, lp: list, logits: torch.Tensor):
        """log-softmax of the raw logits for the rows that asked for logprobs and their
        top-k alternatives (device tensors; copied to the host only when the step's
        tokens are read)."""
        rows = torch.tensor([r for r, _ in lp], device=logits.device)
        kmax = max(1, max(k for _, k in lp))
        lsm = torch.log_softmax(logits.index_select(0, rows).float(), dim=-1)
        topv, topi = lsm.topk(min(kmax, lsm.shape[-1]), dim=-1)
        return lp, rows, lsm, topv, topi

    @staticmethod
    def _logprobs_post(pre, res: torch.Tensor):
        lp, rows, lsm, topv, topi = pre
        chosen = lsm.gather(1, res.index_select(0, rows).view(-1, 1)).view(-1)
        return lp, chosen, topv, topi

    def take_logprobs(self):
        lp, self._last_lp = getattr(self, "_last_lp", None), None
        return lp

    def tokens_to_host(self, res: torch.Tensor):
        """Start the D2H copy of sampled ids into a pinned (double-buffered) host
        buffer; returns (host view, event) -- read after event.synchronize()."""
        buf = self.tok_host[self._tok_flip][: res.shape[0]]
        self._tok_flip ^= 1
        if not self.is_gpu:
            buf.copy_(res)
            return buf, None
        buf.copy_(res, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return buf, ev

    # ------------------------------------------------------------------ hipGraph capture
    @torch.inference_mode()
    def capture_graphs(self) -> float:
        """Capture decode forward + LM head for each batch bucket (largest first,
        sharing one memory pool).  Returns seconds spent."""
        self.buckets = graph_buckets(self.graph_max_bs)
        if self.is_gpu:
            # K9: per decode bucket and weight shape, hipBLASLt or the skinny GEMM --
            # whichever measured faster on this model's weights (ops/gemm.py)
            from ..ops import gemm
            # offline K9m selections for this model, where a table was made (the start-up
            # tuner then times only what the table does not cover)
            gemm.load_dg_table(self.mcfg.name, self.ps.tp_size)
            ns = getattr(self.model, "fused_norm_shapes", lambda: set())()
            # the linear layers' weights: an untied embedding table shares lm_head's shape
            # but is never a GEMM operand (and is not packed: timed with it, lm_head could
            # never take a packed K9m tile)
            tied = getattr(self.mcfg, "tie_embeddings", False)
            lin = [p for n, p in self.model.named_parameters()
                   if p.dim() == 2 and (tied or "embed" not in n)]
            gemm.tune_skinny(lin, self.buckets, norm_shapes=ns,
                             silu_shapes=getattr(self.model, "silu_shapes", lambda: set())(),
                             tail_shapes=getattr(self.model, "tail_shapes", lambda: set())(),
                             qkv_dims=getattr(self.model, "qkv_dims", lambda: {})(),
                             rs_shapes=getattr(self.model, "_rs_w", None) is not None)
        whole = self.model.first and self.model.last
        if (not self.use_graphs or not (whole or self.pp_link is not None)
                or not getattr(self.model, "graph_safe", True)):
            self.use_graphs = False
            return 0.0
        if self.ps.tp_size > 1 and comm.get_custom_allreduce() is None:
            pass  # RCCL all-reduce is capturable on ROCm (torch registers the graph stream)
        t0 = time.time()
        L, mb = self.L, self.max_blocks
        nkv = self.model.local_kv_heads()
        # a valid idle decode state: ctx_len 0 rows (write zeros), slot -1
        self.next_host_bufs()
        self.h64.zero_()
        self.h32.zero_()
        self.h64[L.slots:L.slots + self.graph_max_bs] = -1
        self.h64[L.lidx:L.lidx + self.graph_max_bs] = torch.arange(self.graph_max_bs)
        self.d64.copy_(self.h64)
        self.d32.copy_(self.h32)
        torch.cuda.synchronize()
        self.graph_pool = torch.cuda.graph_pool_handle()
        for B in sorted(self.buckets, reverse=True):
            z = ops.decode_grid_z(B, nkv, self.max_model_len)
            meta = self._meta(B, 0, 0, B, 0, self.max_model_len, z=z)

            def step_body(B=B, meta=meta):
                # PP stages: receive from the previous stage / send to the next one as
                # kernels over peer memory, so the whole stage step is one replay (host
                # link: the graph reads / writes static rows, moved around the replay)
                hin = self.pp_link.recv(B) if not self.model.first else None
                h = self._forward(B, meta, hin)
                if not self.model.last:
                    self.pp_link.send(*h)
                    return None
                # graph rows sample their own hidden row (build_plan sets lidx = 0..B-1 for
                # every graph step): no gather launch in the replay
                return self.model.compute_logits(h, gather=not self.vp)
            for _ in range(2):   # warm up (allocator, library handles) outside capture;
                step_body()      # PP: every stage runs the same warm-ups, in bucket order
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.graph_pool):
                logits = step_body()
            self.graphs[B] = (g, logits)
        torch.cuda.synchronize()
        return time.time() - t0
