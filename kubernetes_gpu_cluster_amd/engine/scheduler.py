"""Continuous-batching scheduler with chunked prefill and recompute preemption.

Each step has a token budget (``max_num_batched_tokens``) and a sequence cap
(``max_num_seqs``).  Policy (decode-first, as in vLLM's V1 scheduler):

1. Running sequences, FCFS: a decoding sequence takes 1 token; a sequence still in
   (chunked) prefill takes min(remaining, budget).  If the KV pool cannot grow,
   the newest running sequence is preempted (blocks freed, re-queued at the front
   of the waiting queue, recomputed later) until the allocation fits.
2. If nothing was preempted, waiting sequences are admitted FCFS while budget,
   the sequence cap and free blocks (with a small watermark) allow.

A scheduled unit is (sequence, n_tokens): tokens [num_computed, num_computed+n)
are run; if that reaches the end of the sequence, a new token is sampled.  With
prefix caching, an admitted sequence first takes the cached blocks of its longest
cached prefix and starts computing after them.
"""
from __future__ import annotations

import collections
import dataclasses
import time
from typing import Optional

from .block_manager import BlockManager
from .sequence import SeqStatus, Sequence


@dataclasses.dataclass
class ScheduledBatch:
    prefills: list[tuple[Sequence, int]]      # (seq, n_tokens), n may be 1 for 1-token prompts
    decodes: list[Sequence]                   # one token each
    preempted: list[Sequence]

    @property
    def num_tokens(self) -> int:
        return sum(n for _, n in self.prefills) + len(self.decodes)

    @property
    def is_empty(self) -> bool:
        return not self.prefills and not self.decodes

    def all_seqs(self) -> list[tuple[Sequence, int]]:
        return self.prefills + [(s, 1) for s in self.decodes]


class Scheduler:
    def __init__(self, block_manager: BlockManager, max_num_seqs: int, token_budget: int,
                 max_model_len: int, chunked_prefill: bool = True, prefill_first: bool = False,
                 max_defer_steps: int = 8, max_decode_gap_ms: float = 0.0):
        self.bm = block_manager
        # prefill-first: while prompts wait and a sequence slot is free, decoding sequences
        # sit the step out and the whole token budget goes to prefill (lower TTFT under a
        # burst, at the cost of the running sequences' TPOT).  Bounded: after
        # max_defer_steps consecutive steps that skipped decodes (or once a running
        # sequence has waited max_decode_gap_ms for a token), the next step decodes every
        # running sequence and prefill takes what is left of the budget -- under continuous
        # arrivals the running streams never starve.
        self.prefill_first = prefill_first
        self.max_defer_steps = max(0, max_defer_steps)
        self.max_decode_gap_s = max(0.0, max_decode_gap_ms) / 1e3
        self._deferred = 0              # consecutive steps whose decodes sat out
        self._skipped = 0
        self.max_num_seqs = max_num_seqs
        self.token_budget = token_budget
        self.max_model_len = max_model_len
        self.chunked = chunked_prefill
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.running: list[Sequence] = []
        self.num_preemptions = 0

    def add(self, seq: Sequence) -> None:
        self.waiting.append(seq)

    def abort(self, request_id: str) -> Optional[Sequence]:
        for q in (self.running, self.waiting):
            for s in list(q):
                if s.request_id == request_id:
                    q.remove(s)
                    self.bm.free_seq(s)
                    s.status = SeqStatus.FINISHED
                    s.finish_reason = "abort"
                    return s
        return None

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def _preempt(self, seq: Sequence) -> None:
        self.bm.free_seq(seq)
        seq.num_computed = 0
        seq.status = SeqStatus.WAITING
        seq.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(seq)

    def _decode_overdue(self) -> bool:
        if self.max_decode_gap_s <= 0:
            return False
        now = time.monotonic()
        return any(s.last_token_time is not None and now - s.last_token_time > self.max_decode_gap_s
                   for s in self.running)

    def schedule(self) -> ScheduledBatch:
        defer = (self.prefill_first and bool(self.waiting)
                 and len(self.running) < self.max_num_seqs
                 and self._deferred < self.max_defer_steps and not self._decode_overdue())
        self._skipped = 0
        batch = self._schedule(defer)
        if defer and batch.is_empty:
            # nothing admissible (e.g. the KV pool is full): decode as usual
            self._skipped = 0
            batch = self._schedule(False)
        self._deferred = self._deferred + 1 if self._skipped else 0
        return batch

    def _schedule(self, defer_decodes: bool) -> ScheduledBatch:
        budget = self.token_budget
        prefills: list[tuple[Sequence, int]] = []
        decodes: list[Sequence] = []
        preempted: list[Sequence] = []
        i = 0
        while i < len(self.running) and budget > 0:
            seq = self.running[i]
            remaining = seq.num_tokens - seq.num_computed
            if defer_decodes and remaining == 1:
                self._skipped += 1
                i += 1
                continue
            n = 1 if remaining == 1 else min(remaining, budget)
            scheduled = True
            while not self.bm.can_allocate(seq, seq.num_computed + n):
                victim = self.running.pop()
                self._preempt(victim)
                preempted.append(victim)
                if victim is seq:
                    scheduled = False
                    break
            if not scheduled:
                break
            self.bm.allocate(seq, seq.num_computed + n)
            if n == 1 and remaining == 1:
                decodes.append(seq)
            else:
                prefills.append((seq, n))
            budget -= n
            i += 1
        if not preempted:
            bs = self.bm.block_size
            while self.waiting and budget > 0 and len(self.running) < self.max_num_seqs:
                seq = self.waiting[0]
                # prefix caching: leading full blocks already in the cache are not recomputed
                hits = self.bm.cached_prefix_blocks(seq) if self.bm.prefix_caching else []
                start = seq.num_computed + len(hits) * bs
                remaining = seq.num_tokens - start
                n = min(remaining, budget)
                if n < remaining and not self.chunked:
                    break
                if not self.bm.can_admit(seq, start + n, hits):
                    break
                self.waiting.popleft()
                if self.bm.prefix_caching:
                    self.bm.note_query(seq)
                    if hits:
                        seq.num_computed += self.bm.take_prefix(seq, hits)
                self.bm.allocate(seq, seq.num_computed + n)
                seq.status = SeqStatus.RUNNING
                self.running.append(seq)
                prefills.append((seq, n))
                budget -= n
        return ScheduledBatch(prefills, decodes, preempted)

    def finish(self, seq: Sequence, reason: str) -> None:
        seq.status = SeqStatus.FINISHED
        seq.finish_reason = reason
        self.bm.free_seq(seq)
        try:
            self.running.remove(seq)
        except ValueError:
            pass


class VirtualSchedulers:
    """Pipeline parallelism: one scheduler per micro-batch ("virtual engine") over the
    shared KV pool.  The engine launches micro-batch v's step, then v+1's, ... and only
    returns to v once v's tokens are back from the last stage, so with ``pp_size``
    micro-batches every stage has work (vLLM's virtual-engine scheme).  A sequence stays
    in the micro-batch it was admitted to (``seq.vengine``); new requests go to the one
    with the fewest sequences.  Each holds at most ``max_num_seqs // n`` sequences, and
    each step still has the full token budget."""

    def __init__(self, n: int, block_manager: BlockManager, max_num_seqs: int, token_budget: int,
                 max_model_len: int, chunked_prefill: bool = True, prefill_first: bool = False,
                 max_defer_steps: int = 8, max_decode_gap_ms: float = 0.0):
        per = max(1, max_num_seqs // n)
        self.scheds = [Scheduler(block_manager, per, token_budget, max_model_len, chunked_prefill,
                                 prefill_first, max_defer_steps, max_decode_gap_ms)
                       for _ in range(n)]

    def __len__(self) -> int:
        return len(self.scheds)

    def add(self, seq: Sequence) -> None:
        v = min(range(len(self.scheds)),
                key=lambda i: len(self.scheds[i].running) + len(self.scheds[i].waiting))
        seq.vengine = v
        self.scheds[v].add(seq)

    def abort(self, request_id: str) -> Optional[Sequence]:
        for sc in self.scheds:
            s = sc.abort(request_id)
            if s is not None:
                return s
        return None

    def has_work(self) -> bool:
        return any(sc.has_work() for sc in self.scheds)

    def schedule_v(self, v: int) -> ScheduledBatch:
        return self.scheds[v].schedule()

    def finish(self, seq: Sequence, reason: str) -> None:
        self.scheds[getattr(seq, "vengine", 0)].finish(seq, reason)

    @property
    def running(self) -> list[Sequence]:
        return [s for sc in self.scheds for s in sc.running]

    @property
    def waiting(self) -> list[Sequence]:
        return [s for sc in self.scheds for s in sc.waiting]

    @property
    def num_preemptions(self) -> int:
        return sum(sc.num_preemptions for sc in self.scheds)
