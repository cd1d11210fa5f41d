"""Per-request logits processing before sampling (vLLM / OpenAI semantics):

* ``presence_penalty`` / ``frequency_penalty`` over the tokens generated so far;
* ``repetition_penalty`` over prompt + generated tokens (positive logits divided,
  negative multiplied);
* ``logit_bias`` (token id -> additive bias);
* ``min_p``: drop tokens whose probability is below ``min_p`` x the top probability.

Only the rows of requests that use one of these are touched, so the common path
(none used) costs nothing.  Token statistics live on the device: one int32 count row
and one prompt bitmap row per running-sequence slot.  They are allocated on first use
and updated with a scatter after each sampling step, so the host never walks token
lists for a decode step.  A sequence (re)entering a slot, on admission or after
recompute preemption, has its row rebuilt from its token lists.
"""
from __future__ import annotations

from typing import Optional

import torch


def needs_processing(p) -> bool:
    return bool(p.presence_penalty or p.frequency_penalty or p.repetition_penalty != 1.0
                or p.logit_bias or p.min_p > 0.0)


def needs_counts(p) -> bool:
    return bool(p.presence_penalty or p.frequency_penalty or p.repetition_penalty != 1.0)


class LogitsProcessor:
    def __init__(self, max_seqs: int, vocab: int, device: torch.device):
        self.max_seqs, self.vocab, self.device = max_seqs, vocab, device
        self.counts: Optional[torch.Tensor] = None      # [slots, V] int32: generated tokens
        self.prompt_mask: Optional[torch.Tensor] = None  # [slots, V] bool: prompt tokens

    def _ensure(self) -> None:
        if self.counts is None:
            self.counts = torch.zeros(self.max_seqs, self.vocab, dtype=torch.int32, device=self.device)
            self.prompt_mask = torch.zeros(self.max_seqs, self.vocab, dtype=torch.bool,
                                           device=self.device)

    def init_slot(self, slot: int, prompt: list[int], output: list[int]) -> None:
        """(Re)build a slot's statistics from the sequence's token lists."""
        self._ensure()
        self.counts[slot].zero_()
        self.prompt_mask[slot].zero_()
        if prompt:
            self.prompt_mask[slot, torch.tensor(prompt, device=self.device)] = True
        out = [t for t in output if t >= 0]
        if out:
            idx = torch.tensor(out, device=self.device)
            self.counts[slot].index_add_(0, idx, torch.ones_like(idx, dtype=torch.int32))

    def apply(self, logits: torch.Tensor, rows: list[tuple]) -> None:
        """In place on ``logits`` [S, V]; rows = [(row, slot, SamplingParams)]."""
        V = min(logits.shape[-1], self.vocab)
        dev = logits.device
        r = torch.tensor([x[0] for x in rows], device=dev)
        sub = logits.index_select(0, r).float()
        pen = [(i, x) for i, x in enumerate(rows) if needs_counts(x[2])]
        if pen:
            self._ensure()
            j = torch.tensor([i for i, _ in pen], device=dev)
            slots = torch.tensor([x[1] for _, x in pen], device=dev)
            pen = [x for _, x in pen]
            cnt = self.counts.index_select(0, slots)[:, :V].float()
            pm = self.prompt_mask.index_select(0, slots)[:, :V]
            pres = torch.tensor([x[2].presence_penalty for x in pen], device=dev)[:, None]
            freq = torch.tensor([x[2].frequency_penalty for x in pen], device=dev)[:, None]
            rep = torch.tensor([x[2].repetition_penalty for x in pen], device=dev)[:, None]
            s = sub.index_select(0, j)[:, :V]
            seen = (cnt > 0) | pm
            s = torch.where(seen & (s > 0), s / rep, torch.where(seen, s * rep, s))
            s = s - freq * cnt - pres * (cnt > 0).float()
            sub[j, :V] = s
        for i, (_, _, p) in enumerate(rows):
            if p.logit_bias:
                ids = torch.tensor([int(k) for k in p.logit_bias], device=dev)
                vals = torch.tensor([float(v) for v in p.logit_bias.values()], device=dev)
                ok = ids < V
                sub[i].index_add_(0, ids[ok], vals[ok])
        mp = [(i, p.min_p, p.temperature) for i, (_, _, p) in enumerate(rows) if p.min_p > 0]
        if mp:
            j = torch.tensor([m[0] for m in mp], device=dev)
            t = torch.tensor([max(m[2], 1e-5) if m[2] > 0 else 1.0 for m in mp], device=dev)[:, None]
            pm = torch.tensor([m[1] for m in mp], device=dev)[:, None]
            s = sub.index_select(0, j)
            prob = torch.softmax(s / t, dim=-1)
            keep = prob >= pm * prob.max(dim=-1, keepdim=True).values
            sub[j] = torch.where(keep, s, torch.full_like(s, float("-inf")))
        logits.index_copy_(0, r, sub.to(logits.dtype))

    def update(self, rows: list[tuple], sampled: torch.Tensor) -> None:
        """Count each penalised row's new token (device scatter, no host sync)."""
        pen = [(x[0], x[1]) for x in rows if needs_counts(x[2])]
        if not pen:
            return
        dev = sampled.device
        j = torch.tensor([p[0] for p in pen], device=dev)
        slots = torch.tensor([p[1] for p in pen], device=dev)
        tok = sampled.index_select(0, j).clamp_(0, self.vocab - 1)
        self.counts.index_put_((slots, tok), torch.ones_like(tok, dtype=torch.int32), accumulate=True)
