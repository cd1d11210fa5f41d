"""A GPU-free stand-in for ``LLMEngine`` with the serving engine's step timing.

Used to load-test and profile everything above the engine -- the engine-core pipe,
the OpenAI API server, detokenisation and SSE, the router, the benchmark client --
on a CPU-only machine, and as a fault-injection target in tests.  Select it in the
API server's engine-core process with ``KGC_FAKE_ENGINE=1`` (default timing) or
``KGC_FAKE_ENGINE=<base_ms>,<us_per_token>,<us_per_decode_seq>``.

Scheduling follows the real scheduler's policy: FCFS, running sequences decode one
token per step, then waiting prompts are prefilled in chunks within
``max_num_batched_tokens`` while at most ``max_num_seqs`` run.  A step sleeps

    base_ms + us_per_token * tokens_in_step + us_per_decode_seq * decoding_seqs

which, with the defaults, reproduces the measured Llama-3-8B TP=1 engine on one
MI355X (profiles/llama3-8b_tp1_bench_kernels.txt): ~11 ms for a 256-sequence decode
step, ~150 ms for a 16384-token prefill chunk.
"""
from __future__ import annotations

import os
import random
import time
from dataclasses import dataclass, field
from typing import Optional

from ..models.configs import resolve_model
from ..utils.metrics import EngineMetrics
from .config import EngineConfig
from .worker import default_max_model_len


@dataclass
class _Req:
    rid: str
    prompt_len: int
    max_tokens: int
    arrival: float
    prefilled: int = 0
    out: list = field(default_factory=list)
    first_token_time: Optional[float] = None


@dataclass
class FakeOutput:
    request_id: str
    new_token_ids: list
    finished: bool
    finish_reason: Optional[str]
    arrival_time: float
    first_token_time: Optional[float]
    finish_time: Optional[float]
    num_preemptions: int = 0
    logprobs: Optional[list] = None
    num_output_tokens: int = 0


def timing_from_env(spec: str) -> tuple[float, float, float]:
    parts = [float(x) for x in spec.split(",")] if spec not in ("", "1") else []
    base_ms, us_tok, us_seq = (parts + [3.7, 8.9, 12.0][len(parts):])[:3]
    return base_ms, us_tok, us_seq


class FakeEngine:
    def __init__(self, cfg: EngineConfig, timing: Optional[tuple[float, float, float]] = None):
        self.cfg = cfg
        self.mcfg, _ = resolve_model(cfg.model)
        self.max_model_len = default_max_model_len(cfg)
        self.base_ms, self.us_tok, self.us_seq = timing or timing_from_env(
            os.environ.get("KGC_FAKE_ENGINE", "1"))
        self.max_seqs = cfg.max_num_seqs
        self.budget = cfg.token_budget()
        self.waiting: list[_Req] = []
        self.running: list[_Req] = []
        self.metrics = EngineMetrics(model_name=cfg.served_model_name or cfg.model)
        self.rng = random.Random(0)

    def add_request(self, prompt_ids, params, request_id: str, arrival_time=None):
        if len(prompt_ids) >= self.max_model_len:
            raise ValueError(f"prompt of {len(prompt_ids)} tokens >= max_model_len")
        self.waiting.append(_Req(request_id, len(prompt_ids), params.max_tokens or 16,
                                 arrival_time if arrival_time is not None else time.monotonic()))

    def abort(self, request_id: str) -> None:
        self.waiting = [r for r in self.waiting if r.rid != request_id]
        self.running = [r for r in self.running if r.rid != request_id]

    def has_unfinished(self) -> bool:
        return bool(self.waiting or self.running)

    def step(self) -> list[FakeOutput]:
        decodes = [r for r in self.running if r.prefilled >= r.prompt_len]
        budget = self.budget - len(decodes)
        prefill = []
        for r in self.running:                       # chunked prefills in flight first
            if r.prefilled < r.prompt_len and budget > 0:
                n = min(budget, r.prompt_len - r.prefilled)
                prefill.append((r, n))
                budget -= n
        while self.waiting and budget > 0 and len(self.running) < self.max_seqs:
            r = self.waiting.pop(0)
            self.running.append(r)
            n = min(budget, r.prompt_len)
            prefill.append((r, n))
            budget -= n
        tokens = len(decodes) + sum(n for _, n in prefill)
        time.sleep((self.base_ms + self.us_tok * 1e-3 * tokens
                    + self.us_seq * 1e-3 * len(decodes)) * 1e-3)
        now = time.monotonic()
        outs = []
        emit = list(decodes)
        for r, n in prefill:
            r.prefilled += n
            if r.prefilled >= r.prompt_len:
                emit.append(r)
        for r in emit:
            tok = self.rng.randrange(100, max(101, self.mcfg.vocab_size - 100))
            r.out.append(tok)
            if r.first_token_time is None:
                r.first_token_time = now
            done = len(r.out) >= r.max_tokens
            outs.append(FakeOutput(r.rid, [tok], done, "length" if done else None, r.arrival,
                                   r.first_token_time, now if done else None,
                                   num_output_tokens=len(r.out)))
            if done:
                self.running.remove(r)
        return outs

    def shutdown(self) -> None:
        pass
