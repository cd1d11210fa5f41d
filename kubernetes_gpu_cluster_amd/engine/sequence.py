"""Request / sequence state and sampling parameters (OpenAI semantics)."""
from __future__ import annotations

import dataclasses
import enum
import itertools
import time
from typing import Optional

_seq_ids = itertools.count()


@dataclasses.dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    max_tokens: Optional[int] = 16
    min_tokens: int = 0
    stop_token_ids: list[int] = dataclasses.field(default_factory=list)
    stop: list[str] = dataclasses.field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None
    n: int = 1
    logprobs: Optional[int] = None
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0
    min_p: float = 0.0
    logit_bias: Optional[dict] = None
    needs_proc: bool = dataclasses.field(default=False, init=False, repr=False)

    def __post_init__(self):
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not 0 < self.top_p <= 1:
            raise ValueError("top_p must be in (0, 1]")
        if self.top_k == 0 or self.top_k < -1:
            raise ValueError("top_k must be -1 (disabled) or >= 1")
        if self.max_tokens is not None and self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.n < 1:
            raise ValueError("n must be >= 1")
        if not -2.0 <= self.presence_penalty <= 2.0 or not -2.0 <= self.frequency_penalty <= 2.0:
            raise ValueError("presence_penalty / frequency_penalty must be in [-2, 2]")
        if self.repetition_penalty <= 0:
            raise ValueError("repetition_penalty must be > 0")
        if not 0.0 <= self.min_p <= 1.0:
            raise ValueError("min_p must be in [0, 1]")
        if self.logit_bias:
            for k, v in self.logit_bias.items():
                if not -100 <= float(v) <= 100:
                    raise ValueError("logit_bias values must be in [-100, 100]")
                int(k)
        # penalties / bias / min_p need the driver-side logits processor
        self.needs_proc = bool(self.presence_penalty or self.frequency_penalty
                               or self.repetition_penalty != 1.0 or self.logit_bias
                               or self.min_p > 0.0)


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


class Sequence:
    __slots__ = ("seq_id", "request_id", "prompt_token_ids", "output_token_ids", "params",
                 "status", "block_ids", "num_computed", "arrival_time", "first_token_time",
                 "finish_time", "finish_reason", "seed", "num_preemptions", "max_tokens",
                 "slot", "last_token_time", "token_times", "prompt_text", "stream",
                 "num_pending", "proc_slot", "block_keys", "num_registered", "vengine")

    def __init__(self, request_id: str, prompt_token_ids: list[int], params: SamplingParams,
                 arrival_time: Optional[float] = None, max_model_len: int = 1 << 30):
        self.seq_id = next(_seq_ids)
        self.request_id = request_id
        self.prompt_token_ids = list(prompt_token_ids)
        self.output_token_ids: list[int] = []
        self.params = params
        self.status = SeqStatus.WAITING
        self.block_ids: list[int] = []
        self.num_computed = 0                 # tokens whose KV is in the cache
        self.arrival_time = time.monotonic() if arrival_time is None else arrival_time
        self.first_token_time: Optional[float] = None
        self.last_token_time: Optional[float] = None
        self.finish_time: Optional[float] = None
        self.finish_reason: Optional[str] = None
        self.seed = params.seed if params.seed is not None else (self.seq_id * 0x9E3779B1) & 0x7FFFFFFF
        self.num_preemptions = 0
        room = max_model_len - len(self.prompt_token_ids)
        self.max_tokens = room if params.max_tokens is None else min(params.max_tokens, room)
        self.slot = -1
        self.token_times: list[float] = []
        self.prompt_text: Optional[str] = None
        self.stream = None
        self.num_pending = 0                  # trailing sampled tokens still on the GPU
        self.proc_slot = -1                   # slot whose penalty statistics are built
        self.block_keys: list[bytes] = []       # prefix-cache keys of its full blocks
        self.num_registered = 0               # leading blocks published to the prefix cache
        self.vengine = 0                      # PP micro-batch (engine/scheduler.VirtualSchedulers)

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_token_ids) + len(self.output_token_ids)

    @property
    def num_prompt(self) -> int:
        return len(self.prompt_token_ids)

    def token_at(self, i: int) -> int:
        n = len(self.prompt_token_ids)
        return self.prompt_token_ids[i] if i < n else self.output_token_ids[i - n]

    def tokens_slice(self, a: int, b: int) -> list[int]:
        n = len(self.prompt_token_ids)
        if b <= n:
            return self.prompt_token_ids[a:b]
        if a >= n:
            return self.output_token_ids[a - n:b - n]
        return self.prompt_token_ids[a:] + self.output_token_ids[: b - n]

    @property
    def is_prefilling(self) -> bool:
        return self.num_computed < self.num_tokens - 1 or (
            self.num_computed < self.num_prompt)

    @property
    def finished(self) -> bool:
        return self.status == SeqStatus.FINISHED


@dataclasses.dataclass
class RequestOutput:
    """Per-step output of one request.  ``output_token_ids`` is a view of the
    sequence's token list cut at the tokens resolved so far (no O(n) copy per step;
    the list only grows past ``num_output_tokens`` or is truncated beyond it)."""
    request_id: str
    prompt_token_ids: list[int]
    new_token_ids: list[int]
    _ids: list[int]
    num_output_tokens: int
    finished: bool
    finish_reason: Optional[str] = None
    arrival_time: float = 0.0
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    num_preemptions: int = 0
    # per new token, when the request asked for logprobs:
    # (token id, logprob, [(alternative id, logprob)] top-k)
    logprobs: Optional[list] = None

    @property
    def output_token_ids(self) -> list[int]:
        return self._ids[:self.num_output_tokens]

    @property
    def ttft(self) -> Optional[float]:
        return None if self.first_token_time is None else self.first_token_time - self.arrival_time
