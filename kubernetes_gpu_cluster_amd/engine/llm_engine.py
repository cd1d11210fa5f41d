"""LLMEngine: request intake, the schedule -> execute -> update step loop, and the
offline ``LLM.generate`` API.

One call to ``step()`` = one engine iteration (the serving hot loop of SURVEY.md
§3.5): the scheduler picks a continuous batch (decodes + chunked prefills), the
driver packs it into a StepPlan, every rank runs it, and sampled tokens are
appended; stop conditions (EOS unless ignore_eos, stop_token_ids, max_tokens,
max_model_len) finish sequences and free their KV blocks.
"""
from __future__ import annotations

import collections
import itertools
import logging
import os
import time
from typing import Iterable, Optional, Union

from ..models import resolve_model
from ..utils.metrics import EngineMetrics
from .block_manager import BlockManager
from .config import EngineConfig
from .scheduler import Scheduler, VirtualSchedulers
from .sequence import RequestOutput, SamplingParams, SeqStatus, Sequence
from .worker import TokenFuture, LocalExecutor, MultiprocExecutor, default_max_model_len

log = logging.getLogger("kgc.engine")
_PENDING = -1          # placeholder for a sampled token still on the GPU


class _StepProfiler:
    """``KGC_TORCH_PROFILE=dir[:start[:steps]]``: record engine steps start..start+steps
    with torch.profiler (CPU + HIP activity) and write a Chrome trace into dir."""

    def __init__(self, out_dir: str, start: int, steps: int):
        self.dir, self.start, self.stop, self.n, self.p = out_dir, start, start + steps, 0, None

    @classmethod
    def from_env(cls):
        spec = os.environ.get("KGC_TORCH_PROFILE")
        if not spec:
            return None
        parts = spec.split(":")
        return cls(parts[0], int(parts[1]) if len(parts) > 1 else 20,
                   int(parts[2]) if len(parts) > 2 else 10)

    def tick(self) -> None:
        import torch
        if self.n == self.start:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.p = torch.profiler.profile(activities=acts, record_shapes=False)
            self.p.__enter__()
        elif self.n == self.stop and self.p is not None:
            self.p.__exit__(None, None, None)
            os.makedirs(self.dir, exist_ok=True)
            path = os.path.join(self.dir, f"engine_steps_{self.start}_{self.stop}.json")
            self.p.export_chrome_trace(path)
            log.info("torch profiler trace: %s", path)
            self.p = None
        self.n += 1


class LLMEngine:
    def __init__(self, cfg: EngineConfig, executor=None):
        self.cfg = cfg
        self.mcfg, _ = resolve_model(cfg.model)
        self.max_model_len = default_max_model_len(cfg)
        if executor is None:
            executor = LocalExecutor(cfg) if cfg.world_size == 1 else MultiprocExecutor(cfg)
        self.executor = executor
        t0 = time.time()
        nb = executor.profile()
        # like vLLM: refuse to start when not even one max-length sequence fits
        # (otherwise requests would wait forever for blocks that never free up)
        cap = (nb - 1) * cfg.block_size
        if cap < self.max_model_len:
            executor.shutdown()
            raise ValueError(
                f"KV cache holds {max(cap, 0)} tokens ({nb} blocks of {cfg.block_size}), less than "
                f"max_model_len={self.max_model_len}: raise --gpu-memory-utilization, lower "
                f"--max-model-len, use --kv-cache-dtype fp8, or add tensor parallelism")
        executor.init_cache(nb)
        self.graph_s = executor.capture()
        self.num_blocks = nb
        runner = executor.runner
        self.bm = BlockManager(nb, cfg.block_size, cfg.max_num_seqs, runner.max_blocks,
                               enable_prefix_caching=cfg.enable_prefix_caching)
        # PP > 1: one micro-batch per stage in flight (engine/scheduler.VirtualSchedulers)
        self.pp_depth = int(getattr(executor, "pipeline_depth", 1))
        if self.pp_depth > 1:
            self.scheduler = VirtualSchedulers(self.pp_depth, self.bm, cfg.max_num_seqs,
                                               cfg.token_budget(), self.max_model_len,
                                               cfg.enable_chunked_prefill, cfg.prefill_first,
                                               cfg.prefill_first_max_defer,
                                               cfg.prefill_first_max_gap_ms)
        else:
            self.scheduler = Scheduler(self.bm, cfg.max_num_seqs, cfg.token_budget(),
                                       self.max_model_len, cfg.enable_chunked_prefill,
                                       cfg.prefill_first, cfg.prefill_first_max_defer,
                                       cfg.prefill_first_max_gap_ms)
        self._pp_inflight: list = [None] * self.pp_depth
        self._vnext = 0
        self.seqs: dict[str, Sequence] = {}
        self._ids = itertools.count()
        self.metrics = EngineMetrics()
        self.eos = self.mcfg.eos_token_id
        self.async_mode = cfg.async_output and getattr(executor, "supports_async", False)
        self._inflight = None
        self._debug = os.environ.get("KGC_DEBUG", "0") == "1"
        self._prof = _StepProfiler.from_env()
        self._host_t = (collections.defaultdict(float)
                        if os.environ.get("KGC_HOST_TIMING", "0") == "1" else None)
        self.init_s = time.time() - t0
        log.info("engine ready: %d KV blocks x %d tokens, graphs %.1fs", nb, cfg.block_size,
                 self.graph_s)

    # ------------------------------------------------------------------ requests
    def add_request(self, prompt_token_ids: list[int], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None, arrival_time: Optional[float] = None) -> Sequence:
        params = params or SamplingParams()
        rid = request_id if request_id is not None else f"req-{next(self._ids)}"
        if not prompt_token_ids:
            raise ValueError("empty prompt")
        if len(prompt_token_ids) >= self.max_model_len:
            raise ValueError(f"prompt of {len(prompt_token_ids)} tokens exceeds max_model_len "
                             f"{self.max_model_len}")
        if max(prompt_token_ids) >= self.mcfg.vocab_size or min(prompt_token_ids) < 0:
            raise ValueError("prompt token id out of vocabulary range")
        if self.pp_depth > 1 and params.logprobs is not None:
            # the pipelined path returns only the sampled ids from the last stage
            raise ValueError("logprobs are not supported with pipeline_parallel_size > 1")
        seq = Sequence(rid, prompt_token_ids, params, arrival_time, self.max_model_len)
        self.seqs[rid] = seq
        self.scheduler.add(seq)
        self.metrics.on_arrival()
        return seq

    def coalescing(self) -> bool:
        """A burst is being admitted: nothing is running or in flight, and the waiting
        prompts fill less than one step's token budget (the engine-core loop then keeps
        admitting arrivals for a moment before it steps: entrypoints/engine_core.py)."""
        s = self.scheduler
        if self.pp_depth > 1 or not s.waiting or s.running or self._inflight is not None:
            return False
        budget, tot = self.cfg.token_budget(), 0
        for seq in s.waiting:
            tot += seq.num_tokens - seq.num_computed
            if tot >= budget:
                return False
        return True

    def inflight_coalescing(self) -> bool:
        """A prefill-only step of at least half the token budget is still running on the
        GPU, and the prompts waiting now (possibly none) fill less than the next step's
        budget: under a burst the rest is still arriving, so the engine-core loop may
        keep admitting arrivals before it launches the next step (a partial prefill, or
        with nothing waiting at that instant, a decode step the prefill-first policy would
        then interleave with the burst's remaining chunks)."""
        inf = self._inflight
        if inf is None or self.pp_depth > 1:
            return False
        fut, _, plan, _, _ = inf
        budget = self.cfg.token_budget()
        if plan.D or plan.Tp < budget // 2 or fut.done():
            return False
        s = self.scheduler
        if len(s.running) >= self.cfg.max_num_seqs:
            return False
        tot = 0
        for seq in s.waiting:
            tot += seq.num_tokens - seq.num_computed
            if tot >= budget:
                return False
        return True

    def abort(self, request_id: str) -> None:
        s = self.scheduler.abort(request_id)
        self.seqs.pop(request_id, None)
        if s is not None:
            self.metrics.on_finish(s)

    def has_unfinished(self) -> bool:
        return (self.scheduler.has_work() or self._inflight is not None
                or any(x is not None for x in self._pp_inflight))

    # ------------------------------------------------------------------ step
    def step(self) -> list[RequestOutput]:
        """One engine iteration.  In async mode (default, TP x PP with PP == 1) the
        step launches batch N and then processes the tokens of batch N-1 while batch N
        runs on the GPU: decode inputs come from the device-side last-token table, so
        host bookkeeping (sampled-token append, stop checks, scheduling) overlaps GPU
        execution.  EOS / stop-token finishes are therefore seen one step late (the
        extra token is discarded); length finishes are exact."""
        if self._debug:
            self.bm.check_invariants(list(self.scheduler.running))
        if self._prof is not None:
            self._prof.tick()
        if self.pp_depth > 1:
            return self._step_pipelined()
        if not self.async_mode:
            return self._step_sync()
        launched = None
        ht = self._host_t
        h0 = time.perf_counter() if ht is not None else 0.0
        batch = self.scheduler.schedule()
        if not batch.is_empty:
            t0 = time.monotonic()
            h1 = time.perf_counter() if ht is not None else 0.0
            plan, samplers = self.executor.runner.build_plan(batch.prefills, batch.decodes,
                                                             self.bm.table, device_tokens=True)
            h2 = time.perf_counter() if ht is not None else 0.0
            fut = self.executor.execute_async(plan)
            h3 = time.perf_counter() if ht is not None else 0.0
            launched = self._launched(batch, plan, samplers, fut, t0)
            if ht is not None:
                ht["schedule"] += h1 - h0
                ht["build_plan"] += h2 - h1
                ht["launch"] += h3 - h2
                h0 = time.perf_counter()
        if self._inflight is not None:
            if ht is not None:
                w0 = time.perf_counter()
                self._inflight[0].result()
                ht["wait"] += time.perf_counter() - w0
                h0b = time.perf_counter()
            outs = self._process(self._inflight)
            if ht is not None:
                ht["process"] += time.perf_counter() - h0b
                ht["steps"] += 1
        else:
            outs = []
        self._inflight = launched
        return outs

    def host_timing(self) -> Optional[dict]:
        """KGC_HOST_TIMING=1: seconds the host spent per engine step in scheduling,
        building the step plan, launching (upload + graph replay + sampler enqueue),
        waiting for the previous step's tokens, and processing them (async mode)."""
        if self._host_t is None:
            return None
        n = max(1, self._host_t["steps"])
        return {k: (round(v / n * 1e6, 1) if k != "steps" else v) for k, v in self._host_t.items()}

    def _step_pipelined(self) -> list[RequestOutput]:
        """PP > 1: micro-batch v = this step's turn.  Its previous step's tokens are read
        first (they left the last stage while the other micro-batches ran), then its next
        step is scheduled and handed to stage 0, and the call returns without waiting."""
        v = self._vnext
        self._vnext = (v + 1) % self.pp_depth
        outs: list[RequestOutput] = []
        if self._pp_inflight[v] is not None:
            outs = self._process(self._pp_inflight[v])
            self._pp_inflight[v] = None
        batch = self.scheduler.schedule_v(v)
        if not batch.is_empty:
            t0 = time.monotonic()
            plan, samplers = self.executor.runner.build_plan(batch.prefills, batch.decodes,
                                                             self.bm.table)
            fut = self.executor.execute_pipelined(plan)
            self._pp_inflight[v] = self._launched(batch, plan, samplers, fut, t0)
        return outs

    def _launched(self, batch, plan, samplers, fut, t0):
        """Host bookkeeping of a step handed to the device before its tokens are known."""
        for seq, n in batch.prefills:
            seq.num_computed += n
        for seq in batch.decodes:
            seq.num_computed += 1
        for seq in samplers:
            seq.output_token_ids.append(_PENDING)
            seq.num_pending += 1
        if self.bm.prefix_caching:      # publish blocks whose token ids are all known
            for seq, _ in batch.prefills:
                self.bm.register_full_blocks(seq, seq.num_tokens - seq.num_pending)
        for seq in samplers:
            if len(seq.output_token_ids) >= seq.max_tokens or seq.num_tokens >= self.max_model_len:
                # finished by length: release now (stream order protects the KV
                # blocks still being written by the in-flight step)
                self.scheduler.finish(seq, "length")
                self.seqs.pop(seq.request_id, None)
        return (fut, samplers, plan, t0, len(batch.preempted))

    def _process(self, inflight) -> list[RequestOutput]:
        fut, samplers, plan, t0, npre = inflight
        tokens = fut.result()
        lps = fut.logprobs() if plan.lp else {}
        now = time.monotonic()
        outs: list[RequestOutput] = []
        for row, (seq, tok) in enumerate(zip(samplers, tokens)):
            if seq.finish_reason not in (None, "length"):
                continue        # finished earlier (EOS seen one step late) or aborted
            if seq.num_pending == 0:
                continue
            idx = len(seq.output_token_ids) - seq.num_pending
            seq.num_pending -= 1
            seq.output_token_ids[idx] = tok
            if self.bm.prefix_caching and seq.slot >= 0:
                self.bm.register_full_blocks(seq, seq.num_tokens - seq.num_pending)
            if seq.first_token_time is None:
                seq.first_token_time = now
            seq.last_token_time = now
            reason = seq.finish_reason if seq.finished else self._check_stop(seq, tok)
            if reason is not None and not seq.finished:
                # EOS / stop token: drop tokens launched after this one
                del seq.output_token_ids[idx + 1:]
                seq.num_pending = 0
                self.scheduler.finish(seq, reason)
                self.seqs.pop(seq.request_id, None)
            if reason is not None and seq.num_pending == 0:
                seq.finish_time = now
                self.metrics.on_finish(seq)
                done = True
            else:
                done = False
            o = RequestOutput(seq.request_id, seq.prompt_token_ids, [tok],
                              seq.output_token_ids, idx + 1, done, reason if done else None,
                              seq.arrival_time, seq.first_token_time, seq.finish_time,
                              seq.num_preemptions)
            if row in lps:
                o.logprobs = [(tok, lps[row][0], lps[row][1])]
            outs.append(o)
        self.metrics.on_step(plan, now - t0, len(samplers), self.bm.usage(),
                             len(self.scheduler.running), len(self.scheduler.waiting), npre)
        if self.bm.prefix_caching:
            self.metrics.on_prefix_cache(self.bm.query_tokens, self.bm.hit_tokens)
        return outs

    def _step_sync(self) -> list[RequestOutput]:
        batch = self.scheduler.schedule()
        if batch.is_empty:
            return []
        t0 = time.monotonic()
        plan, samplers = self.executor.runner.build_plan(batch.prefills, batch.decodes, self.bm.table)
        tokens = self.executor.execute(plan)
        lps = TokenFuture(None, lp=self.executor.runner.take_logprobs()).logprobs() if plan.lp else {}
        now = time.monotonic()
        for seq, n in batch.prefills:
            seq.num_computed += n
        for seq in batch.decodes:
            seq.num_computed += 1
        outs: list[RequestOutput] = []
        if self.bm.prefix_caching:
            for seq, _ in batch.prefills:
                self.bm.register_full_blocks(seq, seq.num_tokens)
        for row, (seq, tok) in enumerate(zip(samplers, tokens)):
            seq.output_token_ids.append(tok)
            if self.bm.prefix_caching:
                self.bm.register_full_blocks(seq, seq.num_tokens)
            if seq.first_token_time is None:
                seq.first_token_time = now
            seq.last_token_time = now
            reason = self._check_stop(seq, tok)
            if reason is not None:
                seq.finish_time = now
                self.scheduler.finish(seq, reason)
                self.seqs.pop(seq.request_id, None)
                self.metrics.on_finish(seq)
            o = RequestOutput(seq.request_id, seq.prompt_token_ids, [tok],
                              seq.output_token_ids, len(seq.output_token_ids),
                              reason is not None, reason,
                              seq.arrival_time, seq.first_token_time, seq.finish_time,
                              seq.num_preemptions)
            if row in lps:
                o.logprobs = [(tok, lps[row][0], lps[row][1])]
            outs.append(o)
        self.metrics.on_step(plan, now - t0, len(samplers), self.bm.usage(),
                             len(self.scheduler.running), len(self.scheduler.waiting),
                             len(batch.preempted))
        return outs

    def _check_stop(self, seq: Sequence, tok: int) -> Optional[str]:
        p = seq.params
        n = len(seq.output_token_ids)
        if n >= seq.max_tokens:
            return "length"
        if seq.num_tokens >= self.max_model_len:
            return "length"
        if n < p.min_tokens:
            return None
        if not p.ignore_eos and tok == self.eos:
            return "stop"
        if tok in p.stop_token_ids:
            return "stop"
        return None

    def shutdown(self) -> None:
        path = self.metrics.dump_trace()      # KGC_TRACE=path: per-step spans (Chrome trace)
        if path:
            log.info("engine step trace: %s", path)
        self.executor.shutdown()


class LLM:
    """Offline batch generation (token ids in, token ids out; a tokenizer is used
    when one is available locally)."""

    def __init__(self, model: str = "llama-3-8b", **kw):
        self.engine = LLMEngine(EngineConfig(model=model, **kw))
        from ..utils.tokenizer import get_tokenizer
        self.tokenizer = get_tokenizer(model, self.engine.mcfg)

    def generate(self, prompts: Iterable[Union[str, list[int]]],
                 params: Union[SamplingParams, list[SamplingParams], None] = None
                 ) -> list[RequestOutput]:
        prompts = list(prompts)
        if not isinstance(params, list):
            params = [params or SamplingParams()] * len(prompts)
        ids = []
        for i, (p, sp) in enumerate(zip(prompts, params)):
            toks = self.tokenizer.encode(p) if isinstance(p, str) else p
            self.engine.add_request(toks, sp, request_id=str(i))
            ids.append(str(i))
        final: dict[str, RequestOutput] = {}
        lps: dict[str, list] = {}
        while self.engine.has_unfinished():
            for o in self.engine.step():
                if o.logprobs:
                    lps.setdefault(o.request_id, []).extend(o.logprobs)
                if o.finished:
                    final[o.request_id] = o
        for rid, o in final.items():
            o.logprobs = lps.get(rid)
        return [final[i] for i in ids]

    def shutdown(self):
        self.engine.shutdown()
