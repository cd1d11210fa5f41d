"""Engine observability: Prometheus metrics + an optional Chrome-trace step timeline.

Exposed at the API server's ``/metrics`` (SURVEY.md §5 "Metrics"): TTFT / TPOT /
e2e latency histograms, prompt & generation token counters, running / waiting
sequences, KV-cache usage, preemptions.  Metric names follow vLLM's
``vllm:``-prefixed names so existing production-stack dashboards keep working.
Set ``KGC_TRACE=/path/trace.json`` to dump per-step spans (chrome://tracing).
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Optional

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram

_LAT = (0.001, 0.005, 0.01, 0.02, 0.04, 0.06, 0.08, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0,
        7.5, 10.0, 20.0, 40.0, 80.0)


class EngineMetrics:
    def __init__(self, registry: Optional[CollectorRegistry] = None, model_name: str = "model"):
        self.registry = registry or CollectorRegistry()
        lab = ["model_name"]
        r = self.registry
        self.ttft = Histogram("vllm:time_to_first_token_seconds", "TTFT", lab, buckets=_LAT, registry=r)
        self.tpot = Histogram("vllm:time_per_output_token_seconds", "TPOT", lab, buckets=_LAT, registry=r)
        self.e2e = Histogram("vllm:e2e_request_latency_seconds", "e2e", lab, buckets=_LAT, registry=r)
        self.prompt_toks = Counter("vllm:prompt_tokens", "prompt tokens", lab, registry=r)
        self.gen_toks = Counter("vllm:generation_tokens", "generated tokens", lab, registry=r)
        self.running = Gauge("vllm:num_requests_running", "running", lab, registry=r)
        self.waiting = Gauge("vllm:num_requests_waiting", "waiting", lab, registry=r)
        self.kv_usage = Gauge("vllm:gpu_cache_usage_perc", "KV usage", lab, registry=r)
        self.preempt = Counter("vllm:num_preemptions", "preemptions", lab, registry=r)
        self.finished = Counter("vllm:request_success", "finished requests", lab + ["finished_reason"],
                                registry=r)
        self.step_time = Histogram("kgc:engine_step_seconds", "engine step wall time", lab,
                                   buckets=_LAT, registry=r)
        self.prefix_queries = Counter("vllm:prefix_cache_queries", "prompt tokens looked up in "
                                      "the prefix cache", lab, registry=r)
        self.prefix_hits = Counter("vllm:prefix_cache_hits", "prompt tokens served from the "
                                   "prefix cache", lab, registry=r)
        self.prefix_rate = Gauge("vllm:gpu_prefix_cache_hit_rate", "prefix cache hit rate",
                                 lab, registry=r)
        self._pq = self._ph = 0
        self.model = model_name
        self.total_gen = 0
        self.total_prompt = 0
        self.steps = 0
        self._trace_path = os.environ.get("KGC_TRACE")
        self._trace: list = []
        self._lock = threading.Lock()

    def on_arrival(self) -> None:
        pass

    def on_step(self, plan, dt: float, n_gen: int, kv: float, running: int, waiting: int,
                preempted: int) -> None:
        m = self.model
        self.steps += 1
        self.total_gen += n_gen
        self.total_prompt += plan.Tp
        self.gen_toks.labels(m).inc(n_gen)
        self.prompt_toks.labels(m).inc(plan.Tp)
        self.running.labels(m).set(running)
        self.waiting.labels(m).set(waiting)
        self.kv_usage.labels(m).set(kv)
        self.step_time.labels(m).observe(dt)
        if preempted:
            self.preempt.labels(m).inc(preempted)
        if self._trace_path:
            now = time.monotonic() * 1e6
            self._trace.append({"name": f"step T={plan.T} P={plan.P} D={plan.D} B={plan.B}",
                                "ph": "X", "ts": now - dt * 1e6, "dur": dt * 1e6, "pid": 0,
                                "tid": 0})

    def on_prefix_cache(self, queries: int, hits: int) -> None:
        """Cumulative token counts from the block manager."""
        m = self.model
        if queries > self._pq:
            self.prefix_queries.labels(m).inc(queries - self._pq)
            self.prefix_hits.labels(m).inc(hits - self._ph)
            self._pq, self._ph = queries, hits
            self.prefix_rate.labels(m).set(hits / queries)

    def on_finish(self, seq) -> None:
        m = self.model
        if seq.first_token_time is not None:
            self.ttft.labels(m).observe(seq.first_token_time - seq.arrival_time)
            n = len(seq.output_token_ids)
            if n > 1 and seq.last_token_time is not None:
                self.tpot.labels(m).observe((seq.last_token_time - seq.first_token_time) / (n - 1))
        if seq.finish_time is not None:
            self.e2e.labels(m).observe(seq.finish_time - seq.arrival_time)
        self.finished.labels(m, seq.finish_reason or "unknown").inc()

    def dump_trace(self) -> Optional[str]:
        if not self._trace_path:
            return None
        with open(self._trace_path, "w") as f:
            json.dump({"traceEvents": self._trace}, f)
        return self._trace_path
