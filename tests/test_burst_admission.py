"""Burst admission (entrypoints/engine_core.py): the engine-core loop keeps admitting a
burst's arrivals before it steps while ``LLMEngine.coalescing`` (idle engine, waiting
prompts under one step's token budget) or ``LLMEngine.inflight_coalescing`` (a large
prefill-only step still on the device, the next step would be a partial prefill) holds.
CPU engine, tiny random model."""
import pytest

from kubernetes_gpu_cluster_amd.engine.config import EngineConfig
from kubernetes_gpu_cluster_amd.engine.llm_engine import LLMEngine
from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams


@pytest.fixture(scope="module")
def eng():
    cfg = EngineConfig(model="tiny-llama", random_init=True, max_model_len=256, max_num_seqs=8,
                       max_num_batched_tokens=128, device="cpu", dtype="float32")
    e = LLMEngine(cfg)
    yield e
    e.shutdown()


class _Fut:
    def __init__(self, done):
        self._done = done

    def done(self):
        return self._done


class _Plan:
    def __init__(self, Tp, D):
        self.Tp, self.D = Tp, D


def _drain(e):
    while e.has_unfinished():
        e.step()


def test_idle_coalescing_until_one_step_of_prompts(eng):
    _drain(eng)
    assert not eng.coalescing()                       # nothing waiting
    p = SamplingParams(max_tokens=2, temperature=0.0)
    eng.add_request(list(range(3, 43)), p)            # 40 tokens < 128
    assert eng.coalescing()
    eng.add_request(list(range(3, 43)), p)            # 80
    assert eng.coalescing()
    eng.add_request(list(range(3, 53)), p)            # 130 >= 128: a full step waits
    assert not eng.coalescing()
    eng.step()                                        # something runs now
    assert not eng.coalescing()
    _drain(eng)


def test_inflight_coalescing_needs_a_large_prefill_in_flight(eng):
    _drain(eng)
    p = SamplingParams(max_tokens=2, temperature=0.0)
    budget = eng.cfg.token_budget()
    try:
        eng._inflight = (_Fut(False), [], _Plan(budget, 0), 0.0, 0)
        assert eng.inflight_coalescing()              # nothing waiting yet: still arriving
        eng.add_request(list(range(3, 43)), p)
        assert eng.inflight_coalescing()              # a partial next step
        eng._inflight = (_Fut(True), [], _Plan(budget, 0), 0.0, 0)
        assert not eng.inflight_coalescing()          # the device step is done: launch now
        eng._inflight = (_Fut(False), [], _Plan(budget, 3), 0.0, 0)
        assert not eng.inflight_coalescing()          # decodes in flight: steady state
        eng._inflight = (_Fut(False), [], _Plan(budget // 4, 0), 0.0, 0)
        assert not eng.inflight_coalescing()          # a small prefill in flight
        eng._inflight = (_Fut(False), [], _Plan(budget, 0), 0.0, 0)
        eng.add_request(list(range(3, 103)), p)       # 140 >= budget
        assert not eng.inflight_coalescing()
    finally:
        eng._inflight = None
    _drain(eng)
