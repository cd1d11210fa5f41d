"""Engine core on the CPU: block manager, continuous-batching scheduler
(decode-first, chunked prefill, recompute preemption, aborts, max-model-len), and
the engine loop end to end with KGC_DEBUG invariants and the torch-profiler hook."""
import os

import numpy as np
import pytest

from kubernetes_gpu_cluster_amd.engine.block_manager import BlockManager
from kubernetes_gpu_cluster_amd.engine.scheduler import Scheduler
from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams, Sequence


def _seq(rid, n, max_tokens=8):
    return Sequence(rid, list(range(3, 3 + n)), SamplingParams(max_tokens=max_tokens))


# ---------------------------------------------------------------------------- block manager
def test_block_manager_alloc_free_and_table():
    bm = BlockManager(num_blocks=9, block_size=4, max_seqs=3, max_blocks_per_seq=4)
    a, b = _seq("a", 5), _seq("b", 3)
    assert bm.can_allocate(a, 5)
    bm.allocate(a, 5)                 # 2 blocks
    bm.allocate(b, 3)                 # 1 block
    assert len(a.block_ids) == 2 and len(b.block_ids) == 1 and 0 not in a.block_ids + b.block_ids
    assert bm.table[a.slot, :2].tolist() == a.block_ids
    bm.check_invariants([a, b])
    assert bm.num_free == 8 - 3
    bm.allocate(a, 8)                 # still 2 blocks
    assert len(a.block_ids) == 2
    assert not bm.can_allocate(a, 17)             # > max_blocks_per_seq
    bm.free_seq(a)
    assert a.slot == -1 and a.block_ids == [] and bm.num_free == 7
    bm.check_invariants([b])
    assert np.all(bm.table[0] == 0) or np.all(bm.table[1] == 0)


def test_block_manager_invariants_catch_corruption():
    bm = BlockManager(6, 4, 2, 4)
    a, b = _seq("a", 8), _seq("b", 4)
    bm.allocate(a, 8)
    bm.allocate(b, 4)
    b.block_ids.append(a.block_ids[0])            # shared block
    with pytest.raises(AssertionError):
        bm.check_invariants([a, b])
    b.block_ids.pop()
    bm.free.append(a.block_ids[0])                # owned and free
    with pytest.raises(AssertionError):
        bm.check_invariants([a, b])
    bm.free.pop()
    bm.free.pop()                                 # leaked block
    with pytest.raises(AssertionError):
        bm.check_invariants([a, b])


# ---------------------------------------------------------------------------- scheduler
def _drive(sched, seqs, steps):
    """Fake model runner: every scheduled unit completes; samplers get one token."""
    trace = []
    for _ in range(steps):
        batch = sched.schedule()
        trace.append(batch)
        for seq, n in batch.prefills:
            seq.num_computed += n
            if seq.num_computed == seq.num_tokens:
                seq.output_token_ids.append(7)
        for seq in batch.decodes:
            seq.num_computed += 1
            seq.output_token_ids.append(7)
        for seq in list(sched.running):
            if len(seq.output_token_ids) >= seq.max_tokens:
                sched.finish(seq, "length")
        sched.bm.check_invariants(sched.running)
        if not sched.has_work():
            break
    return trace


def test_chunked_prefill_respects_budget_and_decode_first():
    bm = BlockManager(64, 4, 4, 16)
    sched = Scheduler(bm, max_num_seqs=4, token_budget=10, max_model_len=64)
    long, short = _seq("long", 23, 3), _seq("short", 4, 3)
    sched.add(long)
    sched.add(short)
    trace = _drive(sched, [long, short], 50)
    assert all(b.num_tokens <= 10 for b in trace)
    first = trace[0]
    assert first.prefills == [(long, 10)]          # chunk of the long prompt only
    # once the long prompt samples, later steps put its decode first
    for b in trace:
        if b.decodes and b.prefills:
            assert b.decodes[0] is long or long not in [s for s, _ in b.prefills]
    assert len(long.output_token_ids) == 3 and len(short.output_token_ids) == 3
    assert not sched.has_work() and bm.num_free == 63


def test_preemption_recompute_when_kv_runs_out():
    bm = BlockManager(num_blocks=7, block_size=4, max_seqs=4, max_blocks_per_seq=8)   # 6 usable
    sched = Scheduler(bm, max_num_seqs=4, token_budget=64, max_model_len=64)
    seqs = [_seq(f"s{i}", 7, 12) for i in range(3)]
    for s in seqs:
        sched.add(s)
    trace = _drive(sched, seqs, 200)
    assert sched.num_preemptions > 0
    assert any(b.preempted for b in trace)
    assert all(len(s.output_token_ids) == 12 for s in seqs)
    assert bm.num_free == 6


def test_abort_and_max_seqs():
    bm = BlockManager(64, 4, 2, 16)
    sched = Scheduler(bm, max_num_seqs=2, token_budget=100, max_model_len=64)
    a, b, c = _seq("a", 5), _seq("b", 5), _seq("c", 5)
    for s in (a, b, c):
        sched.add(s)
    batch = sched.schedule()
    assert len(batch.prefills) == 2 and len(sched.waiting) == 1   # cap of 2 running
    assert sched.abort("b") is b and b.finish_reason == "abort" and b.block_ids == []
    assert sched.abort("zzz") is None
    bm.check_invariants(sched.running)


# ---------------------------------------------------------------------------- engine loop
def _llm(**kw):
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    base = dict(device="cpu", dtype="float32", random_init=True, max_model_len=128,
                max_num_seqs=4, max_num_batched_tokens=48, seed=1)
    base.update(kw)
    return LLM("tiny-llama", **base)


def test_engine_preemption_matches_ample_kv(monkeypatch):
    """Greedy outputs are identical with a KV pool so small that sequences get
    preempted and recomputed; KGC_DEBUG checks block invariants every step."""
    monkeypatch.setenv("KGC_DEBUG", "1")
    prompts = [[5 + i, 6, 7, 8, 9, 10, 11] * 3 for i in range(4)]
    sp = SamplingParams(temperature=0, max_tokens=20, ignore_eos=True)
    ample = _llm(num_gpu_blocks_override=64, block_size=16, max_model_len=64)
    ref = [o.output_token_ids for o in ample.generate(prompts, sp)]
    ample.shutdown()
    tight = _llm(num_gpu_blocks_override=6, block_size=16, max_model_len=64)
    got = [o.output_token_ids for o in tight.generate(prompts, sp)]
    npre = tight.engine.scheduler.num_preemptions
    tight.shutdown()
    assert npre > 0
    assert got == ref


def test_engine_async_equals_sync():
    prompts = [[5, 6, 7], [9] * 30, [11, 12]]
    sp = [SamplingParams(temperature=0.8, seed=s, max_tokens=9, ignore_eos=True) for s in (1, 2, 3)]
    outs = []
    for async_output in (True, False):
        llm = _llm(num_gpu_blocks_override=64, block_size=16, async_output=async_output)
        assert llm.engine.async_mode == async_output
        outs.append([o.output_token_ids for o in llm.generate(prompts, sp)])
        llm.shutdown()
    assert outs[0] == outs[1]


def test_engine_stop_tokens_and_max_model_len():
    llm = _llm(num_gpu_blocks_override=64, block_size=16)
    o = llm.generate([[5, 6, 7]], SamplingParams(temperature=0, max_tokens=30, ignore_eos=True))[0]
    stop_tok = o.output_token_ids[4]
    first = o.output_token_ids.index(stop_tok)
    o2 = llm.generate([[5, 6, 7]], SamplingParams(temperature=0, max_tokens=30,
                                                  stop_token_ids=[stop_tok]))[0]
    assert o2.finish_reason == "stop" and o2.output_token_ids == o.output_token_ids[:first + 1]
    with pytest.raises(ValueError):
        llm.engine.add_request(list(range(200)), SamplingParams())
    o3 = llm.generate([list(range(3, 123))], SamplingParams(max_tokens=50, ignore_eos=True))[0]
    assert len(o3.output_token_ids) == 128 - 120 and o3.finish_reason == "length"
    llm.shutdown()


def test_torch_profiler_hook(tmp_path, monkeypatch):
    monkeypatch.setenv("KGC_TORCH_PROFILE", f"{tmp_path}:1:3")
    llm = _llm(num_gpu_blocks_override=64, block_size=16)
    llm.generate([[5, 6, 7]], SamplingParams(max_tokens=8, ignore_eos=True))
    llm.shutdown()
    files = os.listdir(tmp_path)
    assert files == ["engine_steps_1_4.json"]


def test_engine_fp8_kv_cache_cpu():
    """--kv-cache-dtype fp8: the cache holds float8_e4m3fn, twice the blocks fit in the
    same bytes, and greedy output stays close to the bf16/fp32-cache engine (e4m3 keeps
    3 mantissa bits, so a late near-tie may flip)."""
    import torch
    prompts = [[5 + i, 6, 7, 8, 9, 10, 11] * 3 for i in range(3)]
    sp = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)
    ref = _llm(num_gpu_blocks_override=64, block_size=16)
    a = [o.output_token_ids for o in ref.generate(prompts, sp)]
    bpb = ref.engine.executor.runner.kv_bytes_per_block()
    ref.shutdown()
    f8 = _llm(num_gpu_blocks_override=64, block_size=16, kv_cache_dtype="fp8")
    r = f8.engine.executor.runner
    assert r.kv.dtype == torch.float8_e4m3fn and r.kv_bytes_per_block() * 4 == bpb  # fp32 -> fp8
    b = [o.output_token_ids for o in f8.generate(prompts, sp)]
    f8.shutdown()
    assert all(x[0] == y[0] for x, y in zip(a, b))
    same = sum(p == q for x, y in zip(a, b) for p, q in zip(x, y))
    assert same >= 0.6 * sum(len(x) for x in a)


def test_engine_refuses_kv_smaller_than_one_sequence():
    with pytest.raises(ValueError, match="max_model_len"):
        _llm(num_gpu_blocks_override=4, block_size=16, max_model_len=128)


# ---------------------------------------------------------------------------- prefix caching
def test_prefix_cache_block_manager():
    bm = BlockManager(16, 4, 4, 8, enable_prefix_caching=True)
    a = _seq("a", 10)                       # blocks: [0..3] [4..7] [8..9]
    bm.allocate(a, 10)
    a.num_computed = 10
    bm.register_full_blocks(a, a.num_tokens)
    assert a.num_registered == 2
    b = Sequence("b", list(range(3, 13)) + [99], SamplingParams())   # same first 10 tokens
    hits = bm.cached_prefix_blocks(b)
    assert hits == a.block_ids[:2]
    assert bm.can_admit(b, 11, hits)
    assert bm.take_prefix(b, hits) == 8
    bm.allocate(b, 11)
    bm.check_invariants([a, b])
    assert bm.ref[hits[0]] == 2
    bm.free_seq(a)
    assert bm.ref[hits[0]] == 1 and not bm.evictable   # b still holds the shared blocks
    bm.check_invariants([b])
    bm.free_seq(b)
    assert len(bm.evictable) == 2                      # cached contents kept for reuse
    bm.check_invariants([])
    # allocation drains never-cached blocks first, then evicts LRU cached blocks
    c = _seq("c", 4 * 8)
    bm.allocate(c, 4 * 8)
    d = _seq("d", 4 * 7)
    assert bm.can_allocate(d, 28)
    bm.allocate(d, 28)
    assert not bm.evictable and not bm.block_of     # both cached blocks evicted
    bm.check_invariants([c, d])


def test_prefix_cache_forced_collision_recomputes():
    """Every key collides: a prompt with different tokens must not reuse another
    prompt's KV (verified hit), and the same prompt still hits."""
    bm = BlockManager(16, 4, 4, 8, enable_prefix_caching=True)
    bm.block_key = lambda parent, toks: b"\x00" * 16          # worst case: one key for all
    a = _seq("a", 10)
    bm.allocate(a, 10)
    a.num_computed = 10
    bm.register_full_blocks(a, a.num_tokens)
    other = Sequence("o", list(range(50, 61)), SamplingParams())
    assert bm.cached_prefix_blocks(other) == []
    assert bm.collisions == 1
    same = Sequence("s", list(range(3, 7)) + [99] * 7, SamplingParams())
    assert bm.cached_prefix_blocks(same) == a.block_ids[:1]   # block 0 matches, block 1 not


def test_prefix_cache_keys_are_salted_per_process():
    a = BlockManager(8, 4, 2, 4, enable_prefix_caching=True)
    b = BlockManager(8, 4, 2, 4, enable_prefix_caching=True)
    assert a.block_key(b"", [1, 2, 3, 4]) != b.block_key(b"", [1, 2, 3, 4])
    assert len(a.block_key(b"", [1, 2, 3, 4])) == 16


def test_missing_weights_refuse_to_start(tmp_path):
    """No silent random init: a preset name, a preset-basename path that does not exist
    (failed hostPath mount) or a dir without safetensors all fail unless random weights
    are requested explicitly (--load-format dummy)."""
    from kubernetes_gpu_cluster_amd.models import WeightsNotFoundError, check_weights
    from kubernetes_gpu_cluster_amd.entrypoints import api_server
    for name in ("qwen3-0.6b", "/models/Qwen3-0.6B", "meta-llama/Meta-Llama-3-8B"):
        with pytest.raises(WeightsNotFoundError):
            check_weights(name, random_weights=False)
        check_weights(name, random_weights=True)
    (tmp_path / "config.json").write_text('{"model_type": "llama", "num_hidden_layers": 1, '
                                          '"hidden_size": 64, "num_attention_heads": 2, '
                                          '"intermediate_size": 128, "vocab_size": 256}')
    with pytest.raises(WeightsNotFoundError):
        check_weights(str(tmp_path), random_weights=False)
    with pytest.raises(WeightsNotFoundError):          # the server exits before any engine
        api_server.main(["/models/Qwen3-0.6B", "--device", "cpu"])
    with pytest.raises(WeightsNotFoundError):
        _llm_plain = __import__("kubernetes_gpu_cluster_amd.engine.llm_engine",
                                fromlist=["LLM"]).LLM
        _llm_plain("tiny-llama", device="cpu", dtype="float32", max_model_len=64)


def test_engine_prefix_cache_hits_and_parity(monkeypatch):
    """Shared-prefix prompts: the second wave reuses cached blocks (fewer computed
    tokens) and produces exactly the tokens of an engine without prefix caching."""
    monkeypatch.setenv("KGC_DEBUG", "1")
    shared = list(range(7, 7 + 40))
    prompts = [shared + [100 + i, 101 + i, 102] for i in range(3)]
    sp = SamplingParams(temperature=0, max_tokens=10, ignore_eos=True)
    off = _llm(num_gpu_blocks_override=64, block_size=16, enable_prefix_caching=False)
    ref = [o.output_token_ids for o in off.generate(prompts, sp)]
    off.shutdown()
    on = _llm(num_gpu_blocks_override=64, block_size=16, enable_prefix_caching=True)
    first = [o.output_token_ids for o in on.generate(prompts[:1], sp)]
    rest = [o.output_token_ids for o in on.generate(prompts, sp)]
    bm = on.engine.bm
    assert bm.hit_tokens >= 3 * 32        # every prompt of wave 2 reused 2 full blocks
    on.shutdown()
    assert first[0] == ref[0]
    assert rest == ref


def test_engine_prefix_cache_with_preemption(monkeypatch):
    monkeypatch.setenv("KGC_DEBUG", "1")
    prompts = [[5 + i, 6, 7, 8, 9, 10, 11] * 3 for i in range(4)]
    sp = SamplingParams(temperature=0, max_tokens=20, ignore_eos=True)
    a = _llm(num_gpu_blocks_override=64, block_size=16, max_model_len=64,
             enable_prefix_caching=False)
    ref = [o.output_token_ids for o in a.generate(prompts, sp)]
    a.shutdown()
    b = _llm(num_gpu_blocks_override=6, block_size=16, max_model_len=64, enable_prefix_caching=True)
    got = [o.output_token_ids for o in b.generate(prompts, sp)]
    assert b.engine.scheduler.num_preemptions > 0
    b.shutdown()
    assert got == ref


def test_prefill_first_policy():
    """--prefill-first: while prompts wait for a slot, running sequences skip their decode
    and the budget goes to prefill; with nothing admissible they decode as usual, and the
    output is the same as the default policy (greedy)."""
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    sp = SamplingParams(temperature=0, max_tokens=4, ignore_eos=True)
    bm = BlockManager(64, 16, 8, 16, enable_prefix_caching=False)
    sc = Scheduler(bm, 8, 32, 256, True, prefill_first=True)
    a = Sequence("a", list(range(3, 19)), sp, None, 256)
    sc.add(a)
    b1 = sc.schedule()
    assert [s.request_id for s, _ in b1.prefills] == ["a"]
    a.num_computed += 16
    a.output_token_ids.append(7)            # a now decodes
    sc.add(Sequence("b", list(range(3, 35)), sp, None, 256))
    b2 = sc.schedule()                       # b waits: a sits out, b takes the budget
    assert not b2.decodes and [s.request_id for s, _ in b2.prefills] == ["b"]
    b3 = sc.schedule()                       # nothing waiting: a decodes again
    assert [s.request_id for s in b3.decodes] == ["a"]
    prompts = [[5 + i, 6, 7, 8] * 3 for i in range(6)]
    outs = []
    for pf in (False, True):
        llm = LLM("tiny-llama", random_init=True, device="cpu", dtype="float32",
                  max_model_len=128, max_num_seqs=4, max_num_batched_tokens=16,
                  prefill_first=pf)
        outs.append([o.output_token_ids for o in llm.generate(prompts, SamplingParams(
            temperature=0, max_tokens=6, ignore_eos=True))])
        llm.shutdown()
    assert outs[0] == outs[1]


@pytest.mark.parametrize("k", [1, 3, 8])
def test_prefill_first_bounded_deferral(k):
    """--prefill-first under continuous arrivals (one new prompt every step, a free slot
    always available): every running sequence still decodes at least once every k + 1
    steps (--prefill-first-max-defer k), so TPOT stays bounded."""
    sp = SamplingParams(temperature=0, max_tokens=1000, ignore_eos=True)
    bm = BlockManager(4096, 16, 64, 64, enable_prefix_caching=False)
    sc = Scheduler(bm, 64, 64, 1024, True, prefill_first=True, max_defer_steps=k)
    last_decode: dict[str, int] = {}
    worst = 0
    for step in range(40):
        sc.add(Sequence(f"r{step}", list(range(3, 19)), sp, None, 1024))
        b = sc.schedule()
        for s, n in b.prefills:
            s.num_computed += n
            if s.num_computed == s.num_tokens:
                s.output_token_ids.append(7)
                last_decode[s.request_id] = step
        for s in b.decodes:
            s.num_computed += 1
            s.output_token_ids.append(7)
            last_decode[s.request_id] = step
        for s in sc.running:
            if s.request_id in last_decode:
                worst = max(worst, step - last_decode[s.request_id])
    assert worst <= k + 1, worst
    assert len(sc.running) > 10


def test_prefill_first_gap_bound(monkeypatch):
    """--prefill-first-max-gap-ms: a running stream that has waited longer than the gap
    is decoded in the next step even while prompts keep arriving."""
    from kubernetes_gpu_cluster_amd.engine import scheduler as sched_mod
    sp = SamplingParams(temperature=0, max_tokens=100, ignore_eos=True)
    bm = BlockManager(256, 16, 8, 16, enable_prefix_caching=False)
    sc = Scheduler(bm, 8, 32, 256, True, prefill_first=True, max_defer_steps=100,
                   max_decode_gap_ms=50)
    clock = [1000.0]
    monkeypatch.setattr(sched_mod.time, "monotonic", lambda: clock[0])
    a = Sequence("a", list(range(3, 19)), sp, None, 256)
    sc.add(a)
    sc.schedule()
    a.num_computed += 16
    a.output_token_ids.append(7)
    a.last_token_time = clock[0]
    sc.add(Sequence("b", list(range(3, 19)), sp, None, 256))
    assert not sc.schedule().decodes            # within the gap: a sits out
    clock[0] += 0.2
    sc.add(Sequence("c", list(range(3, 19)), sp, None, 256))
    assert [s.request_id for s in sc.schedule().decodes] == ["a"]


def test_step_plan_header_carries_the_tp_overlap_split():
    """The TP prefill overlap split is decided once by the driver (build_plan) and sent in
    the broadcast header, so every TP rank splits the same way whatever its environment;
    the header length matches what the worker loop unpacks."""
    import numpy as np
    from kubernetes_gpu_cluster_amd.engine.model_runner import StepPlan
    from kubernetes_gpu_cluster_amd.engine.worker import N_HDR
    z = np.zeros(1)
    p = StepPlan(40, 40, 2, 0, 2, 3, 0, 0, 0, 0, 1, 1, z, z, z)
    h = p.header()
    assert len(h) == N_HDR and h[-1] == 1
    q = StepPlan(*h, z, z, z)
    assert q.split == 1 and q.vp == 1 and q.T == 40
