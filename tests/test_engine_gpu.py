"""Engine-level checks on the MI355X: model parity through the HIP kernels,
hipGraph decode replay == eager, async engine loop, Llama-3-8B-dims smoke."""
import os

import pytest
import torch

from kubernetes_gpu_cluster_amd.engine.config import EngineConfig
from kubernetes_gpu_cluster_amd.engine.llm_engine import LLMEngine
from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams
from kubernetes_gpu_cluster_amd.models import PRESETS, build_model, full_state_dict_random
from kubernetes_gpu_cluster_amd.engine.model_runner import ModelRunner
from kubernetes_gpu_cluster_amd.parallel.state import ParallelState, set_state

from test_model_parity import _engine_logits, _hf_model

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-qwen3", "tiny-qwen2", "tiny-mixtral",
                                  "tiny-llama-gqa8"])
def test_gpu_logits_match_hf(gpu, name):
    cfg = PRESETS[name]
    sd = full_state_dict_random(cfg, seed=2, std=0.05)
    hf, _ = _hf_model(cfg, sd)
    set_state(ParallelState(device=gpu))
    model = build_model(cfg, torch.bfloat16, gpu)
    model.load_weights(sd.items())
    runner = ModelRunner(model, cfg, torch.bfloat16, gpu, block_size=16, max_model_len=256,
                         max_num_seqs=4, token_budget=128, enforce_eager=True)
    runner.init_kv_cache(48)
    g = torch.Generator().manual_seed(0)
    prompt = torch.randint(3, cfg.vocab_size, (70,), generator=g).tolist()
    extra = torch.randint(3, cfg.vocab_size, (4,), generator=g).tolist()
    with torch.no_grad():
        ref = hf(torch.tensor([prompt + extra])).logits[0].float()
    got = _engine_logits(model, runner, prompt, [33, 37], extra).float().cpu()
    scale = ref.abs().max().item()
    pos_err = (got - ref).abs().max(-1).values
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    ok = (pos_err < 0.03 * scale + 1e-3) & (cos > 0.999)
    if cfg.is_moe:
        # bf16 rounding can flip a top-2 expert choice at a near-tie (the same happens
        # with the CPU reference in bf16): allow a few positions to route differently
        assert ok.float().mean() >= 0.93, (pos_err.max(), ok.float().mean())
    else:
        assert bool(ok.all()), (pos_err.max().item(), scale, cos.min().item())


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-qwen2", "tiny-qwen3"])
def test_gpu_logits_match_hf_fused_small_m(gpu, name):
    """The fused small-M decoder (norms inside the skinny GEMMs, residual adds in their
    epilogues) against HF: prefill chunks of 13 and 7 tokens and 1-token decode steps
    all take the fused path once the skinny plan covers every projection."""
    from kubernetes_gpu_cluster_amd.ops import gemm
    cfg = PRESETS[name]
    sd = full_state_dict_random(cfg, seed=3, std=0.05)
    hf, _ = _hf_model(cfg, sd)
    set_state(ParallelState(device=gpu))
    model = build_model(cfg, torch.bfloat16, gpu)
    model.load_weights(sd.items())
    runner = ModelRunner(model, cfg, torch.bfloat16, gpu, block_size=16, max_model_len=256,
                         max_num_seqs=4, token_budget=128, enforce_eager=True)
    runner.init_kv_cache(48)
    norm_ws, acc_ws = model._fused_weights()
    gemm.clear_plan()
    try:
        for M in (13, 7, 1):      # a plan as if tuning had measured the fused layer faster
            for w in norm_ws:
                N, K = w.shape
                gemm._plan_norm[(M, N, K)] = ((1, 1, 4, True), 1.0)
                gemm._chosen_us[(M, N, K)] = 2.0
                gemm._rms_us[(M, K)] = 1.0
            for w in acc_ws:
                gemm._plan[(M, *w.shape)] = (1, 1, 4, True)
            assert model._fused_cfgs(M) is not None
        g = torch.Generator().manual_seed(1)
        prompt = torch.randint(3, cfg.vocab_size, (20,), generator=g).tolist()
        extra = torch.randint(3, cfg.vocab_size, (4,), generator=g).tolist()
        with torch.no_grad():
            ref = hf(torch.tensor([prompt + extra])).logits[0].float()
        got = _engine_logits(model, runner, prompt, [13, 7], extra).float().cpu()
    finally:
        gemm.clear_plan()
    scale = ref.abs().max().item()
    pos_err = (got - ref).abs().max(-1).values
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert bool(((pos_err < 0.03 * scale + 1e-3) & (cos > 0.999)).all()), \
        (pos_err.max().item(), scale, cos.min().item())


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-llama-gqa8"])
def test_gpu_logits_match_hf_norm_free_small_m(gpu, name):
    """The norm-free small-M decoder (models/llama.py _forward_rs: o / down add into the
    residual and leave its sums of squares, qkv / gate_up run on gamma-folded weights with
    a per-row rsqrt scale; K9 SK_ACC_SS / SK_RSCALE(_SILU)) against HF: prefill chunks of
    13 and 7 tokens and 1-token decode steps all take it."""
    from kubernetes_gpu_cluster_amd.ops import gemm
    cfg = PRESETS[name]
    sd = full_state_dict_random(cfg, seed=4, std=0.05)
    hf, _ = _hf_model(cfg, sd)
    set_state(ParallelState(device=gpu))
    model = build_model(cfg, torch.bfloat16, gpu)
    model.load_weights(sd.items())
    assert model.fold_rs_weights() > 0
    runner = ModelRunner(model, cfg, torch.bfloat16, gpu, block_size=16, max_model_len=256,
                         max_num_seqs=4, token_budget=128, enforce_eager=True)
    runner.init_kv_cache(48)
    gemm.clear_plan()
    try:
        (nq, kq), (no, ko), (ng, kg), (nd, kd) = model._rs_shapes()
        for M in (13, 7, 1):      # configurations as the start-up tuning records them
            gemm._best_sk[(M, nq, kq)] = (1, 2, 4, False)
            gemm._best_sk[(M, no, ko)] = (1, 1, 4, True)
            gemm._best_silu[(M, ng, kg)] = (1, 2, 4, False)
            gemm._best_sk[(M, nd, kd)] = (1, 1, 8, False)
            assert model._rs_cfgs(M) is not None
            if M != 13:   # layer 0's input norm inside its qkv GEMM (SK_NORM) at M = 7 / 1
                gemm._plan_norm[(M, nq, kq)] = ((1, 2, 4, False), 1.0)
                gemm._chosen_us[(M, nq, kq)] = 10.0
                gemm._rms_us[(M, kq)] = 5.0
                assert gemm.norm_fused_cfg(M, nq, kq) == (1, 2, 4, False)
        g = torch.Generator().manual_seed(1)
        prompt = torch.randint(3, cfg.vocab_size, (20,), generator=g).tolist()
        extra = torch.randint(3, cfg.vocab_size, (4,), generator=g).tolist()
        with torch.no_grad():
            ref = hf(torch.tensor([prompt + extra])).logits[0].float()
        got = _engine_logits(model, runner, prompt, [13, 7], extra).float().cpu()
    finally:
        gemm.clear_plan()
    scale = ref.abs().max().item()
    pos_err = (got - ref).abs().max(-1).values
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert bool(((pos_err < 0.03 * scale + 1e-3) & (cos > 0.999)).all()), \
        (pos_err.max().item(), scale, cos.min().item())


def _tiny_engine(**kw):
    PRESETS.setdefault("llama-3-8b-2l", PRESETS["llama-3-8b"].shrink(name="llama-3-8b-2l",
                                                                     num_layers=2))
    base = dict(model="llama-3-8b-2l", random_init=True, max_model_len=1024, max_num_seqs=16,
                max_num_batched_tokens=2048, num_gpu_blocks_override=512, cuda_graph_max_bs=16)
    base.update(kw)
    return LLMEngine(EngineConfig(**base))


def _run(eng, prompts, params):
    seqs = [eng.add_request(p, sp) for p, sp in zip(prompts, params)]
    while eng.has_unfinished():
        eng.step()
    return [s.output_token_ids for s in seqs]


def test_graph_equals_eager_and_async_equals_sync(gpu):
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(100, 128000, (n,), generator=g).tolist() for n in (5, 77, 300, 1)]
    params = [SamplingParams(temperature=1.0, seed=i, max_tokens=12, ignore_eos=True)
              for i in range(len(prompts))]
    outs = {}
    for eager in (True, False):
        for am in (False, True):
            eng = _tiny_engine(enforce_eager=eager, async_output=am)
            outs[(eager, am)] = _run(eng, prompts, params)
            if not eager:
                assert eng.executor.runner.stats["graph_steps"] > 0
            del eng
            torch.cuda.empty_cache()
    base = outs[(True, False)]
    for k, v in outs.items():
        # sampling noise is counter-based, so identical logits give identical tokens;
        # hipBLASLt may pick a different kernel for a padded graph bucket, so allow a
        # rare late divergence but require the first tokens to agree
        for a, b in zip(v, base):
            assert len(a) == len(b) == 12
            assert a[:4] == b[:4], (k, a, b)


def _run_lp(eng, prompts, params):
    """Greedy runs with top-2 logprobs per generated token: {request: [(tok, lp, top2)]}."""
    seqs = [eng.add_request(p, sp) for p, sp in zip(prompts, params)]
    lps = {s.request_id: [] for s in seqs}
    while eng.has_unfinished():
        for o in eng.step():
            if o.logprobs:
                lps[o.request_id].extend(o.logprobs)
    return [(s.output_token_ids, lps[s.request_id]) for s in seqs]


def _assert_greedy_agrees(got, base, n_first, tie=0.05):
    """Greedy continuations agree on the first n_first tokens -- except at a near-tie:
    where they first differ, the base run's top-2 logprob gap must be < ``tie`` and the
    other run's token must be the base run's runner-up (kernels with different rounding,
    e.g. a graph bucket's GEMM choice or split-context factor, may break a tie either
    way; after that the two continuations are different texts and are not compared)."""
    (a, _), (b, lpb) = got, base
    for i in range(min(n_first, len(a), len(b))):
        if a[i] == b[i]:
            continue
        tok, lp, top = lpb[i]
        alts = dict(top)
        assert a[i] in alts, (i, a, b, top)
        assert abs(lp - alts[a[i]]) < tie, (i, a, b, top)
        return


def test_decode_rope_fused_equals_unfused(gpu, monkeypatch):
    """Decode steps with RoPE + KV write inside the paged-decode kernel give the same
    greedy tokens as rope_kv_write + paged_decode, eager and replayed from hipGraphs
    (up to a near-tie, see _assert_greedy_agrees)."""
    from kubernetes_gpu_cluster_amd.models import llama
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(100, 128000, (n,), generator=g).tolist() for n in (9, 150, 33)]
    params = [SamplingParams(temperature=0.0, max_tokens=16, ignore_eos=True, logprobs=2)
              for _ in prompts]
    outs = {}
    for fused in (False, True):
        monkeypatch.setattr(llama, "_decode_rope_fused", fused)
        for eager in (True, False):
            eng = _tiny_engine(enforce_eager=eager)
            outs[(fused, eager)] = _run_lp(eng, prompts, params)
            del eng
            torch.cuda.empty_cache()
    base = outs[(False, True)]
    for k, v in outs.items():
        for got, ref in zip(v, base):
            assert len(got[0]) == 16 and len(got[1]) == 16
            _assert_greedy_agrees(got, ref, 8)


def test_prefill_rope_fused_equals_unfused(gpu, monkeypatch):
    """Prefill-only steps with q RoPE inside the prefill attention kernel (and a k / v-only
    rope_kv_write) give the same greedy tokens as the unfused path; mixed prefill + decode
    steps keep the unfused path, so chunked prompts cover both (up to a near-tie)."""
    from kubernetes_gpu_cluster_amd.models import llama
    g = torch.Generator().manual_seed(7)
    prompts = [torch.randint(100, 128000, (n,), generator=g).tolist() for n in (9, 300, 150)]
    params = [SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True, logprobs=2)
              for _ in prompts]
    outs = {}
    for fused in (False, True):
        monkeypatch.setattr(llama, "_prefill_rope_fused", fused)
        eng = _tiny_engine(enforce_eager=False)
        outs[fused] = _run_lp(eng, prompts, params)
        del eng
        torch.cuda.empty_cache()
    for got, ref in zip(outs[True], outs[False]):
        assert len(got[0]) == 12
        _assert_greedy_agrees(got, ref, 8)


def test_engine_preemption_recompute(gpu):
    """A KV pool too small for the batch forces recompute preemption; every request
    still completes with the requested length."""
    eng = _tiny_engine(num_gpu_blocks_override=40, max_num_seqs=8, block_size=32)
    g = torch.Generator().manual_seed(2)
    prompts = [torch.randint(100, 128000, (200,), generator=g).tolist() for _ in range(8)]
    params = [SamplingParams(max_tokens=60, ignore_eos=True, seed=i) for i in range(8)]
    outs = _run(eng, prompts, params)
    assert all(len(o) == 60 for o in outs)
    assert eng.scheduler.num_preemptions > 0
    assert eng.bm.num_free == eng.bm.num_blocks - 1


def _write_hf_dir(tmp_path, cfg, std=0.08, seed=5):
    import json
    import os
    from safetensors.torch import save_file
    d = str(tmp_path / "m")
    os.makedirs(d)
    save_file({k: v.contiguous() for k, v in full_state_dict_random(cfg, seed=seed, std=std).items()},
              os.path.join(d, "model.safetensors"))
    json.dump({"model_type": "llama", "hidden_size": cfg.hidden_size,
               "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
               "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
               "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
               "max_position_embeddings": 512, "rope_theta": cfg.rope_theta,
               "rms_norm_eps": cfg.rms_eps, "eos_token_id": 2, "bos_token_id": 1},
              open(os.path.join(d, "config.json"), "w"))
    return d


def _teacher_forced_deltas(d, prompts, runs):
    """TP = 1 evaluates, by prefill, every prefix that the TP = N run decoded from:
    prompt + its first j generated tokens, j = 0 .. n-1.  For each position returns
    |logprob_N(y_j) - logprob_1(y_j)| (y_j = the token TP = N chose there) and whether
    y_j is TP = 1's argmax or a near-tie of it (0.05 nats)."""
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    reqs, keys = [], []
    for i, (p, (toks, lps)) in enumerate(zip(prompts, runs)):
        for j in range(len(toks)):
            reqs.append(p + toks[:j])
            keys.append((i, j))
    llm = LLM(d, device="cuda", dtype="bfloat16", tensor_parallel_size=1, enforce_eager=True,
              max_model_len=256, max_num_seqs=16, max_num_batched_tokens=512,
              num_gpu_blocks_override=128, enable_prefix_caching=False)
    try:
        res = llm.generate(reqs, [SamplingParams(temperature=0, max_tokens=1, logprobs=5)] *
                           len(reqs))
    finally:
        llm.shutdown()
    out = []
    for (i, j), r in zip(keys, res):
        toks, lps = runs[i]
        y, lp_n = toks[j], lps[j][1]
        top1 = dict(r.logprobs[0][2])
        best = max(top1.values())
        lp_1 = top1.get(y)
        out.append((i, j, None if lp_1 is None else abs(lp_n - lp_1),
                    lp_1 is not None and best - lp_1 < 0.05))
    return out


@pytest.mark.parametrize("tp,eager,name,overlap,xgmi,perturb",
                         [(2, True, "tiny-llama", False, True, False),
                          (2, False, "tiny-llama", False, True, False),
                          (2, False, "tiny-llama", True, True, False),
                          (4, False, "tiny-llama", False, True, False),
                          (8, True, "tiny-llama-gqa8", False, False, False),
                          (2, False, "tiny-llama", False, True, True)])
def test_tp_on_one_gpu_matches_tp1(gpu, tmp_path, monkeypatch, tp, eager, name, overlap, xgmi,
                                   perturb):
    """The tensor-parallel engine on the GPU against TP = 1, TEACHER-FORCED: TP ranks share
    cuda:0 (gloo process group, since RCCL refuses two ranks on one device), sharded
    QKV/MLP/vocab layers, the xGMI all-reduce kernel over IPC buffers for the row-parallel
    sums, multiprocess workers.  eager=False is the production decode path:
    hipGraph-captured decode buckets with the xGMI all-reduce INSIDE the graphs.
    overlap: the 100-token first prefill step runs as two halves whose all-reduces are in
    flight while the other half computes (KGC_TP_OVERLAP_MIN_TOKENS lowered to 16).  TP = 4
    replicates tiny-llama's 2 kv heads over 4 ranks.  TP = 8 (BASELINE config 3's degree:
    one kv head per rank, the per-rank attention shape of 70B at TP = 8) runs every GPU
    kernel of the 8-rank engine with its sums over gloo (KGC_CUSTOM_AR=0, eager); the
    xGMI kernels' NR = 8 forms are proven by the single-launch world emulation and the
    phantom rank (test_allreduce_gpu.py).

    The oracle: TP = N decodes greedily and reports the logprob of every token it chose;
    TP = 1 then prefills each prefix TP = N decoded from (the same tokens, not its own
    continuation) and must give each chosen token the same logprob within 0.1 nats and
    rank it first (or within a 0.05-nat near-tie).  A second TP = N pass without logprobs
    (vocab-parallel sampling, no logits all-gather) must choose the same tokens.
    perturb: rank 1 adds noise to its o_proj shards (KGC_FAULT_PERTURB_TP_RANK) -- the
    oracle must then FAIL, i.e. it does catch one wrong shard."""
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    cfg = PRESETS[name]
    d = _write_hf_dir(tmp_path, cfg)
    prompts = [list(range(3, 40)), [5, 6, 7] * 20, [9, 10, 11]]
    n_out = 8
    monkeypatch.setenv("KGC_DIST_BACKEND", "gloo")
    if not xgmi:
        monkeypatch.setenv("KGC_CUSTOM_AR", "0")
    if overlap:
        monkeypatch.setenv("KGC_TP_OVERLAP_MIN_TOKENS", "16")
    if perturb:
        monkeypatch.setenv("KGC_FAULT_PERTURB_TP_RANK", "1")
        monkeypatch.setenv("KGC_TESTING", "1")
    llm = LLM(d, device="cuda", dtype="bfloat16", tensor_parallel_size=tp, enforce_eager=eager,
              max_model_len=256, max_num_seqs=4, max_num_batched_tokens=128,
              num_gpu_blocks_override=64)
    try:
        from kubernetes_gpu_cluster_amd.parallel import comm
        car = comm.get_custom_allreduce()
        if xgmi:
            assert car is not None and car.world == tp, f"xGMI all-reduce not set up for TP={tp}"
            # the per-size policy was timed on this box at start-up (every rank agrees on it:
            # the times are MAX-reduced) and it is what the captured graphs launched
            cal = car.calibration
            assert car.table and cal["rows"][0] == 1 and cal["rows"][-1] >= 4, cal
            # chosen on hipGraph REPLAY times (the decode graphs' launch pattern), with the
            # eager times and their delta logged beside them; no uncapturable gloo 'rccl'
            assert cal["timing"] == "graph", cal
            assert len(cal["graph_minus_eager_us"]["one"]) == len(cal["rows"]), cal
            assert all(v is None for v in cal["us"]["rccl"]), cal
            assert all(p != "rccl" for _, p, _ in car.table), car.table
            table_forms = {f for _, p, fu in car.table for f in (p, fu)}
        else:
            assert car is None, "KGC_CUSTOM_AR=0 must leave every sum to the process group"
        res = llm.generate(prompts, [SamplingParams(temperature=0, max_tokens=n_out,
                                                    ignore_eos=True, logprobs=5)] * 3)
        runs = [(o.output_token_ids, o.logprobs) for o in res]
        plain = llm.generate(prompts, [SamplingParams(temperature=0, max_tokens=n_out,
                                                      ignore_eos=True)] * 3)
        st = llm.engine.executor.runner.stats
        if car is not None:
            car.check()         # a time-out on ANY rank is raised in every rank's word
            assert sum(car.launches.values()) > 0, "the xGMI kernels never ran"
            # the decode graphs' messages are table sizes: their launches followed it;
            # past the table (prefill-sized messages) the largest entry's bandwidth form is
            # extrapolated, never the one-shot default unless the table chose it
            assert sum(car.table_launches.values()) > 0, (dict(car.launches), car.table)
            assert set(car.table_launches) <= table_forms, (dict(car.table_launches),
                                                            car.table)
            if car.table[-1][1] != "one":
                assert car.launches["one"] == car.table_launches["one"], (
                    dict(car.launches), car.table)
            if table_forms & {"fused1", "fused2"}:
                assert car.fused_calls > 0, "fused all-reduce + add + RMSNorm never ran"
        if os.environ.get("KGC_VP_SAMPLING", "1") != "0":
            assert st["vp_steps"] > 0, st
        if not eager:
            assert st["graph_steps"] > 0, st
    finally:
        llm.shutdown()
    for (toks, _), o in zip(runs, plain):
        assert o.output_token_ids == toks, "vocab-parallel sampling chose other tokens"
    monkeypatch.delenv("KGC_FAULT_PERTURB_TP_RANK", raising=False)
    deltas = _teacher_forced_deltas(d, prompts, runs)
    bad = [(i, j, dlt, top) for i, j, dlt, top in deltas if dlt is None or dlt > 0.1 or not top]
    worst = max((dlt for _, _, dlt, _ in deltas if dlt is not None), default=None)
    if perturb:
        assert bad, f"one perturbed shard went unnoticed (max delta {worst})"
    else:
        assert not bad, (bad, worst)


def test_logprobs_through_decode_graphs(gpu):
    """logprobs come from the graph's static logits buffer: greedy -> the sampled token
    is the top-1 alternative, every value is a log-probability."""
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    llm = LLM("tiny-llama", device="cuda", dtype="bfloat16", random_init=True, max_model_len=256,
              max_num_seqs=8, max_num_batched_tokens=256)
    outs = llm.generate([[5, 6, 7, 8], [9, 10]],
                        [SamplingParams(temperature=0, max_tokens=6, ignore_eos=True, logprobs=3)] * 2)
    assert llm.engine.executor.runner.stats["graph_steps"] > 0
    for o in outs:
        assert len(o.logprobs) == 6
        for tok, lp, top in o.logprobs:
            assert lp <= 1e-6 and len(top) == 3
            assert top[0][0] == tok or abs(top[0][1] - lp) < 1e-3
    llm.shutdown()


def test_fp8_kv_engine_graphs(gpu):
    """--kv-cache-dtype fp8 through the whole engine (graph decode + chunked prefill).
    e4m3 keeps 3 mantissa bits, so greedy tokens of a random-init model (flat logits)
    may differ; the check is that each fp8 first token is among the bf16-cache run's
    top-5 candidates and that the top-1 logprobs agree closely."""
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    prompts = [[5 + i, 6, 7, 8, 9] * 9 for i in range(3)]
    sp = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True, logprobs=5)
    outs = []
    for kvd in ("auto", "fp8"):
        llm = LLM("tiny-llama", device="cuda", dtype="bfloat16", random_init=True, seed=2,
                  max_model_len=256, max_num_seqs=4, max_num_batched_tokens=64,
                  kv_cache_dtype=kvd)
        if kvd == "fp8":
            assert llm.engine.executor.runner.kv.dtype == torch.float8_e4m3fn
        outs.append(llm.generate(prompts, sp))
        assert llm.engine.executor.runner.stats["graph_steps"] > 0
        llm.shutdown()
    for a, b in zip(*outs):
        tok_b, lp_b, _ = b.logprobs[0]
        top_a = a.logprobs[0][2]
        assert tok_b in [t for t, _ in top_a], (a.output_token_ids, b.output_token_ids)
        assert abs(top_a[0][1] - b.logprobs[0][2][0][1]) < 0.15


def _rccl_capture_worker(port):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        x = torch.zeros(1 << 16, dtype=torch.bfloat16, device=dev)
        y = torch.empty(1 << 16, dtype=torch.bfloat16, device=dev)
        dist.all_reduce(x)                       # communicator + warm up outside capture
        dist.all_gather_into_tensor(y, x)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            x.mul_(2)
            dist.all_reduce(x)
            dist.all_gather_into_tensor(y, x)
        for it in range(3):
            src = torch.randint(-50, 50, (1 << 16,), device=dev).to(torch.bfloat16)
            x.copy_(src)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(x, src * 2) and torch.equal(y, src * 2), it
    finally:
        dist.destroy_process_group()


def test_rccl_collectives_capture_in_hipgraph(gpu):
    """A single-rank RCCL process group: all_reduce and all_gather captured into a
    hipGraph and replayed (the decode graphs' collectives at TP > 1 when the xGMI
    kernel is off or a tensor exceeds its buffer)."""
    import socket
    import torch.multiprocessing as tmp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = tmp.get_context("spawn")
    p = ctx.Process(target=_rccl_capture_worker, args=(port,))
    p.start()
    p.join(300)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0


@pytest.mark.parametrize("ep", [2, 4])
def test_mixtral_ep_graphs_on_one_gpu(gpu, tmp_path, monkeypatch, ep):
    """Mixtral with --moe-parallel ep at TP = 2 (two ranks on cuda:0, gloo group): decode
    steps replay hipGraphs with the device-side expert all-to-all inside.  Greedy output
    equals the eager EP engine that exchanges through all_to_all with host-side counts
    (KGC_EP_IPC=0), and starts like TP = 1 (whose sums round differently)."""
    import json
    import os
    from safetensors.torch import save_file
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    cfg = PRESETS["tiny-mixtral"]
    d = str(tmp_path / "m")
    os.makedirs(d)
    save_file({k: v.contiguous() for k, v in full_state_dict_random(cfg, seed=5, std=0.15).items()},
              os.path.join(d, "model.safetensors"))
    json.dump({"model_type": "mixtral", "hidden_size": cfg.hidden_size,
               "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
               "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
               "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
               "max_position_embeddings": 512, "rope_theta": cfg.rope_theta,
               "rms_norm_eps": cfg.rms_eps, "num_local_experts": cfg.num_experts,
               "num_experts_per_tok": cfg.top_k_experts, "eos_token_id": 2, "bos_token_id": 1},
              open(os.path.join(d, "config.json"), "w"))
    prompts = [list(range(3, 40)), [5, 6, 7] * 20, [9, 10, 11]]
    sp = [SamplingParams(temperature=0, max_tokens=8, ignore_eos=True)] * 3
    monkeypatch.setenv("KGC_DIST_BACKEND", "gloo")
    outs = {}
    for tp, ipc in ((1, "1"), (ep, "1"), (ep, "0")):
        monkeypatch.setenv("KGC_EP_IPC", ipc)
        llm = LLM(d, device="cuda", dtype="bfloat16", tensor_parallel_size=tp,
                  moe_parallel="ep", max_model_len=256, max_num_seqs=4, enforce_eager=ipc == "0",
                  max_num_batched_tokens=128, num_gpu_blocks_override=64)
        outs[(tp, ipc)] = [o.output_token_ids for o in llm.generate(prompts, sp)]
        if tp == ep and ipc == "1":
            w = llm.engine.executor.worker
            assert w.ep_a2a is not None, "device-side EP all-to-all not set up"
            assert llm.engine.executor.runner.stats["graph_steps"] > 0
            w.ep_a2a.check()
        llm.shutdown()
    # the device-side exchange (graphs) computes exactly what the host-count all-to-all
    # computes eagerly; vs TP = 1 only rounding differs (near-tie expert flips late on)
    assert outs[(ep, "1")] == outs[(ep, "0")], outs
    assert all(x[:3] == y[:3] for x, y in zip(outs[(1, "1")], outs[(ep, "1")])), outs


def test_pp2_stage_graphs_on_one_gpu(gpu, tmp_path, monkeypatch):
    """PP = 2 on the GPU, two stage ranks on cuda:0: each stage captures its decode step
    (receive kernel -> its layers -> send kernel / LM head) as hipGraphs with the handoff
    over peer memory, the engine keeps both micro-batches in flight, and greedy output
    equals the single-GPU engine (the stage split does not change the arithmetic)."""
    import json
    import os
    from safetensors.torch import save_file
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    cfg = PRESETS["tiny-llama"]
    d = str(tmp_path / "m")
    os.makedirs(d)
    save_file({k: v.contiguous() for k, v in full_state_dict_random(cfg, seed=5, std=0.15).items()},
              os.path.join(d, "model.safetensors"))
    json.dump({"model_type": "llama", "hidden_size": cfg.hidden_size,
               "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
               "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
               "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
               "max_position_embeddings": 512, "rope_theta": cfg.rope_theta,
               "rms_norm_eps": cfg.rms_eps, "eos_token_id": 2, "bos_token_id": 1},
              open(os.path.join(d, "config.json"), "w"))
    prompts = [list(range(3, 40)), [5, 6, 7] * 20, [9, 10, 11], [4] * 9]
    sp = [SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)] * 4
    monkeypatch.setenv("KGC_DIST_BACKEND", "gloo")
    # one arithmetic on both sides: the norm-free small-M layer (PP = 1 only: it needs the
    # whole model on one rank) rounds differently -- gamma folded into the weights, the
    # residual not normalised before its GEMM -- and the random model's near-ties then flip
    # greedy tokens (its own parity is tests/test_engine_gpu.py ..._norm_free_small_m)
    from kubernetes_gpu_cluster_amd.models import llama as llama_mod
    monkeypatch.setattr(llama_mod, "_rs_enabled", False)
    outs = {}
    for pp in (1, 2):
        llm = LLM(d, device="cuda", dtype="bfloat16", pipeline_parallel_size=pp,
                  max_model_len=256, max_num_seqs=4, max_num_batched_tokens=128,
                  num_gpu_blocks_override=64)
        outs[pp] = [o.output_token_ids for o in llm.generate(prompts, sp)]
        if pp == 2:
            r = llm.engine.executor.runner
            assert r.pp_link is not None, "PP peer-memory handoff not set up"
            assert r.stats["graph_steps"] > 0, r.stats
            r.pp_link.check()
        llm.shutdown()
    assert outs[2] == outs[1], outs


@pytest.mark.parametrize("tp,pp", [(2, 1), (1, 2)])
def test_two_node_engine_on_one_gpu(gpu, tmp_path, tp, pp):
    """The multi-pod engine (leader/worker StatefulSet layout) on the GPU: node 0 (the
    driver, this process) and entrypoints.worker_node (node 1, a separate process)
    rendezvous over TCP and run one engine; both ranks use cuda:0 with a gloo group.
    TP = 2 runs eager.  PP = 2 across the two "nodes" runs per-stage decode GRAPHS: the
    stages cannot map each other's memory across pods, so the hidden / residual rows move
    by point-to-point sends between the stages' replays (HostPipelineLink) -- both stages
    must report graph replays.  Greedy output == the single-GPU engine."""
    import json
    import os
    import socket
    import subprocess
    import sys
    from safetensors.torch import save_file
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    cfg = PRESETS["tiny-llama"]
    d = str(tmp_path / "m")
    os.makedirs(d)
    save_file({k: v.contiguous() for k, v in full_state_dict_random(cfg, seed=5, std=0.15).items()},
              os.path.join(d, "model.safetensors"))
    json.dump({"model_type": "llama", "hidden_size": cfg.hidden_size,
               "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
               "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
               "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
               "max_position_embeddings": 512, "rope_theta": cfg.rope_theta,
               "rms_norm_eps": cfg.rms_eps, "eos_token_id": 2, "bos_token_id": 1},
              open(os.path.join(d, "config.json"), "w"))
    prompts = [list(range(3, 40)), [5, 6, 7] * 20]
    sp = [SamplingParams(temperature=0, max_tokens=8, ignore_eos=True)] * 2
    common = dict(device="cuda", dtype="bfloat16", max_model_len=256, max_num_seqs=4,
                  max_num_batched_tokens=128, num_gpu_blocks_override=64, enforce_eager=True)
    ref_llm = LLM(d, **common)
    ref = [o.output_token_ids for o in ref_llm.generate(prompts, sp)]
    ref_llm.shutdown()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, KGC_DIST_BACKEND="gloo")
    stats = tmp_path / "stats"
    stats.mkdir()
    env["KGC_STAGE_STATS_DIR"] = str(stats)
    eager = pp == 1
    worker = subprocess.Popen(
        [sys.executable, "-m", "kubernetes_gpu_cluster_amd.entrypoints.worker_node", d,
         "--tensor-parallel-size", str(tp), "--pipeline-parallel-size", str(pp),
         "--nnodes", "2", "--node-rank", "1",
         "--master-addr", "127.0.0.1", "--master-port", str(port), "--device", "cuda",
         "--dtype", "bfloat16", "--max-model-len", "256", "--max-num-seqs", "4",
         "--max-num-batched-tokens", "128", "--num-gpu-blocks-override", "64"]
        + (["--enforce-eager"] if eager else []),
        cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    saved = {k: os.environ.get(k) for k in ("KGC_DIST_BACKEND", "KGC_STAGE_STATS_DIR")}
    os.environ["KGC_DIST_BACKEND"] = "gloo"
    os.environ["KGC_STAGE_STATS_DIR"] = str(stats)
    try:
        llm = LLM(d, tensor_parallel_size=tp, pipeline_parallel_size=pp, nnodes=2, node_rank=0,
                  master_addr="127.0.0.1", master_port=port,
                  **dict(common, enforce_eager=eager))
        got = [o.output_token_ids for o in llm.generate(prompts, sp)]
        llm.shutdown()
        rc = worker.wait(timeout=120)
    finally:
        for k_, v_ in saved.items():
            if v_ is None:
                os.environ.pop(k_, None)
            else:
                os.environ[k_] = v_
        if worker.poll() is None:
            worker.kill()
    assert rc == 0, worker.stdout.read()[-3000:]
    if pp == 2:
        st = {json.loads(f.read_text())["pp_rank"]: json.loads(f.read_text())
              for f in stats.glob("rank*.json")}
        assert set(st) == {0, 1}, st
        for r in (0, 1):
            assert st[r]["pp_link"] == "HostPipelineLink", st
            assert st[r]["graph_steps"] > 0, st
    same = sum(a == b for x, y in zip(ref, got) for a, b in zip(x, y))
    assert all(x[0] == y[0] for x, y in zip(ref, got)), (ref, got)
    assert same >= 0.8 * sum(len(x) for x in ref), (ref, got)


def test_phantom_ep8_rank_of_mixtral_captures_and_replays(gpu, monkeypatch):
    """KGC_TP_PHANTOM=8 with --moe-parallel ep: one process runs rank 0 of Mixtral 8x7B at
    EP = TP = 8 (2 of its layers) -- BASELINE config 4's per-rank decode step on one GPU.
    Rank 0 owns ONE whole expert; attention is the TP = 8 shard (nq 4, nkv 1).  The decode
    steps replay from hipGraphs with the device-side expert all-to-all (dispatch / receive /
    grouped MLP / return / combine, parallel/expert_a2a.py PhantomExpertAllToAll: peer
    buffers local, their flags pre-raised) and the xGMI all-reduce INSIDE the graphs; no
    barrier times out and the sticky error words stay clear."""
    from kubernetes_gpu_cluster_amd.models.moe import MoEBlock
    from kubernetes_gpu_cluster_amd.parallel import comm
    from kubernetes_gpu_cluster_amd.parallel.expert_a2a import PhantomExpertAllToAll
    from kubernetes_gpu_cluster_amd.parallel.state import get_state
    PRESETS.setdefault("mixtral-8x7b-2l", PRESETS["mixtral-8x7b"].shrink(name="mixtral-8x7b-2l",
                                                                         num_layers=2))
    monkeypatch.setenv("KGC_TP_PHANTOM", "8")
    eng = LLMEngine(EngineConfig(model="mixtral-8x7b-2l", random_init=True, max_model_len=1024,
                                 max_num_seqs=16, max_num_batched_tokens=2048,
                                 num_gpu_blocks_override=256, cuda_graph_max_bs=16,
                                 moe_parallel="ep", allow_phantom=True))
    try:
        s = get_state()
        assert s.phantom and s.tp_size == 8 and s.tp_rank == 0
        m = eng.executor.runner.model
        blk = m.layers[0].mlp
        assert isinstance(blk, MoEBlock) and blk.mode == "ep" and blk.E_local == 1
        assert isinstance(blk.ep_a2a, PhantomExpertAllToAll) and blk.ep_a2a.world == 8
        assert m.local_kv_heads() == 1
        g = torch.Generator().manual_seed(6)
        prompts = [torch.randint(100, 31000, (n,), generator=g).tolist() for n in (7, 64, 200)]
        params = [SamplingParams(temperature=1.0, seed=i, max_tokens=12, ignore_eos=True)
                  for i in range(len(prompts))]
        outs = _run(eng, prompts, params)
        assert all(len(o) == 12 for o in outs)
        st = eng.executor.runner.stats
        assert st["graph_steps"] > 0, st
        blk.ep_a2a.check()
        comm.get_custom_allreduce().check()
    finally:
        eng.shutdown()
        from kubernetes_gpu_cluster_amd.engine.worker import _release_custom_allreduce
        _release_custom_allreduce()
        set_state(ParallelState())


def test_phantom_tp8_rank_of_70b_captures_and_replays(gpu, monkeypatch):
    """KGC_TP_PHANTOM=8: one process runs rank 0 of Llama-3-70B at TP = 8 (2 of its layers)
    -- BASELINE config 3's per-rank decode step on one GPU.  The decode steps replay from
    hipGraphs with the xGMI all-reduce (plain for the embedding, fused add + RMSNorm for
    o / down) INSIDE the graphs; the peers never run, their flags are pre-raised, and no
    barrier times out.  Every non-all-reduce kernel sees the TP = 1 model's shard shapes:
    qkv N = 1280, o K = 1024, gate_up N = 7168, down K = 3584, vocab / 8, one kv head."""
    from kubernetes_gpu_cluster_amd.parallel import comm
    from kubernetes_gpu_cluster_amd.parallel.custom_allreduce import PhantomAllReduce
    from kubernetes_gpu_cluster_amd.parallel.state import get_state
    PRESETS.setdefault("llama-3-70b-2l", PRESETS["llama-3-70b"].shrink(name="llama-3-70b-2l",
                                                                       num_layers=2))
    monkeypatch.setenv("KGC_TP_PHANTOM", "8")
    eng = LLMEngine(EngineConfig(model="llama-3-70b-2l", random_init=True, max_model_len=1024,
                                 max_num_seqs=16, max_num_batched_tokens=2048,
                                 num_gpu_blocks_override=256, cuda_graph_max_bs=16,
                                 allow_phantom=True))
    try:
        s = get_state()
        assert s.phantom and s.tp_size == 8 and s.tp_rank == 0
        m = eng.executor.runner.model
        l0 = m.layers[0]
        full = PRESETS["llama-3-70b"]
        assert tuple(l0.self_attn.qkv_proj.weight.shape) == (
            (full.num_heads + 2 * full.num_kv_heads) // 8 * full.head_dim, full.hidden_size)
        assert tuple(l0.self_attn.o_proj.weight.shape) == (full.hidden_size,
                                                           full.num_heads // 8 * full.head_dim)
        assert tuple(l0.mlp.gate_up_proj.weight.shape) == (2 * full.intermediate_size // 8,
                                                           full.hidden_size)
        assert tuple(l0.mlp.down_proj.weight.shape) == (full.hidden_size,
                                                        full.intermediate_size // 8)
        assert m.local_kv_heads() == 1
        car = comm.get_custom_allreduce()
        assert isinstance(car, PhantomAllReduce) and car.world == 8
        # the phantom's policy is graph-timed too, and the eager-vs-graph delta is logged
        cal = car.calibration
        assert cal is not None and cal["timing"] == "graph" and car.table, cal
        deltas = [v for f in ("one", "two", "fused1") for v in cal["graph_minus_eager_us"][f]
                  if v is not None]
        assert deltas and len(cal["eager_choice_differs"]) == len(cal["rows"]), cal
        g = torch.Generator().manual_seed(4)
        prompts = [torch.randint(100, 128000, (n,), generator=g).tolist() for n in (5, 90, 300)]
        params = [SamplingParams(temperature=1.0, seed=i, max_tokens=12, ignore_eos=True)
                  for i in range(len(prompts))]
        outs = _run(eng, prompts, params)
        assert all(len(o) == 12 for o in outs)
        st = eng.executor.runner.stats
        assert st["graph_steps"] > 0, st
        assert car.fused_calls > 0, "fused all-reduce + add + RMSNorm never ran"
        car.check()
    finally:
        eng.shutdown()
        from kubernetes_gpu_cluster_amd.engine.worker import _release_custom_allreduce
        _release_custom_allreduce()
        set_state(ParallelState())
