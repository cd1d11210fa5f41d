"""Penalties, logit_bias and min_p (engine/logits_processor.py) vs a plain per-row
reference, and their effect end to end (CPU engine, single and TP=2 ranks)."""
import torch

from kubernetes_gpu_cluster_amd.engine.logits_processor import LogitsProcessor
from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams


def _ref(logits, p, prompt, output):
    x = logits.clone().float()
    V = x.shape[0]
    cnt = torch.zeros(V)
    for t in output:
        cnt[t] += 1
    seen = cnt > 0
    for t in prompt:
        seen[t] = True
    if p.repetition_penalty != 1.0:
        x = torch.where(seen & (x > 0), x / p.repetition_penalty,
                        torch.where(seen, x * p.repetition_penalty, x))
    x = x - p.frequency_penalty * cnt - p.presence_penalty * (cnt > 0).float()
    for k, v in (p.logit_bias or {}).items():
        x[int(k)] += v
    if p.min_p > 0:
        pr = torch.softmax(x / (p.temperature if p.temperature > 0 else 1.0), -1)
        x = torch.where(pr >= p.min_p * pr.max(), x, torch.full_like(x, float("-inf")))
    return x


def test_processor_matches_reference():
    g = torch.Generator().manual_seed(0)
    V, S = 50, 5
    logits = torch.randn(S, V, generator=g) * 3
    params = [SamplingParams(presence_penalty=0.7, frequency_penalty=0.3),
              SamplingParams(),                                      # untouched row
              SamplingParams(repetition_penalty=1.3, logit_bias={"3": 5.0, 7: -100}),
              SamplingParams(min_p=0.2, temperature=0.8),
              SamplingParams(presence_penalty=-0.5, repetition_penalty=0.9, min_p=0.05)]
    prompts = [[1, 2, 2], [4], [3, 9, 11], [0], [5, 6]]
    outputs = [[2, 8, 8, 8], [], [9, 12], [1], [6, 6, 13]]
    proc = LogitsProcessor(max_seqs=8, vocab=V, device=torch.device("cpu"))
    rows = [(i, 7 - i, p) for i, p in enumerate(params) if p.needs_proc]
    for i, slot, p in rows:
        proc.init_slot(slot, prompts[i], outputs[i][:-1])
    # the last output token arrives through update() like a sampled token
    sampled = torch.tensor([o[-1] if o else 0 for o in outputs])
    proc.update(rows, sampled)
    got = logits.clone()
    proc.apply(got, rows)
    for i, p in enumerate(params):
        exp = _ref(logits[i], p, prompts[i], outputs[i]) if p.needs_proc else logits[i]
        torch.testing.assert_close(got[i], exp, atol=1e-5, rtol=1e-5)


def _llm(**kw):
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    base = dict(device="cpu", dtype="float32", random_init=True, max_model_len=128,
                max_num_seqs=4, max_num_batched_tokens=64, seed=3, num_gpu_blocks_override=64,
                block_size=16)
    base.update(kw)
    return LLM("tiny-llama", **base)


def test_engine_penalties_bias_minp():
    llm = _llm()
    prompt = [[5, 6, 7, 8]]
    base = llm.generate(prompt, SamplingParams(temperature=0, max_tokens=24, ignore_eos=True))[0]
    pen = llm.generate(prompt, SamplingParams(temperature=0, max_tokens=24, ignore_eos=True,
                                              presence_penalty=2.0, frequency_penalty=2.0))[0]
    assert len(set(pen.output_token_ids)) >= len(set(base.output_token_ids))
    assert len(set(pen.output_token_ids)) > 12          # strongly discouraged repeats
    bias = llm.generate(prompt, SamplingParams(temperature=1.0, max_tokens=6, ignore_eos=True,
                                               logit_bias={42: 100.0}, seed=1))[0]
    assert bias.output_token_ids == [42] * 6
    # min_p = 1 keeps only the argmax: sampling at T=1 == greedy
    mp = llm.generate(prompt, SamplingParams(temperature=1.0, max_tokens=24, ignore_eos=True,
                                             min_p=1.0, seed=5))[0]
    assert mp.output_token_ids == base.output_token_ids
    llm.shutdown()
