"""Model-zoo parity vs the HuggingFace transformers implementations (CPU, fp32).

Both sides load the same unsharded random state dict (models.full_state_dict_random,
HF naming).  Ours runs through the real engine path -- paged KV cache, block tables,
chunked prefill then decode steps with the reference ops -- and its logits at every
computed position must match HF's full-sequence forward.
"""
import pytest
import torch

from kubernetes_gpu_cluster_amd.engine.block_manager import BlockManager
from kubernetes_gpu_cluster_amd.engine.model_runner import ModelRunner
from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams, Sequence
from kubernetes_gpu_cluster_amd.models import PRESETS, build_model, full_state_dict_random
from kubernetes_gpu_cluster_amd.parallel.state import ParallelState, set_state

transformers = pytest.importorskip("transformers")


def _hf_model(cfg, sd):
    T = transformers
    common = dict(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                  num_hidden_layers=cfg.num_layers, num_attention_heads=cfg.num_heads,
                  max_position_embeddings=cfg.max_position, tie_word_embeddings=cfg.tie_embeddings)
    if cfg.arch == "opt":
        c = T.OPTConfig(ffn_dim=cfg.intermediate_size, word_embed_proj_dim=cfg.hidden_size,
                        do_layer_norm_before=True, **common)
        m = T.OPTForCausalLM(c)
        sd = {"model." + k: v for k, v in sd.items()}
    else:
        extra = dict(intermediate_size=cfg.intermediate_size, num_key_value_heads=cfg.num_kv_heads,
                     head_dim=cfg.head_dim, rms_norm_eps=cfg.rms_eps,
                     rope_parameters={"rope_theta": cfg.rope_theta, "rope_type": "default"})
        if cfg.arch == "llama":
            m = T.LlamaForCausalLM(T.LlamaConfig(**common, **extra))
        elif cfg.arch == "qwen2":
            m = T.Qwen2ForCausalLM(T.Qwen2Config(**common, **extra))
        elif cfg.arch == "qwen3":
            m = T.Qwen3ForCausalLM(T.Qwen3Config(**common, **extra))
        elif cfg.arch == "mixtral":
            m = T.MixtralForCausalLM(T.MixtralConfig(num_local_experts=cfg.num_experts,
                                                     num_experts_per_tok=cfg.top_k_experts,
                                                     **common, **extra))
            sd = dict(sd)
            for i in range(cfg.num_layers):
                p = f"model.layers.{i}.block_sparse_moe."
                q = f"model.layers.{i}.mlp."
                E = cfg.num_experts
                w1 = torch.stack([sd.pop(p + f"experts.{e}.w1.weight") for e in range(E)])
                w3 = torch.stack([sd.pop(p + f"experts.{e}.w3.weight") for e in range(E)])
                w2 = torch.stack([sd.pop(p + f"experts.{e}.w2.weight") for e in range(E)])
                sd[q + "experts.gate_up_proj"] = torch.cat([w1, w3], dim=1)
                sd[q + "experts.down_proj"] = w2
                sd[q + "gate.weight"] = sd.pop(p + "gate.weight")
        else:
            raise ValueError(cfg.arch)
        if cfg.tie_embeddings:
            sd = {k: v for k, v in sd.items() if k != "lm_head.weight"}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("lm_head" in k or "rotary" in k for k in missing), missing
    return m.eval(), sd


def _ours(cfg, sd):
    set_state(ParallelState())
    model = build_model(cfg, torch.float32, torch.device("cpu"))
    n = model.load_weights(sd.items())
    assert n > 0
    runner = ModelRunner(model, cfg, torch.float32, torch.device("cpu"), block_size=16,
                         max_model_len=256, max_num_seqs=4, token_budget=128, enforce_eager=True)
    runner.init_kv_cache(48)
    return model, runner


def _engine_logits(model, runner, prompt, chunks, decode_tokens):
    bm = BlockManager(48, 16, 4, runner.max_blocks)
    seq = Sequence("0", prompt, SamplingParams())
    out = []
    def run(prefills, decodes):
        plan, _ = runner.build_plan(prefills, decodes, bm.table)
        runner._upload(plan)
        meta = runner._meta(plan.T, plan.Tp, plan.P, plan.D, plan.W, plan.max_ctx,
                            split=plan.split)
        with torch.inference_mode():
            h = runner._forward(plan.T, meta)
            return model.compute_logits(h)
    for n in chunks:
        bm.allocate(seq, seq.num_computed + n)
        out.append(run([(seq, n)], []))
        seq.num_computed += n
    for t in decode_tokens:
        seq.output_token_ids.append(t)
        bm.allocate(seq, seq.num_computed + 1)
        out.append(run([], [seq]))
        seq.num_computed += 1
    return torch.cat(out, 0)


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-qwen2", "tiny-qwen3", "tiny-opt",
                                  "tiny-mixtral"])
def test_logits_match_hf(name):
    cfg = PRESETS[name]
    sd = full_state_dict_random(cfg, seed=1, std=0.05)
    hf, _ = _hf_model(cfg, sd)
    model, runner = _ours(cfg, sd)
    g = torch.Generator().manual_seed(0)
    prompt = torch.randint(3, cfg.vocab_size, (37,), generator=g).tolist()
    extra = torch.randint(3, cfg.vocab_size, (5,), generator=g).tolist()
    with torch.no_grad():
        ref = hf(torch.tensor([prompt + extra])).logits[0].float()
    got = _engine_logits(model, runner, prompt, [16, 21], extra)   # chunked prefill + 5 decodes
    torch.testing.assert_close(got, ref[: len(prompt) + len(extra)], atol=2e-4, rtol=2e-4)


def test_engine_logprobs_match_log_softmax(tmp_path):
    """Sampled-token logprob and top-k from the runner == log_softmax of the logits
    the model produces for the same prefix (raw logits, before temperature)."""
    import json
    import os
    from safetensors.torch import save_file
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLM
    from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams as SP
    cfg = PRESETS["tiny-llama"]
    sd = full_state_dict_random(cfg, seed=4, std=0.1)
    save_file({k: v.contiguous() for k, v in sd.items()}, str(tmp_path / "model.safetensors"))
    json.dump({"model_type": "llama", "hidden_size": cfg.hidden_size,
               "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
               "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
               "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
               "max_position_embeddings": 512, "rope_theta": cfg.rope_theta,
               "rms_norm_eps": cfg.rms_eps, "eos_token_id": 2, "bos_token_id": 1},
              open(tmp_path / "config.json", "w"))
    llm = LLM(str(tmp_path), device="cpu", dtype="float32", max_model_len=128, max_num_seqs=2,
              max_num_batched_tokens=64, num_gpu_blocks_override=32)
    prompt = [5, 9, 13, 17]
    out = llm.generate([prompt], [SP(temperature=0.7, max_tokens=3, ignore_eos=True, logprobs=4,
                                     seed=3)])[0]
    llm.shutdown()
    assert len(out.logprobs) == 3
    model, runner = _ours(cfg, sd)
    full = prompt + out.output_token_ids
    logits = _engine_logits(model, runner, full, [len(full)], [])
    for i, (tok, lp, top) in enumerate(out.logprobs):
        assert tok == out.output_token_ids[i]
        ref = torch.log_softmax(logits[len(prompt) - 1 + i].float(), -1)
        assert abs(ref[tok].item() - lp) < 1e-3
        assert [a for a, _ in top] == ref.topk(4).indices.tolist()
