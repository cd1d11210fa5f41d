"""Model registry, random initialisation and checkpoint loading.

Offline operation: the GPU box has no network, so models
are built from the preset table (``configs.PRESETS``) and either random-initialised
(``--random-init``, the north-star benchmark mode: "random-init weights") or
loaded from a local HF directory of safetensors shards (the reference mounts
these from hostPath ``/models/...``, ``values-01-minimal-example3.yaml:22-30``).
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
from typing import Iterable, Iterator, Optional

import torch

from .configs import PRESETS, ModelConfig, resolve_model
from .llama import LlamaForCausalLM
from .opt import OPTForCausalLM


def build_model(cfg: ModelConfig, dtype=torch.bfloat16, device=None):
    if cfg.arch == "opt":
        return OPTForCausalLM(cfg, dtype, device)
    return LlamaForCausalLM(cfg, dtype, device)


def _seed_for(name: str, base: int) -> int:
    h = hashlib.blake2b(name.encode(), digest_size=8).digest()
    return (int.from_bytes(h, "little") ^ base) & ((1 << 62) - 1)


@torch.no_grad()
def random_init(model: torch.nn.Module, seed: int = 0, std: float = 0.02) -> None:
    """Deterministic per-parameter random init, generated on the parameter's device
    (fast for 70B-class shards).  Norm weights stay at 1; biases small."""
    for name, p in model.named_parameters():
        if "norm" in name and name.endswith("weight"):
            p.fill_(1.0)
            continue
        g = torch.Generator(device=p.device)
        g.manual_seed(_seed_for(name, seed))
        if p.dtype in (torch.bfloat16, torch.float16, torch.float32):
            tmp = torch.empty(p.shape, dtype=torch.float32, device=p.device)
            tmp.normal_(0.0, std if not name.endswith("bias") else std * 0.1, generator=g)
            p.copy_(tmp)
        else:
            p.zero_()


def full_state_dict_random(cfg: ModelConfig, seed: int = 0, std: float = 0.02,
                           dtype=torch.float32) -> dict[str, torch.Tensor]:
    """An unsharded HF-layout state dict with deterministic random values (CPU).
    Used by the TP/PP parity tests: every rank loads the same full tensors and
    slices its shard through the layers' weight loaders."""
    g = torch.Generator()
    g.manual_seed(seed)

    def rnd(*shape):
        return (torch.randn(*shape, generator=g) * std).to(dtype)

    H, I, d = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    sd: dict[str, torch.Tensor] = {}
    if cfg.arch == "opt":
        sd["decoder.embed_tokens.weight"] = rnd(cfg.vocab_size, H)
        sd["decoder.embed_positions.weight"] = rnd(cfg.max_position + cfg.pos_offset, H)
        for i in range(cfg.num_layers):
            p = f"decoder.layers.{i}."
            for n in "qkv":
                sd[p + f"self_attn.{n}_proj.weight"] = rnd(H, H)
                sd[p + f"self_attn.{n}_proj.bias"] = rnd(H)
            sd[p + "self_attn.out_proj.weight"] = rnd(H, H)
            sd[p + "self_attn.out_proj.bias"] = rnd(H)
            sd[p + "fc1.weight"], sd[p + "fc1.bias"] = rnd(I, H), rnd(I)
            sd[p + "fc2.weight"], sd[p + "fc2.bias"] = rnd(H, I), rnd(H)
            for ln in ("self_attn_layer_norm", "final_layer_norm"):
                sd[p + ln + ".weight"] = 1 + rnd(H)
                sd[p + ln + ".bias"] = rnd(H)
        sd["decoder.final_layer_norm.weight"] = 1 + rnd(H)
        sd["decoder.final_layer_norm.bias"] = rnd(H)
        return sd
    sd["model.embed_tokens.weight"] = rnd(cfg.vocab_size, H)
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        sd[p + "self_attn.q_proj.weight"] = rnd(cfg.num_heads * d, H)
        sd[p + "self_attn.k_proj.weight"] = rnd(cfg.num_kv_heads * d, H)
        sd[p + "self_attn.v_proj.weight"] = rnd(cfg.num_kv_heads * d, H)
        if cfg.qkv_bias:
            sd[p + "self_attn.q_proj.bias"] = rnd(cfg.num_heads * d)
            sd[p + "self_attn.k_proj.bias"] = rnd(cfg.num_kv_heads * d)
            sd[p + "self_attn.v_proj.bias"] = rnd(cfg.num_kv_heads * d)
        sd[p + "self_attn.o_proj.weight"] = rnd(H, cfg.num_heads * d)
        if cfg.qk_norm:
            sd[p + "self_attn.q_norm.weight"] = 1 + rnd(d)
            sd[p + "self_attn.k_norm.weight"] = 1 + rnd(d)
        if cfg.is_moe:
            q = p + "block_sparse_moe."
            sd[q + "gate.weight"] = rnd(cfg.num_experts, H) * 10
            for e in range(cfg.num_experts):
                sd[q + f"experts.{e}.w1.weight"] = rnd(I, H)
                sd[q + f"experts.{e}.w3.weight"] = rnd(I, H)
                sd[q + f"experts.{e}.w2.weight"] = rnd(H, I)
        else:
            sd[p + "mlp.gate_proj.weight"] = rnd(I, H)
            sd[p + "mlp.up_proj.weight"] = rnd(I, H)
            sd[p + "mlp.down_proj.weight"] = rnd(H, I)
        sd[p + "input_layernorm.weight"] = 1 + rnd(H)
        sd[p + "post_attention_layernorm.weight"] = 1 + rnd(H)
    sd["model.norm.weight"] = 1 + rnd(H)
    if not cfg.tie_embeddings:
        sd["lm_head.weight"] = rnd(cfg.vocab_size, H)
    return sd


def iter_safetensors(path: str) -> Iterator[tuple[str, torch.Tensor]]:
    """Stream tensors from every *.safetensors shard in ``path`` (mmap, CPU)."""
    from safetensors import safe_open
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {path}")
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as fh:
            for k in fh.keys():
                yield k, fh.get_tensor(k)


class WeightsNotFoundError(FileNotFoundError):
    """The model names a checkpoint that is not there and random weights were not asked for.

    A pod whose hostPath mount failed (``values-01-minimal-example3.yaml:22-30``) must
    crash-loop, not serve random tokens with HTTP 200."""


def check_weights(model_name: str, random_weights: bool) -> Optional[str]:
    """Resolve the weights directory; raise unless it holds safetensors or random
    weights were requested (``--load-format dummy`` / ``--random-init``)."""
    _, wdir = resolve_model(model_name)
    if random_weights:
        return wdir
    if wdir is None:
        raise WeightsNotFoundError(
            f"model {model_name!r} resolves to a built-in architecture preset with no "
            f"checkpoint: pass --load-format dummy (or --random-init) for random weights, "
            f"or point the model at a directory with config.json + *.safetensors")
    if not glob.glob(os.path.join(wdir, "*.safetensors")):
        raise WeightsNotFoundError(f"no *.safetensors under {wdir!r} (and random weights were "
                                   f"not requested)")
    return wdir


def load_model(model_name: str, dtype=torch.bfloat16, device=None, random_weights: bool = False,
               seed: int = 0, cfg_override: Optional[dict] = None):
    cfg, _ = resolve_model(model_name)
    wdir = check_weights(model_name, random_weights)
    if cfg_override:
        cfg = cfg.shrink(**cfg_override)
    model = build_model(cfg, dtype, device)
    if random_weights:
        random_init(model, seed)
    else:
        model.load_weights(iter_safetensors(wdir))
    model.eval()
    return cfg, model


__all__ = ["PRESETS", "ModelConfig", "resolve_model", "build_model", "random_init",
           "full_state_dict_random", "load_model", "iter_safetensors", "check_weights",
           "WeightsNotFoundError"]
