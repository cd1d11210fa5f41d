"""Built-in model architectures (offline: no HF download on the GPU box).

The reference deploys these models through its Helm values files
(`values-01-minimal-example.yaml:7` OPT-125m, `values-01-minimal-example2.yaml:8`
Qwen3-0.6B, `…4.yaml:8` Qwen-7B, `…5.yaml:8` Qwen3-4B, `…8.yaml:8` Qwen2.5-7B,
`…9.yaml:8` Qwen3-14B) and the north-star configs add Llama-3-8B/70B and
Mixtral-8x7B.  Dimensions are the public HF config values.

A model is resolved from (in order): a preset name, a local directory holding
an HF ``config.json`` (weights loaded from safetensors if present), or an HF
id whose basename matches a preset (``Qwen/Qwen3-0.6B`` -> ``qwen3-0.6b``).
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Optional


@dataclasses.dataclass
class ModelConfig:
    name: str
    arch: str                    # "llama" | "qwen2" | "qwen3" | "qwen" | "opt" | "mixtral"
    num_layers: int
    hidden_size: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int
    max_position: int = 8192
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None
    rms_eps: float = 1e-5
    tie_embeddings: bool = False
    qkv_bias: bool = False
    qk_norm: bool = False        # Qwen3 per-head q/k RMSNorm (kernel K6)
    # OPT
    norm_type: str = "rms"       # "rms" | "layer"
    act: str = "silu"            # "silu" (SwiGLU) | "relu" (OPT)
    learned_pos: bool = False
    pos_offset: int = 0
    mlp_bias: bool = False
    o_bias: bool = False
    # MoE
    num_experts: int = 0
    top_k_experts: int = 0
    bos_token_id: int = 1
    eos_token_id: int = 2

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def num_params(self) -> int:
        h, i, L = self.hidden_size, self.intermediate_size, self.num_layers
        attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
        if self.act == "silu":
            mlp = 3 * h * i
        else:
            mlp = 2 * h * i
        if self.is_moe:
            mlp = mlp * self.num_experts + h * self.num_experts
        emb = self.vocab_size * h * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp) + emb

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.num_kv_heads * self.head_dim * dtype_bytes

    def shrink(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


_LLAMA3_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                   "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}

PRESETS: dict[str, ModelConfig] = {
    # north-star model (BASELINE configs 2, 5)
    "llama-3-8b": ModelConfig("llama-3-8b", "llama", 32, 4096, 32, 8, 128, 14336, 128256,
                              max_position=8192, rope_theta=500000.0, bos_token_id=128000,
                              eos_token_id=128001),
    "llama-3.1-8b": ModelConfig("llama-3.1-8b", "llama", 32, 4096, 32, 8, 128, 14336, 128256,
                                max_position=131072, rope_theta=500000.0,
                                rope_scaling=_LLAMA3_SCALING, bos_token_id=128000,
                                eos_token_id=128001),
    "llama-3-70b": ModelConfig("llama-3-70b", "llama", 80, 8192, 64, 8, 128, 28672, 128256,
                               max_position=8192, rope_theta=500000.0, bos_token_id=128000,
                               eos_token_id=128001),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", "mixtral", 32, 4096, 32, 8, 128, 14336, 32000,
                                max_position=32768, rope_theta=1e6, num_experts=8,
                                top_k_experts=2),
    # reference values-file models
    "opt-125m": ModelConfig("opt-125m", "opt", 12, 768, 12, 12, 64, 3072, 50272,
                            max_position=2048, norm_type="layer", act="relu",
                            learned_pos=True, pos_offset=2, qkv_bias=True, mlp_bias=True,
                            o_bias=True, tie_embeddings=True, bos_token_id=2, eos_token_id=2),
    "qwen3-0.6b": ModelConfig("qwen3-0.6b", "qwen3", 28, 1024, 16, 8, 128, 3072, 151936,
                              max_position=40960, rope_theta=1e6, rms_eps=1e-6,
                              tie_embeddings=True, qk_norm=True, bos_token_id=151643,
                              eos_token_id=151645),
    "qwen3-4b": ModelConfig("qwen3-4b", "qwen3", 36, 2560, 32, 8, 128, 9728, 151936,
                            max_position=40960, rope_theta=1e6, rms_eps=1e-6,
                            tie_embeddings=True, qk_norm=True, bos_token_id=151643,
                            eos_token_id=151645),
    "qwen3-14b": ModelConfig("qwen3-14b", "qwen3", 40, 5120, 40, 8, 128, 17408, 151936,
                             max_position=40960, rope_theta=1e6, rms_eps=1e-6,
                             qk_norm=True, bos_token_id=151643, eos_token_id=151645),
    "qwen2.5-7b": ModelConfig("qwen2.5-7b", "qwen2", 28, 3584, 28, 4, 128, 18944, 152064,
                              max_position=32768, rope_theta=1e6, rms_eps=1e-6, qkv_bias=True,
                              bos_token_id=151643, eos_token_id=151643),
    "qwen-7b": ModelConfig("qwen-7b", "qwen", 32, 4096, 32, 32, 128, 11008, 151936,
                           max_position=8192, rope_theta=10000.0, rms_eps=1e-6, qkv_bias=True,
                           bos_token_id=151643, eos_token_id=151643),
    # tiny configs for tests / CPU plumbing
    "tiny-llama": ModelConfig("tiny-llama", "llama", 2, 256, 4, 2, 64, 512, 1024,
                              max_position=2048, rope_theta=10000.0, bos_token_id=1,
                              eos_token_id=2),
    "tiny-qwen3": ModelConfig("tiny-qwen3", "qwen3", 2, 256, 4, 2, 64, 512, 1024,
                              max_position=2048, rope_theta=1e6, rms_eps=1e-6, qk_norm=True,
                              tie_embeddings=True),
    "tiny-qwen2": ModelConfig("tiny-qwen2", "qwen2", 2, 256, 4, 2, 64, 512, 1024,
                              max_position=2048, rope_theta=1e6, rms_eps=1e-6, qkv_bias=True),
    "tiny-opt": ModelConfig("tiny-opt", "opt", 2, 128, 4, 4, 32, 512, 1024, max_position=512,
                            norm_type="layer", act="relu", learned_pos=True, pos_offset=2,
                            qkv_bias=True, mlp_bias=True, o_bias=True, tie_embeddings=True),
    # TP = 8 rehearsals: 16 q / 2 kv heads of 64 (each kv head replicated on 4 ranks at
    # TP = 8; GPU kernels take head_dim 64 / 128), and Llama-3-70B's head layout (64 q / 8
    # kv, intermediate 3.5 x hidden) scaled down to head_dim 16 (CPU oracle path only)
    "tiny-llama-gqa8": ModelConfig("tiny-llama-gqa8", "llama", 2, 1024, 16, 2, 64, 2048, 1024,
                                   max_position=2048, rope_theta=500000.0, bos_token_id=1,
                                   eos_token_id=2),
    "tiny-llama-70b-shape": ModelConfig("tiny-llama-70b-shape", "llama", 2, 1024, 64, 8, 16,
                                        3584, 1024, max_position=2048, rope_theta=500000.0,
                                        rope_scaling=_LLAMA3_SCALING, bos_token_id=1,
                                        eos_token_id=2),
    "tiny-mixtral": ModelConfig("tiny-mixtral", "mixtral", 2, 256, 4, 2, 64, 384, 1024,
                                max_position=2048, rope_theta=1e6, num_experts=4,
                                top_k_experts=2),
}

# HF repo basenames (lower-cased) -> preset
_ALIASES = {
    "meta-llama-3-8b": "llama-3-8b", "meta-llama-3-8b-instruct": "llama-3-8b",
    "llama-3-8b-instruct": "llama-3-8b", "meta-llama-3.1-8b": "llama-3.1-8b",
    "llama-3.1-8b-instruct": "llama-3.1-8b", "meta-llama-3.1-8b-instruct": "llama-3.1-8b",
    "meta-llama-3-70b": "llama-3-70b", "meta-llama-3-70b-instruct": "llama-3-70b",
    "mixtral-8x7b-v0.1": "mixtral-8x7b", "mixtral-8x7b-instruct-v0.1": "mixtral-8x7b",
    "qwen2.5-7b-instruct": "qwen2.5-7b", "qwen3-0.6b-base": "qwen3-0.6b",
}


def _from_hf_config(d: dict, name: str) -> ModelConfig:
    """Map an HF config.json dict onto ModelConfig."""
    mt = d.get("model_type", "llama")
    if mt == "opt":
        h = d["hidden_size"]
        return ModelConfig(name, "opt", d["num_hidden_layers"], h, d["num_attention_heads"],
                           d["num_attention_heads"], h // d["num_attention_heads"], d["ffn_dim"],
                           d["vocab_size"], max_position=d.get("max_position_embeddings", 2048),
                           norm_type="layer", act="relu", learned_pos=True, pos_offset=2,
                           qkv_bias=True, mlp_bias=True, o_bias=True,
                           tie_embeddings=d.get("tie_word_embeddings", True),
                           bos_token_id=d.get("bos_token_id", 2),
                           eos_token_id=d.get("eos_token_id", 2))
    if mt == "qwen":  # Qwen v1 (trust-remote-code arch)
        h = d["hidden_size"]
        nh = d["num_attention_heads"]
        return ModelConfig(name, "qwen", d["num_hidden_layers"], h, nh, nh, h // nh,
                           d["intermediate_size"] // 2, d["vocab_size"],
                           max_position=d.get("seq_length", 8192),
                           rope_theta=d.get("rotary_emb_base", 10000.0),
                           rms_eps=d.get("layer_norm_epsilon", 1e-6), qkv_bias=True)
    nh = d["num_attention_heads"]
    h = d["hidden_size"]
    arch = {"llama": "llama", "qwen2": "qwen2", "qwen3": "qwen3", "mistral": "llama",
            "mixtral": "mixtral"}.get(mt, "llama")
    eos = d.get("eos_token_id", 2)
    if isinstance(eos, list):
        eos = eos[0]
    return ModelConfig(
        name, arch, d["num_hidden_layers"], h, nh, d.get("num_key_value_heads", nh),
        d.get("head_dim") or h // nh, d["intermediate_size"], d["vocab_size"],
        max_position=d.get("max_position_embeddings", 8192),
        rope_theta=float(d.get("rope_theta", 10000.0)), rope_scaling=d.get("rope_scaling"),
        rms_eps=d.get("rms_norm_eps", 1e-6), tie_embeddings=d.get("tie_word_embeddings", False),
        qkv_bias=(arch == "qwen2") or d.get("attention_bias", False), qk_norm=(arch == "qwen3"),
        num_experts=d.get("num_local_experts", 0), top_k_experts=d.get("num_experts_per_tok", 0),
        bos_token_id=d.get("bos_token_id", 1) or 1, eos_token_id=eos)


def resolve_model(model: str) -> tuple[ModelConfig, Optional[str]]:
    """Return (config, weights_dir_or_None) for a preset name, local dir or HF id."""
    key = model.lower().rstrip("/")
    if key in PRESETS:
        return PRESETS[key], None
    if os.path.isdir(model) and os.path.isfile(os.path.join(model, "config.json")):
        with open(os.path.join(model, "config.json")) as f:
            cfg = _from_hf_config(json.load(f), os.path.basename(model.rstrip("/")))
        return cfg, model
    base = os.path.basename(key)
    base = _ALIASES.get(base, base)
    if base in PRESETS:
        return PRESETS[base], None
    raise ValueError(f"unknown model {model!r}: not a preset ({sorted(PRESETS)}) and no "
                     f"config.json found at that path")
