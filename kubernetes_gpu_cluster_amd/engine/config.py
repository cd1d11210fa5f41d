"""Engine configuration and the vLLM-compatible CLI flag surface.

The reference passes engine flags through Helm ``vllmConfig`` keys and
``extraArgs`` (``values-01-minimal-example8.yaml:23-38``):
``--tensor-parallel-size``, ``--pipeline-parallel-size``, ``--max-model-len``,
``--gpu-memory-utilization``, ``--dtype float16``, ``--disable-custom-all-reduce``,
``--enforce-eager``, ``--trust-remote-code``, ``--kv-cache-dtype``.  All of them are
accepted here with the same spelling (both ``--flag value`` and ``--flag=value``).
"""
from __future__ import annotations

import argparse
import dataclasses
from typing import Optional

import torch

_DTYPES = {"auto": None, "bfloat16": torch.bfloat16, "bf16": torch.bfloat16,
           "float16": torch.float16, "half": torch.float16, "fp16": torch.float16,
           "float32": torch.float32, "float": torch.float32}


KV_CACHE_DTYPES = ("auto", "bfloat16", "bf16", "float16", "fp16", "fp8", "fp8_e4m3")


@dataclasses.dataclass
class EngineConfig:
    model: str = "llama-3-8b"
    served_model_name: Optional[str] = None
    tokenizer: Optional[str] = None
    dtype: str = "auto"
    tensor_parallel_size: int = 1
    pipeline_parallel_size: int = 1
    max_model_len: Optional[int] = None
    gpu_memory_utilization: float = 0.90
    block_size: int = 32
    max_num_seqs: int = 256
    max_num_batched_tokens: Optional[int] = None
    enable_chunked_prefill: bool = True
    prefill_first: bool = False           # decodes sit out while prompts wait (scheduler.py)
    prefill_first_max_defer: int = 8      # ... for at most this many consecutive steps
    prefill_first_max_gap_ms: float = 0.0  # ... or until a running stream waited this long
    enable_prefix_caching: bool = True    # vLLM V1 default: reuse cached KV of shared prefixes
    enforce_eager: bool = False
    disable_custom_all_reduce: bool = False
    trust_remote_code: bool = False
    kv_cache_dtype: str = "auto"
    seed: int = 0
    random_init: bool = False
    num_gpu_blocks_override: Optional[int] = None
    device: str = "auto"                  # auto | cuda | cpu
    moe_parallel: str = "tp"              # tp | ep  (Mixtral expert placement)
    cuda_graph_max_bs: int = 256
    async_output: bool = True             # overlap host bookkeeping with the next step
    num_cpu_blocks: int = 0
    # one engine spread over several nodes / pods (TP x PP ranks split evenly):
    # node 0 runs the API server and ranks [0, g); node k runs ranks [k*g, (k+1)*g)
    # via entrypoints.worker_node; rendezvous at master_addr:master_port
    nnodes: int = 1
    node_rank: int = 0
    master_addr: Optional[str] = None
    master_port: int = 29500
    # KGC_TP_PHANTOM (parallel/state.py init_phantom) is a one-GPU per-rank MEASUREMENT
    # stand-in whose missing peers contribute zeros to every all-reduce: its completions are
    # wrong by construction.  Only bench.py --mode engine and the tests set this; every other
    # entrypoint (API server, LLM) leaves it False, and the worker then refuses the mode.
    allow_phantom: bool = False

    def torch_dtype(self, model_default: torch.dtype = torch.bfloat16) -> torch.dtype:
        d = _DTYPES.get(self.dtype.lower())
        if self.dtype.lower() not in _DTYPES:
            raise ValueError(f"unsupported --dtype {self.dtype}")
        return model_default if d is None else d

    def kv_torch_dtype(self, act: torch.dtype) -> torch.dtype:
        """Cache element type: fp8 e4m3 for --kv-cache-dtype fp8, else the activations'."""
        if self.kv_cache_dtype in ("fp8", "fp8_e4m3"):
            return torch.float8_e4m3fn
        return act

    def resolved_device(self) -> torch.device:
        if self.device == "auto":
            return torch.device("cuda" if torch.cuda.is_available() else "cpu")
        return torch.device(self.device)

    @property
    def world_size(self) -> int:
        return self.tensor_parallel_size * self.pipeline_parallel_size

    @property
    def ranks_per_node(self) -> int:
        if self.world_size % self.nnodes:
            raise ValueError(f"tp*pp={self.world_size} does not split over {self.nnodes} nodes")
        return self.world_size // self.nnodes

    def dist_env(self) -> dict:
        """Rendezvous env shared by every rank of this engine."""
        if self.nnodes > 1 and not self.master_addr:
            raise ValueError("--nnodes > 1 needs --master-addr (node 0's address)")
        return {"MASTER_ADDR": self.master_addr or "127.0.0.1", "MASTER_PORT": str(self.master_port),
                "WORLD_SIZE": str(self.world_size)}

    def token_budget(self) -> int:
        if self.max_num_batched_tokens:
            return self.max_num_batched_tokens
        return 16384 if self.enable_chunked_prefill else max(16384, self.max_model_len or 0)


def add_engine_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    a = p.add_argument
    a("--model", type=str, default=None, help="preset name, local HF dir, or HF id")
    a("--served-model-name", type=str, default=None)
    a("--tokenizer", type=str, default=None)
    a("--dtype", type=str, default="auto")
    a("--tensor-parallel-size", "-tp", type=int, default=1)
    a("--pipeline-parallel-size", "-pp", type=int, default=1)
    a("--max-model-len", type=int, default=None)
    a("--gpu-memory-utilization", type=float, default=0.90)
    a("--block-size", type=int, default=32)
    a("--max-num-seqs", type=int, default=256)
    a("--max-num-batched-tokens", type=int, default=None)
    a("--enable-chunked-prefill", dest="enable_chunked_prefill", action="store_true",
      default=True)
    a("--no-enable-chunked-prefill", dest="enable_chunked_prefill", action="store_false")
    a("--prefill-first", action="store_true",
      help="while prompts wait for a free sequence slot, running sequences skip decode steps "
           "and the token budget goes to prefill (lower TTFT under bursts)")
    a("--prefill-first-max-defer", type=int, default=8,
      help="with --prefill-first: decodes run at least every N+1 steps (bounds TPOT under "
           "continuous arrivals; 8 keeps a 256 x 512-token burst prefill-only)")
    a("--prefill-first-max-gap-ms", type=float, default=0.0,
      help="with --prefill-first: never defer decodes once a running stream has waited this "
           "long for its next token (0 = off)")
    a("--enable-prefix-caching", dest="enable_prefix_caching", action="store_true", default=True)
    a("--no-enable-prefix-caching", dest="enable_prefix_caching", action="store_false")
    a("--enforce-eager", action="store_true")
    a("--disable-custom-all-reduce", action="store_true")
    a("--trust-remote-code", action="store_true")
    a("--kv-cache-dtype", type=str, default="auto",
      help="auto (activation dtype) or fp8 / fp8_e4m3 (half the KV bytes)")
    a("--seed", type=int, default=0)
    a("--random-init", action="store_true", help="random weights (offline benchmarking)")
    a("--load-format", type=str, default="auto", help="'dummy' == --random-init")
    a("--num-gpu-blocks-override", type=int, default=None)
    a("--device", type=str, default="auto")
    a("--moe-parallel", type=str, default="tp", choices=["tp", "ep"])
    a("--cuda-graph-max-bs", type=int, default=256)
    a("--nnodes", type=int, default=1, help="nodes (pods) one engine spans")
    a("--node-rank", type=int, default=0)
    a("--master-addr", type=str, default=None, help="address of node 0 (multi-node)")
    a("--master-port", type=int, default=29500)
    a("--swap-space", type=float, default=0, help="accepted for compatibility (unused)")
    a("--disable-log-requests", action="store_true")
    a("--disable-log-stats", action="store_true")
    return p


def config_from_args(ns: argparse.Namespace) -> EngineConfig:
    if ns.kv_cache_dtype not in KV_CACHE_DTYPES:
        raise ValueError(f"--kv-cache-dtype {ns.kv_cache_dtype} is not supported "
                         f"({'/'.join(KV_CACHE_DTYPES)})")
    return EngineConfig(
        model=ns.model, served_model_name=ns.served_model_name, tokenizer=ns.tokenizer,
        dtype=ns.dtype, tensor_parallel_size=ns.tensor_parallel_size,
        pipeline_parallel_size=ns.pipeline_parallel_size, max_model_len=ns.max_model_len,
        gpu_memory_utilization=ns.gpu_memory_utilization, block_size=ns.block_size,
        max_num_seqs=ns.max_num_seqs, max_num_batched_tokens=ns.max_num_batched_tokens,
        enable_chunked_prefill=ns.enable_chunked_prefill, enforce_eager=ns.enforce_eager,
        prefill_first=ns.prefill_first, prefill_first_max_defer=ns.prefill_first_max_defer,
        prefill_first_max_gap_ms=ns.prefill_first_max_gap_ms,
        enable_prefix_caching=ns.enable_prefix_caching,
        disable_custom_all_reduce=ns.disable_custom_all_reduce,
        trust_remote_code=ns.trust_remote_code, kv_cache_dtype=ns.kv_cache_dtype, seed=ns.seed,
        random_init=ns.random_init or ns.load_format == "dummy",
        num_gpu_blocks_override=ns.num_gpu_blocks_override, device=ns.device,
        moe_parallel=ns.moe_parallel, cuda_graph_max_bs=ns.cuda_graph_max_bs,
        nnodes=ns.nnodes, node_rank=ns.node_rank, master_addr=ns.master_addr,
        master_port=ns.master_port)
