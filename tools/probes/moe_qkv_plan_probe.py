"""Probe: which GEMM path do a Mixtral engine's decode graphs capture at batch 256?
(Round-6 Mixtral anatomy showed qkv and lm_head on hipBLASLt despite K9m plans.)
Records every K9m plan lookup (M, N, K, kind -> plan) while the engine starts (tuning,
graph capture) and runs a few batch-256 decode steps."""
import collections
import logging
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
logging.basicConfig(level=logging.WARNING, stream=sys.stderr, format="%(message)s")


def main():
    import kubernetes_gpu_cluster_amd.ops.gemm as G
    from kubernetes_gpu_cluster_amd.engine.config import EngineConfig
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLMEngine
    from kubernetes_gpu_cluster_amd.engine.sequence import SamplingParams
    from kubernetes_gpu_cluster_amd.models import configs
    name = sys.argv[1] if len(sys.argv) > 1 else "mixtral-8x7b"
    configs.PRESETS[name + "-2l"] = configs.PRESETS[name].shrink(name=name + "-2l", num_layers=2)
    seen = collections.Counter()
    orig = G._dg_plan

    def spy(x, w, kind):
        p = orig(x, w, kind)
        seen[(tuple(x.shape), tuple(w.shape), kind, p, tuple(x.stride()))] += 1
        return p
    G._dg_plan = spy
    eng = LLMEngine(EngineConfig(model=name + "-2l", random_init=True, max_model_len=512,
                                 max_num_seqs=256, max_num_batched_tokens=16384,
                                 cuda_graph_max_bs=256))
    print("plans after start:", {k: v for k, v in G.dgemm_plan().items() if k[0] == 256})
    sp = SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True)
    for i in range(256):
        eng.add_request(list(range(10 + i % 50, 42 + i % 50)), sp)
    while eng.has_unfinished():
        eng.step()
    torch.cuda.synchronize()
    for k, v in sorted(seen.items(), key=lambda kv: (kv[0][0][0], kv[0][2])):
        if k[0][0] >= 200:
            print("lookup", k, "x", v)
    print("runner stats", eng.executor.runner.stats)


if __name__ == "__main__":
    main()
