"""K9 skinny GEMM vs hipBLASLt on a model's decode GEMM shapes (small batch).

    python tools/skinny_bench.py [--model llama-3-8b] [--layers 32] [--ms 1,2,4,8,16,32,64]

Every shape is timed over ``--layers`` distinct weight copies (as in a decode step,
the weights stream from HBM, not the 256 MB Infinity Cache).  One JSON line per
(M, N, K): hipBLASLt us, best skinny config and its us per call, weight TB/s.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--ms", default="1,2,4,8,16,24,32,48,64")
    ap.add_argument("--tp", type=int, default=1)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd.models import configs
    from kubernetes_gpu_cluster_amd.ops import gemm
    from kubernetes_gpu_cluster_amd.utils.gemm_tuning import enable_tuned_gemms
    enable_tuned_gemms(a.model, a.tp)
    c = configs.PRESETS[a.model]
    H, d, tp = c.hidden_size, c.head_dim, a.tp
    shapes = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d // tp, H),
              "o": (H, c.num_heads * d // tp),
              "gate_up": (2 * c.intermediate_size // tp, H),
              "down": (H, c.intermediate_size // tp)}
    dev = torch.device("cuda")
    ms = [int(m) for m in a.ms.split(",")]
    for name, (N, K) in shapes.items():
        ws = [torch.randn(N, K, dtype=torch.bfloat16, device=dev) * 0.02 for _ in range(a.layers)]
        res = gemm.tune_skinny(ws, ms)
        for (M, n, k), (chosen, lib_us, sk_us, sk_cfg) in sorted(res.items()):
            print(json.dumps({"gemm": name, "M": M, "N": n, "K": k, "hipblaslt_us": round(lib_us, 2),
                              "skinny_us": round(sk_us, 2), "skinny_cfg": sk_cfg,
                              "chosen": "skinny" if chosen else "hipblaslt",
                              "skinny_speedup": round(lib_us / sk_us, 3),
                              "skinny_weight_TBps": round(n * k * 2 / sk_us / 1e6, 2),
                              "hipblaslt_weight_TBps": round(n * k * 2 / lib_us / 1e6, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
