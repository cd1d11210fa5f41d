"""Probe: does hipBLASLt run the decode / prefill projections faster with the weight
stored [K, N] (x @ Wt, "NN") than with the nn.Linear layout [N, K] (F.linear, "TN")?
Both layouts are TunableOp-tuned in this process (cold weights: rotating buffers), then
timed over --copies weight copies.

    python tools/gemm_layout_probe.py [--ms 256,16384]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ms", default="256,16384")
    ap.add_argument("--copies", type=int, default=8)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    c = PRESETS[a.model]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    shapes = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H), "o": (H, c.num_heads * d),
              "gate_up": (2 * I, H), "down": (H, I)}
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_duration(30)
    torch.cuda.tunable.set_rotating_buffer_size(512)
    torch.cuda.tunable.set_filename("/tmp/kgc_layout_probe.csv", insert_device_ordinal=False)
    dev = torch.device("cuda")
    for name, (N, K) in shapes.items():
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(a.copies)]
        wts = [w.t().contiguous() for w in ws]
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            F.linear(x, ws[0])          # tune TN
            x @ wts[0]                  # tune NN
            torch.cuda.synchronize()
            n = a.copies if M <= 1024 else 1
            it = max(1, 24 // n)
            t_tn = bench(lambda: [F.linear(x, w) for w in ws[:n]], it) / n
            t_nn = bench(lambda: [x @ w for w in wts[:n]], it) / n
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K,
                              "TN_us": round(t_tn * 1e6, 1), "NN_us": round(t_nn * 1e6, 1),
                              "NN_speedup": round(t_tn / t_nn, 3)}), flush=True)
        del ws, wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
