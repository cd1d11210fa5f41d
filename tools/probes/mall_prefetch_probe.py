"""Probe: does a batch-1 decode GEMM run faster when its weight was read once just before
(so it sits in the 256 MB Infinity Cache / MALL) than from cold HBM?

For each Llama-3-8B projection at M = 1: flush (read a 1 GB scratch buffer: reads leave no dirty lines to write back), optionally
read the weight once (a plain reduction kernel), then time the tuned K9 / hipBLASLt GEMM
between two events.  Reports the median over --reps iterations for both orders.

    python tools/probes/mall_prefetch_probe.py [--reps 30]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--m", type=int, default=1)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.ops import gemm
    ops.load_extension(strict=True)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    ws = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
    gemm.tune_skinny(list(ws.values()), [a.m])
    flush = torch.ones(1 << 28, dtype=torch.int32, device=dev)     # 1 GB, read to evict
    sink = torch.zeros(1, dtype=torch.float32, device=dev)
    for name, w in ws.items():
        x = torch.randn(a.m, w.shape[1], device=dev, dtype=torch.bfloat16)
        res = {}
        for mode in ("cold", "prefetched", "prefetched_half"):
            ts = []
            for _ in range(a.reps + 3):
                sink += flush.sum(dtype=torch.int64).float()
                if mode == "prefetched":
                    sink += w.view(torch.int32).sum(dtype=torch.int64).float()
                elif mode == "prefetched_half":
                    sink += w[: w.shape[0] // 2].view(torch.int32).sum(dtype=torch.int64).float()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gemm.linear(x, w)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            res[mode] = statistics.median(ts[3:])
        mb = w.numel() * 2 / 1e6
        print(json.dumps({"shape": name, "M": a.m, "MB": round(mb, 1),
                          **{k + "_us": round(v, 2) for k, v in res.items()},
                          "cold_TBps": round(mb / res["cold"], 2),
                          "prefetched_TBps": round(mb / res["prefetched"], 2)}),
              flush=True)


if __name__ == "__main__":
    main()
