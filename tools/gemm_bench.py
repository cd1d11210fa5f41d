"""Microbenchmark the projection GEMM shapes of the decode / prefill steps.

    python tools/gemm_bench.py [--model llama-3-8b] [--ms 1,16,64,128,256,512] [--table CSV]

Reports per shape: time, weight-streaming TB/s and TFLOP/s for F.linear
(hipBLASLt) -- the baseline the hand-written decode GEMM must beat.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def shapes(model):
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    c = PRESETS[model]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    return {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H), "o": (H, c.num_heads * d),
            "gate_up": (2 * I, H), "down": (H, I), "lm_head": (c.vocab_size, H)}


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ms", default="1,16,64,128,256,512,4096")
    ap.add_argument("--backend", default="hipblaslt")
    ap.add_argument("--table", default=None, help="TunableOp results CSV to apply (read-only)")
    ap.add_argument("--copies", type=int, default=1,
                    help="rotate over this many weight copies (>1: weights stream from HBM, "
                         "not the 256 MB Infinity Cache, as in a decode step)")
    a = ap.parse_args()
    if a.backend != "hipblaslt":
        torch.backends.cuda.preferred_blas_library(a.backend)
    if a.table:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(False)
        torch.cuda.tunable.set_filename(a.table, insert_device_ordinal=False)
        assert torch.cuda.tunable.read_file(a.table), a.table
    dev = torch.device("cuda")
    res = []
    for name, (N, K) in shapes(a.model).items():
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(a.copies)]
        for M in [int(x) for x in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)

            def run():
                for w in ws:
                    F.linear(x, w)
            t = bench(run, iters=max(1, 50 // a.copies)) / a.copies
            row = {"shape": name, "M": M, "N": N, "K": K,
                   "backend": "tunableop-table" if a.table else a.backend,
                   "us": round(t * 1e6, 2), "w_TBps": round(N * K * 2 / t / 1e12, 2),
                   "TFLOPs": round(2 * M * N * K / t / 1e12, 1)}
            print(json.dumps(row), flush=True)
            res.append(row)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
