"""K10 sampler microbenchmark: Gumbel-max over a Llama-3 vocabulary.

    python tools/sample_bench.py [--vocab 128256] [--batches 1,8,64,256]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--batches", default="1,8,64,256")
    ap.add_argument("--stamps", action="store_true",
                    help="print the cooperative kernel's phase stamps (workgroup 0 of row 0)")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    dev = torch.device("cuda")
    for B in [int(b) for b in a.batches.split(",")]:
        for mode in ("temperature", "greedy", "top_p", "top_k", "top_k_p"):
            logits = torch.randn(B, a.vocab, device=dev).to(torch.bfloat16)
            temp = torch.full((B,), 0.0 if mode == "greedy" else 1.0, device=dev)
            top_k = torch.full((B,), 50 if mode in ("top_k", "top_k_p") else -1, dtype=torch.int32, device=dev)
            top_p = torch.full((B,), 0.9 if mode in ("top_p", "top_k_p") else 1.0, device=dev)
            seeds = torch.arange(B, dtype=torch.int64, device=dev)
            out = ops.sample(logits, temp, top_k, top_p, seeds)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(20):
                    ops.sample(logits, temp, top_k, top_p, seeds, out=out)
            g.replay()
            torch.cuda.synchronize()
            t = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t) / 20 * 1e6
            rec = {"op": "sample", "mode": mode, "B": B, "V": a.vocab, "us": round(us, 2)}
            if a.stamps and mode in ("top_p", "top_k", "top_k_p"):
                k = torch.ops.kgc
                k.sample_stamps_enable(True)
                ops.sample(logits, temp, top_k, top_p, seeds, out=out)
                torch.cuda.synchronize()
                st = k.sample_stamps()
                k.sample_stamps_enable(False)
                # 100 MHz wall clock: 10 ns per tick; phases never reached stay 0
                rec["phase_us"] = {i: round((st[i] - st[0]) / 100, 2) for i in range(1, 13)
                                   if st[i] >= st[0] > 0}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
