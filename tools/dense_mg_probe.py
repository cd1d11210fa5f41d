"""Probe: the K14 grouped-GEMM kernel run as a dense decode GEMM (one 'expert', identity
row map), split-K S slices, weights rotated over 16 copies (HBM-resident).

    python tools/dense_mg_probe.py [--m 256]
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
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--copies", type=int, default=16)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    k = ops._k()
    dev = torch.device("cuda")
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for name, (N, K) in shapes.items():
        ws = [torch.randn(1, N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(a.copies)]
        for M in a.m:
            bm = 128
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ids = torch.arange(M, dtype=torch.int32, device=dev)
            be = torch.zeros(M // bm, dtype=torch.int32, device=dev)
            meta = torch.tensor([M // bm], dtype=torch.int32, device=dev)
            ref = x.float() @ ws[-1][0].float().t()   # run() leaves the last copy's product
            for S in (1, 2, 4, 8):
                if K // 64 < S:
                    continue
                if S > 1:
                    c = torch.empty(S, M, N, dtype=torch.float32, device=dev)
                else:
                    c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)

                def run():
                    for w in ws:
                        k.moe_gemm(c, x, w, ids, be, meta, M, 1, bm, False, S > 1, S)
                run()
                torch.cuda.synchronize()
                out = c.sum(0) if S > 1 else c.float()
                err = ((out - ref).abs().max() / ref.abs().max()).item()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(3):
                        run()
                g.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.replay()
                torch.cuda.synchronize()
                us = (time.perf_counter() - t0) / (3 * a.copies) * 1e6
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "S": S, "us": round(us, 2),
                                  "w_TBps": round(N * K * 2 / us / 1e6, 2), "rel_err": round(err, 5)}),
                      flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
