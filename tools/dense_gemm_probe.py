"""Probe: dense split-K decode GEMM with XCD-mapped K-slices (``dense_gemm_splitk``) vs
hipBLASLt (``F.linear``), weights rotated over --copies copies (HBM-resident).  Times the
GEMM alone and GEMM + ``splitk_reduce`` (fp32 slices -> bf16).

    python tools/dense_gemm_probe.py [--m 128 256] [--s 2 4 8] [--bm 64 128]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[128, 256])
    ap.add_argument("--s", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--bm", type=int, nargs="+", default=[64, 128])
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    k = ops._k()
    dev = torch.device("cuda")
    allshapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
                 "down": (4096, 14336)}
    for name in a.shapes.split(","):
        N, K = allshapes[name]
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(a.copies)]
        for M in a.m:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ref = x.float() @ ws[-1].float().t()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

            def lin():
                for w in ws:
                    torch.matmul(x, w.t(), out=out)
            us = timed(lin, 3) / a.copies * 1e6
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "backend": "hipblaslt",
                              "us": round(us, 2), "w_TBps": round(N * K * 2 / us / 1e6, 2)}),
                  flush=True)
            for bm in a.bm:
                for S in a.s:
                    cs = torch.empty(S, M, N, device=dev, dtype=torch.float32)

                    def gem():
                        for w in ws:
                            k.dense_gemm_splitk(cs, x, w, bm)

                    def gem_red():
                        for w in ws:
                            k.dense_gemm_splitk(cs, x, w, bm)
                            k.splitk_reduce(out, cs)
                    gem_red()
                    torch.cuda.synchronize()
                    err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                    t1 = timed(gem, 3) / a.copies * 1e6
                    t2 = timed(gem_red, 3) / a.copies * 1e6
                    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "backend": "dense_splitk_xcd",
                                      "bm": bm, "S": S, "us_gemm": round(t1, 2),
                                      "us_gemm_reduce": round(t2, 2),
                                      "w_TBps": round(N * K * 2 / t2 / 1e6, 2),
                                      "rel_err": round(err, 5)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
