"""K9w (weights private per wave, tools/research/gemm_wv.hip) against the engine's K9m at
the decode GEMM shapes, same box, same timing: every shape's weights in --copies distinct
HBM copies (a decode step streams each weight once, never from the 256 MB Infinity Cache),
replayed from a hipGraph.

    python tools/research/build.py && python tools/research/wv_bench.py [--ms 256]

One JSON line per (shape, kernel, config): us per GEMM, weight TB/s, max relative error
against an fp32 product of the first copy.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ms", default="256")
    ap.add_argument("--copies", type=int, default=8)
    ap.add_argument("--shapes", default="gate_up,lm_head,down,qkv,o")
    a = ap.parse_args()
    import build as research_build
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    ops.load_extension(strict=True)
    r = research_build.load()
    k = torch.ops.kgc
    c = PRESETS[a.model]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    allshapes = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H, 0),
                 "o": (H, c.num_heads * d, 0), "gate_up": (2 * I, H, 2), "down": (H, I, 0),
                 "lm_head": (c.vocab_size, H, 1)}
    dev = torch.device("cuda")
    for name in a.shapes.split(","):
        N, K, epi = allshapes[name]
        copies = a.copies if N * K * 2 < (1 << 30) else 2
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        wb = N * K * 2
        silu = epi == 2
        for M in (int(m) for m in a.ms.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ref = x.float() @ ws[0].float().t()
            want = F.silu(ref[:, : N // 2]) * ref[:, N // 2:] if silu else ref
            # splits: gate_up / lm_head run unsplit (SiLU and bf16 outputs), the rest fp32 slices
            splits = (1,) if epi else (2, 4, 8)
            rows = []
            # K9m split-loader 256 x 128 (cfg 8) and 4-loader 256 x 128 (cfg 6), packed
            pk = []
            for w in ws:
                p = torch.empty(N // 128, K // 64, 8192, dtype=w.dtype, device=dev)
                k.dgemm_pack(p, w, silu)
                pk.append(p)
            for cfg in (8, 6):
                for S in splits:
                    C = (torch.empty(S, M, N, device=dev) if epi == 0 else
                         torch.empty(M, N // 2 if silu else N, device=dev, dtype=torch.bfloat16))
                    k.dgemm(C, x, pk[0], cfg, epi)
                    got = C.sum(0) if epi == 0 else C.float()

                    def run(C=C, cfg=cfg):
                        for p in pk:
                            k.dgemm(C, x, p, cfg, epi)
                    t = bench(run, max(1, 32 // copies)) / copies
                    rows.append(("k9m", cfg, S, t, got))
            del pk
            wv = []
            for w in ws:
                p = torch.empty(N // 256, K // 64, 16384, dtype=w.dtype, device=dev)
                r.wv_pack(p, w, silu)
                wv.append(p)
            for depth in (2, 3):
                for S in splits:
                    C = (torch.empty(S, M, N, device=dev) if epi == 0 else
                         torch.empty(M, N // 2 if silu else N, device=dev, dtype=torch.bfloat16))
                    r.dgemm_wv(C, x, wv[0], depth, epi)
                    got = C.sum(0) if epi == 0 else C.float()

                    def run(C=C, depth=depth):
                        for p in wv:
                            r.dgemm_wv(C, x, p, depth, epi)
                    t = bench(run, max(1, 32 // copies)) / copies
                    rows.append(("k9w", depth, S, t, got))
            del wv
            for kern, cfg, S, t, got in rows:
                err = ((got - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kernel": kern,
                                  "cfg": cfg, "S": S, "us": round(t * 1e6, 2),
                                  "w_TBps": round(wb / t / 1e12, 2),
                                  "rel_err": float(f"{err:.2e}")}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
