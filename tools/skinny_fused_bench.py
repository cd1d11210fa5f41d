"""K9 fused epilogues vs separate kernels at small M (weights rotated over --layers copies,
so they stream from HBM as in a decode step).

    python tools/skinny_fused_bench.py [--model llama-3-8b] [--ms 1,4,16]

Per (shape, M): rms_norm + skinny GEMM vs the SK_NORM skinny GEMM (qkv, gate_up), and
skinny GEMM + residual add vs the SK_ACC skinny GEMM (o, down), us per layer.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--ms", default="1,4,16")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.models import configs
    from kubernetes_gpu_cluster_amd.ops import gemm
    c = configs.PRESETS[a.model]
    H, d = c.hidden_size, c.head_dim
    shapes = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H, "norm"),
              "o": (H, c.num_heads * d, "acc"),
              "gate_up": (2 * c.intermediate_size, H, "norm"),
              "down": (H, c.intermediate_size, "acc")}
    dev = torch.device("cuda")
    ms = [int(m) for m in a.ms.split(",")]
    gamma = (torch.rand(H, device=dev) + 0.5).to(torch.bfloat16)
    for name, (N, K, kind) in shapes.items():
        ws = [torch.randn(N, K, dtype=torch.bfloat16, device=dev) * 0.02 for _ in range(a.layers)]
        gemm.clear_plan()
        gemm.tune_skinny(ws, ms, norm_shapes={(N, K)} if kind == "norm" else ())
        for M in ms:
            cfg = gemm.skinny_cfg(M, N, K)
            if cfg is None:
                continue
            x = torch.randn(M, K, dtype=torch.bfloat16, device=dev)
            res = torch.randn(M, N, dtype=torch.bfloat16, device=dev)
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            if kind == "norm":
                def sep():
                    for w in ws:
                        gemm.skinny_gemm(ops.rms_norm(x, gamma, 1e-5), w, None, cfg, out)

                ncfg = gemm._plan_norm[(M, N, K)][0]

                def fused():
                    for w in ws:
                        gemm.skinny_norm(x, w, None, gamma, 1e-5, ncfg)
            else:
                def sep():
                    for w in ws:
                        gemm.skinny_gemm(x, w, None, cfg, out)
                        res.add_(out)

                def fused():
                    for w in ws:
                        gemm.skinny_accum(res, x, w, None, cfg)
            t_sep, t_fused = _time(sep) / len(ws), _time(fused) / len(ws)
            t_plain = _time(lambda: [gemm.skinny_gemm(x, w, None, cfg, out) for w in ws]) / len(ws)
            nc = gemm._plan_norm.get((M, N, K), (None,))[0]
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "epilogue": kind, "cfg": cfg,
                              "norm_cfg": nc, "rms_norm_us": round(gemm._rms_us.get((M, K), 0), 2),
                              "plain_gemm_us": round(t_plain, 2), "separate_us": round(t_sep, 2),
                              "fused_us": round(t_fused, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()
    gemm.clear_plan()


if __name__ == "__main__":
    main()
