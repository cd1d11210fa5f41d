"""Grouped-GEMM MoE block vs the per-expert hipBLASLt loop, Mixtral-8x7B shapes.

    python tools/moe_bench.py [--tokens 256 1024 8192]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[64, 256, 1024, 8192])
    ap.add_argument("--H", type=int, default=4096)
    ap.add_argument("--I", type=int, default=14336)
    ap.add_argument("--E", type=int, default=8)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--no-loop", action="store_true", help="skip the per-expert hipBLASLt loop")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.models.moe import grouped_expert_mlp
    dev = torch.device("cuda")
    dt = torch.bfloat16
    w13 = torch.randn(a.E, 2 * a.I, a.H, device=dev, dtype=dt) * 0.02
    w2 = torch.randn(a.E, a.H, a.I, device=dev, dtype=dt) * 0.02
    wbytes = (w13.numel() + w2.numel()) * 2
    # K14m's packed per-expert copies (ops.moe_pack)
    w13p, w2p = ops.moe_pack(w13, True), ops.moe_pack(w2, False)
    for T in a.tokens:
        x = torch.randn(T, a.H, device=dev, dtype=dt)
        tw, tid = ops.moe_topk_softmax(torch.randn(T, a.E, device=dev), a.k)
        exp = ops.fused_moe(x, w13, w2, tw, tid).float()
        t_nat = timeit(lambda: ops.fused_moe(x, w13, w2, tw, tid))
        t_loop = timeit(lambda: grouped_expert_mlp(x, w13, w2, tw, tid)) if not a.no_loop else 0
        flops = 2 * T * a.k * 3 * a.H * a.I
        npairs = T * a.k
        bm = int(os.environ.get("KGC_MOE_BM", 0)) or (64 if npairs <= 40 * a.E else 128)
        S = ops.moe_splitk(npairs, a.E, a.H, a.I, bm)
        row = {"T": T, "bm": bm, "splitk": S, "native_us": round(t_nat * 1e6, 1),
               "loop_us": round(t_loop * 1e6, 1),
               "native_TFLOPs": round(flops / t_nat / 1e12, 1),
               "native_w_TBps": round(wbytes / t_nat / 1e12, 2)}
        for kbm, kbn in ((64, 256), (96, 256), (128, 256), (64, 128), (96, 128), (128, 128)):
            os.environ["KGC_MOE_BM"] = str(kbm)
            os.environ["KGC_MOE_BN"] = str(kbn)
            got = ops.fused_moe(x, w13, w2, tw, tid, w13p=w13p, w2p=w2p).float()
            err = ((got - exp).abs().max() / exp.abs().max().clamp_min(1e-6)).item()
            t = timeit(lambda: ops.fused_moe(x, w13, w2, tw, tid, w13p=w13p, w2p=w2p))
            row[f"k14m_bm{kbm}_bn{kbn}_us"] = round(t * 1e6, 1)
            row[f"k14m_bm{kbm}_bn{kbn}_w_TBps"] = round(wbytes / t / 1e12, 2)
            row[f"k14m_bm{kbm}_bn{kbn}_S"] = ops.moe_dgemm_splitk(npairs, a.E, a.H, a.I, kbm, kbn)
            row[f"k14m_bm{kbm}_bn{kbn}_rel_err"] = float(f"{err:.2e}")
        os.environ.pop("KGC_MOE_BM", None)
        os.environ.pop("KGC_MOE_BN", None)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
