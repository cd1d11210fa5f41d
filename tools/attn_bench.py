"""Decode / prefill attention microbenchmark on realistic serving shapes.

    python tools/attn_bench.py [--batch 256] [--ctx 640] [--nq 32 --nkv 8] [--rope S]

Reports time per call and the KV bytes streamed per second (the decode kernel is
HBM-bound: every cached K/V byte of every sequence is read once per step).
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=30):
    for _ in range(3):
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=640)
    ap.add_argument("--nq", type=int, default=32)
    ap.add_argument("--nkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--max-len", type=int, default=4096)
    ap.add_argument("--ragged", type=float, default=0.25,
                    help="context lengths uniform in [ctx*(1-r), ctx] (0: all equal, as in bench.py)")
    ap.add_argument("--z", type=int, default=0, help="force the z-split (0: engine heuristic)")
    ap.add_argument("--copies", type=int, default=0,
                    help="KV copies cycled per call (0: enough for 1.5 GB, past the Infinity Cache)")
    ap.add_argument("--rope", type=int, default=-1,
                    help=">= 0: also time rope_kv_write + decode vs the fused decode kernel "
                         "(0: bf16 QKV, S > 0: S fp32 split-K slices)")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    dev = torch.device("cuda")
    B, d, bs = a.batch, a.d, a.bs
    nblk = math.ceil(a.ctx / bs)
    NB1 = B * nblk + 16
    # L "layers": disjoint copies of the KV blocks, one per call in turn, so the timed
    # calls stream from HBM as a decode step's layers do -- one copy of a small shape
    # (e.g. 84 MB at B = 256, one kv head) stays in the 256 MB Infinity Cache between
    # back-to-back calls and times the cache, not HBM
    per_copy = NB1 * a.nkv * bs * d * 2 * 2
    L = a.copies or max(1, math.ceil((1536 << 20) / per_copy))
    NB = NB1 * L
    kc = torch.randn(NB, a.nkv, bs, d, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(NB, a.nkv, bs // 8, d, 8, device=dev, dtype=torch.bfloat16)
    maxb = math.ceil(a.max_len / bs)
    perm = torch.randperm(NB1 - 1, device=dev)[: B * nblk] + 1
    bt = torch.zeros(B, maxb, dtype=torch.int32, device=dev)
    bt[:, :nblk] = perm.view(B, nblk).int()
    bts = [torch.where(bt > 0, bt + l * NB1, bt).contiguous() for l in range(L)]
    # ragged contexts around --ctx (uniform +-25%)
    ctx = (a.ctx * (1 - a.ragged + a.ragged * torch.rand(B, device=dev))).int().clamp(1, nblk * bs)
    q = torch.randn(B, a.nq, d, device=dev, dtype=torch.bfloat16)
    ws = ops.decode_partials(B, a.nq, d, maxb, bs, dev)
    z = a.z or ops.decode_grid_z(B, a.nkv, a.max_len)
    out = ops.paged_attention_decode(q, kc, vc, bt, ctx, d ** -0.5, ws, z)
    from kubernetes_gpu_cluster_amd.ops import reference as R
    n = min(B, 8)
    ref = R.paged_attention_decode(q[:n].float(), kc.float(), vc.float(), bt[:n], ctx[:n], d ** -0.5)
    err = (out[:n].float() - ref).abs().max().item()
    it = [0]

    def layer_bt():
        it[0] += 1
        return bts[it[0] % L]
    t = timeit(lambda: ops.paged_attention_decode(q, kc, vc, layer_bt(), ctx, d ** -0.5, ws, z),
               iters=max(30, 2 * L))
    kv_bytes = int(ctx.sum()) * a.nkv * d * 2 * 2
    print(json.dumps({"kernel": "paged_decode", "batch": B, "ctx_mean": float(ctx.float().mean()),
                      "z": z, "max_err": round(err, 4), "us": round(t * 1e6, 2), "kv_TBps": round(kv_bytes / t / 1e12, 3),
                      "kv_copies": L, "min_chunks": os.environ.get("KGC_DECODE_MIN_CHUNKS"),
                      "nq": a.nq, "nkv": a.nkv}))
    if a.rope >= 0:
        # rope_kv_write + paged_decode vs the fused decode kernel, the QKV projection
        # handed over as bf16 (--rope 0) or as S K9m split-K slices (--rope S)
        N = (a.nq + 2 * a.nkv) * d
        S = a.rope
        qkv = (torch.randn(S, B, N, device=dev) if S else
               torch.randn(B, N, device=dev, dtype=torch.bfloat16))
        pos = (ctx - 1).long()
        slots = (bt.gather(1, ((ctx - 1) // bs).long().unsqueeze(1)).squeeze(1).long() * bs
                 + ((ctx - 1) % bs).long())
        cs = R.rope_cos_sin_cache(d, a.max_len, 5e5).to(dev)
        nq, nkv = a.nq, a.nkv

        def unfused(btl=None):
            btl = bt if btl is None else btl
            qq = ops.rope_kv_write(qkv, pos, cs, kc, vc, slots, nq, nkv, d, dtype=torch.bfloat16)
            return ops.paged_attention_decode(qq, kc, vc, btl, ctx, d ** -0.5, ws, z)

        def fused(btl=None):
            btl = bt if btl is None else btl
            return ops.paged_attention_decode_rope(qkv, pos, cs, kc, vc, slots, nq, nkv, d, btl,
                                                   ctx, d ** -0.5, workspace=ws, grid_z=z,
                                                   dtype=torch.bfloat16)
        e = (unfused().float() - fused().float()).abs().max().item()
        tu = timeit(lambda: unfused(layer_bt()), iters=max(30, 2 * L))
        tf = timeit(lambda: fused(layer_bt()), iters=max(30, 2 * L))
        print(json.dumps({"kernel": "rope_kv + paged_decode vs paged_decode_rope", "batch": B,
                          "ctx_mean": float(ctx.float().mean()), "z": z, "S": S,
                          "unfused_us": round(tu * 1e6, 2), "fused_us": round(tf * 1e6, 2),
                          "max_diff": round(e, 5)}))


if __name__ == "__main__":
    main()
