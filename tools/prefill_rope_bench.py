"""Prefill-chunk RoPE / KV write and K2 attention, timed in a hipGraph at engine shapes.

    python tools/prefill_rope_bench.py [--prompts 32] [--len 512]

One JSON line per variant: rope_kv_write (q + k + v), the k / v-only write the fused path
uses, K2 on a rotated q, and K2 rotating q itself (prefill_attention_rope).  Run under
KGC_ROPE_KVG=0 / 1 to A/B the 8-token-group K / V writer.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(2):
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
    return best * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--len", type=int, default=512)
    ap.add_argument("--nq", type=int, default=32)
    ap.add_argument("--nkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--bs", type=int, default=32)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.ops import reference as ref
    dev = torch.device("cuda")
    P, L, nq, nkv, d, bs = a.prompts, a.len, a.nq, a.nkv, a.d, a.bs
    T = P * L
    nbp = math.ceil(L / bs)
    nb = P * nbp + 8
    kc = torch.zeros(nb, nkv, bs, d, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(nb, nkv, bs // 8, d, 8, device=dev, dtype=torch.bfloat16)
    perm = torch.randperm(nb - 1)[: P * nbp] + 1
    bt = perm.view(P, nbp).int().to(dev)
    pos = torch.arange(L).repeat(P)
    slots = (bt.cpu().long().repeat_interleave(bs, dim=1)[:, :L] * bs
             + torch.arange(L) % bs).reshape(-1)
    pos, slots = pos.to(dev), slots.to(dev)
    qkv = torch.randn(T, (nq + 2 * nkv) * d, device=dev, dtype=torch.bfloat16)
    cs = ref.rope_cos_sin_cache(d, 8192, 500000.0).to(dev)
    qsl = torch.arange(0, T + 1, L, dtype=torch.int32, device=dev)
    sl = torch.full((P,), L, dtype=torch.int32, device=dev)
    ws, wm = ops.prefill_work_list([L] * P, [L] * P)
    ws = torch.tensor(ws, dtype=torch.int32, device=dev)
    wm = torch.tensor(wm, dtype=torch.int32, device=dev)
    q = ops.rope_kv_write(qkv, pos, cs, kc, vc, slots, nq, nkv, d)
    tag = {"kvg": os.environ.get("KGC_ROPE_KVG", "1"), "T": T}
    res = {
        "rope_kv_write": timeit(lambda: ops.rope_kv_write(qkv, pos, cs, kc, vc, slots, nq, nkv, d)),
        "kv_write_rope (k/v only)": timeit(lambda: ops.kv_write_rope(qkv, pos, cs, kc, vc, slots,
                                                                     nq, nkv, d)),
        "prefill_attention": timeit(lambda: ops.prefill_attention(q, kc, vc, bt, qsl, sl,
                                                                  d ** -0.5, ws, wm)),
        "prefill_attention_rope": timeit(lambda: ops.prefill_attention_rope(
            qkv, cs, kc, vc, bt, qsl, sl, d ** -0.5, nq, d, ws, wm)),
    }
    for k, v in res.items():
        print(json.dumps(dict(tag, op=k, us=round(v, 1))), flush=True)


if __name__ == "__main__":
    main()
