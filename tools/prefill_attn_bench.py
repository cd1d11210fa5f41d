"""K2 prefill attention microbenchmark: causal prefill over the paged KV cache at
prompt lengths 512 .. 32K (Llama-3-8B heads: 32 q / 8 kv x 128), one-head-per-workgroup
kernel (KGC_PREFILL_GQA=0) vs the GQA-shared kernel (=1), one-shot grid
(KGC_PREFILL_PERSIST=0) and persistent walk (=1).

    python tools/prefill_attn_bench.py [--nq 32 --nkv 8] [--shapes 32x512,8x2048,2x8192,1x16384]
                                       [--chunked 32768]

A shape ``NxL`` is N fresh prompts of L tokens in one prefill step (L <= the 16K-token
chunk); ``--chunked T`` adds a T-token prompt's last 16K-token chunk (16K queries against
all T keys).  Reports ms per call and causal TFLOP/s (4 * d * nq * sum over queries of
the keys each attends to).
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
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
    ap.add_argument("--nq", type=int, default=32)
    ap.add_argument("--nkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--shapes", default="32x512,8x2048,2x8192,1x16384")
    ap.add_argument("--chunked", type=int, default=32768)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    ops.load_extension(strict=True)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cases = []
    for sh in a.shapes.split(","):
        n, L = (int(x) for x in sh.split("x"))
        cases.append((f"{n}x{L}", [L] * n, [L] * n))
    if a.chunked:
        cases.append((f"chunk16k@{a.chunked}", [a.chunked], [min(16384, a.chunked)]))
    for name, seq_lens, qlens in cases:
        nblk = [math.ceil(s / a.bs) for s in seq_lens]
        tot = sum(nblk) + 1
        kc = (torch.randn(tot, a.nkv, a.bs, a.d, device=dev) * 0.5).to(torch.bfloat16)
        vc = torch.randn(tot, a.nkv, a.bs // 8, a.d, 8, device=dev).to(torch.bfloat16)
        bt = torch.zeros(len(seq_lens), max(nblk), dtype=torch.int32)
        k = 1
        for i, n in enumerate(nblk):
            bt[i, :n] = torch.arange(k, k + n)
            k += n
        bt = bt.to(dev)
        qsl = [0]
        for q in qlens:
            qsl.append(qsl[-1] + q)
        q = torch.randn(qsl[-1], a.nq, a.d, device=dev, dtype=torch.bfloat16)
        qsl_t = torch.tensor(qsl, dtype=torch.int32, device=dev)
        sl_t = torch.tensor(seq_lens, dtype=torch.int32, device=dev)
        ws, wm = ops.prefill_work_list(qlens, seq_lens)
        ws_t = torch.tensor(ws, dtype=torch.int32, device=dev)
        wm_t = torch.tensor(wm, dtype=torch.int32, device=dev)
        out = torch.empty_like(q)
        keys = sum(sum(s - ql + i + 1 for i in range(ql)) for s, ql in zip(seq_lens, qlens))
        flop = 4.0 * a.d * a.nq * keys
        res = {}
        for gqa, persist in (("0", "0"), ("1", "0"), ("1", "1")):
            os.environ["KGC_PREFILL_GQA"] = gqa
            os.environ["KGC_PREFILL_PERSIST"] = persist

            def run():
                ops.prefill_attention(q, kc, vc, bt, qsl_t, sl_t, a.d ** -0.5, ws_t, wm_t, out)
            t = timeit(run)
            res[gqa + persist] = t
            print(json.dumps({"case": name, "nq": a.nq, "nkv": a.nkv, "gqa_kernel": gqa == "1",
                              "persistent": persist == "1",
                              "ms": round(t * 1e3, 3), "TFLOPs": round(flop / t / 1e12, 1)}),
                  flush=True)
        print(json.dumps({"case": name, "speedup_gqa": round(res["00"] / res["10"], 3),
                          "speedup_persistent": round(res["10"] / res["11"], 3)}), flush=True)
        del kc, vc, q, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
