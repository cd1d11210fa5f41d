"""Prefill-chunk GEMMs of one model, timed the way a chunked-prefill step runs them.

    python tools/prefill_gemm_probe.py [--model llama-3-8b] [--tokens 16384] [--layers 8]

For each projection at M = --tokens: hipBLASLt's default pick vs the tuned table
(profiles/tunableop), isolated (one weight, repeated) and as a layer sequence
(qkv -> o -> gate_up -> down over --layers distinct weight sets, as the forward pass
streams them).  Prints one JSON line per measurement: ms and PF/s.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5,
                    help="timed calls per measurement (200+: sustained, power-managed clocks)")
    ap.add_argument("--tables", default="default,tuned")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    from kubernetes_gpu_cluster_amd.utils.gemm_tuning import enable_tuned_gemms
    c = PRESETS[a.model]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    shapes = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H), "o": (H, c.num_heads * d),
              "gate_up": (2 * I, H), "down": (H, I)}
    dev = torch.device("cuda")
    M = a.tokens
    ws = {n: [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(a.layers)]
          for n, (N, K) in shapes.items()}
    xs = {n: torch.randn(M, K, device=dev, dtype=torch.bfloat16) for n, (N, K) in shapes.items()}
    flops = {n: 2.0 * M * N * K for n, (N, K) in shapes.items()}

    def report(kind, table, ms, fl):
        print(json.dumps({"kind": kind, "table": table, "M": M, "ms": round(ms, 3),
                          "PFps": round(fl / ms / 1e12, 3)}), flush=True)

    for table in a.tables.split(","):
        if table == "tuned" and not enable_tuned_gemms(a.model, 1):
            print(json.dumps({"error": "tuned table not loaded"}))
            break
        for n in shapes:
            w, x = ws[n][0], xs[n]
            report(n, table, timed(lambda: F.linear(x, w), a.reps), flops[n])

        def layer_seq():
            for i in range(a.layers):
                for n in shapes:
                    F.linear(xs[n], ws[n][i])
        ms = timed(layer_seq, reps=max(3, a.reps // 20)) / a.layers
        report("layer", table, ms, sum(flops.values()))


if __name__ == "__main__":
    main()
