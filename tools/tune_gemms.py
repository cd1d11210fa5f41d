"""Offline hipBLASLt kernel selection for the decode-graph GEMM shapes (PyTorch
TunableOp), written to a CSV the engine loads read-only at start-up.

hipBLASLt's default heuristic picks poorly for the skinny decode shapes (M = the
graph batch bucket): e.g. Llama-3-8B down_proj at M=128 runs 59 us by default vs
42 us with the best solution.  Every shape a captured decode graph replays is
known in advance (bucket x {qkv, o, gate_up, down, lm_head}), so they are tuned
once per (model, TP degree, ROCm/hipBLASLt build) and shipped in profiles/tunableop/.

    python tools/tune_gemms.py --model llama-3-8b [--tp 1] [--max-bs 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--max-bs", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--prefill-m", type=int, nargs="*", default=[],
                    help="also tune these token counts (full chunked-prefill steps run exactly "
                         "--max-num-batched-tokens tokens)")
    ap.add_argument("--append", action="store_true", help="keep the rows already in --out")
    ap.add_argument("--min-bs", type=int, default=1, help="only tune buckets >= this")
    ap.add_argument("--rotating-mb", type=int, default=0,
                    help="TunableOp rotating input buffers of this many MB: > 256 MB (the "
                         "Infinity Cache) times every candidate on cold weights, as a decode "
                         "graph runs them")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd.utils.gemm_tuning import default_table_path
    out = a.out or default_table_path(a.model, a.tp)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    import torch
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(out, insert_device_ordinal=False)
    if a.append and os.path.exists(out):
        torch.cuda.tunable.read_file(out)
    torch.cuda.tunable.set_max_tuning_duration(60)
    if a.rotating_mb:
        torch.cuda.tunable.set_rotating_buffer_size(a.rotating_mb)
    import torch.nn.functional as F
    from kubernetes_gpu_cluster_amd.engine.model_runner import graph_buckets
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    c = PRESETS[a.model]
    tp = a.tp
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    nkv = max(1, c.num_kv_heads // tp)
    shapes = {"qkv": ((c.num_heads // tp + 2 * nkv) * d, H), "o": (H, c.num_heads * d // tp),
              "gate_up": (2 * I // tp, H), "down": (H, I // tp),
              "lm_head": (-(-c.vocab_size // (64 * tp)) * 64 if tp > 1 else c.vocab_size, H)}
    dev = torch.device("cuda")
    for name, (N, K) in shapes.items():
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        ms = [m for m in graph_buckets(a.max_bs) if m >= a.min_bs]
        for M in ms + [m for m in a.prefill_m if name != "lm_head"]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            F.linear(x, w)
            torch.cuda.synchronize()
            print(f"  {name} M={M}", flush=True)   # progress (a long silent run looks hung)
        print(f"tuned {name} N={N} K={K} for {len(graph_buckets(a.max_bs))} buckets", flush=True)
    print(out)   # TunableOp writes the results file at process exit


if __name__ == "__main__":
    main()
