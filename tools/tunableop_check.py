"""Does a TunableOp selection for a prefill-chunk GEMM hold up in sustained use?

    python tools/tunableop_check.py [--shape gate_up] [--tokens 16384] [--reps 100]

Times F.linear at M = --tokens for one Llama-3-8B projection with hipBLASLt's default
pick, then lets TunableOp tune that one shape in-process (written to a scratch CSV), then
times the tuned selection the same way (100+ back-to-back calls: sustained clocks).
Prints one JSON line per phase plus the selection TunableOp recorded.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="gate_up")
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    c = PRESETS["llama-3-8b"]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    N, K = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H), "o": (H, c.num_heads * d),
            "gate_up": (2 * I, H), "down": (H, I)}[a.shape]
    dev = torch.device("cuda")
    M = a.tokens
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K

    def rep(phase, ms):
        print(json.dumps({"shape": a.shape, "M": M, "phase": phase, "ms": round(ms, 3),
                          "PFps": round(fl / ms / 1e12, 3)}), flush=True)

    rep("default", timed(lambda: F.linear(x, w), a.reps))
    path = os.path.join(tempfile.mkdtemp(), "tuned.csv")
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(path, insert_device_ordinal=False)
    torch.cuda.tunable.set_max_tuning_duration(20)
    torch.cuda.tunable.set_max_tuning_iterations(10)
    t0 = time.time()
    F.linear(x, w)                      # tunes this signature
    torch.cuda.synchronize()
    tune_s = time.time() - t0
    torch.cuda.tunable.tuning_enable(False)
    rep("tuned", timed(lambda: F.linear(x, w), a.reps))
    sel = [str(r) for r in torch.cuda.tunable.get_results()]
    print(json.dumps({"shape": a.shape, "tune_s": round(tune_s, 1), "selection": sel}), flush=True)
    torch.cuda.tunable.enable(False)
    rep("default_again", timed(lambda: F.linear(x, w), a.reps))


if __name__ == "__main__":
    main()
