"""TunableOp selection of the chunked-prefill GEMMs (M = --tokens) timed at the
power-managed clock they actually run at.

Back-to-back prefill GEMMs settle at the chip's 1400 W limit (~1.75 GHz,
profiles/prefill_gemm_clock_power_r4.txt), so a short tuning burst at full clock ranks
solutions by speed, not by work per joule, and its picks ran no faster sustained
(profiles/README.md "Prefill GEMMs are power-bound").  Here the chip is first held at
its sustained state by a few seconds of the layer's GEMMs, and every candidate is then
timed over --tune-ms of back-to-back calls, so the ranking is the sustained one.

    PYTORCH_TUNABLEOP_VERBOSE=1 python tools/tune_prefill_sustained.py --out X.csv
    KGC_GEMM_TABLE=X.csv python tools/prefill_gemm_probe.py --tables default,tuned --reps 200
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--out", required=True)
    ap.add_argument("--tune-ms", type=int, default=300)
    ap.add_argument("--heat-s", type=float, default=4.0)
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    c = PRESETS[a.model]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    shapes = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H), "o": (H, c.num_heads * d),
              "gate_up": (2 * I, H), "down": (H, I)}
    dev = torch.device("cuda")
    M = a.tokens
    ws = {n: torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
          for n, (N, K) in shapes.items()}
    xs = {n: torch.randn(M, K, device=dev, dtype=torch.bfloat16) for n, (N, K) in shapes.items()}

    def layer():
        for n in shapes:
            F.linear(xs[n], ws[n])

    # hold the chip at its sustained (power-limited) state before and between shapes
    def heat(sec):
        t0 = time.time()
        while time.time() - t0 < sec:
            for _ in range(20):
                layer()
            torch.cuda.synchronize()

    heat(a.heat_s)
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(a.out, insert_device_ordinal=False)
    torch.cuda.tunable.set_max_tuning_duration(a.tune_ms)
    torch.cuda.tunable.set_max_tuning_iterations(1000)
    for n in a.shapes.split(","):
        t0 = time.time()
        F.linear(xs[n], ws[n])
        torch.cuda.synchronize()
        print(f"tuned {n} M={M} in {time.time() - t0:.0f} s", flush=True)
        torch.cuda.tunable.tuning_enable(False)
        heat(1.0)
        torch.cuda.tunable.tuning_enable(True)
    print(a.out, flush=True)      # TunableOp writes the results file at process exit


if __name__ == "__main__":
    main()
