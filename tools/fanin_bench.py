"""K9m fan-in epilogue (EPI_FANIN, the norm-free mid-M layer's o / down) against the
regular tail it replaces, on Llama-3-8B shapes: the engine tuner's own measurement
(ops/gemm.py _tune_dgemm kind "tail" + _tune_fanin), with every candidate logged.

    python tools/fanin_bench.py --ms 256 --layers 32 > fanin.jsonl
"""
import argparse
import json
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubernetes_gpu_cluster_amd.ops import gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="256")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--shapes", default="4096x4096,4096x14336")
    a = ap.parse_args()
    logging.basicConfig(level=logging.DEBUG, stream=sys.stderr, format="%(message)s")
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for sh in a.shapes.split(","):
        N, K = (int(v) for v in sh.split("x"))
        ws = [torch.randn(N, K, dtype=torch.bfloat16, device=dev) * K ** -0.5
              for _ in range(a.layers)]
        gemm.pack_decode_weights(ws, [])
        res = {}
        ms = [int(m) for m in a.ms.split(",")]
        gemm._tune_dgemm(ws, N, K, ms, 0.97, 3, res, "tail", fanin=True)
        for M in ms:
            t = res.get((M, N, K, "tail"))
            f = gemm._plan_fanin.get((M, N, K))
            print(json.dumps({"M": M, "N": N, "K": K, "tail_plan": t and list(t[0] or []),
                              "tail_k9m_us": t and round(t[2], 2),
                              "tail_lib_us": t and round(t[1], 2),
                              "fanin": f and {"cfg": f[0], "S": f[1], "us": round(f[2], 2),
                                              "tail_graphed_us": round(f[3], 2)}}), flush=True)
        gemm._packed.clear()
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
