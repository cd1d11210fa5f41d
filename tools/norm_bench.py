"""RMSNorm / fused add+RMSNorm microbenchmark at decode and prefill row counts.

    python tools/norm_bench.py [--h 4096] [--rows 1,64,256,16384]

Times back-to-back calls on distinct activations inside one hipGraph (as in a decode
graph) and checks the output against the fp32 reference."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=4096)
    ap.add_argument("--rows", default="1,64,256,16384")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    from kubernetes_gpu_cluster_amd.ops import reference as ref
    dev = torch.device("cuda")
    for rows in [int(r) for r in a.rows.split(",")]:
        L = 32 if rows <= 4096 else 4
        xs = [torch.randn(rows, a.h, dtype=torch.bfloat16, device=dev) for _ in range(L)]
        rs = [torch.randn(rows, a.h, dtype=torch.bfloat16, device=dev) for _ in range(L)]
        w = torch.randn(a.h, dtype=torch.bfloat16, device=dev)
        x0, r0 = xs[0].clone(), rs[0].clone()
        o, r = ops.fused_add_rms_norm(x0, r0, w, 1e-5)
        eo, er = ref.fused_add_rms_norm(xs[0].cpu(), rs[0].cpu(), w.cpu(), 1e-5)
        err = max((o.cpu().float() - eo.float()).abs().max().item(),
                  (r.cpu().float() - er.float()).abs().max().item())

        def run():
            for x, rr in zip(xs, rs):
                ops.fused_add_rms_norm(x, rr, w, 1e-5)
        run()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run()
        g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t) / 5 / L * 1e6
        print(json.dumps({"op": "fused_add_rms_norm", "rows": rows, "H": a.h, "us": round(us, 2),
                          "TBps": round(4 * rows * a.h * 2 / us / 1e6, 2),
                          "max_err": round(err, 4),
                          "variant": os.environ.get("KGC_NORM_VARIANT", "1")}), flush=True)


if __name__ == "__main__":
    main()
