"""K9r full-K ring decode GEMM (tools/research/gemm_ring.hip) vs hipBLASLt and K9m.

    python tools/ring_bench.py [--model llama-3-8b] [--ms 256] [--copies 16]
                               [--shapes qkv,o,gate_up,down] [--cfgs 0,1,...] [--g 0|16|32]

Every projection of the model at batch M: hipBLASLt (torch.mm) and each K9r tile config
(bm, bn, S, epilogue), timed inside a hipGraph over ``--copies`` distinct weight copies
so the weights stream from HBM as in a decode step.  Weights are packed per config with
G = BN (``--g`` overrides the row-group size).  Each configuration is first checked
against an fp32 reference; one JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def shapes(model):
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    c = PRESETS[model]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    return {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * d, H), "o": (H, c.num_heads * d),
            "gate_up": (2 * I, H), "down": (H, I)}


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(5):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--ms", default="256")
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--cfgs", default=None)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--g", type=int, default=0, help="row-group size of the packing (0 = BN)")
    ap.add_argument("--no-lib", action="store_true")
    ap.add_argument("--xpad", type=int, default=0,
                    help="activation row stride K + xpad elements (L2 channel spread probe)")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    ops.load_extension(strict=True)
    # K9r lives in the research library (tools/research/build.py), not the engine's
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "research"))
    import build as research_build
    k = research_build.load()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ncfg = k.ring_num_cfgs()
    want = None if not a.cfgs else {int(c) for c in a.cfgs.split(",")}
    for name, (N, K) in shapes(a.model).items():
        if name not in a.shapes.split(","):
            continue
        copies = a.copies if N * K * 2 * a.copies < 6e9 else max(2, int(3e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        wb = N * K * 2
        for M in [int(x) for x in a.ms.split(",")]:
            x = torch.randn(M, K + a.xpad, device=dev, dtype=torch.bfloat16)[:, :K]
            ref = x.float() @ ws[0].float().t()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            if not a.no_lib:
                def lib():
                    for w in ws:
                        torch.mm(x, w.t(), out=out)
                t = bench(lib, max(1, 64 // copies)) / copies
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kernel": "hipblaslt",
                                  "us": round(t * 1e6, 2), "w_TBps": round(wb / t / 1e12, 2),
                                  "TFLOPs": round(2 * M * N * K / t / 1e12, 1)}), flush=True)
            for cid in range(ncfg):
                if want is not None and cid not in want:
                    continue
                bm, bn, thr, ns = k.ring_cfg_info(cid)
                if N % bn or bm > 2 * M:
                    continue
                G = a.g or bn
                if bn % G:
                    continue
                epis = [1, 2] if name == "gate_up" else [1]
                for silu in sorted(set(e == 2 for e in epis)):
                    ps = []
                    for w in ws:
                        p = torch.empty(N // G, K // 64, G * 64, device=dev, dtype=w.dtype)
                        k.ring_pack(p, w, silu)
                        ps.append(p)
                    runs = []
                    if silu:
                        runs.append((1, 2))
                    else:
                        runs += [(S, 1 if S == 1 else 0) for S in
                                 (int(s) for s in a.splits.split(",")) if S <= K // 64]
                    for S, epi in runs:
                        if epi == 0:
                            C = torch.empty(S, M, N, device=dev, dtype=torch.float32)
                        elif epi == 1:
                            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                        else:
                            C = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                        k.ring_gemm(C, x, ps[0], cid, epi)
                        if epi == 0:
                            got, wnt = C.sum(0), ref
                        elif epi == 1:
                            got, wnt = C.float(), ref
                        else:
                            I = N // 2
                            wnt = F.silu(ref[:, :I]) * ref[:, I:]
                            got = C.float()
                        err = ((got - wnt).abs().max() / wnt.abs().max().clamp_min(1e-6)).item()

                        def run(C=C, cid=cid, epi=epi, ps=ps):
                            for p in ps:
                                k.ring_gemm(C, x, p, cid, epi)
                        t = bench(run, max(1, 64 // copies)) / copies
                        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kernel": "k9r",
                                          "xpad": a.xpad,
                                          "cfg": cid, "bm": bm, "bn": bn, "threads": thr,
                                          "slots": ns, "G": G, "S": S, "epi": epi,
                                          "us": round(t * 1e6, 2),
                                          "w_TBps": round(wb / t / 1e12, 2),
                                          "TFLOPs": round(2 * M * N * K / t / 1e12, 1),
                                          "rel_err": float(f"{err:.2e}"), "ok": err < 2e-2}),
                              flush=True)
                    del ps
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
