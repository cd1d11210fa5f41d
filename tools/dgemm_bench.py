"""K9m mid-batch decode GEMM (csrc/kernels/gemm_decode.hip) vs hipBLASLt.

    python tools/dgemm_bench.py [--model llama-3-8b] [--ms 128,256] [--copies 16]
                                [--shapes qkv,o,gate_up,down,lm_head] [--table CSV]

For every projection of the model and batch M: hipBLASLt (F.linear, optionally with a
TunableOp table) and every K9m configuration (bm, bn, S, epilogue), each timed inside a
hipGraph over ``--copies`` distinct weight copies so the weights stream from HBM as in a
decode step.  The numbers include what each path needs to hand its consumer the same
thing: for split-K (S > 1) the fp32 slices only (the consumers sum them), so the reduce
kernels are listed separately.  Every configuration is first checked against an fp32
reference.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def shapes(model, tp=1):
    """(N, K) of each projection of one TP rank's shard (tp = 1: the whole model)."""
    from kubernetes_gpu_cluster_amd.models.configs import PRESETS
    c = PRESETS[model]
    H, I, d = c.hidden_size, c.intermediate_size, c.head_dim
    nq, nkv = c.num_heads // tp, max(1, c.num_kv_heads // tp)
    return {"qkv": ((nq + 2 * nkv) * d, H), "o": (H, nq * d),
            "gate_up": (2 * I // tp, H), "down": (H, I // tp), "lm_head": (c.vocab_size // tp, H)}


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
    for _ in range(3):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1, help="time one TP rank's shard shapes")
    ap.add_argument("--ms", default="256")
    ap.add_argument("--copies", type=int, default=16)
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--table", default=None)
    ap.add_argument("--splits", default="1,2,3,4,6,8")
    ap.add_argument("--only", default=None,
                    help="cfg:S:epi -- time just this configuration (profiling runs)")
    ap.add_argument("--no-lib", action="store_true", help="skip the hipBLASLt baseline")
    ap.add_argument("--cfgs", default=None, help="comma list: only these tile configs")
    ap.add_argument("--reduce", action="store_true",
                    help="time split-K candidates with their splitk_reduce to bf16")
    ap.add_argument("--max-grid", type=int, default=264,
                    help="skip split-K candidates with more workgroups than this")
    ap.add_argument("--ablate", default=None,
                    help="S value: time the packed 256 x 128 tile with modes full / no-MFMA / "
                         "no-DMA / no-A-DMA / no-B-DMA at this split")
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd import ops
    ops.load_extension(strict=True)
    k = torch.ops.kgc
    if a.table:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(False)
        torch.cuda.tunable.set_filename(a.table, insert_device_ordinal=False)
        torch.cuda.tunable.read_file(a.table)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for name, (N, K) in shapes(a.model, a.tp).items():
        if name not in a.shapes.split(","):
            continue
        copies = a.copies if N * K * 2 * a.copies < 8e9 else max(2, int(4e9 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        # packed copies (dgemm_pack) for the packed tile configs; gate_up packed both ways
        def packed(silu):
            out = []
            for w in ws:
                p = torch.empty(N // 128, K // 64, 8192, device=dev, dtype=w.dtype)
                k.dgemm_pack(p, w, silu)
                out.append(p)
            return out
        want_cfgs = None if not a.cfgs else {int(c) for c in a.cfgs.split(",")}
        wps = {False: packed(False)}
        if name == "gate_up":
            wps[True] = packed(True)
        for M in [int(x) for x in a.ms.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ref = (x.float() @ ws[0].float().t())
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

            def lib():
                for w in ws:
                    torch.mm(x, w.t(), out=out)
            wb = N * K * 2
            if not a.no_lib:
                t = bench(lib, max(1, 64 // copies)) / copies
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kernel": "hipblaslt",
                                  "us": round(t * 1e6, 2), "w_TBps": round(wb / t / 1e12, 2),
                                  "TFLOPs": round(2 * M * N * K / t / 1e12, 1)}), flush=True)
            if a.ablate:
                S = int(a.ablate)
                C = torch.empty(S, M, N, device=dev, dtype=torch.float32)
                for mode, mname in enumerate(["full", "no_mfma", "no_dma", "no_a", "no_b"]):
                    def run(mode=mode):
                        for w in wps[False]:
                            k.dgemm_ablate(C, x, w, mode)
                    t = bench(run, max(1, 64 // copies)) / copies
                    print(json.dumps({"shape": name, "M": M, "S": S, "ablate": mname,
                                      "us": round(t * 1e6, 2)}), flush=True)
                continue
            cfgs = []
            for cid in range(k.dgemm_num_cfgs()):
                bm, bn, pk = k.dgemm_cfg_info(cid)
                if (bm == 256 and M <= 128) or N % bn or (want_cfgs is not None and cid not in want_cfgs):
                    continue
                tiles = ((M + bm - 1) // bm) * (N // bn)
                for S in [int(s) for s in a.splits.split(",")]:
                    if K // 64 < S or (S > 1 and tiles * S > a.max_grid):
                        continue
                    cfgs.append((cid, S, 0 if S > 1 else 1))
                if name == "gate_up" and (k.dgemm_cfg_epis(cid) >> 2) & 1:
                    cfgs.append((cid, 1, 2))
            if a.only:
                cfgs = [tuple(int(v) for v in a.only.split(":"))]
            for cid, S, epi in cfgs:
                bm, bn, pk = k.dgemm_cfg_info(cid)
                wl = wps[epi == 2] if pk else ws
                if epi == 0:
                    C = torch.empty(S, M, N, device=dev, dtype=torch.float32)
                elif epi == 1:
                    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                else:
                    C = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                k.dgemm(C, x, wl[0], cid, epi)
                if epi == 0:
                    got = C.sum(0)
                    want = ref
                elif epi == 1:
                    got, want = C.float(), ref
                else:
                    I = N // 2
                    want = F.silu(ref[:, :I]) * ref[:, I:]
                    got = C.float()
                err = ((got - want).abs().max() / want.abs().max().clamp_min(1e-6)).item()
                ok = err < 2e-2

                red = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

                def run(C=C, cid=cid, epi=epi, wl=wl, red=red):
                    for w in wl:
                        k.dgemm(C, x, w, cid, epi)
                        if epi == 0 and a.reduce:
                            k.splitk_reduce(red, C)
                t = bench(run, max(1, 64 // copies)) / copies
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kernel": "k9m",
                                  "cfg": cid, "bm": bm, "bn": bn, "packed": pk, "S": S, "epi": epi,
                                  "with_reduce": bool(a.reduce and epi == 0),
                                  "us": round(t * 1e6, 2), "w_TBps": round(wb / t / 1e12, 2),
                                  "TFLOPs": round(2 * M * N * K / t / 1e12, 1),
                                  "rel_err": float(f"{err:.2e}"), "ok": ok}), flush=True)
        del ws, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
