"""Offline K9m selection table for one model (ops/gemm.py ``load_dg_table``): the engine's
own start-up tuner (``tune_skinny`` -> ``_tune_dgemm``, every candidate timed with its
consumer over every layer's copy of the weight) run with many more interleaved refinement
rounds, on random weights of the model's decode-GEMM shapes, at the decode-graph buckets
K9m serves (M = 65 .. max).  Writes profiles/tunableop/k9m_<model>_tp1_gfx950.json.

    python tools/tune_dgemm_table.py --model llama-3-8b [--max-bs 256] [--rounds 15]
"""
import argparse
import json
import logging
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--max-bs", type=int, default=256)
    ap.add_argument("--refine", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--ms", default="", help="comma list (default: the K9m graph buckets)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    os.environ["KGC_DGEMM_REFINE"] = str(a.refine)
    os.environ["KGC_DGEMM_REFINE_ROUNDS"] = str(a.rounds)
    os.environ["KGC_DGEMM_TABLE"] = "0"
    logging.basicConfig(level=logging.INFO, stream=sys.stderr, format="%(message)s")
    import torch
    from kubernetes_gpu_cluster_amd.engine.model_runner import graph_buckets
    from kubernetes_gpu_cluster_amd.models import load_model
    from kubernetes_gpu_cluster_amd.ops import gemm
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    mcfg, model = load_model(a.model, torch.bfloat16, dev, True, seed=0)
    silu = list(model.silu_weights())
    skip = {id(x) for x in silu}
    plain = [p for n, p in model.named_parameters() if p.dim() == 2 and id(p) not in skip
             and (mcfg.tie_embeddings or "embed" not in n)]
    gemm.pack_decode_weights(plain, silu)
    ms = ([int(m) for m in a.ms.split(",")] if a.ms else
          [m for m in graph_buckets(a.max_bs) if gemm.SKINNY_MAX_M < m <= gemm.DG_MAX_M])
    t0 = time.time()
    res = gemm.tune_skinny(plain + silu, ms,
                           silu_shapes=model.silu_shapes(), tail_shapes=model.tail_shapes(),
                           qkv_dims=model.qkv_dims())
    path = a.out or gemm.dg_table_path(mcfg.name, 1)
    n = gemm.save_dg_table(path, res, {
        "model": mcfg.name, "tp": 1, "arch": "gfx950", "ms": ms, "refine": a.refine,
        "rounds": a.rounds, "device": torch.cuda.get_device_name(0),
        "seconds": round(time.time() - t0, 1),
        "note": "tools/tune_dgemm_table.py: the start-up tuner with more refinement rounds"})
    print(json.dumps({"table": path, "entries": n, "seconds": round(time.time() - t0, 1)}))


if __name__ == "__main__":
    main()
