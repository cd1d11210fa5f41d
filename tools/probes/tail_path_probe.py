"""Probe: which branch ``gemm.linear_add_rms`` (o / down projection + residual add + RMSNorm)
takes in the batch-256 decode forward of the Llama-3-8B engine, and why.  Builds the
engine as ``bench.py --mode engine`` does (random init, start-up tuning, graphs), then
runs ONE eager decode forward at B = 256 with linear_add_rms wrapped to log its operands
and plan lookups.

    python tools/probes/tail_path_probe.py [--model llama-3-8b] [--m 256]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--m", type=int, default=256)
    a = ap.parse_args()
    from kubernetes_gpu_cluster_amd.engine.config import EngineConfig
    from kubernetes_gpu_cluster_amd.engine.llm_engine import LLMEngine
    from kubernetes_gpu_cluster_amd.ops import gemm
    torch.cuda.set_device(0)
    cfg = EngineConfig(model=a.model, random_init=True, seed=0, max_num_seqs=256,
                       max_num_batched_tokens=16384, allow_phantom=True)
    eng = LLMEngine(cfg)
    runner = eng.executor.runner
    model = runner.model
    calls = []
    orig = gemm.linear_add_rms

    def traced(x, w, residual, gamma, eps):
        p = gemm._dg_plan(x, w, "tail")
        calls.append({"x": list(x.shape), "x_stride": list(x.stride()), "x_cuda": x.is_cuda,
                      "w": list(w.shape), "res_contig": residual.is_contiguous(),
                      "res_stride": list(residual.stride()), "tail_plan": p,
                      "accnorm": gemm._plan_accnorm.get((x.shape[0], w.shape[0], w.shape[1]))})
        return orig(x, w, residual, gamma, eps)
    gemm.linear_add_rms = traced
    B = a.m
    meta = runner._meta(B, 0, 0, B, 0, runner.max_model_len, z=1)
    print(json.dumps({"tail_fusable": bool(model._tail_fusable(torch.empty(B, 1, device="cuda"))),
                      "plan_dg_tail_keys": sorted(str(k) for k in gemm.dgemm_plan() if k[3] == "tail"
                                                  and k[0] == B)}), flush=True)
    with torch.inference_mode():
        runner._forward(B, meta, None)
    torch.cuda.synchronize()
    for c in calls[:4]:
        print(json.dumps(c, default=str), flush=True)
    print(json.dumps({"calls": len(calls)}), flush=True)
    eng.shutdown() if hasattr(eng, "shutdown") else None


if __name__ == "__main__":
    main()
