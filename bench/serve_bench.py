"""Service-level benchmark: output tokens/s and TTFT/TPOT through the OpenAI HTTP API
and the router -- the path a client of the K8s ``vllm-router-service`` takes
(BASELINE.json: "Llama-3-8B K8s service").  vLLM ``benchmark_serving`` shape:
``--num-prompts`` synthetic random-token prompts of ``--input-len`` tokens, streamed
``/v1/completions`` with ``ignore_eos`` and ``max_tokens = --output-len``, all sent at
once (``--request-rate inf``) or as a Poisson process.

Against a running service:
    python bench/serve_bench.py --base-url http://vllm-router-service:80
Self-contained on one node (one engine per GPU + one router over all of them, like
the dpN deployment):
    python bench/serve_bench.py --launch --gpus 1 --model llama-3-8b
(``bench.py`` is the driver's headline harness: one router over every replica, timed
bursts between barriers, engine-side figures alongside.  This script adds the Poisson
arrival shape, ``--request-rate R``, whose p99 TPOT / ITL show decode starvation.)
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubernetes_gpu_cluster_amd.benchmarks import serving_client as sc  # noqa: E402


async def run_client(a, prompts_seed: int) -> dict:
    prompts = sc.random_prompts(a.num_prompts, a.input_len, a.vocab, prompts_seed)
    async with sc.new_session() as s:
        res, t0, t1 = await sc.run_wave(s, a.base_url, a.model, prompts, a.output_len,
                                        a.request_rate, seed=a.seed)
    out = {"metric": "service output tokens/sec + p50 TTFT", "unit": "output_tokens/s"}
    out.update(sc.summarize(res, t1 - t0))
    out["config"] = {"model": a.model, "num_prompts": a.num_prompts, "input_len": a.input_len,
                     "output_len": a.output_len, "request_rate": a.request_rate}
    return out


def launch(a) -> list:
    procs, backends = [], []
    for g in range(a.gpus):
        port = a.engine_port + g
        procs.append(sc.start_api_server(
            a.model, port, str(g), ["--load-format", "dummy", "--max-num-seqs", str(a.max_num_seqs),
                                    "--max-model-len", str(a.max_model_len)] + a.engine_args))
        backends.append(f"http://127.0.0.1:{port}")
    if a.no_router:
        asyncio.run(sc.wait_healthy(backends, a.startup_timeout, procs))
        a.base_url = backends[0]
        return procs
    procs.append(sc.start_router(a.router_port, backends))
    asyncio.run(sc.wait_healthy(backends + [f"http://127.0.0.1:{a.router_port}"],
                                a.startup_timeout, procs))
    a.base_url = f"http://127.0.0.1:{a.router_port}"
    return procs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base-url", default="http://127.0.0.1:8080")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--num-prompts", type=int, default=256)
    ap.add_argument("--input-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--request-rate", type=float, default=float("inf"))
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--warmup-prompts", type=int, default=8)
    ap.add_argument("--launch", action="store_true", help="start engines + router locally")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--engine-port", type=int, default=8100)
    ap.add_argument("--router-port", type=int, default=8080)
    ap.add_argument("--no-router", action="store_true", help="--launch: hit engine 0 directly")
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--startup-timeout", type=float, default=900)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("engine_args", nargs=argparse.REMAINDER, help="extra engine flags after --")
    a = ap.parse_args()
    a.engine_args = [x for x in a.engine_args if x != "--"]
    procs = launch(a) if a.launch else []
    try:
        if a.warmup_prompts:
            w = argparse.Namespace(**vars(a))
            w.num_prompts, w.output_len = a.warmup_prompts, 16
            asyncio.run(run_client(w, a.seed + 1))
        out = asyncio.run(run_client(a, a.seed))
        out["n_engines"] = a.gpus if a.launch else None
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    finally:
        sc.stop(procs, grace=30)


if __name__ == "__main__":
    main()
