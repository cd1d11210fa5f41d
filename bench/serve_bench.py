"""Service-level benchmark: output tokens/s and TTFT/TPOT through the OpenAI HTTP API
and the router -- the path a client of the K8s ``vllm-router-service`` takes
(BASELINE.json: "Llama-3-8B K8s service").  vLLM ``benchmark_serving`` shape:
``--num-prompts`` synthetic random-token prompts of ``--input-len`` tokens, streamed
``/v1/completions`` with ``ignore_eos`` and ``max_tokens = --output-len``, all sent at
once (``--request-rate inf``) or as a Poisson process.

Against a running service:
    python bench/serve_bench.py --base-url http://vllm-router-service:80
Self-contained on one node (one engine per GPU + the router, like the dpN deployment):
    python bench/serve_bench.py --launch --gpus 1 --model llama-3-8b
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import signal
import statistics
import subprocess
import sys
import time

import aiohttp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else float("nan")


async def one_request(session, url, model, prompt, out_len, res):
    body = {"model": model, "prompt": prompt, "max_tokens": out_len, "ignore_eos": True,
            "stream": True, "temperature": 1.0}
    t0 = time.perf_counter()
    ttft, last, chunks, itl = None, t0, 0, []
    async with session.post(url + "/v1/completions", json=body) as r:
        if r.status != 200:
            res.append({"ok": False, "status": r.status})
            return
        async for raw in r.content:
            line = raw.decode().strip()
            if not line.startswith("data:") or line == "data: [DONE]":
                continue
            now = time.perf_counter()
            if ttft is None:
                ttft = now - t0
            else:
                itl.append(now - last)
            last = now
            chunks += 1
    res.append({"ok": True, "ttft": ttft, "e2e": last - t0, "tokens": out_len, "itl": itl})


async def run_client(a) -> dict:
    rng = random.Random(a.seed)
    prompts = [[rng.randrange(100, a.vocab) for _ in range(a.input_len)]
               for _ in range(a.num_prompts)]
    res: list = []
    conn = aiohttp.TCPConnector(limit=0)
    timeout = aiohttp.ClientTimeout(total=None, sock_read=600)
    async with aiohttp.ClientSession(connector=conn, timeout=timeout) as s:
        tasks = []
        t0 = time.perf_counter()
        for p in prompts:
            tasks.append(asyncio.create_task(one_request(s, a.base_url, a.model, p, a.output_len, res)))
            if a.request_rate != float("inf"):
                await asyncio.sleep(rng.expovariate(a.request_rate))
        await asyncio.gather(*tasks)
        dur = time.perf_counter() - t0
    ok = [r for r in res if r["ok"]]
    toks = sum(r["tokens"] for r in ok)
    tpot = [(r["e2e"] - r["ttft"]) / max(1, r["tokens"] - 1) for r in ok]
    return {"metric": "service output tokens/sec + p50 TTFT", "value": round(toks / dur, 2),
            "unit": "output_tokens/s", "completed": len(ok), "failed": len(res) - len(ok),
            "duration_s": round(dur, 3), "p50_ttft_ms": round(1e3 * pct([r["ttft"] for r in ok], 0.5), 2),
            "p99_ttft_ms": round(1e3 * pct([r["ttft"] for r in ok], 0.99), 2),
            "p50_tpot_ms": round(1e3 * pct(tpot, 0.5), 3),
            "p50_itl_ms": round(1e3 * statistics.median([x for r in ok for x in r["itl"]] or [0]), 3),
            "config": {"model": a.model, "num_prompts": a.num_prompts, "input_len": a.input_len,
                       "output_len": a.output_len, "request_rate": a.request_rate}}


async def wait_healthy(urls, timeout_s):
    deadline = time.time() + timeout_s
    async with aiohttp.ClientSession() as s:
        for u in urls:
            while True:
                try:
                    async with s.get(u + "/health") as r:
                        if r.status == 200:
                            break
                except aiohttp.ClientError:
                    pass
                if time.time() > deadline:
                    raise TimeoutError(f"{u} not healthy after {timeout_s}s")
                await asyncio.sleep(2)


def launch(a) -> list[subprocess.Popen]:
    procs, backends = [], []
    env0 = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    for g in range(a.gpus):
        port = a.engine_port + g
        env = dict(env0, HIP_VISIBLE_DEVICES=str(g))
        cmd = [sys.executable, "-m", "kubernetes_gpu_cluster_amd.entrypoints.api_server", a.model,
               "--port", str(port), "--host", "127.0.0.1", "--load-format", "dummy",
               "--max-num-seqs", str(a.max_num_seqs), "--max-model-len", str(a.max_model_len),
               "--uvicorn-log-level", "warning"] + a.engine_args
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
        backends.append(f"http://127.0.0.1:{port}")
    if a.no_router:
        asyncio.run(wait_healthy(backends, a.startup_timeout))
        a.base_url = backends[0]
        return procs
    cmd = [sys.executable, "-m", "kubernetes_gpu_cluster_amd.router.router", "--host", "127.0.0.1",
           "--port", str(a.router_port), "--backends", ",".join(backends)]
    procs.append(subprocess.Popen(cmd, env=env0, start_new_session=True))
    asyncio.run(wait_healthy(backends + [f"http://127.0.0.1:{a.router_port}"], a.startup_timeout))
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
            asyncio.run(run_client(w))
        out = asyncio.run(run_client(a))
        out["n_engines"] = a.gpus if a.launch else None
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    finally:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)


if __name__ == "__main__":
    main()
