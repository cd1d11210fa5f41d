"""Streaming OpenAI-completions load generator (the vLLM ``benchmark_serving`` shape).

A *wave* is ``len(prompts)`` streamed ``/v1/completions`` requests with
``ignore_eos`` and ``max_tokens = output_len``, sent at once (request rate inf) or as a
Poisson process.  TTFT is send -> first SSE data event of a request; TPOT is
(last event - first event) / (tokens - 1).  Prompts are token-id lists, so no
tokenizer is involved on either side.

Also the service launcher used by ``bench.py`` and ``bench/serve_bench.py``: API
server and router as fresh child processes (own sessions, so one ``killpg`` ends an
API server together with its engine core and ranks).  The launching process never
touches the GPU.
"""
from __future__ import annotations

import asyncio
import json
import os
import random
import signal
import statistics
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Optional

import aiohttp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else float("nan")


def random_prompts(n: int, input_len: int, vocab: int, seed: int) -> list[list[int]]:
    rng = random.Random(seed)
    return [[rng.randrange(100, vocab - 100) for _ in range(input_len)] for _ in range(n)]


@dataclass
class Result:
    ok: bool
    status: int = 200
    ttft: Optional[float] = None
    e2e: float = 0.0
    tokens: int = 0
    itl: list = field(default_factory=list)


async def one_request(session: aiohttp.ClientSession, url: str, model: str, prompt,
                      out_len: int, temperature: float = 1.0) -> Result:
    """One streamed completion.  Tokens are counted from what arrived: the
    ``stream_options.include_usage`` event (completion_tokens) that the server sends
    before ``[DONE]``.  A stream cut short (no usage event or no [DONE]) is a failed
    request that credits no tokens -- never ``max_tokens`` on faith."""
    body = {"model": model, "prompt": prompt, "max_tokens": out_len, "ignore_eos": True,
            "stream": True, "temperature": temperature,
            "stream_options": {"include_usage": True}}
    t0 = time.monotonic()
    ttft, last, itl = None, t0, []
    ntok, done = None, False
    async with session.post(url + "/v1/completions", json=body) as r:
        if r.status != 200:
            await r.read()
            return Result(False, r.status)
        async for raw in r.content:
            if not raw.startswith(b"data:"):
                continue
            if raw.startswith(b"data: [DONE]"):
                done = True
                continue
            if b'"usage"' in raw and b'"choices": []' in raw:
                try:
                    ntok = int(json.loads(raw[5:])["usage"]["completion_tokens"])
                except (ValueError, KeyError, TypeError):
                    pass
                continue
            now = time.monotonic()
            if ttft is None:
                ttft = now - t0
            else:
                itl.append(now - last)
            last = now
    ok = ttft is not None and done and ntok is not None
    return Result(ok, 200, ttft, last - t0, ntok if ok else 0, itl)


async def run_wave(session, url: str, model: str, prompts, out_len: int,
                   request_rate: float = float("inf"), seed: int = 0,
                   temperature: float = 1.0) -> tuple[list[Result], float, float]:
    """-> (results, wave start, wave end) with host ``time.monotonic()`` stamps."""
    rng = random.Random(seed)
    t0 = time.monotonic()
    tasks = []
    for p in prompts:
        tasks.append(asyncio.create_task(one_request(session, url, model, p, out_len, temperature)))
        if request_rate != float("inf"):
            await asyncio.sleep(rng.expovariate(request_rate))
    res = await asyncio.gather(*tasks)
    return list(res), t0, time.monotonic()


def new_session() -> aiohttp.ClientSession:
    return aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0),
                                 timeout=aiohttp.ClientTimeout(total=None, sock_read=900))


def summarize(res: list[Result], duration: float) -> dict:
    ok = [r for r in res if r.ok]
    toks = sum(r.tokens for r in ok)
    tpot = [(r.e2e - r.ttft) / max(1, r.tokens - 1) for r in ok]
    return {"value": round(toks / duration, 2) if duration > 0 else 0.0,
            "completed": len(ok), "failed": len(res) - len(ok), "duration_s": round(duration, 3),
            "p50_ttft_ms": round(1e3 * pct([r.ttft for r in ok], 0.5), 2),
            "p99_ttft_ms": round(1e3 * pct([r.ttft for r in ok], 0.99), 2),
            "p50_tpot_ms": round(1e3 * pct(tpot, 0.5), 3),
            "p99_tpot_ms": round(1e3 * pct(tpot, 0.99), 3),
            "p50_itl_ms": round(1e3 * statistics.median([x for r in ok for x in r.itl] or [0]), 3),
            "p99_itl_ms": round(1e3 * pct([x for r in ok for x in r.itl], 0.99), 3),
            "max_itl_ms": round(1e3 * max([x for r in ok for x in r.itl] or [0]), 3)}


def engine_figures(reqs: list, windows: list[tuple[float, float]]) -> dict:
    """Engine-side figures of the requests that arrived inside the timed ``windows``
    (``/kgc/engine_stats`` records: arrival at the engine, first token, finish, tokens).
    Per wave the engine span is first arrival -> last finish."""
    toks, span, ttft, tpot = 0, 0.0, [], []
    for lo, hi in windows:
        w = [r for r in reqs if lo <= r[0] <= hi and r[1] is not None and r[2] is not None]
        if not w:
            continue
        toks += sum(r[3] for r in w)
        span += max(r[2] for r in w) - min(r[0] for r in w)
        ttft += [r[1] - r[0] for r in w]
        tpot += [(r[2] - r[1]) / max(1, r[3] - 1) for r in w]
    return {"engine_tokens": toks, "engine_span_s": span,
            "engine_ttft": ttft, "engine_tpot": tpot}


# ---------------------------------------------------------------------------- launcher
# the launcher may itself be a torch.distributed.run rank (bench.py --gpus N): its
# rendezvous variables must not leak into a server that builds its own TP world
_LAUNCHER_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                  "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME",
                  "MASTER_ADDR", "MASTER_PORT")


def _env(extra: dict) -> dict:
    env = {k: v for k, v in os.environ.items()
           if k not in _LAUNCHER_VARS and not k.startswith("TORCHELASTIC_")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.update(extra)
    return env


def start_api_server(model: str, port: int, devices: Optional[str], engine_args: list[str],
                     log=None) -> subprocess.Popen:
    """``devices``: HIP_VISIBLE_DEVICES of the server (None: inherit)."""
    cmd = [sys.executable, "-m", "kubernetes_gpu_cluster_amd.entrypoints.api_server", model,
           "--port", str(port), "--host", "127.0.0.1", "--uvicorn-log-level", "warning"] + engine_args
    extra = {} if devices is None else {"HIP_VISIBLE_DEVICES": devices}
    return subprocess.Popen(cmd, env=_env(extra), start_new_session=True, stdout=log,
                            stderr=subprocess.STDOUT if log is not None else None)


def start_router(port: int, backends: list[str], log=None, workers: int = 1) -> subprocess.Popen:
    cmd = [sys.executable, "-m", "kubernetes_gpu_cluster_amd.router.router", "--host", "127.0.0.1",
           "--port", str(port), "--backends", ",".join(backends), "--workers", str(workers)]
    return subprocess.Popen(cmd, env=_env({}), start_new_session=True, stdout=log,
                            stderr=subprocess.STDOUT if log is not None else None)


async def wait_healthy(urls: list[str], timeout_s: float, procs=(), progress=None) -> None:
    """Poll ``/health`` until 200; fail early when a launched process exits."""
    deadline = time.monotonic() + timeout_s
    last_note = time.monotonic()
    async with aiohttp.ClientSession() as s:
        for u in urls:
            while True:
                try:
                    async with s.get(u + "/health", timeout=aiohttp.ClientTimeout(total=5)) as r:
                        if r.status == 200:
                            break
                except (aiohttp.ClientError, asyncio.TimeoutError):
                    pass
                for p in procs:
                    if p.poll() is not None:
                        raise RuntimeError(f"{' '.join(p.args[:4])} exited with {p.returncode} "
                                           f"before {u} became healthy")
                if time.monotonic() > deadline:
                    raise TimeoutError(f"{u} not healthy after {timeout_s:.0f}s")
                if progress is not None and time.monotonic() - last_note > 20:
                    progress(f"waiting for {u}/health ({time.monotonic() - deadline + timeout_s:.0f}s)")
                    last_note = time.monotonic()
                await asyncio.sleep(1.0)


def cpu_seconds(pid: int) -> float:
    """user + system CPU time of a process and all its descendants (router workers)."""
    import psutil
    try:
        root = psutil.Process(pid)
        tot = 0.0
        for p in [root] + root.children(recursive=True):
            try:
                t = p.cpu_times()
                tot += t.user + t.system
            except psutil.NoSuchProcess:
                pass
        return tot
    except psutil.NoSuchProcess:
        return 0.0


def stop(procs: list[subprocess.Popen], grace: float = 60.0) -> list[Optional[int]]:
    """SIGTERM every process group (API server -> graceful uvicorn stop -> engine core
    shutdown), SIGKILL what is left after ``grace`` seconds."""
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
    return [p.returncode for p in procs]
