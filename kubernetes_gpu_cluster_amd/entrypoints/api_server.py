"""OpenAI-compatible HTTP server for the engine (the reference's serving pods run
``vllm serve``).

Routes: ``POST /v1/completions``, ``POST /v1/chat/completions`` (both with SSE
streaming), ``GET /v1/models``, ``GET /health`` (liveness/readiness probes),
``GET /metrics`` (Prometheus), ``GET /version``.

    python -m kubernetes_gpu_cluster_amd.entrypoints.api_server --model llama-3-8b \\
        --random-init --host 0.0.0.0 --port 8000 [--tensor-parallel-size 8 ...]

Every engine flag of ``engine.config.add_engine_args`` is accepted, including
the reference values files' ``extraArgs`` (``--dtype float16``,
``--disable-custom-all-reduce``, ``--enforce-eager``, ``--trust-remote-code``, ...).
"""
from __future__ import annotations

import argparse
import asyncio
import dataclasses
import json
import logging
import os
import socket
import threading
import time
import uuid
from typing import Any, Optional, Union

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from pydantic import BaseModel, ConfigDict, Field
from starlette.background import BackgroundTask

from .. import __version__
from ..engine.config import EngineConfig, add_engine_args, config_from_args
from ..engine.sequence import SamplingParams
from ..utils.tokenizer import get_tokenizer
from .async_engine import AsyncLLMEngine, EngineDeadError

log = logging.getLogger("kgc.api")


class _Lenient(BaseModel):
    model_config = ConfigDict(extra="allow")


class TokenizeRequest(_Lenient):
    model: Optional[str] = None
    prompt: Optional[str] = None
    messages: Optional[list[dict]] = None
    add_generation_prompt: bool = True


class DetokenizeRequest(_Lenient):
    model: Optional[str] = None
    tokens: list[int]


class CompletionRequest(_Lenient):
    model: Optional[str] = None
    prompt: Union[str, list[str], list[int], list[list[int]]]
    max_tokens: Optional[int] = 16
    temperature: Optional[float] = 1.0
    top_p: Optional[float] = 1.0
    top_k: Optional[int] = -1
    n: int = 1
    stream: bool = False
    stream_options: Optional[dict] = None
    stop: Optional[Union[str, list[str]]] = None
    stop_token_ids: Optional[list[int]] = None
    seed: Optional[int] = None
    ignore_eos: bool = False
    min_tokens: int = 0
    echo: bool = False
    logprobs: Optional[int] = None
    presence_penalty: Optional[float] = 0.0
    frequency_penalty: Optional[float] = 0.0
    repetition_penalty: Optional[float] = 1.0
    min_p: Optional[float] = 0.0
    logit_bias: Optional[dict[str, float]] = None
    user: Optional[str] = None


class ChatMessage(_Lenient):
    role: str
    content: Union[str, list[dict[str, Any]], None] = ""


class ChatCompletionRequest(_Lenient):
    model: Optional[str] = None
    messages: list[ChatMessage]
    max_tokens: Optional[int] = None
    max_completion_tokens: Optional[int] = None
    temperature: Optional[float] = 1.0
    top_p: Optional[float] = 1.0
    top_k: Optional[int] = -1
    n: int = 1
    stream: bool = False
    stream_options: Optional[dict] = None
    stop: Optional[Union[str, list[str]]] = None
    stop_token_ids: Optional[list[int]] = None
    seed: Optional[int] = None
    ignore_eos: bool = False
    min_tokens: int = 0
    logprobs: bool = False
    top_logprobs: Optional[int] = None
    presence_penalty: Optional[float] = 0.0
    frequency_penalty: Optional[float] = 0.0
    repetition_penalty: Optional[float] = 1.0
    min_p: Optional[float] = 0.0
    logit_bias: Optional[dict[str, float]] = None
    user: Optional[str] = None


MAX_LOGPROBS = 20


def _err(status: int, msg: str, typ: str = "invalid_request_error") -> JSONResponse:
    return JSONResponse({"object": "error", "message": msg, "type": typ, "code": status},
                        status_code=status)


class _Detok:
    """Incremental detokenizer with stop-string truncation.

    Decodes only a short window per update (tokens since the last emitted text, plus
    a few before for merge context), so a streamed response costs O(n), not O(n^2)
    full re-decodes.  A window ending in U+FFFD (an incomplete multi-byte sequence)
    is held back until the next token completes it.  With stop strings, the last
    ``max(len(stop)) - 1`` characters are withheld from the stream until they can no
    longer start a stop string, so a stop string split over two updates is never
    partially emitted; ``flush()`` releases them at the end."""

    CONTEXT = 5

    def __init__(self, tok, stops: list[str]):
        self.tok, self.stops = tok, [s for s in stops if s]
        self.text = ""          # accepted text (truncated at a stop string)
        self.stopped = False
        self._emitted = 0       # characters of self.text already returned
        self._hold = max((len(s) for s in self.stops), default=1) - 1
        self._prefix = 0        # window start (context tokens already decoded)
        self._read = 0          # tokens whose text is already in self.text

    def update(self, ids: list[int]) -> str:
        if self.stopped or len(ids) <= self._read:
            return ""
        before = self.tok.decode(ids[self._prefix:self._read]) if self._read > self._prefix else ""
        after = self.tok.decode(ids[self._prefix:])
        if after.endswith("\ufffd") or not after.startswith(before):
            return ""
        self._read = len(ids)
        self._prefix = max(0, self._read - self.CONTEXT)
        old = len(self.text)
        self.text += after[len(before):]
        if self.stops:
            start = max(0, old - self._hold)      # a stop may straddle old text and delta
            hits = [i for i in (self.text.find(s, start) for s in self.stops) if i >= 0]
            if hits:
                self.text = self.text[:min(hits)]
                self.stopped = True
                return self.flush()
        end = len(self.text) - self._hold
        if end <= self._emitted:
            return ""
        out = self.text[self._emitted:end]
        self._emitted = end
        return out

    def flush(self) -> str:
        out = self.text[self._emitted:]
        self._emitted = len(self.text)
        return out


def build_app(engine: AsyncLLMEngine, tokenizer, served_name: str, max_model_len: int,
              api_key: Optional[str] = None) -> FastAPI:
    app = FastAPI(title="kgc OpenAI-compatible server", version=__version__)
    created = int(time.time())

    if api_key:
        # vLLM's --api-key: every /v1 route wants "Authorization: Bearer <key>"; /health,
        # /metrics, /version and (de)tokenize stay open for probes and scrapers
        import hmac
        want = f"Bearer {api_key}".encode()

        @app.middleware("http")
        async def check_api_key(request, call_next):
            if request.method != "OPTIONS" and request.url.path.startswith("/v1"):
                got = request.headers.get("authorization", "").encode()
                if not hmac.compare_digest(got, want):
                    return JSONResponse({"error": "Unauthorized"}, status_code=401)
            return await call_next(request)

    def params_from(req, max_tokens: Optional[int], logprobs: Optional[int] = None) -> SamplingParams:
        stops = req.stop if isinstance(req.stop, list) else ([req.stop] if req.stop else [])
        if logprobs is not None and not 0 <= logprobs <= MAX_LOGPROBS:
            raise ValueError(f"logprobs must be in [0, {MAX_LOGPROBS}]")
        return SamplingParams(temperature=req.temperature if req.temperature is not None else 1.0,
                              top_p=req.top_p if req.top_p is not None else 1.0,
                              top_k=req.top_k if req.top_k not in (None, 0) else -1,
                              max_tokens=max_tokens, min_tokens=req.min_tokens,
                              stop_token_ids=list(req.stop_token_ids or []), stop=stops,
                              ignore_eos=req.ignore_eos, seed=req.seed, n=req.n,
                              logprobs=logprobs,
                              presence_penalty=req.presence_penalty or 0.0,
                              frequency_penalty=req.frequency_penalty or 0.0,
                              repetition_penalty=req.repetition_penalty or 1.0,
                              min_p=req.min_p or 0.0,
                              logit_bias={int(k): float(v) for k, v in (req.logit_bias or {}).items()}
                              or None)

    def close_all(gens) -> None:
        """Abort every submitted choice that has not finished (no-op for finished ones)."""
        for g in gens:
            g.close()

    def tok_str(t: int) -> str:
        return tokenizer.decode([t])

    def usage_chunk(final_fn, np_: int, nc: int) -> str:
        """stream_options.include_usage: the last event before [DONE], no choices."""
        body = final_fn("", None, np_, nc)
        body["choices"] = []
        if body["object"] == "chat.completion":
            body["object"] = "chat.completion.chunk"
        return "data: " + json.dumps(body) + "\n\n"

    async def run(ids: list[int], sp: SamplingParams, rid: str, stream_fn, final_fn, stream: bool,
                  include_usage: bool = False):
        """One engine request per choice (n > 1 fans out with seeds seed+i); choices stream
        interleaved, each chunk tagged with its choice index."""
        n = sp.n
        subs = [dataclasses.replace(sp, n=1, seed=None if sp.seed is None else sp.seed + i)
                for i in range(n)]
        rids = [rid if n == 1 else f"{rid}-{i}" for i in range(n)]
        # submit every choice before the response starts (EngineDeadError -> 503 here)
        gens = [engine.generate(ids, subs[i], rids[i]) for i in range(n)]
        if stream and n == 1:
            # one coroutine per stream: engine output -> detok -> SSE bytes, no task or
            # queue hop (the per-token path dominates the API process at 256 streams)
            async def sse1():
                detok = _Detok(tokenizer, sp.stop)
                gen = gens[0]
                nc = 0
                try:
                    async for out in gen:
                        nc = len(out.output_token_ids)
                        delta = detok.update(out.output_token_ids)
                        reason = out.finish_reason if out.finished else None
                        if detok.stopped:
                            reason = "stop"
                        elif reason:
                            delta += detok.flush()
                        if delta or reason or out.logprobs:
                            yield stream_fn(delta, reason, out.logprobs, 0)
                        if detok.stopped:
                            break
                except EngineDeadError as e:
                    yield f"data: {json.dumps({'error': str(e)})}\n\n"
                finally:
                    await gen.aclose()
                if include_usage:
                    yield usage_chunk(final_fn, len(ids), nc)
                yield "data: [DONE]\n\n"
            return StreamingResponse(sse1(), media_type="text/event-stream",
                                     background=BackgroundTask(close_all, gens))
        if stream:
            q: asyncio.Queue = asyncio.Queue()

            ncs = [0] * n

            async def pump(i):
                detok = _Detok(tokenizer, subs[i].stop)
                gen = gens[i]
                try:
                    async for out in gen:
                        ncs[i] = len(out.output_token_ids)
                        delta = detok.update(out.output_token_ids)
                        reason = out.finish_reason if out.finished else None
                        if detok.stopped:
                            reason = "stop"
                        elif reason:
                            delta += detok.flush()
                        if delta or reason or out.logprobs:
                            await q.put((i, delta, reason, out.logprobs))
                        if detok.stopped:
                            await gen.aclose()
                            break
                except EngineDeadError as e:
                    await q.put((i, None, None, e))
                finally:
                    await q.put((i, None, "__done__", None))

            async def sse():
                tasks = [asyncio.create_task(pump(i)) for i in range(n)]
                done = 0
                try:
                    while done < n:
                        i, delta, reason, lps = await q.get()
                        if reason == "__done__":
                            done += 1
                            continue
                        if isinstance(lps, BaseException):
                            yield f"data: {json.dumps({'error': str(lps)})}\n\n"
                            continue
                        yield stream_fn(delta, reason, lps, i)
                    if include_usage:
                        yield usage_chunk(final_fn, len(ids), sum(ncs))
                    yield "data: [DONE]\n\n"
                finally:
                    for t in tasks:
                        t.cancel()
            return StreamingResponse(sse(), media_type="text/event-stream",
                                     background=BackgroundTask(close_all, gens))

        async def one(i):
            detok = _Detok(tokenizer, subs[i].stop)
            gen = gens[i]
            last, lps = None, []
            async for out in gen:
                last = out
                if out.logprobs:
                    lps.extend(out.logprobs)
                detok.update(out.output_token_ids)
                if detok.stopped:
                    await gen.aclose()
                    break
            reason = "stop" if detok.stopped else (last.finish_reason if last else None)
            return detok.text, reason, (len(last.output_token_ids) if last else 0), lps
        try:
            res = await asyncio.gather(*[one(i) for i in range(n)])
        finally:
            close_all(gens)      # a failed or cancelled sibling leaves the others unread
        text, reason, nc, lps = res[0]
        body = final_fn(text, reason, len(ids), sum(r[2] for r in res),
                        lps if sp.logprobs is not None else None)
        if n > 1:
            choices = []
            for i, (t_i, r_i, _, l_i) in enumerate(res):
                one_body = final_fn(t_i, r_i, len(ids), 0, l_i if sp.logprobs is not None else None)
                c = one_body["choices"][0]
                c["index"] = i
                choices.append(c)
            body["choices"] = choices
        return JSONResponse(body)

    def completion_logprobs(lps, offset0: int = 0):
        """legacy completions shape: tokens / token_logprobs / top_logprobs / text_offset"""
        if lps is None:
            return None
        toks, vals, tops, offs = [], [], [], []
        off = offset0
        for t, lp, top in lps:
            s = tok_str(t)
            toks.append(s)
            vals.append(lp)
            tops.append({tok_str(a): v for a, v in top})
            offs.append(off)
            off += len(s)
        return {"tokens": toks, "token_logprobs": vals, "top_logprobs": tops, "text_offset": offs}

    def chat_logprobs(lps):
        if lps is None:
            return None

        def ent(t, lp):
            s = tok_str(t)
            return {"token": s, "logprob": lp, "bytes": list(s.encode("utf-8"))}
        return {"content": [dict(ent(t, lp), top_logprobs=[ent(a, v) for a, v in top])
                            for t, lp, top in lps]}

    def prompt_ids(p) -> list[int]:
        return tokenizer.encode(p) if isinstance(p, str) else [int(x) for x in p]

    async def completions_batch(req: CompletionRequest, prompts: list):
        """A list of prompts in one /v1/completions request (as vLLM / OpenAI accept it):
        choice index = prompt * n + choice; streamed chunks interleave, tagged by index."""
        all_ids = [prompt_ids(p) for p in prompts]
        for ids in all_ids:
            if len(ids) >= max_model_len:
                raise ValueError(f"prompt has {len(ids)} tokens; max_model_len is {max_model_len}")
        sp = params_from(req, req.max_tokens, req.logprobs)
        n, rid = sp.n, f"cmpl-{uuid.uuid4().hex}"
        want_lp = req.logprobs is not None
        prefixes = [((p if isinstance(p, str) else tokenizer.decode(ids)) if req.echo else "")
                    for p, ids in zip(prompts, all_ids)]
        subs, gens = [], []
        for pi, ids in enumerate(all_ids):
            for i in range(n):
                sub = dataclasses.replace(sp, n=1, seed=None if sp.seed is None else sp.seed + i)
                subs.append(sub)
                gens.append(engine.generate(ids, sub, f"{rid}-{pi}-{i}"))

        async def drain(k, q=None):
            detok = _Detok(tokenizer, subs[k].stop)
            gen, last, lps = gens[k], None, []
            try:
                async for out in gen:
                    last = out
                    delta = detok.update(out.output_token_ids)
                    reason = out.finish_reason if out.finished else None
                    if detok.stopped:
                        reason = "stop"
                    elif reason:
                        delta += detok.flush()
                    if out.logprobs:
                        lps.extend(out.logprobs)
                    if q is not None and (delta or reason or out.logprobs):
                        await q.put((k, delta, reason, out.logprobs))
                    if detok.stopped:
                        await gen.aclose()
                        break
            except EngineDeadError as e:
                if q is None:
                    raise
                await q.put((k, None, None, e))
            finally:
                if q is not None:
                    await q.put((k, None, "__done__", None))
            reason = "stop" if detok.stopped else (last.finish_reason if last else None)
            return detok.text, reason, (len(last.output_token_ids) if last else 0), lps

        if req.stream:
            q: asyncio.Queue = asyncio.Queue()
            head = f'data: {{"id": "{rid}", "object": "text_completion", "created": '
            model_js = json.dumps(served_name)

            async def sse():
                tasks = [asyncio.create_task(drain(k, q)) for k in range(len(gens))]
                done = 0
                try:
                    while done < len(gens):
                        k, delta, reason, lps = await q.get()
                        if reason == "__done__":
                            done += 1
                            continue
                        if isinstance(lps, BaseException):
                            yield f"data: {json.dumps({'error': str(lps)})}\n\n"
                            continue
                        lp = json.dumps(completion_logprobs(lps or [])) if want_lp else "null"
                        yield (f'{head}{int(time.time())}, "model": {model_js}, "choices": '
                               f'[{{"index": {k}, "text": {json.dumps(delta)}, "logprobs": '
                               f'{lp}, "finish_reason": {json.dumps(reason)}}}]}}\n\n')
                    yield "data: [DONE]\n\n"
                finally:
                    for t in tasks:
                        t.cancel()
            return StreamingResponse(sse(), media_type="text/event-stream",
                                     background=BackgroundTask(close_all, gens))
        try:
            res = await asyncio.gather(*[drain(k) for k in range(len(gens))])
        finally:
            close_all(gens)
        choices = []
        for k, (text, reason, _, lps) in enumerate(res):
            pre = prefixes[k // n]
            choices.append({"index": k, "text": pre + text,
                            "logprobs": completion_logprobs(lps, len(pre)) if want_lp else None,
                            "finish_reason": reason})
        np_ = sum(len(ids) for ids in all_ids)
        nc = sum(r[2] for r in res)
        return JSONResponse({"id": rid, "object": "text_completion", "created": int(time.time()),
                             "model": served_name, "choices": choices,
                             "usage": {"prompt_tokens": np_, "completion_tokens": nc,
                                       "total_tokens": np_ + nc}})

    @app.post("/v1/completions")
    async def completions(req: CompletionRequest):
        if not 1 <= req.n <= 16:
            return _err(400, "n must be in [1, 16]")
        prompts = req.prompt
        if isinstance(prompts, list) and prompts and isinstance(prompts[0], (str, list)):
            if len(prompts) > 1:
                try:
                    return await completions_batch(req, prompts)
                except EngineDeadError as e:
                    return _err(503, f"engine unavailable: {e}", "server_error")
                except ValueError as e:
                    return _err(400, str(e))
            prompts = prompts[0]
        ids = prompt_ids(prompts)
        if len(ids) >= max_model_len:
            return _err(400, f"prompt has {len(ids)} tokens; max_model_len is {max_model_len}")
        try:
            sp = params_from(req, req.max_tokens, req.logprobs)
        except ValueError as e:
            return _err(400, str(e))
        rid = f"cmpl-{uuid.uuid4().hex}"
        prefix = (prompts if isinstance(prompts, str) else tokenizer.decode(ids)) if req.echo else ""
        want_lp = req.logprobs is not None

        head = f'data: {{"id": "{rid}", "object": "text_completion", "created": '
        model_js = json.dumps(served_name)

        def chunk(delta, reason, lps=None, index=0):
            """One SSE event; the constant head is formatted once per request."""
            lp = json.dumps(completion_logprobs(lps or [])) if want_lp else "null"
            return (f'{head}{int(time.time())}, "model": {model_js}, "choices": [{{"index": '
                    f'{index}, "text": {json.dumps(delta)}, "logprobs": {lp}, "finish_reason": '
                    f'{json.dumps(reason)}}}]}}\n\n')

        def final(text, reason, np_, nc, lps=None):
            return {"id": rid, "object": "text_completion", "created": int(time.time()),
                    "model": served_name,
                    "choices": [{"index": 0, "text": prefix + text,
                                 "logprobs": completion_logprobs(lps, len(prefix)),
                                 "finish_reason": reason}],
                    "usage": {"prompt_tokens": np_, "completion_tokens": nc,
                              "total_tokens": np_ + nc}}
        try:
            return await run(ids, sp, rid, chunk, final, req.stream,
                             bool((req.stream_options or {}).get("include_usage")))
        except EngineDeadError as e:
            return _err(503, f"engine unavailable: {e}", "server_error")
        except ValueError as e:
            return _err(400, str(e))

    @app.post("/v1/chat/completions")
    async def chat(req: ChatCompletionRequest):
        if not 1 <= req.n <= 16:
            return _err(400, "n must be in [1, 16]")
        msgs = []
        for m in req.messages:
            c = m.content
            if isinstance(c, list):
                c = "".join(p.get("text", "") for p in c if isinstance(p, dict))
            msgs.append({"role": m.role, "content": c or ""})
        text = tokenizer.apply_chat_template(msgs, add_generation_prompt=True)
        ids = tokenizer.encode(text)
        if len(ids) >= max_model_len:
            return _err(400, f"prompt has {len(ids)} tokens; max_model_len is {max_model_len}")
        try:
            sp = params_from(req, req.max_completion_tokens or req.max_tokens,
                             (req.top_logprobs or 0) if req.logprobs else None)
        except ValueError as e:
            return _err(400, str(e))
        rid = f"chatcmpl-{uuid.uuid4().hex}"
        first = [True]

        def chunk(delta, reason, lps=None, index=0):
            d = {"content": delta}
            if first[0]:
                d["role"] = "assistant"
                first[0] = False
            c = {"index": index, "delta": d, "finish_reason": reason}
            if req.logprobs:
                c["logprobs"] = chat_logprobs(lps or [])
            return "data: " + json.dumps({"id": rid, "object": "chat.completion.chunk",
                                          "created": int(time.time()), "model": served_name,
                                          "choices": [c]}) + "\n\n"

        def final(text, reason, np_, nc, lps=None):
            return {"id": rid, "object": "chat.completion", "created": int(time.time()),
                    "model": served_name,
                    "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                                 "logprobs": chat_logprobs(lps),
                                 "finish_reason": reason}],
                    "usage": {"prompt_tokens": np_, "completion_tokens": nc,
                              "total_tokens": np_ + nc}}
        try:
            return await run(ids, sp, rid, chunk, final, req.stream,
                             bool((req.stream_options or {}).get("include_usage")))
        except EngineDeadError as e:
            return _err(503, f"engine unavailable: {e}", "server_error")
        except ValueError as e:
            return _err(400, str(e))

    @app.post("/tokenize")
    async def tokenize(req: TokenizeRequest):
        """vLLM's /tokenize: a prompt, or chat messages rendered with the chat template."""
        if req.messages is not None:
            msgs = [{"role": m.get("role", "user"), "content": m.get("content") or ""}
                    for m in req.messages]
            text = tokenizer.apply_chat_template(msgs,
                                                 add_generation_prompt=req.add_generation_prompt)
        elif req.prompt is not None:
            text = req.prompt
        else:
            return _err(400, "tokenize needs 'prompt' or 'messages'")
        ids = tokenizer.encode(text)
        return {"count": len(ids), "max_model_len": max_model_len, "tokens": ids}

    @app.post("/detokenize")
    async def detokenize(req: DetokenizeRequest):
        vocab = getattr(tokenizer, "vocab_size", None)
        if vocab and any(not 0 <= t < vocab for t in req.tokens):
            return _err(400, f"token ids must be in [0, {vocab})")
        return {"prompt": tokenizer.decode(list(req.tokens))}

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": served_name, "object": "model",
                                            "created": created, "owned_by": "kgc",
                                            "root": served_name, "parent": None,
                                            "max_model_len": max_model_len}]}

    @app.get("/health")
    async def health():
        if not engine.is_alive:
            return PlainTextResponse("engine dead", status_code=503)
        return PlainTextResponse("ok")

    @app.api_route("/ping", methods=["GET", "POST"])
    async def ping():
        """vLLM's /ping (SageMaker-style liveness): same answer as /health."""
        return await health()

    @app.get("/kgc/engine_stats")
    async def engine_stats(since: float = 0.0):
        """Engine-side timings of requests that arrived at or after ``since`` (host
        ``time.monotonic()``) and have finished: (arrival, first token, finish, tokens)."""
        return JSONResponse(await engine.engine_stats(since))

    @app.get("/metrics")
    async def metrics():
        return PlainTextResponse(await engine.metrics_text(),
                                 media_type="text/plain; version=0.0.4")

    @app.get("/version")
    async def version():
        return {"version": __version__}

    return app


def make_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="kgc OpenAI-compatible server")
    p.add_argument("model_tag", nargs="?", default=None, help="model (positional, like vllm serve)")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--uvicorn-log-level", default="info")
    p.add_argument("--api-key", default=os.environ.get("VLLM_API_KEY"),
                   help="require 'Authorization: Bearer <key>' on /v1 routes (env VLLM_API_KEY)")
    p.add_argument("--engine-in-process", action="store_true",
                   help="run the engine loop on a thread of this process instead of a "
                        "separate engine-core process")
    p.add_argument("--api-server-count", type=int, default=0,
                   help="API processes sharing the port (SO_REUSEPORT) in front of one "
                        "engine core; >1 spreads detokenisation / SSE of many concurrent "
                        "streams over several CPUs (0: min(4, CPUs / 4))")
    add_engine_args(p)
    return p


def _reuseport_socket(host: str, port: int) -> socket.socket:
    s = socket.socket(socket.AF_INET6 if ":" in host else socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    return s


def _serve(ns, cfg: EngineConfig, connect=None, core_proc=None, sock=None) -> None:
    """One API process: an engine (private core, shared core at ``connect``, or
    in-process thread) behind uvicorn; with a shared core it exits when the core does."""
    import uvicorn
    logging.basicConfig(level=logging.INFO)
    if ns.engine_in_process:
        eng = AsyncLLMEngine(cfg)
    else:
        from .engine_core import EngineCoreClient
        eng = EngineCoreClient(cfg, connect=connect, core_proc=core_proc)
    tok = get_tokenizer(cfg.model, eng.engine.mcfg, cfg.tokenizer,
                        allow_synthetic=cfg.random_init)
    name = cfg.served_model_name or cfg.model
    app = build_app(eng, tok, name, eng.engine.max_model_len, ns.api_key)
    server = uvicorn.Server(uvicorn.Config(app, host=ns.host, port=ns.port,
                                           log_level=ns.uvicorn_log_level))
    dead = threading.Event()

    def watchdog():
        # the engine (core process, its TP/PP ranks, or the in-process loop) died: stop
        # serving and exit non-zero so the pod restarts (engine/health.py); /health
        # answers 503 meanwhile
        while not server.should_exit:
            time.sleep(0.5)
            if not eng.is_alive:
                logging.getLogger("kgc.api").critical("engine is dead; shutting down")
                dead.set()
                server.should_exit = True
    threading.Thread(target=watchdog, name="kgc-api-watchdog", daemon=True).start()
    try:
        server.run(sockets=[sock] if sock is not None else None)
    finally:
        if dead.is_set():
            t = threading.Thread(target=eng.shutdown, daemon=True)
            t.start()
            t.join(10)
        else:
            eng.shutdown()
    if dead.is_set():
        raise SystemExit(3)


def _serve_worker(ns, cfg: EngineConfig, connect) -> None:
    _serve(ns, cfg, connect=connect, sock=_reuseport_socket(ns.host, ns.port))


def main(argv=None) -> None:
    ns = make_parser().parse_args(argv)
    ns.model = ns.model or ns.model_tag or "llama-3-8b"
    cfg = config_from_args(ns)
    # fail before any engine process or GPU is touched: a missing hostPath checkpoint
    # exits non-zero so the pod crash-loops instead of serving random tokens
    from ..models import check_weights
    check_weights(cfg.model, cfg.random_init)
    n = ns.api_server_count or min(4, max(1, (os.cpu_count() or 1) // 4))
    if n == 1 or ns.engine_in_process:
        _serve(ns, cfg)
        return
    import multiprocessing as mp
    import secrets
    import shutil
    import tempfile
    from .engine_core import start_core
    tmp = tempfile.mkdtemp(prefix="kgc-core-")
    connect = (os.path.join(tmp, "core.sock"), secrets.token_bytes(32))
    core = start_core(cfg, connect[0], connect[1], n)
    ctx = mp.get_context("spawn")
    workers = [ctx.Process(target=_serve_worker, args=(ns, cfg, connect), name=f"kgc-api-{i}")
               for i in range(1, n)]
    for w in workers:
        w.start()
    try:
        _serve(ns, cfg, connect=connect, core_proc=core,
               sock=_reuseport_socket(ns.host, ns.port))
    finally:
        for w in workers:
            w.join(30)
            if w.is_alive():
                w.terminate()
        shutil.rmtree(tmp, ignore_errors=True)
    if core.exitcode not in (0, None):
        raise SystemExit(3)


if __name__ == "__main__":
    main()
