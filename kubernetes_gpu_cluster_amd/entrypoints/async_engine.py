"""Thread-backed async facade over LLMEngine for the HTTP server.

The engine loop (schedule -> execute -> update) runs on one background thread;
request submission, abort and per-request output streams cross to the asyncio
loop through thread-safe queues (``loop.call_soon_threadsafe``).  GPU waits in the
engine release the GIL, so the HTTP event loop keeps serving while a step runs.
"""
from __future__ import annotations

import asyncio
import collections
import logging
import queue
import threading
import time
import traceback
from typing import AsyncIterator, Optional

from ..engine.config import EngineConfig
from ..engine.llm_engine import LLMEngine
from ..engine.sequence import RequestOutput, SamplingParams

log = logging.getLogger("kgc.async_engine")


class EngineDeadError(RuntimeError):
    pass


def _merge(prev, nxt) -> None:
    """Fold an earlier (undelivered) step output into the next one of the same request."""
    nxt.new_token_ids = prev.new_token_ids + nxt.new_token_ids
    if prev.logprobs or nxt.logprobs:
        nxt.logprobs = (prev.logprobs or []) + (nxt.logprobs or [])


class DoneLog:
    """Engine-side timing of finished requests -- (arrival, first token, finish, output
    tokens), all ``time.monotonic()`` of the serving host -- for ``GET
    /kgc/engine_stats``: the engine-level counterpart of what an HTTP client measures
    (bench.py reports both)."""

    def __init__(self, maxlen: int = 1 << 17):
        self.log: collections.deque = collections.deque(maxlen=maxlen)
        self.steps = 0
        self.step_s = 0.0

    def on_step(self, outs, dt: float) -> None:
        self.steps += 1
        self.step_s += dt
        for o in outs:
            if o.finished:
                self.log.append((o.arrival_time, o.first_token_time, o.finish_time,
                                 o.num_output_tokens))

    def snapshot(self, since: float = 0.0) -> dict:
        return {"now": time.monotonic(), "steps": self.steps, "step_busy_s": self.step_s,
                "requests": [r for r in list(self.log) if r[0] >= since]}


class RequestStream:
    """The output stream of one submitted request (``generate``).  Every exit that leaves
    the request unfinished aborts it in the engine: ``aclose()`` / ``close()``, a
    cancelled or failed consumer, and a stream that is dropped without ever being
    iterated (a client that disconnects before the response starts, a sibling choice
    whose task raised) -- the request was submitted eagerly, so without this it would
    keep decoding to max_tokens in a batch slot nobody reads."""

    def __init__(self, request_id: str, q: asyncio.Queue, on_close, on_drop=None):
        self.request_id = request_id
        self._q = q
        self._on_close = on_close           # on_close(request_id, abort: bool)
        # on_drop(request_id): the finalizer's abort -- it must take NO lock (a cyclic GC
        # pass can run __del__ on a thread that already holds the engine client's send
        # lock or a queue's mutex, e.g. while pickling inside _send): the owner only
        # records the id lock-free and aborts it later from a normal context
        self._on_drop = on_drop
        self._closed = False

    def __aiter__(self):
        return self

    async def __anext__(self) -> RequestOutput:
        if self._closed:
            raise StopAsyncIteration
        try:
            item = await self._q.get()
        except BaseException:
            self.close()
            raise
        # coalesce: if the consumer fell behind, merge the queued steps into one output
        # (token lists are cumulative), so a slow HTTP stream costs one event per wake-up
        q = self._q
        while not isinstance(item, BaseException) and not item.finished and not q.empty():
            nxt = q.get_nowait()
            if not isinstance(nxt, BaseException):
                _merge(item, nxt)
            item = nxt
        if isinstance(item, BaseException):
            self._end(abort=False)          # rejected, or the engine is gone
            raise item
        if item.finished:
            self._end(abort=False)
        return item

    def _end(self, abort: bool) -> None:
        if not self._closed:
            self._closed = True
            self._on_close(self.request_id, abort)

    def close(self) -> None:
        self._end(abort=True)

    async def aclose(self) -> None:
        self.close()

    def __del__(self):
        if self._closed:
            return
        self._closed = True
        try:
            if self._on_drop is not None:
                self._on_drop(self.request_id)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def _deliver(items) -> None:
    for q, o in items:
        q.put_nowait(o)


class AsyncLLMEngine:
    def __init__(self, cfg: EngineConfig, engine: Optional[LLMEngine] = None):
        self.cfg = cfg
        self.engine = engine or LLMEngine(cfg)
        self._new: queue.Queue = queue.Queue()
        # request ids to abort: a deque (append / popleft are atomic and lock-free), so a
        # stream finalizer can add to it from any context (RequestStream.__del__)
        self._aborts: collections.deque = collections.deque()
        self._streams: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self._wake = threading.Event()
        self._stop = False
        self.error: Optional[BaseException] = None
        self.last_step_time = time.monotonic()
        self.done_log = DoneLog()
        self._thread = threading.Thread(target=self._loop, name="kgc-engine", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ engine thread
    def _push(self, rid: str, item) -> None:
        ent = self._streams.get(rid)
        if ent is not None:
            loop, q = ent
            loop.call_soon_threadsafe(q.put_nowait, item)

    def _push_step(self, outs) -> None:
        """Hand a whole step's outputs to the event loop in ONE thread-safe call (not one
        wake-up per request: at batch 256 that is 256 self-pipe writes per step)."""
        by_loop: dict = {}
        for o in outs:
            ent = (self._streams.pop(o.request_id, None) if o.finished
                   else self._streams.get(o.request_id))
            if ent is not None:
                by_loop.setdefault(ent[0], []).append((ent[1], o))
        for loop, items in by_loop.items():
            loop.call_soon_threadsafe(_deliver, items)

    def _loop(self) -> None:
        eng = self.engine
        try:
            while not self._stop:
                while True:
                    try:
                        rid, ids, params, t = self._new.get_nowait()
                    except queue.Empty:
                        break
                    try:
                        eng.add_request(ids, params, request_id=rid, arrival_time=t)
                    except Exception as e:  # noqa: BLE001 - reported to the request
                        self._push(rid, e)
                while self._aborts:
                    eng.abort(self._aborts.popleft())
                if eng.has_unfinished():
                    t0 = time.monotonic()
                    outs = eng.step()
                    self.last_step_time = time.monotonic()
                    # logged BEFORE the outputs reach the event loop: a client that reads a
                    # request's [DONE] and then asks /kgc/engine_stats must find it there
                    # (pushed first, a descheduled engine thread left the last request of a
                    # wave out of the bench's engine-side window under CPU load)
                    self.done_log.on_step(outs, self.last_step_time - t0)
                    self._push_step(outs)
                else:
                    self._wake.wait(0.05)
                    self._wake.clear()
        except BaseException as e:  # noqa: BLE001
            self.error = e
            log.error("engine loop died: %s", traceback.format_exc())
            for rid in list(self._streams):
                self._push(rid, EngineDeadError(str(e)))

    # ------------------------------------------------------------------ asyncio side
    @property
    def is_alive(self) -> bool:
        return self._thread.is_alive() and self.error is None

    def generate(self, prompt_ids: list[int], params: SamplingParams,
                 request_id: str) -> AsyncIterator[RequestOutput]:
        """Submit now (from the request handler) and return the output stream."""
        if not self.is_alive:
            raise EngineDeadError(str(self.error))
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        self._streams[request_id] = (loop, q)
        self._new.put((request_id, prompt_ids, params, time.monotonic()))
        self._wake.set()
        return RequestStream(request_id, q, self._close_stream, self._drop_stream)

    def _close_stream(self, request_id: str, abort: bool) -> None:
        self._streams.pop(request_id, None)
        if abort:
            self.abort(request_id)

    def _drop_stream(self, request_id: str) -> None:
        """Finalizer path: lock-free (dict pop and deque append); the engine thread picks
        the abort up within one loop iteration (it waits at most 50 ms when idle)."""
        self._streams.pop(request_id, None)
        self._aborts.append(request_id)

    def abort(self, request_id: str) -> None:
        self._aborts.append(request_id)
        self._wake.set()

    async def metrics_text(self) -> str:
        from prometheus_client import generate_latest
        return generate_latest(self.engine.metrics.registry).decode()

    async def engine_stats(self, since: float = 0.0) -> dict:
        return self.done_log.snapshot(since)

    def shutdown(self) -> None:
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=30)
        self.engine.shutdown()
