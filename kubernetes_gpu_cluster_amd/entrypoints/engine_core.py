"""Engine core in its own process, for the HTTP server.

With the engine loop on a thread of the API-server process, the scheduler and
plan building (~1-2 ms per step at batch 256) compete for one GIL with request
parsing, detokenisation and SSE writes for 256 streams.  Once that Python work
exceeds a decode step, the GPU idles.  ``EngineCoreClient`` starts
``LLMEngine`` in a separate spawned process.  The API process never touches the
GPU, so spawning stays safe.  The two talk over one duplex pipe:

* API -> core: ``add`` / ``abort`` / ``metrics`` / ``shutdown`` messages, non-blocking
  for the event loop;
* core -> API: ONE ``out`` message per engine step, carrying every request's newly
  resolved tokens.  A reader thread delivers it to the event loop with one
  thread-safe call.

At 256 concurrent streams one API process is itself CPU-bound (detokenisation,
JSON and SSE writes for every token of every stream each ~11 ms step), so
``--api-server-count N`` runs N API processes on one port (SO_REUSEPORT) in front of
ONE engine core: the core accepts N connections on a unix socket and sends each
frontend only the outputs of the requests it submitted.

The interface matches ``AsyncLLMEngine``: ``generate``, ``abort``, ``is_alive``,
``shutdown``, ``metrics_text``, ``mcfg``, ``max_model_len``.  ``build_app`` therefore
accepts either.  ``--engine-in-process`` selects the thread-backed engine instead.
"""
from __future__ import annotations

import asyncio
import collections
import itertools
import logging
import multiprocessing as mp
import os
import threading
import time
import traceback
from multiprocessing.connection import wait as mp_wait
from typing import AsyncIterator, Optional

from ..engine.config import EngineConfig
from ..engine.sequence import RequestOutput, SamplingParams
from .async_engine import DoneLog, EngineDeadError, RequestStream, _deliver

log = logging.getLogger("kgc.engine_core")


# ---------------------------------------------------------------------------- core process
class _Intake(threading.Thread):
    """Receives the frontends' messages while the engine steps: a burst of requests is
    unpickled and queued during the GPU step, not after it, so the core loop admits
    everything that arrived at the next step boundary with no receive work of its own
    (the loop only drains this queue).  Connections are only READ here; every send
    stays on the core loop's thread."""

    def __init__(self, conns: list):
        super().__init__(name="kgc-core-intake", daemon=True)
        self.conns = list(conns)
        self.q: collections.deque = collections.deque()
        self.wake = threading.Event()
        self.stop = False

    def run(self) -> None:
        while self.conns and not self.stop:
            for c in mp_wait(self.conns, 0.1):
                try:
                    msg = c.recv()
                except (EOFError, OSError):
                    self.conns.remove(c)
                    msg = None              # the frontend went away
                self.q.append((c, msg, time.monotonic()))
                self.wake.set()
        self.q.append((None, None, time.monotonic()))   # no frontend left
        self.wake.set()


def _drain(intake: "_Intake", eng, conns: list, owner: dict, adds, done) -> bool:
    """Handle every message the intake thread queued.  Returns False on shutdown.
    ``adds`` gets (receive time, frontend stamp) per admitted request."""
    while intake.q:
        c, msg, t_recv = intake.q.popleft()
        if c is None:
            conns.clear()
            return True
        if msg is None:
            if c in conns:
                conns.remove(c)        # a frontend went away: drop its requests
            for rid in [r for r, oc in owner.items() if oc is c]:
                owner.pop(rid)
                eng.abort(rid)
            continue
        kind = msg[0]
        if kind == "add":
            _, rid, ids, params, arrival = msg
            adds.append((t_recv, arrival))
            try:
                eng.add_request(ids, params, request_id=rid, arrival_time=arrival)
                owner[rid] = c
            except Exception as e:  # noqa: BLE001 - reported to that request
                c.send(("reject", rid, f"{type(e).__name__}: {e}"))
        elif kind == "abort":
            owner.pop(msg[1], None)
            eng.abort(msg[1])
        elif kind == "metrics":
            from prometheus_client import generate_latest
            c.send(("metrics", msg[1], generate_latest(eng.metrics.registry).decode()))
        elif kind == "stats":
            c.send(("stats", msg[1], done.snapshot(msg[2])))
        elif kind == "shutdown":
            return False
    return True


def _make_engine(cfg: EngineConfig):
    if os.environ.get("KGC_FAKE_ENGINE"):
        # GPU-free timing model of the engine (engine/fake.py): load-tests the
        # API / router / client path above the engine on a CPU-only machine
        from ..engine.fake import FakeEngine
        return FakeEngine(cfg)
    from ..engine.llm_engine import LLMEngine
    return LLMEngine(cfg)


def _core_main(cfg: EngineConfig, conn, listen: Optional[tuple] = None) -> None:
    """``conn``: the pipe to a single frontend; or, with ``listen = (address, authkey,
    n)``, accept ``n`` frontend connections (``--api-server-count``) and route every
    request's outputs back to the frontend that submitted it."""
    logging.basicConfig(level=logging.INFO)
    # the API process owns termination: a SIGTERM / Ctrl-C to the process group (pod stop)
    # reaches it, it stops serving and tells the core to shut down; the core also ends
    # when every frontend connection is gone (EOF), so it never outlives the server
    import signal
    signal.signal(signal.SIGTERM, signal.SIG_IGN)
    signal.signal(signal.SIGINT, signal.SIG_IGN)
    conns = [conn] if conn is not None else []
    listener = None
    if listen is not None:
        from multiprocessing.connection import Listener
        listener = Listener(listen[0], authkey=listen[1])
    try:
        eng = _make_engine(cfg)
    except BaseException:  # noqa: BLE001
        tb = traceback.format_exc()
        if listener is not None:
            for _ in range(listen[2]):
                try:
                    listener.accept().send(("dead", tb))
                except OSError:
                    break
        else:
            conn.send(("dead", tb))
        return
    ready_msg = ("ready", {"mcfg": eng.mcfg, "max_model_len": eng.max_model_len})
    if listener is not None:
        for _ in range(listen[2]):        # each frontend may start serving once attached
            conns.append(listener.accept())
            conns[-1].send(ready_msg)
        listener.close()
    else:
        conn.send(ready_msg)
    owner: dict = {}          # request id -> connection of the frontend that submitted it
    # host-time accounting of the core loop, logged at exit: where a step's host time goes
    # besides the engine step itself (inbox handling, output fan-out to the frontends)
    st = {"iters": 0, "steps": 0, "step_s": 0.0, "send_s": 0.0, "inbox_s": 0.0,
          "coalesce_waits": 0}
    # Burst admission (KGC_COALESCE_MS, default 40; KGC_COALESCE_GAP_MS, default 3): when
    # an idle engine receives a burst (a wave of requests through the router: 256 arrive
    # over ~50 ms), stepping at once ran the first 1, 6 and 7 requests as three small
    # prefill steps and left a 19-request remainder after the full 16K-token chunks: 11
    # prefill steps instead of 8, plus a decode step forced into a chunk by the prefill-
    # first deferral bound (profiles/README.md "Round 6: burst admission").  While
    # nothing is running and the waiting prompts fill less than one step's token budget,
    # the loop keeps admitting as long as requests keep arriving (gaps under GAP ms), for
    # at most COALESCE ms.  Under continuous load something is always running, so this
    # never delays a step there.
    coalesce_s = float(os.environ.get("KGC_COALESCE_MS", "40")) / 1e3
    gap_s = float(os.environ.get("KGC_COALESCE_GAP_MS", "3")) / 1e3
    coalescing = getattr(eng, "coalescing", lambda: False)
    inflight_coalescing = getattr(eng, "inflight_coalescing", lambda: False)
    gap_inflight_s = float(os.environ.get("KGC_COALESCE_INFLIGHT_GAP_MS", "10")) / 1e3
    # (core receive time, frontend stamp) of the latest requests (bounded: a server runs
    # for weeks)
    adds: collections.deque = collections.deque(maxlen=1 << 16)
    done = DoneLog()
    intake = _Intake(conns)
    intake.start()
    try:
        running = True
        while running and conns:
            idle = not eng.has_unfinished()
            st["iters"] += 1
            ti = time.perf_counter()
            # drain what the intake thread queued; block briefly only when idle
            if idle and not intake.q:
                intake.wake.wait(0.05)
            intake.wake.clear()
            running = _drain(intake, eng, conns, owner, adds, done) and running
            # a burst is being admitted (nothing runs yet and the waiting prompts fill
            # less than one prefill step): keep admitting while requests keep arriving
            if running and coalesce_s > 0 and coalescing():
                t_end = time.monotonic() + coalesce_s
                n0 = len(adds)
                while running and coalescing():
                    rem = t_end - time.monotonic()
                    if rem <= 0:
                        break
                    # a lone request waits at most GAP for a follower; once followers
                    # come (a burst), pauses of up to INFLIGHT_GAP are tolerated
                    gap = gap_s if len(adds) - n0 < 2 else gap_inflight_s
                    if not intake.q and not intake.wake.wait(min(gap, rem)):
                        break                  # the arrivals paused: start the step
                    intake.wake.clear()
                    running = _drain(intake, eng, conns, owner, adds, done) and running
                    st["coalesce_waits"] += 1
            # ... and while a large prefill step is on the GPU: the next step would be a
            # partial prefill of what has arrived so far, so admit further arrivals until
            # the step's budget fills, the arrivals pause (GAP_INFLIGHT ms since the last
            # one) or the GPU step completes -- the next step is launched before the GPU
            # goes idle, except when the in-flight step finishes first
            if (running and coalesce_s > 0 and adds
                    and time.monotonic() - adds[-1][0] < gap_inflight_s
                    and inflight_coalescing()):
                t_end = time.monotonic() + 0.5
                while running and inflight_coalescing():
                    now = time.monotonic()
                    if now >= t_end or (adds and now - adds[-1][0] > gap_inflight_s):
                        break
                    if not intake.q and not intake.wake.wait(0.001):
                        continue               # re-check: the GPU step may have completed
                    intake.wake.clear()
                    running = _drain(intake, eng, conns, owner, adds, done) and running
                    st["coalesce_waits"] += 1
            if not idle:
                st["inbox_s"] += time.perf_counter() - ti
            if running and eng.has_unfinished():
                by_conn: dict = {}
                t1 = time.perf_counter()
                outs = eng.step()
                t2 = time.perf_counter()
                st["steps"] += 1
                st["step_s"] += t2 - t1
                done.on_step(outs, t2 - t1)
                for o in outs:
                    c = owner.get(o.request_id)
                    if c is None:
                        continue
                    if o.finished:
                        owner.pop(o.request_id, None)
                    by_conn.setdefault(c, []).append(
                        (o.request_id, o.new_token_ids, o.finished, o.finish_reason,
                         o.arrival_time, o.first_token_time, o.finish_time,
                         o.num_preemptions, o.logprobs))
                for c, items in by_conn.items():
                    try:
                        c.send(("out", items))
                    except OSError:
                        pass
                st["send_s"] += time.perf_counter() - t2
    except BaseException:  # noqa: BLE001
        tb = traceback.format_exc()
        log.error("engine core died: %s", tb)
        for c in conns:
            try:
                c.send(("dead", tb))
            except OSError:
                pass
        # never recover in place (engine/health.py): give the shutdown a bounded chance
        # (it may block on a collective with a dead rank), then exit non-zero
        t = threading.Thread(target=eng.shutdown, daemon=True)
        t.start()
        t.join(10)
        os._exit(1)
    intake.stop = True
    log.info("core loop: %d iterations, %d engine steps; host time: step %.2f s, output "
             "fan-out %.2f s, inbox %.2f s; burst-admission waits %d", st["iters"],
             st["steps"], st["step_s"], st["send_s"], st["inbox_s"], st["coalesce_waits"])
    if adds:
        lat = sorted(r - a for r, a in adds)
        log.info("core intake (last %d requests): %.3f s first -> last receive; frontend -> core "
                 "latency p50 %.2f ms, max %.2f ms", len(adds), adds[-1][0] - adds[0][0],
                 1e3 * lat[len(lat) // 2], 1e3 * lat[-1])
    eng.shutdown()


def start_core(cfg: EngineConfig, address: str, authkey: bytes, n_frontends: int):
    """Start an engine core serving ``n_frontends`` API processes over the unix socket
    ``address`` (``--api-server-count``); each attaches with
    ``EngineCoreClient(cfg, connect=(address, authkey))``."""
    ctx = mp.get_context("spawn")
    proc = ctx.Process(target=_core_main, args=(cfg, None, (address, authkey, n_frontends)),
                       name="kgc-engine-core")
    proc.start()
    return proc


# ---------------------------------------------------------------------------- API side
class _Stream:
    __slots__ = ("loop", "q", "prompt", "ids")

    def __init__(self, loop, q, prompt):
        self.loop, self.q, self.prompt, self.ids = loop, q, prompt, []


class EngineCoreClient:
    def __init__(self, cfg: EngineConfig, startup_timeout: float = 3600.0,
                 connect: Optional[tuple] = None, core_proc=None):
        """Spawn a private engine core (default), or attach to a shared one at
        ``connect = (address, authkey)``; ``core_proc`` is given in the process that
        started the shared core (liveness and shutdown)."""
        self.cfg = cfg
        if connect is None:
            ctx = mp.get_context("spawn")
            self._conn, child = ctx.Pipe(duplex=True)
            self._proc = ctx.Process(target=_core_main, args=(cfg, child), name="kgc-engine-core")
            self._proc.start()
            child.close()
        else:
            from multiprocessing.connection import Client
            self._proc = core_proc
            deadline = time.monotonic() + startup_timeout
            while True:              # the core binds its socket before loading weights
                try:
                    self._conn = Client(connect[0], authkey=connect[1])
                    break
                except (FileNotFoundError, ConnectionRefusedError):
                    if time.monotonic() > deadline:
                        raise RuntimeError("engine core socket never appeared")
                    time.sleep(0.2)
        if not self._conn.poll(startup_timeout):
            if self._proc is not None:
                self._proc.kill()
            raise RuntimeError("engine core did not start in time")
        kind, info = self._conn.recv()
        if kind != "ready":
            if self._proc is not None:
                self._proc.join(10)
            raise RuntimeError(f"engine core failed to start:\n{info}")
        self.mcfg = info["mcfg"]
        self.max_model_len = info["max_model_len"]
        self.error: Optional[str] = None
        self._streams: dict[str, _Stream] = {}
        self._send_lock = threading.Lock()
        # streams dropped unfinished (RequestStream.__del__): aborted from a normal context,
        # never from the finalizer, which may run while this thread holds _send_lock
        self._dropped: collections.deque = collections.deque()
        self._metrics_waiters: dict[int, tuple] = {}
        self._tokens = itertools.count()
        self._reader = threading.Thread(target=self._read_loop, name="kgc-core-reader", daemon=True)
        self._reader.start()

    # the api server reads these through ``engine.engine`` in thread mode
    @property
    def engine(self):
        return self

    def _send(self, msg) -> None:
        """msg None: only the aborts of dropped streams."""
        with self._send_lock:
            while self._dropped:
                self._conn.send(("abort", self._dropped.popleft()))
            if msg is not None:
                self._conn.send(msg)

    def _read_loop(self) -> None:
        try:
            while True:
                msg = self._conn.recv()
                kind = msg[0]
                if kind == "out":
                    by_loop: dict = {}
                    for rid, new, fin, reason, arr, ftt, ft, npre, lps in msg[1]:
                        st = self._streams.get(rid) if not fin else self._streams.pop(rid, None)
                        if st is None:
                            continue
                        st.ids.extend(new)
                        o = RequestOutput(rid, st.prompt, new, st.ids, len(st.ids), fin, reason,
                                          arr, ftt, ft, npre, lps)
                        by_loop.setdefault(st.loop, []).append((st.q, o))
                    for loop, items in by_loop.items():
                        loop.call_soon_threadsafe(_deliver, items)
                elif kind == "reject":
                    st = self._streams.get(msg[1])
                    if st is not None:
                        st.loop.call_soon_threadsafe(st.q.put_nowait, ValueError(msg[2]))
                elif kind in ("metrics", "stats"):
                    w = self._metrics_waiters.pop(msg[1], None)
                    if w is not None:
                        loop, fut = w
                        loop.call_soon_threadsafe(fut.set_result, msg[2])
                elif kind == "dead":
                    self.error = msg[1]
                    break
        except (EOFError, OSError) as e:
            self.error = self.error or f"engine core connection lost: {e}"
        log.error("engine core is gone: %s", self.error)
        err = EngineDeadError("engine core died")
        for st in list(self._streams.values()):
            st.loop.call_soon_threadsafe(st.q.put_nowait, err)

    @property
    def is_alive(self) -> bool:
        return self.error is None and (self._proc is None or self._proc.is_alive())

    def generate(self, prompt_ids: list[int], params: SamplingParams,
                 request_id: str) -> AsyncIterator[RequestOutput]:
        """Submit NOW (from the request handler, before the response starts streaming: a
        burst of arrivals reaches the core while the frontend is still parsing the rest)
        and return the request's output stream."""
        if not self.is_alive:
            raise EngineDeadError(str(self.error))
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        self._streams[request_id] = _Stream(loop, q, list(prompt_ids))
        self._send(("add", request_id, list(prompt_ids), params, time.monotonic()))
        return RequestStream(request_id, q, self._close_stream, self._drop_stream)

    def _close_stream(self, request_id: str, abort: bool) -> None:
        self._streams.pop(request_id, None)
        if abort and self.is_alive:
            self.abort(request_id)

    def _drop_stream(self, request_id: str) -> None:
        """Finalizer path, lock-free: record the id and schedule the abort on the stream's
        event loop (call_soon_threadsafe appends to the loop's ready deque and writes its
        self-pipe -- no lock); _send also drains the backlog before its next message."""
        st = self._streams.pop(request_id, None)
        self._dropped.append(request_id)
        if st is not None:
            try:
                st.loop.call_soon_threadsafe(self._drain_dropped)
            except RuntimeError:        # loop closed: the next _send drains it
                pass

    def _drain_dropped(self) -> None:
        if self._dropped and self.is_alive:
            try:
                self._send(None)
            except OSError:
                pass

    def abort(self, request_id: str) -> None:
        try:
            self._send(("abort", request_id))
        except OSError:
            pass

    async def metrics_text(self) -> str:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        tok = next(self._tokens)
        self._metrics_waiters[tok] = (loop, fut)
        self._send(("metrics", tok))
        return await asyncio.wait_for(fut, 10)

    async def engine_stats(self, since: float = 0.0) -> dict:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        tok = next(self._tokens)
        self._metrics_waiters[tok] = (loop, fut)
        self._send(("stats", tok, since))
        return await asyncio.wait_for(fut, 10)

    def shutdown(self) -> None:
        if self._proc is None:            # attached to a shared core: just detach
            try:
                self._conn.close()
            except OSError:
                pass
            return
        try:
            self._send(("shutdown",))
        except OSError:
            pass
        self._proc.join(60)
        if self._proc.is_alive():
            self._proc.kill()
