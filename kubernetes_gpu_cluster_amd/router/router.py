"""Request router in front of the engine pods (the reference's production-stack
router behind ``svc/vllm-router-service`` port 80; ``old_README.md:1175,1473-1476``).

* Backend discovery: a static list (``--backends``), Kubernetes pod discovery
  through the API server (``--k8s-label-selector``, in-cluster service-account
  credentials; pods labelled ``app.kubernetes.io/component=serving-engine`` by the
  chart), or DNS of a headless Service (``--dns-service``).
* Model-aware routing: each backend's ``/v1/models`` is polled; a request goes to
  a healthy backend serving its ``model`` (any backend if unspecified).
* Policies: ``least-outstanding`` (default), ``round-robin``, ``session`` (sticky by
  the ``x-session-id`` header / ``user`` field, consistent hashing).
* Failure handling: periodic ``/health`` probes eject unhealthy backends; a
  connection error or 5xx before any byte was relayed is retried on another
  backend (failover); SSE streams are relayed chunk by chunk.
* ``/v1/models`` (union), ``/health``, ``/metrics`` (router Prometheus metrics).
* ``--workers K``: K router processes accept on ONE port (SO_REUSEPORT) and share the
  backends' in-flight counts through shared memory (each worker owns one row of a
  [K x slots] table and least-outstanding reads the column sums), so the DP replicas
  behind one service endpoint stay balanced while the SSE relaying -- one event per
  token per stream -- is spread over K cores instead of saturating one.
"""
from __future__ import annotations

import argparse
import asyncio
import bisect
import hashlib
import itertools
import json
import logging
import os
import sys
import ssl
import time
from typing import Optional

import aiohttp
from aiohttp import web
from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

log = logging.getLogger("kgc.router")

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class Backend:
    def __init__(self, url: str):
        self.url = url.rstrip("/")
        self.healthy = True
        self.outstanding = 0
        self.models: set[str] = set()
        self.fails = 0
        self.last_ok = 0.0

    def __repr__(self):
        return f"Backend({self.url}, healthy={self.healthy}, out={self.outstanding})"


class SharedOutstanding:
    """In-flight requests per backend, shared by the worker processes of one router:
    a RawArray of [workers x slots] int64, row w written only by worker w (no lock, no
    lost updates); a backend's global count is its column sum.  Backends map to slots
    by URL hash (a collision only merges two backends' counts)."""

    SLOTS = 1024

    def __init__(self, workers: int):
        import multiprocessing as mp
        self.workers = workers
        self.arr = mp.RawArray("q", workers * self.SLOTS)
        # pick + reserve is one critical section across the workers: a burst of
        # simultaneous arrivals is spread exactly evenly (a DP replica that gets even a
        # few requests over its max_num_seqs serves them as a second, serial wave)
        self.lock = mp.Lock()
        self.row = 0

    @classmethod
    def slot(cls, url: str) -> int:
        return int.from_bytes(hashlib.blake2b(url.encode(), digest_size=4).digest(), "big") % cls.SLOTS

    def add(self, url: str, d: int) -> None:
        self.arr[self.row * self.SLOTS + self.slot(url)] += d

    def total(self, url: str) -> int:
        j = self.slot(url)
        return sum(self.arr[w * self.SLOTS + j] for w in range(self.workers))


class Router:
    def __init__(self, backends: list[str], policy: str = "least-outstanding",
                 health_interval: float = 5.0, fail_threshold: int = 2,
                 k8s_selector: Optional[str] = None, k8s_namespace: Optional[str] = None,
                 k8s_port: int = 8000, dns_service: Optional[str] = None, max_retries: int = 2,
                 request_timeout: float = 3600.0, backend_api_key: Optional[str] = None,
                 shared: Optional[SharedOutstanding] = None):
        self.shared = shared
        # engines started with --api-key: the router's own /v1/models polls carry the key
        # (client requests are proxied with their own Authorization header)
        self._poll_headers = ({"Authorization": f"Bearer {backend_api_key}"}
                              if backend_api_key else {})
        self.backends: dict[str, Backend] = {u.rstrip("/"): Backend(u) for u in backends}
        self.policy = policy
        self.health_interval = health_interval
        self.fail_threshold = fail_threshold
        self.k8s_selector, self.k8s_namespace, self.k8s_port = k8s_selector, k8s_namespace, k8s_port
        self.dns_service = dns_service
        self.max_retries = max_retries
        self.timeout = aiohttp.ClientTimeout(total=request_timeout, sock_connect=5)
        self._rr = itertools.count()
        self.session: Optional[aiohttp.ClientSession] = None
        self._tasks: list[asyncio.Task] = []
        r = self.registry = CollectorRegistry()
        self.m_req = Counter("kgc_router_requests", "requests", ["backend", "status"], registry=r)
        self.m_lat = Histogram("kgc_router_request_seconds", "latency", ["route"], registry=r)
        self.m_out = Gauge("kgc_router_outstanding", "in-flight per backend", ["backend"], registry=r)
        self.m_healthy = Gauge("kgc_router_healthy_backends", "healthy backends", registry=r)
        self.m_retry = Counter("kgc_router_retries", "failover retries", registry=r)

    # ------------------------------------------------------------------ lifecycle
    async def start(self, app=None):
        # no connection cap: aiohttp's default (100 total) would silently queue every
        # request past the 100th, starving an engine that batches 256+ sequences
        conn = aiohttp.TCPConnector(limit=0, limit_per_host=0, keepalive_timeout=60)
        self.session = aiohttp.ClientSession(timeout=self.timeout, connector=conn)
        await self.refresh_discovery()
        await self.check_health()
        self._tasks.append(asyncio.create_task(self._health_loop()))

    async def stop(self, app=None):
        for t in self._tasks:
            t.cancel()
        if self.session:
            await self.session.close()

    async def _health_loop(self):
        while True:
            await asyncio.sleep(self.health_interval)
            try:
                await self.refresh_discovery()
                await self.check_health()
            except Exception as e:  # noqa: BLE001
                log.warning("health loop: %s", e)

    # ------------------------------------------------------------------ discovery
    async def refresh_discovery(self):
        urls = None
        if self.k8s_selector:
            urls = await self._k8s_pods()
        elif self.dns_service:
            urls = await self._dns()
        if urls is None:
            return
        for u in urls:
            self.backends.setdefault(u, Backend(u))
        for u in list(self.backends):
            if u not in urls:
                del self.backends[u]

    async def _k8s_pods(self) -> Optional[list[str]]:
        host = os.environ.get("KUBERNETES_SERVICE_HOST")
        if not host or not os.path.exists(f"{SA_DIR}/token"):
            return None
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        ns = self.k8s_namespace or open(f"{SA_DIR}/namespace").read().strip()
        token = open(f"{SA_DIR}/token").read().strip()
        ctx = ssl.create_default_context(cafile=f"{SA_DIR}/ca.crt")
        url = f"https://{host}:{port}/api/v1/namespaces/{ns}/pods"
        async with self.session.get(url, params={"labelSelector": self.k8s_selector},
                                    headers={"Authorization": f"Bearer {token}"}, ssl=ctx) as r:
            data = await r.json()
        return pods_to_urls(data, self.k8s_port)

    async def _dns(self) -> Optional[list[str]]:
        host, _, port = self.dns_service.partition(":")
        loop = asyncio.get_running_loop()
        try:
            infos = await loop.getaddrinfo(host, int(port or 8000))
        except OSError:
            return []
        return sorted({f"http://{i[4][0]}:{i[4][1]}" for i in infos})

    # ------------------------------------------------------------------ health
    async def _probe(self, b: Backend):
        try:
            async with self.session.get(b.url + "/health", timeout=aiohttp.ClientTimeout(total=3)) as r:
                ok = r.status == 200
            if ok and not b.models:
                async with self.session.get(b.url + "/v1/models", headers=self._poll_headers,
                                            timeout=aiohttp.ClientTimeout(total=3)) as r:
                    if r.status == 200:
                        b.models = {m["id"] for m in (await r.json()).get("data", [])}
        except Exception:  # noqa: BLE001
            ok = False
        if ok:
            b.fails, b.healthy, b.last_ok = 0, True, time.monotonic()
        else:
            b.fails += 1
            if b.fails >= self.fail_threshold:
                b.healthy = False

    async def check_health(self):
        await asyncio.gather(*(self._probe(b) for b in list(self.backends.values())))
        self.m_healthy.set(sum(b.healthy for b in self.backends.values()))

    # ------------------------------------------------------------------ selection
    def candidates(self, model: Optional[str]) -> list[Backend]:
        hs = [b for b in self.backends.values() if b.healthy]
        if model:
            m = [b for b in hs if not b.models or model in b.models]
            if m:
                return m
        return hs

    def pick(self, model: Optional[str], session_key: Optional[str] = None,
             exclude: set = frozenset()) -> Optional[Backend]:
        """Choose a backend and count the request against it (``release`` undoes it)."""
        cs = [b for b in self.candidates(model) if b.url not in exclude]
        if not cs:
            return None
        if self.shared is None:
            b = self._choose(cs, session_key, {b.url: b.outstanding for b in cs})
        else:
            with self.shared.lock:
                b = self._choose(cs, session_key, None)
                self.shared.add(b.url, 1)
        b.outstanding += 1
        self.m_out.labels(b.url).set(b.outstanding)
        return b

    def release(self, b: Backend) -> None:
        b.outstanding -= 1
        if self.shared is not None:
            self.shared.add(b.url, -1)
        self.m_out.labels(b.url).set(b.outstanding)

    def _choose(self, cs: list[Backend], session_key: Optional[str], load) -> Backend:
        if self.policy == "round-robin":
            return cs[next(self._rr) % len(cs)]
        if self.policy == "session" and session_key:
            return consistent_pick(cs, session_key)
        if load is None:
            load = {b.url: self.shared.total(b.url) for b in cs}
        lo = min(load.values())
        ties = [b for b in cs if load[b.url] == lo]
        return ties[next(self._rr) % len(ties)]

    # ------------------------------------------------------------------ proxy
    async def proxy(self, request: web.Request) -> web.StreamResponse:
        t0 = time.monotonic()
        body = await request.read()
        model = skey = None
        try:
            j = json.loads(body) if body else {}
            model = j.get("model")
            skey = request.headers.get("x-session-id") or j.get("user")
        except (ValueError, AttributeError):
            pass
        tried: set = set()
        for attempt in range(self.max_retries + 1):
            b = self.pick(model, skey, tried)
            if b is None:
                return web.json_response({"error": "no healthy backend" + (f" for model {model}" if model else "")},
                                         status=503)
            tried.add(b.url)
            resp: Optional[web.StreamResponse] = None
            try:
                hdrs = {k: v for k, v in request.headers.items()
                        if k.lower() not in ("host", "content-length", "transfer-encoding")}
                async with self.session.request(request.method, b.url + request.path_qs,
                                                data=body, headers=hdrs) as up:
                    if up.status >= 500 and attempt < self.max_retries:
                        b.fails += 1
                        self.m_req.labels(b.url, str(up.status)).inc()
                        self.m_retry.inc()
                        continue
                    resp = web.StreamResponse(status=up.status, headers={
                        k: v for k, v in up.headers.items()
                        if k.lower() in ("content-type", "cache-control")})
                    await resp.prepare(request)
                    async for chunk in up.content.iter_any():
                        await resp.write(chunk)
                    await resp.write_eof()
                    self.m_req.labels(b.url, str(up.status)).inc()
                    self.m_lat.labels(request.path).observe(time.monotonic() - t0)
                    return resp
            except (aiohttp.ClientConnectionError, asyncio.TimeoutError) as e:
                self.m_req.labels(b.url, "conn_error").inc()
                b.fails += 1
                if b.fails >= self.fail_threshold:
                    b.healthy = False
                if resp is not None:       # bytes already relayed: cannot fail over
                    return resp
                self.m_retry.inc()
                log.warning("backend %s failed (%s); failing over", b.url, e)
            finally:
                self.release(b)
        return web.json_response({"error": "all backends failed"}, status=502)

    async def models(self, request: web.Request) -> web.Response:
        seen, data = set(), []
        for b in self.backends.values():
            if not b.healthy:
                continue
            for m in sorted(b.models):
                if m not in seen:
                    seen.add(m)
                    data.append({"id": m, "object": "model", "owned_by": "kgc"})
        return web.json_response({"object": "list", "data": data})

    async def health(self, request: web.Request) -> web.Response:
        n = sum(b.healthy for b in self.backends.values())
        return web.Response(text=f"ok ({n} healthy backends)", status=200 if n else 503)

    async def metrics(self, request: web.Request) -> web.Response:
        return web.Response(body=generate_latest(self.registry), content_type="text/plain")

    def app(self) -> web.Application:
        a = web.Application(client_max_size=64 << 20)
        a.router.add_get("/v1/models", self.models)
        a.router.add_get("/health", self.health)
        a.router.add_get("/metrics", self.metrics)
        a.router.add_route("*", "/v1/{tail:.*}", self.proxy)
        a.router.add_post("/tokenize", self.proxy)       # vLLM's (de)tokenizer endpoints
        a.router.add_post("/detokenize", self.proxy)
        a.on_startup.append(self.start)
        a.on_cleanup.append(self.stop)
        return a


def pods_to_urls(pod_list: dict, port: int) -> list[str]:
    """Ready, running pods with an IP -> base URLs."""
    urls = []
    for p in pod_list.get("items", []):
        st = p.get("status", {})
        if st.get("phase") != "Running" or not st.get("podIP"):
            continue
        conds = {c.get("type"): c.get("status") for c in st.get("conditions", [])}
        if conds.get("Ready") == "False":
            continue
        urls.append(f"http://{st['podIP']}:{port}")
    return sorted(urls)


def consistent_pick(backends: list[Backend], key: str, vnodes: int = 64) -> Backend:
    ring = []
    for b in backends:
        for v in range(vnodes):
            h = int.from_bytes(hashlib.md5(f"{b.url}#{v}".encode()).digest()[:8], "big")
            ring.append((h, b))
    ring.sort(key=lambda x: x[0])
    h = int.from_bytes(hashlib.md5(key.encode()).digest()[:8], "big")
    i = bisect.bisect([r[0] for r in ring], h)
    return ring[i % len(ring)][1]


def main(argv=None):
    p = argparse.ArgumentParser(description="kgc request router")
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8080)
    p.add_argument("--backends", default="", help="comma-separated engine base URLs")
    p.add_argument("--k8s-label-selector", default=None)
    p.add_argument("--k8s-namespace", default=None)
    p.add_argument("--k8s-port", type=int, default=8000)
    p.add_argument("--dns-service", default=None, help="headless service host[:port]")
    p.add_argument("--routing-logic", "--policy", dest="policy", default="least-outstanding",
                   choices=["least-outstanding", "round-robin", "session"])
    p.add_argument("--health-interval", type=float, default=5.0)
    p.add_argument("--access-log", action="store_true", help="log every proxied request")
    p.add_argument("--backend-api-key", default=os.environ.get("VLLM_API_KEY"),
                   help="bearer key for the router's own /v1/models polls of engines that "
                        "run with --api-key (env VLLM_API_KEY)")
    p.add_argument("--workers", type=int, default=1,
                   help="router processes sharing the port (SO_REUSEPORT) and the backends' "
                        "in-flight counts; 0 = one per 2 CPUs, at most 8")
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if not a.access_log:
        logging.getLogger("aiohttp.access").setLevel(logging.WARNING)
    workers = a.workers if a.workers > 0 else max(1, min(8, (os.cpu_count() or 2) // 2))

    def serve(shared: Optional[SharedOutstanding]):
        r = Router([u for u in a.backends.split(",") if u], a.policy, a.health_interval,
                   k8s_selector=a.k8s_label_selector, k8s_namespace=a.k8s_namespace,
                   k8s_port=a.k8s_port, dns_service=a.dns_service,
                   backend_api_key=a.backend_api_key, shared=shared)
        # the banner goes to stderr: a launcher's stdout (bench.py's one JSON line) stays clean
        web.run_app(r.app(), host=a.host, port=a.port, reuse_port=workers > 1,
                    print=None if workers > 1 else
                    (lambda *m, **k: print(*m, file=sys.stderr, flush=True)))

    if workers == 1:
        serve(None)
        return
    shared = SharedOutstanding(workers)
    run_workers(workers, shared, serve)


def run_workers(workers: int, shared: SharedOutstanding, serve) -> None:
    """Fork ``workers`` processes that each run ``serve(shared)`` on the same port; the
    parent waits, forwards SIGTERM / SIGINT, and exits non-zero if any worker dies."""
    import signal
    pids = []
    for w in range(workers):
        pid = os.fork()
        if pid == 0:
            shared.row = w
            rc = 1                      # a worker that raises (bind failure, crash) exits 1
            try:
                serve(shared)
                rc = 0
            except BaseException:       # noqa: BLE001 - reported, then a non-zero exit
                import traceback
                traceback.print_exc()
            finally:
                os._exit(rc)
        pids.append(pid)

    def stop(signum, frame):
        for pid in pids:
            try:
                os.kill(pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rc = 0
    for _ in pids:
        try:
            _, status = os.wait()
        except ChildProcessError:
            break
        if os.waitstatus_to_exitcode(status) not in (0, -signal.SIGTERM):
            rc = 1
            stop(None, None)
    raise SystemExit(rc)


if __name__ == "__main__":
    main()
