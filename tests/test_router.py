"""Router: discovery, model-aware least-outstanding routing, failover, SSE relay."""
import asyncio
import json

from aiohttp import web
from aiohttp.test_utils import TestClient, TestServer

from kubernetes_gpu_cluster_amd.router.router import Router, consistent_pick, pods_to_urls, Backend


def fake_engine(name: str, model: str = "m", fail: bool = False):
    app = web.Application()
    app["hits"] = 0

    async def health(r):
        return web.Response(text="ok")

    async def models(r):
        return web.json_response({"data": [{"id": model}]})

    async def comp(r):
        app["hits"] += 1
        if fail:
            return web.Response(status=500, text="boom")
        body = await r.json()
        if body.get("stream"):
            resp = web.StreamResponse(headers={"content-type": "text/event-stream"})
            await resp.prepare(r)
            for i in range(3):
                await resp.write(f"data: {json.dumps({'i': i, 'be': name})}\n\n".encode())
            await resp.write(b"data: [DONE]\n\n")
            await resp.write_eof()
            return resp
        return web.json_response({"backend": name, "model": body.get("model")})

    app.router.add_get("/health", health)
    app.router.add_get("/v1/models", models)
    app.router.add_post("/v1/completions", comp)

    async def tokenize(r):
        body = await r.json()
        return web.json_response({"backend": name, "count": len(body.get("prompt", ""))})
    app.router.add_post("/tokenize", tokenize)
    return app


async def _scenario():
    servers = [TestServer(fake_engine("a", "m1")), TestServer(fake_engine("b", "m1")),
               TestServer(fake_engine("c", "m2")), TestServer(fake_engine("bad", "m1", fail=True))]
    for s in servers:
        await s.start_server()
    urls = [str(s.make_url("")) for s in servers]
    r = Router(urls, health_interval=3600)
    client = TestClient(TestServer(r.app()))
    await client.start_server()
    try:
        # model union
        j = await (await client.get("/v1/models")).json()
        assert {m["id"] for m in j["data"]} == {"m1", "m2"}
        # m2 only on c
        for _ in range(3):
            j = await (await client.post("/v1/completions", json={"model": "m2", "prompt": "x"})).json()
            assert j["backend"] == "c"
        # m1 spread over a, b (and 'bad' fails over)
        seen = set()
        for _ in range(12):
            resp = await client.post("/v1/completions", json={"model": "m1", "prompt": "x"})
            assert resp.status == 200
            seen.add((await resp.json())["backend"])
        assert seen == {"a", "b"}
        assert r.m_retry._value.get() > 0
        # /tokenize is routed by model like the /v1 endpoints
        j = await (await client.post("/tokenize", json={"model": "m2", "prompt": "abc"})).json()
        assert j["backend"] == "c" and j["count"] == 3
        # SSE relay
        resp = await client.post("/v1/completions", json={"model": "m1", "stream": True})
        text = await resp.text()
        assert text.count("data: ") == 4 and text.strip().endswith("[DONE]")
        # a dead backend is ejected by health probes
        await servers[0].close()
        await r.check_health()
        await r.check_health()
        assert not r.backends[urls[0].rstrip("/")].healthy
        for _ in range(4):
            j = await (await client.post("/v1/completions", json={"model": "m1"})).json()
            assert j["backend"] == "b"
        h = await client.get("/health")
        assert h.status == 200
        m = await (await client.get("/metrics")).text()
        assert "kgc_router_requests_total" in m
    finally:
        await client.close()
        for s in servers:
            await s.close()


def test_router_end_to_end():
    asyncio.run(_scenario())


def test_pods_to_urls_and_consistent_hash():
    pods = {"items": [
        {"status": {"phase": "Running", "podIP": "10.0.0.2", "conditions": [{"type": "Ready", "status": "True"}]}},
        {"status": {"phase": "Pending", "podIP": "10.0.0.3"}},
        {"status": {"phase": "Running", "podIP": "10.0.0.4", "conditions": [{"type": "Ready", "status": "False"}]}},
    ]}
    assert pods_to_urls(pods, 8000) == ["http://10.0.0.2:8000"]
    bs = [Backend(f"http://h{i}:1") for i in range(4)]
    picks = {k: consistent_pick(bs, k).url for k in ("u1", "u2", "u3")}
    assert picks == {k: consistent_pick(bs, k).url for k in picks}   # stable


async def _concurrency_scenario(n=300):
    """More concurrent streams than aiohttp's default connector cap (100): all must be
    in flight at the backend at the same time, none queued in the router."""
    app = web.Application()
    state = {"live": 0, "peak": 0}
    gate = asyncio.Event()

    async def health(r):
        return web.Response(text="ok")

    async def models(r):
        return web.json_response({"data": [{"id": "m"}]})

    async def comp(r):
        state["live"] += 1
        state["peak"] = max(state["peak"], state["live"])
        if state["live"] >= n:
            gate.set()
        resp = web.StreamResponse(headers={"content-type": "text/event-stream"})
        await resp.prepare(r)
        await asyncio.wait_for(gate.wait(), 30)
        await resp.write(b"data: {}\n\ndata: [DONE]\n\n")
        await resp.write_eof()
        state["live"] -= 1
        return resp

    app.router.add_get("/health", health)
    app.router.add_get("/v1/models", models)
    app.router.add_post("/v1/completions", comp)
    be = TestServer(app)
    await be.start_server()
    r = Router([str(be.make_url(""))], health_interval=3600)
    client = TestClient(TestServer(r.app()))
    await client.start_server()
    import aiohttp
    sess = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0))
    try:
        async def one():
            async with sess.post(client.make_url("/v1/completions"),
                                 json={"model": "m", "stream": True}) as resp:
                return await resp.text()
        outs = await asyncio.gather(*[one() for _ in range(n)])
        assert all(o.endswith("[DONE]\n\n") for o in outs)
        assert state["peak"] == n
    finally:
        await sess.close()
        await client.close()
        await be.close()


def test_router_has_no_connection_cap():
    asyncio.run(_concurrency_scenario())


async def _multiworker_scenario(nbe=4, per=64, workers=3):
    """``--workers K``: K router processes on one port (SO_REUSEPORT) share the backends'
    in-flight counts, so a burst of nbe * per simultaneous streams lands exactly ``per``
    on every backend (a replica given more than its max_num_seqs would serve the surplus
    as a second, serial wave)."""
    import os
    import socket
    import subprocess
    import sys
    import time
    import aiohttp
    import psutil
    n = nbe * per
    hits = [0] * nbe
    gate = asyncio.Event()

    def make(i):
        app = web.Application()

        async def health(r):
            return web.Response(text="ok")

        async def models(r):
            return web.json_response({"data": [{"id": "m"}]})

        async def comp(r):
            hits[i] += 1
            if sum(hits) >= n:
                gate.set()
            resp = web.StreamResponse(headers={"content-type": "text/event-stream"})
            await resp.prepare(r)
            await asyncio.wait_for(gate.wait(), 60)
            await resp.write(f"data: {i}\n\ndata: [DONE]\n\n".encode())
            await resp.write_eof()
            return resp
        app.router.add_get("/health", health)
        app.router.add_get("/v1/models", models)
        app.router.add_post("/v1/completions", comp)
        return app

    bes = [TestServer(make(i)) for i in range(nbe)]
    for b in bes:
        await b.start_server()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    proc = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_cluster_amd.router.router",
                             "--host", "127.0.0.1", "--port", str(port), "--workers", str(workers),
                             "--backends", ",".join(str(b.make_url("")) for b in bes)],
                            cwd=root, env=dict(os.environ, PYTHONPATH=root))
    url = f"http://127.0.0.1:{port}"
    sess = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0, force_close=True))
    try:
        deadline = time.monotonic() + 60
        while True:
            try:
                async with sess.get(url + "/health") as r:
                    if r.status == 200:
                        break
            except aiohttp.ClientError:
                pass
            assert time.monotonic() < deadline and proc.poll() is None
            await asyncio.sleep(0.2)
        assert len(psutil.Process(proc.pid).children()) == workers

        async def one():
            async with sess.post(url + "/v1/completions", json={"model": "m", "stream": True}) as r:
                return await r.text()
        outs = await asyncio.gather(*[one() for _ in range(n)])
        assert all(o.endswith("[DONE]\n\n") for o in outs)
        assert hits == [per] * nbe, hits
    finally:
        await sess.close()
        proc.terminate()
        proc.wait(30)
        for b in bes:
            await b.close()
    assert proc.returncode == 0, proc.returncode


def test_router_workers_share_load_exactly():
    asyncio.run(_multiworker_scenario())


def test_run_workers_exits_nonzero_when_a_worker_raises():
    import os
    """A forked router worker whose serve() raises (bind failure, crash) exits 1, and the
    parent stops the others and exits non-zero -- never a silent 0."""
    import subprocess
    import sys
    code = r'''
import os, sys, time
from kubernetes_gpu_cluster_amd.router.router import run_workers, SharedOutstanding

def serve(shared):
    if shared.row == 1:
        raise OSError("address already in use")
    time.sleep(30)

try:
    run_workers(2, SharedOutstanding(2), serve)
except SystemExit as e:
    sys.exit(e.code)
'''
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 1, (r.returncode, r.stderr[-2000:])
    assert "address already in use" in r.stderr
