"""bench.py's driver contract on the CPU path: one JSON line from rank 0, whole-job
aggregates, 1 rank and 2 ranks (torch.distributed.run, gloo) for dp and tp; the default
service mode launches API server + router per replica and streams over HTTP."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--model", "tiny-llama", "--num-prompts", "4", "--input-len", "16",
         "--output-len", "4", "--max-num-seqs", "4", "--max-num-batched-tokens", "64",
         "--max-model-len", "128", "--steps", "1", "--warmup", "1"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_single_rank():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1"] + SMALL, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    # stdout is the driver's contract: that ONE line and nothing else (the router's
    # aiohttp banner once went there too)
    assert [l for l in r.stdout.splitlines() if l.strip()] == [r.stdout.strip()], r.stdout
    j = lines[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in j
    assert j["n_gpus"] == 1 and j["value"] > 0 and j["config"]["parallelism"] == "dp1"
    # service mode (default): HTTP/SSE numbers plus the engine-side view of the same requests
    assert j["mode"].startswith("service") and j["failed"] == 0 and j["completed"] == 4
    assert j["engine_output_tokens"] == 4 * 4 and j["engine_tok_s"] > 0
    assert j["p50_ttft_ms"] >= j["engine_p50_ttft_ms"] > 0


def test_bench_engine_mode():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--mode", "engine"] + SMALL,
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json_lines(r.stdout)[0]
    assert j["value"] > 0 and j["engine_steps"] > 0 and "mode" not in j


@pytest.mark.parametrize("tp", [1, 2])
def test_bench_two_ranks(tp):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--tp", str(tp)] + SMALL
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == 2
    if tp == 1:
        assert j["config"]["parallelism"] == "dp2" and j["config"]["global_batch"] == 8
        assert j["engine_steps"] > 0
        # ONE service endpoint: rank 0's router (a worker per replica) over both replicas
        assert j["config"]["endpoint"].startswith("one router (2 replica(s))")
        assert j["router_workers"] == 2 and j["router_cpu_util"] is not None
        assert j["engine_output_tokens"] == 8 * 4
    else:
        assert j["config"]["parallelism"] == "tp2" and j["config"]["global_batch"] == 4


def test_client_counts_received_tokens_not_max_tokens():
    """The load generator credits the tokens the server reports in the include_usage
    event before [DONE]; a stream cut short is a failed request worth 0 tokens, so a
    truncating server makes the measured value drop instead of being credited
    max_tokens per request."""
    import asyncio
    import json as _json
    from aiohttp import web
    from aiohttp.test_utils import TestServer
    from kubernetes_gpu_cluster_amd.benchmarks import serving_client as sc

    def app(truncate_every: int):
        state = {"n": 0}

        async def comp(r):
            body = await r.json()
            assert body["stream_options"] == {"include_usage": True}
            state["n"] += 1
            cut = truncate_every and state["n"] % truncate_every == 0
            resp = web.StreamResponse(headers={"content-type": "text/event-stream"})
            await resp.prepare(r)
            n = body["max_tokens"]
            for i in range(n if not cut else 2):
                await resp.write(f'data: {{"choices": [{{"text": "t{i}"}}]}}\n\n'.encode())
            if not cut:
                u = {"choices": [], "usage": {"prompt_tokens": 3, "completion_tokens": n}}
                await resp.write(f"data: {_json.dumps(u)}\n\ndata: [DONE]\n\n".encode())
            await resp.write_eof()
            return resp
        a = web.Application()
        a.router.add_post("/v1/completions", comp)
        return a

    async def run(truncate_every):
        srv = TestServer(app(truncate_every))
        await srv.start_server()
        try:
            async with sc.new_session() as s:
                res, t0, t1 = await sc.run_wave(s, str(srv.make_url("")).rstrip("/"), "m",
                                                [[5, 6, 7]] * 8, 6)
        finally:
            await srv.close()
        return res

    full = asyncio.run(run(0))
    assert all(r.ok and r.tokens == 6 for r in full)
    cut = asyncio.run(run(2))
    assert sum(r.ok for r in cut) == 4 and sum(r.tokens for r in cut) == 4 * 6
    assert sc.summarize(cut, 1.0)["value"] < sc.summarize(full, 1.0)["value"]


def test_fake_engine_dp4_one_router_keeps_up():
    """Router fan-in at DP = 4: four replicas whose engine cores are the
    GPU-free timing model (engine/fake.py, Llama-3-8B step times), all client load
    through rank 0's single multi-worker router.  The service must deliver what the
    engines produce: service tok/s / engine tok/s >= 0.95 with nothing failed.
    The 8-replica, full-config run is recorded in profiles/router_fanin_fake_dp8.jsonl."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "4",
           "--device", "cpu", "--model", "llama-3-8b", "--num-prompts", "128", "--input-len", "256",
           "--output-len", "128", "--steps", "1", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, KGC_FAKE_ENGINE="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_lines(r.stdout)[0]
    assert j["failed"] == 0 and j["completed"] == 4 * 128
    assert j["engine_output_tokens"] == 4 * 128 * 128
    assert j["config"]["endpoint"].startswith("one router (4 replica(s))")
    assert j["router_workers"] == 4
    # the ratio is a throughput claim about the router: it holds on an unloaded host (the
    # driver's serial run); beside 7 other xdist workers the 4 replicas, the router workers
    # and the client compete for 8 CPUs, which measures the host, not the router
    if os.environ.get("PYTEST_XDIST_WORKER") is None:
        assert j["service_vs_engine"] >= 0.95, j
