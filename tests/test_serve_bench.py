"""bench/serve_bench.py end to end on CPU: engine server + router subprocesses, streamed
completions through the router, one JSON result line."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_serve_bench_launch_cpu(tmp_path):
    out = tmp_path / "r.json"
    cmd = [sys.executable, os.path.join(ROOT, "bench", "serve_bench.py"), "--launch", "--gpus", "1",
           "--model", "tiny-llama", "--num-prompts", "6", "--input-len", "24", "--output-len", "5",
           "--max-model-len", "128", "--vocab", "1000", "--warmup-prompts", "1",
           "--engine-port", str(_free_port()), "--router-port", str(_free_port()),
           "--startup-timeout", "240", "--json-out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["completed"] == 6 and res["failed"] == 0
    assert res["value"] > 0 and res["p50_ttft_ms"] > 0
