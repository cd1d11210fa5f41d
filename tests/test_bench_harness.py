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
    else:
        assert j["config"]["parallelism"] == "tp2" and j["config"]["global_batch"] == 4
