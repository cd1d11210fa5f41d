"""Fault injection on the CPU path (gloo): multi-rank failures end the serving process
with a non-zero exit instead of hanging or serving garbage (engine/health.py).  The
reference relies on Kubernetes restarting pods whose health checks fail
(/root/reference/multi-cp.md:66-72,102-111); these tests pin our half of that contract."""
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.request

import psutil
import pytest

from kubernetes_gpu_cluster_amd.engine import health

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _get(url, timeout=2.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status
    except urllib.error.HTTPError as e:
        return e.code
    except OSError:
        return None


def _rank_process(root_pid: int):
    """The spawned TP rank: a grandchild of the API server (server -> engine core ->
    rank 1); RANK is set after spawn, so /proc environ cannot name it."""
    for core in psutil.Process(root_pid).children():
        for p in core.children():
            try:
                cmd = " ".join(p.cmdline())
            except (psutil.NoSuchProcess, psutil.AccessDenied):
                continue
            if "spawn_main" in cmd and "resource_tracker" not in cmd:
                return p
    return None


@pytest.mark.timeout(300)
def test_tp_rank_death_exits_api_server(tmp_path):
    """TP=2 API server; SIGKILL rank 1 while a stream is running -> the server process
    exits non-zero within 30 s (and answers 503 on /health meanwhile)."""
    port = _port()
    log = open(tmp_path / "server.log", "w")
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1", KGC_STEP_TIMEOUT="60")
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_cluster_amd.entrypoints.api_server",
                          "tiny-llama", "--load-format", "dummy", "--device", "cpu",
                          "--dtype", "float32", "--tensor-parallel-size", "2",
                          "--max-model-len", "256", "--max-num-seqs", "4",
                          "--api-server-count", "1", "--host", "127.0.0.1",
                          "--port", str(port)], stdout=log, stderr=subprocess.STDOUT, env=env,
                         cwd=REPO)
    try:
        t0 = time.time()
        while _get(f"http://127.0.0.1:{port}/health") != 200:
            assert p.poll() is None, (tmp_path / "server.log").read_text()
            assert time.time() - t0 < 180, "server never became healthy"
            time.sleep(0.5)
        rank1 = _rank_process(p.pid)
        assert rank1 is not None, "rank 1 process not found"

        def stream():
            body = json.dumps({"prompt": [5, 6, 7], "max_tokens": 200, "stream": True,
                               "ignore_eos": True}).encode()
            req = urllib.request.Request(f"http://127.0.0.1:{port}/v1/completions", body,
                                         {"content-type": "application/json"})
            try:
                with urllib.request.urlopen(req, timeout=60) as r:
                    for _ in r:
                        pass
            except OSError:
                pass
        th = threading.Thread(target=stream, daemon=True)
        th.start()
        time.sleep(1.0)
        os.kill(rank1.pid, signal.SIGKILL)
        killed = time.time()
        rc = p.wait(timeout=30)
        assert rc != 0, f"server exited 0 after a rank died\n{(tmp_path / 'server.log').read_text()}"
        assert time.time() - killed < 30
        # either the rank watchdog saw the exit code first, or the collective with the
        # dead peer failed first and the core died on that step -- both end the server
        text = (tmp_path / "server.log").read_text()
        assert ("exited with code" in text or "engine core died" in text
                or "engine is dead" in text), text[-3000:]
    finally:
        if p.poll() is None:
            p.kill()
        for c in psutil.Process().children(recursive=True):
            try:
                c.kill()
            except psutil.NoSuchProcess:
                pass
        log.close()


class _FakeProc:
    def __init__(self, code=None):
        self.exitcode, self.pid, self.name = code, 1234, "rank-1"


def test_watchdog_reports_dead_rank_and_stuck_step():
    hits = []
    w = health.RankWatchdog([_FakeProc()], step_timeout=0.2, poll=0.05,
                            on_fatal=lambda c, m: hits.append((c, m)))
    assert w.check_once() is None
    w.step_begin()
    time.sleep(0.3)
    code, msg = w.check_once()
    assert code == health.EXIT_STEP_TIMEOUT and "no progress" in msg
    w.step_end()
    assert w.check_once() is None                 # progress resets the deadline
    w.procs[0].exitcode = -9
    code, msg = w.check_once()
    assert code == health.EXIT_RANK_DEAD and "-9" in msg
    w.start()
    time.sleep(0.3)
    assert hits and hits[0][0] == health.EXIT_RANK_DEAD
    w.stop()


def test_parent_watch_fires_when_parent_changes(monkeypatch):
    hits = []
    ppids = iter([100, 100, 1])
    monkeypatch.setattr(os, "getppid", lambda: next(ppids, 1))
    health.watch_parent(poll=0.01, on_fatal=lambda c, m: hits.append(c))
    time.sleep(0.2)
    assert hits == [health.EXIT_PARENT_DEAD]
