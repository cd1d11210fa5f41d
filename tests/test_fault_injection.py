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


def test_adaptive_step_timeout():
    """Without KGC_STEP_TIMEOUT the limit is the warm-up grace for the first steps, then
    max(floor, 10 x the longest step seen) -- tens of seconds, not ten minutes."""
    w = health.RankWatchdog([], poll=0.05, on_fatal=lambda c, m: None)
    w.fixed_timeout = None
    w.floor, w.warmup_timeout = 1.0, 5.0
    assert w.step_timeout == 5.0
    for _ in range(health.WARMUP_STEPS):
        w.step_begin()
        time.sleep(0.01)
        w.step_end()
    assert w.steps_done == health.WARMUP_STEPS
    assert w.step_timeout == 1.0                       # floor: 10 x ~10 ms < 1 s
    w.longest_step = 0.5
    assert w.step_timeout == 5.0
    w.step_begin()
    w._last -= 6.0                                     # a step wedged for 6 s
    code, msg = w.check_once()
    assert code == health.EXIT_STEP_TIMEOUT and "longest 0.5 s" in msg


class _Store:
    def __init__(self):
        self.d = {}
        self.fail = False

    def add(self, k, v):
        if self.fail:
            raise RuntimeError("connection reset by peer")
        self.d[k] = self.d.get(k, 0) + v
        return self.d[k]


def test_heartbeats_both_directions():
    """Driver side: a rank whose heartbeat counter stops moving is reported dead after
    KGC_HEARTBEAT_TIMEOUT.  Rank side: when the store (the driver's process) fails, the
    rank exits EXIT_PARENT_DEAD -- unless a clean shutdown stopped the heartbeat first."""
    st = _Store()
    hb = health.Heartbeat(st, 3, period=0.02, timeout=5, on_fatal=lambda c, m: hits.append(c))
    hits = []
    hb.start()
    w = health.RankWatchdog([], step_timeout=0, poll=0.05, on_fatal=lambda c, m: None)
    w.watch_heartbeats(st, [3])
    w.hb_timeout = 0.3
    for _ in range(10):
        assert w.check_once() is None
        time.sleep(0.05)
    hb.stop()
    time.sleep(0.05)
    assert w.check_once() is None                      # sees the last bump
    time.sleep(0.4)
    code, msg = w.check_once()
    assert code == health.EXIT_RANK_DEAD and "rank 3" in msg
    assert not hits                                    # a stopped heartbeat never fires
    hits2 = []
    st2 = _Store()
    hb2 = health.Heartbeat(st2, 5, period=0.02, timeout=5,
                           on_fatal=lambda c, m: hits2.append(c)).start()
    time.sleep(0.1)
    st2.fail = True
    time.sleep(2.5)                                    # the 2 s clean-shutdown grace
    assert hits2 == [health.EXIT_PARENT_DEAD]
    hb2.stop()


def _two_node_server(tmp_path, port, mport):
    env = dict(os.environ, PYTHONPATH=REPO, KGC_HEARTBEAT_TIMEOUT="10")
    common = ["--load-format", "dummy", "--device", "cpu", "--dtype", "float32",
              "--tensor-parallel-size", "2", "--nnodes", "2", "--master-addr", "127.0.0.1",
              "--master-port", str(mport), "--max-model-len", "256", "--max-num-seqs", "4"]
    slog = open(tmp_path / "server.log", "w")
    wlog = open(tmp_path / "worker.log", "w")
    server = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_cluster_amd.entrypoints.api_server",
                               "tiny-llama", "--node-rank", "0", "--api-server-count", "1",
                               "--host", "127.0.0.1", "--port", str(port)] + common,
                              stdout=slog, stderr=subprocess.STDOUT, env=env, cwd=REPO,
                              start_new_session=True)
    worker = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_cluster_amd.entrypoints.worker_node",
                               "tiny-llama", "--node-rank", "1"] + common,
                              stdout=wlog, stderr=subprocess.STDOUT, env=env, cwd=REPO,
                              start_new_session=True)
    t0 = time.time()
    while _get(f"http://127.0.0.1:{port}/health") != 200:
        assert server.poll() is None, (tmp_path / "server.log").read_text()[-3000:]
        assert worker.poll() is None, (tmp_path / "worker.log").read_text()[-3000:]
        assert time.time() - t0 < 180, "two-node server never became healthy"
        time.sleep(0.5)
    return server, worker, (slog, wlog)


def _start_stream(port):
    def stream():
        body = json.dumps({"prompt": [5, 6, 7], "max_tokens": 200, "stream": True,
                           "ignore_eos": True}).encode()
        req = urllib.request.Request(f"http://127.0.0.1:{port}/v1/completions", body,
                                     {"content-type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=120) as r:
                for _ in r:
                    pass
        except OSError:
            pass
    th = threading.Thread(target=stream, daemon=True)
    th.start()
    time.sleep(1.0)


def _kill_tree(*procs):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass


@pytest.mark.timeout(300)
def test_remote_rank_death_ends_driver(tmp_path):
    """Two-node TP=2 engine (API server = node 0, worker_node = node 1, CPU/gloo): SIGKILL
    the rank on node 1 mid-stream -> the API server exits non-zero within 60 s, and so
    does the worker node."""
    server, worker, logs = _two_node_server(tmp_path, _port(), _port())
    try:
        ranks = [c for c in psutil.Process(worker.pid).children()
                 if "spawn_main" in " ".join(c.cmdline()) and "resource_tracker" not in " ".join(c.cmdline())]
        assert ranks, "node-1 rank not found"
        _start_stream(int(server.args[server.args.index("--port") + 1]))
        os.kill(ranks[0].pid, signal.SIGKILL)
        killed = time.time()
        rc = server.wait(timeout=90)
        assert rc != 0 and time.time() - killed < 60, (tmp_path / "server.log").read_text()[-3000:]
        assert worker.wait(timeout=30) != 0
    finally:
        _kill_tree(server, worker)
        for f in logs:
            f.close()


@pytest.mark.timeout(300)
def test_driver_death_ends_worker_node(tmp_path):
    """The driver's pod dies (SIGKILL of the whole API-server process group): the rank on
    node 1 loses its heartbeat store and exits, ending the worker node non-zero."""
    server, worker, logs = _two_node_server(tmp_path, _port(), _port())
    try:
        os.killpg(server.pid, signal.SIGKILL)
        killed = time.time()
        rc = worker.wait(timeout=90)
        assert rc != 0 and time.time() - killed < 60, (tmp_path / "worker.log").read_text()[-3000:]
    finally:
        _kill_tree(server, worker)
        for f in logs:
            f.close()


def _replica_store_rank(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubernetes_gpu_cluster_amd.parallel.state import init_parallel
    ps = init_parallel(2, 1)                 # 2 ranks per replica -> 2 replicas in 4 ranks
    st = health.replica_store(ps)
    default = health.rendezvous_store()
    base = ps.global_base
    if rank == base:
        dist.barrier()                       # the worker of this replica has beaten
        beats = st.add(f"kgc_hb/{rank + 1}", 0)
        in_default = default.add(f"kgc_hb/{rank + 1}", 0)
        with open(os.path.join(outdir, f"r{rank}"), "w") as f:
            json.dump({"own": st is not default, "beats": beats, "in_default": in_default}, f)
    else:
        hb = health.Heartbeat(st, rank, period=0.02, timeout=30, on_fatal=lambda c, m: None).start()
        time.sleep(0.3)
        hb.stop()
        dist.barrier()
    dist.barrier()
    dist.destroy_process_group()


def test_replicas_heartbeat_into_their_own_driver(tmp_path):
    """Data-parallel replicas sharing one world: each replica's ranks heart-beat into a
    store hosted by THAT replica's driver, not into the rendezvous store of global rank 0
    -- so the loss of replica 0's node cannot end replica 1."""
    import torch.multiprocessing as mp
    mp.start_processes(_replica_store_rank, args=(4, _port(), str(tmp_path)), nprocs=4,
                       join=True, start_method="spawn")
    r2 = json.load(open(tmp_path / "r2"))
    assert r2["own"] and r2["beats"] > 0 and r2["in_default"] == 0, r2
    r0 = json.load(open(tmp_path / "r0"))
    assert r0["own"] and r0["beats"] > 0, r0
