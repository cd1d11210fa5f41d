"""Failure detection for multi-rank engines: exit, never hang and never recover in place.

The reference leaves restart semantics to Kubernetes and its health checks
(keepalived's ``check_apiserver.sh`` with ``fall 10 rise 2``, haproxy ``/healthz`` probes:
/root/reference/multi-cp.md:66-72,102-111; vLLM pods restarted by their Deployment).  The
engine's part of that contract is to turn every fatal condition into a prompt, non-zero
process exit -- which the API server turns into its own non-zero exit and a 503 on
``/health`` -- so the pod restarts instead of serving wrong tokens or hanging:

* a TP / PP rank process dies       -> the driver's ``RankWatchdog`` sees its exit code
                                       and ends the driver (EXIT_RANK_DEAD);
* a step makes no progress for       -> the same watchdog ends the driver
  ``KGC_STEP_TIMEOUT`` seconds         (EXIT_STEP_TIMEOUT): an RCCL collective waiting
                                       on a dead or wedged peer never returns;
* the xGMI all-reduce barrier gave   -> the sticky error word is copied to the host after
  up on a peer (allreduce.hip)          every step and ``AllReduceFailed`` is raised when
                                       the step's result is read (never silently summing
                                       stale peer data);
* the driver dies                   -> every spawned rank's ``watch_parent`` thread ends
                                       that rank (EXIT_PARENT_DEAD) instead of leaving it
                                       blocked in a broadcast forever;
* a rank on ANOTHER node (pod) dies  -> its heartbeat counter in the rendezvous TCPStore
  or hangs                             (hosted by the driver) stops moving; the driver's
                                       watchdog ends the driver after
                                       ``KGC_HEARTBEAT_TIMEOUT`` (15 s) -- the same check
                                       covers torchrun-launched ranks (ExternalExecutor),
                                       whose exit codes the driver cannot see;
* the driver's node (pod) dies       -> the remote ranks' heartbeat writes fail or stall
                                       and those ranks exit (EXIT_PARENT_DEAD), which ends
                                       their worker_node pod.

The step timeout adapts to the engine: ``KGC_STEP_TIMEOUT`` pins it; otherwise it is
``KGC_STEP_TIMEOUT_WARMUP`` (300 s) for the first steps (lazy kernel / library set-up)
and then max(``KGC_STEP_TIMEOUT_FLOOR`` (30 s), 10 x the longest step seen) -- a wedged
collective is reported in tens of seconds, not the ten minutes of a fixed bound.

``os._exit`` is deliberate: the thread that notices is not the one blocked in the
collective, and a clean interpreter shutdown would wait on it.
"""
from __future__ import annotations

import logging
import os
import sys
import threading
import time
from typing import Callable, Optional

log = logging.getLogger("kgc.health")

EXIT_RANK_DEAD = 70
EXIT_STEP_TIMEOUT = 71
EXIT_PARENT_DEAD = 72


class AllReduceFailed(RuntimeError):
    """A custom all-reduce barrier timed out waiting for a peer: results are invalid."""


def die(code: int, msg: str) -> None:
    log.critical(msg)
    try:
        sys.stderr.write(f"kgc: FATAL: {msg} (exit {code})\n")
        sys.stderr.flush()
    finally:
        os._exit(code)


WARMUP_STEPS = 8


def step_timeout_s() -> Optional[float]:
    """The pinned step timeout (``KGC_STEP_TIMEOUT``), or None: adaptive."""
    v = os.environ.get("KGC_STEP_TIMEOUT")
    return float(v) if v not in (None, "") else None


def heartbeat_timeout_s() -> float:
    return float(os.environ.get("KGC_HEARTBEAT_TIMEOUT", "15"))


def _hb_key(rank: int) -> str:
    return f"kgc_hb/{rank}"


class RankWatchdog:
    """Driver-side monitor of the spawned rank processes, of step progress, and of the
    heartbeats of ranks it did not spawn (other nodes, torchrun)."""

    def __init__(self, procs: list, step_timeout: Optional[float] = None, poll: float = 0.5,
                 on_fatal: Callable[[int, str], None] = die):
        self.procs = list(procs)
        self.fixed_timeout = step_timeout_s() if step_timeout is None else step_timeout
        self.floor = float(os.environ.get("KGC_STEP_TIMEOUT_FLOOR", "30"))
        self.warmup_timeout = float(os.environ.get("KGC_STEP_TIMEOUT_WARMUP", "300"))
        self.poll = poll
        self.on_fatal = on_fatal
        self._inflight = 0
        self._last = time.monotonic()
        self.steps_done = 0
        self.longest_step = 0.0
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._hb_store = None
        self._hb: dict[int, list] = {}          # rank -> [last value, last change time]
        self.hb_timeout = heartbeat_timeout_s()

    @property
    def step_timeout(self) -> float:
        if self.fixed_timeout is not None:
            return self.fixed_timeout
        if self.steps_done < WARMUP_STEPS:
            return self.warmup_timeout
        return max(self.floor, 10.0 * self.longest_step)

    # progress bookkeeping (called by the executor)
    def step_begin(self) -> None:
        with self._lock:
            if self._inflight == 0:
                self._last = time.monotonic()
            self._inflight += 1

    def step_end(self) -> None:
        with self._lock:
            now = time.monotonic()
            if self._inflight:
                self.longest_step = max(self.longest_step, now - self._last)
                self.steps_done += 1
            self._inflight = max(0, self._inflight - 1)
            self._last = now

    def watch_heartbeats(self, store, ranks) -> "RankWatchdog":
        """Also require every rank in ``ranks`` to keep bumping its heartbeat counter in
        ``store`` (``start_heartbeat``)."""
        now = time.monotonic()
        self._hb_store = store
        self._hb = {int(r): [None, now] for r in ranks}
        return self

    def _check_heartbeats(self) -> Optional[tuple[int, str]]:
        if self._hb_store is None or self.hb_timeout <= 0:
            return None
        now = time.monotonic()
        for r, st in self._hb.items():
            try:
                v = self._hb_store.add(_hb_key(r), 0)
            except Exception as e:  # noqa: BLE001 - the store lives in this process
                return EXIT_RANK_DEAD, f"heartbeat store unreadable: {e}"
            if v != st[0]:
                st[0], st[1] = v, now
            elif now - st[1] > self.hb_timeout:
                return EXIT_RANK_DEAD, (f"engine rank {r} sent no heartbeat for {now - st[1]:.0f} s "
                                        f"(KGC_HEARTBEAT_TIMEOUT={self.hb_timeout:.0f}): its process "
                                        f"or its node is gone")
        return None

    def start(self) -> "RankWatchdog":
        self._thread = threading.Thread(target=self._run, name="kgc-rank-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def check_once(self) -> Optional[tuple[int, str]]:
        for i, p in enumerate(self.procs):
            code = p.exitcode
            if code is not None:
                return EXIT_RANK_DEAD, (f"engine rank process {getattr(p, 'name', i)} "
                                        f"(pid {p.pid}) exited with code {code}")
        with self._lock:
            stalled = time.monotonic() - self._last
            lim = self.step_timeout
            if self._inflight and lim > 0 and stalled > lim:
                return EXIT_STEP_TIMEOUT, (f"engine step made no progress for {stalled:.0f} s "
                                           f"(limit {lim:.0f} s after {self.steps_done} steps, "
                                           f"longest {self.longest_step:.1f} s): a collective "
                                           f"is waiting on a dead or wedged peer")
        return self._check_heartbeats()

    def _run(self) -> None:
        while not self._stop.wait(self.poll):
            bad = self.check_once()
            if bad is not None and not self._stop.is_set():
                self.on_fatal(*bad)
                return


def watch_parent(poll: float = 1.0, on_fatal: Callable[[int, str], None] = die) -> threading.Thread:
    """In a spawned rank: end this process when its parent (the driver) is gone."""
    parent = os.getppid()

    def run():
        while True:
            time.sleep(poll)
            if os.getppid() != parent:
                on_fatal(EXIT_PARENT_DEAD, f"engine driver (pid {parent}) is gone; rank {os.getpid()} exits")
                return
    t = threading.Thread(target=run, name="kgc-parent-watch", daemon=True)
    t.start()
    return t


class Heartbeat:
    """A non-driver rank's heartbeat: bump ``kgc_hb/<rank>`` in its replica's TCPStore
    (``replica_store``: served from the replica driver's process) every ``period`` s.  When a bump fails, or none
    has succeeded for ``timeout`` s (the driver's node vanished without a TCP reset),
    the rank exits (EXIT_PARENT_DEAD) -- unless ``stop()`` was called first (a clean
    shutdown tears the store down right after telling the ranks to exit)."""

    def __init__(self, store, rank: int, period: float = 1.0, timeout: Optional[float] = None,
                 on_fatal: Callable[[int, str], None] = die):
        self.store, self.rank, self.period = store, rank, period
        self.timeout = heartbeat_timeout_s() if timeout is None else timeout
        self.on_fatal = on_fatal
        self._ok = time.monotonic()
        self._stop = threading.Event()

    def start(self) -> "Heartbeat":
        for fn, name in ((self._beat, "kgc-heartbeat"), (self._guard, "kgc-heartbeat-guard")):
            threading.Thread(target=fn, name=name, daemon=True).start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _fatal(self, msg: str) -> None:
        # a clean exit may race the store's teardown: give the main thread a moment
        if self._stop.wait(2.0):
            return
        self.on_fatal(EXIT_PARENT_DEAD, f"rank {self.rank}: {msg}")

    def _beat(self) -> None:
        while not self._stop.is_set():
            try:
                self.store.add(_hb_key(self.rank), 1)
                self._ok = time.monotonic()
            except Exception as e:  # noqa: BLE001
                self._fatal(f"engine driver unreachable ({e})")
                return
            self._stop.wait(self.period)

    def _guard(self) -> None:
        while not self._stop.wait(self.period):
            if self.timeout > 0 and time.monotonic() - self._ok > self.timeout:
                self._fatal(f"no heartbeat reached the engine driver for "
                            f"{time.monotonic() - self._ok:.0f} s")
                return


def replica_store(ps):
    """The heartbeat store of THIS engine replica (tp x pp ranks starting at
    ``ps.global_base``).  When the process group is exactly one replica this is the
    rendezvous store.  When several data-parallel replicas share one world, the default
    store is hosted by global rank 0 (or the torchrun agent) -- the node of replica 0 --
    so heart-beating into it would tie every replica's ranks to that node: its loss
    would end all replicas.  Each replica's driver therefore hosts a TCPStore of its own
    (published under ``kgc/hb_store/<base>`` in the default store) and its ranks connect
    to it.  Called by every rank of the replica (the driver first creates the store, the
    others block until it is published).  None without a process group."""
    import torch.distributed as dist
    default = rendezvous_store()
    if default is None:
        return None
    n = ps.tp_size * ps.pp_size
    if dist.get_world_size() == n:
        return default
    import datetime
    base = getattr(ps, "global_base", 0)
    key = f"kgc/hb_store/{base}"
    to = datetime.timedelta(seconds=float(os.environ.get("KGC_HB_STORE_TIMEOUT", 1800)))
    if dist.get_rank() == base:
        host = _local_ip()
        st = dist.TCPStore(host, 0, is_master=True, timeout=to, wait_for_workers=False)
        default.set(key, f"{host}:{st.port}")
        return st
    default.wait([key], to)
    host, port = default.get(key).decode().rsplit(":", 1)
    return dist.TCPStore(host, int(port), is_master=False, timeout=to)


def _local_ip() -> str:
    """The address this host uses to reach the rendezvous master (MASTER_ADDR)."""
    import socket
    master = os.environ.get("MASTER_ADDR", "127.0.0.1")
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as sk:
            sk.connect((master, 1))
            return sk.getsockname()[0]
    except OSError:
        return "127.0.0.1"


def rendezvous_store():
    """The default process group's TCPStore (hosted by rank 0), or None."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return None
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001
        return None
