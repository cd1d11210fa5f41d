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
                                       blocked in a broadcast forever.

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


def step_timeout_s() -> float:
    return float(os.environ.get("KGC_STEP_TIMEOUT", "600"))


class RankWatchdog:
    """Driver-side monitor of the spawned rank processes and of step progress."""

    def __init__(self, procs: list, step_timeout: Optional[float] = None, poll: float = 0.5,
                 on_fatal: Callable[[int, str], None] = die):
        self.procs = list(procs)
        self.step_timeout = step_timeout_s() if step_timeout is None else step_timeout
        self.poll = poll
        self.on_fatal = on_fatal
        self._inflight = 0
        self._last = time.monotonic()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # progress bookkeeping (called by the executor)
    def step_begin(self) -> None:
        with self._lock:
            if self._inflight == 0:
                self._last = time.monotonic()
            self._inflight += 1

    def step_end(self) -> None:
        with self._lock:
            self._inflight = max(0, self._inflight - 1)
            self._last = time.monotonic()

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
            if self._inflight and self.step_timeout > 0 and stalled > self.step_timeout:
                return EXIT_STEP_TIMEOUT, (f"engine step made no progress for {stalled:.0f} s "
                                           f"(KGC_STEP_TIMEOUT={self.step_timeout:.0f}): a "
                                           f"collective is waiting on a dead or wedged peer")
        return None

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
