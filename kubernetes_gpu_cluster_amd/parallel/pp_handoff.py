"""Pipeline-stage handoff over xGMI peer memory (C5), graph-capturable.

Eager steps (prefill chunks) pass activations between stages with RCCL send/recv
(``comm.pp_send`` / ``pp_recv``).  Decode steps instead end with a send kernel that
writes the stage's hidden + residual rows straight into the next stage's IPC ring
buffer and begin with a receive kernel on the next stage (``csrc/kernels/pp_handoff.hip``),
so every stage -- first, middle or last -- replays its whole decode step (receive,
layers, send / LM head) as one hipGraph.  Credits and availability are step counters in
device memory; the ring has ``R`` slots, so a stage may run ``R`` micro-batches ahead.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..engine.health import AllReduceFailed
from .custom_allreduce import _agree

log = logging.getLogger("kgc.pp")


class PipelineHandoff:
    """Collective constructor over the model ranks' gloo ``cpu_group``: every rank maps
    its next stage's receive ring (to send) and its previous stage's send signal (to
    return credits)."""

    def __init__(self, ps, device: torch.device, max_rows: int, hidden: int, dtype: torch.dtype,
                 slots: int = 2):
        from .. import ops
        ops.load_extension(strict=True)
        k = torch.ops.kgc
        self.device, self.R = device, int(slots)
        esz = torch.finfo(dtype).bits // 8
        self.slot_bytes = (max_rows * hidden * esz + 15) // 16 * 16
        self.first, self.last = ps.is_first_pp, ps.is_last_pp
        self._own, self._opened = 0, []
        handle, err = None, None
        try:
            with torch.cuda.device(device):
                sb = int(k.pp_signal_bytes())
                self._own = int(k.ar_alloc(2 * sb + self.R * 2 * self.slot_bytes))
                handle = k.ar_get_handle(self._own).tolist()
        except Exception as e:  # noqa: BLE001
            err = e
        group = ps.cpu_group
        if not _agree(err is None, group):
            self.close()
            raise RuntimeError(f"PP handoff buffer allocation failed: {err}")
        n = dist.get_world_size(group)
        gathered: list = [None] * n
        dist.all_gather_object(gathered, handle, group=group)
        me = ps.pp_rank * ps.tp_size + ps.tp_rank            # index within the model ranks

        def open_(i):
            p = int(k.ar_open_handle(torch.tensor(gathered[i], dtype=torch.uint8)))
            self._opened.append(p)
            return p
        try:
            with torch.cuda.device(device):
                nxt = open_(me + ps.tp_size) if not self.last else 0
                prv = open_(me - ps.tp_size) if not self.first else 0
        except Exception as e:  # noqa: BLE001
            err = e
        if not _agree(err is None, group):
            self.close()
            raise RuntimeError(f"PP handoff peer mapping failed: {err}")
        self.own_send_sig, self.own_recv_sig = self._own, self._own + sb
        self.own_data = self._own + 2 * sb
        self.next_recv_sig, self.next_data = (nxt + sb, nxt + 2 * sb) if nxt else (0, 0)
        self.prev_send_sig = prv
        # static receive targets: a graph replays into fixed addresses
        self.h_in = torch.zeros(max_rows, hidden, dtype=dtype, device=device)
        self.r_in = torch.zeros(max_rows, hidden, dtype=dtype, device=device)
        self.max_rows = max_rows
        self._err_host: Optional[torch.Tensor] = None

    def pre_replay(self, rows: int) -> None:
        """Nothing: the receive kernel is inside the stage's graph."""

    def post_replay(self, rows: int) -> None:
        """Nothing: the send kernel is inside the stage's graph."""

    def send(self, h: torch.Tensor, r: torch.Tensor) -> None:
        torch.ops.kgc.pp_send(h.contiguous(), r.contiguous(), self.next_data, self.next_recv_sig,
                              self.own_send_sig, self.slot_bytes, self.R)

    def recv(self, rows: int) -> tuple[torch.Tensor, torch.Tensor]:
        h, r = self.h_in[:rows], self.r_in[:rows]
        torch.ops.kgc.pp_recv(h, r, self.own_data, self.own_recv_sig, self.prev_send_sig,
                              self.slot_bytes, self.R)
        return h, r

    def check(self) -> None:
        err = int(torch.ops.kgc.pp_read_err(self.own_send_sig)) | int(
            torch.ops.kgc.pp_read_err(self.own_recv_sig))
        if err:
            raise AllReduceFailed("PP handoff: the neighbouring stage never arrived")

    _ERR_OFFSET = 16            # PpSignal::err (csrc/kernels/pp_handoff.hip)

    def enqueue_err_read(self) -> None:
        """Queue async copies of both sticky error words behind the current step."""
        if self._err_host is None:
            self._err_host = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        k = torch.ops.kgc
        k.u32_copy_async(self.own_send_sig + self._ERR_OFFSET, self._err_host, 0)
        k.u32_copy_async(self.own_recv_sig + self._ERR_OFFSET, self._err_host, 1)

    def raise_if_failed(self, slot=None) -> None:
        if self._err_host is not None and int(self._err_host.sum()):
            raise AllReduceFailed("PP handoff: the neighbouring stage never arrived "
                                  "(a PP rank is dead or wedged); the engine stops")

    def close(self) -> None:
        if self._own or self._opened:
            torch.cuda.synchronize(self.device)
            for p in self._opened:
                torch.ops.kgc.ar_close_handle(p)
            if self._own:
                torch.ops.kgc.ar_free(self._own)
            self._own = 0
            self._opened = []


class HostPipelineLink:
    """Stage handoff for per-stage decode graphs when the stages cannot map each other's
    memory -- pods on different nodes (``nnodes > 1``; KubeRay's multi-pod PP in the
    reference, /root/reference/values-01-minimal-example4.yaml:17-18,42-46).  The stage's
    decode step is still ONE graph replay, over static tensors: the graph reads its input
    rows from ``h_in`` / ``r_in`` and copies its output rows into ``h_out`` / ``r_out``; the
    rows move between replays by point-to-point send / recv on the stream (RCCL over the
    pod network; gloo stages them through the host in the one-GPU test harness).
    Warm-up calls outside capture communicate as the replays will, so every stage runs
    the same sequence."""

    def __init__(self, ps, device: torch.device, max_rows: int, hidden: int,
                 dtype: torch.dtype):
        self.first, self.last = ps.is_first_pp, ps.is_last_pp
        self.max_rows = max_rows
        z = lambda: torch.zeros(max_rows, hidden, dtype=dtype, device=device)  # noqa: E731
        self.h_in, self.r_in, self.h_out, self.r_out = z(), z(), z(), z()

    @staticmethod
    def _capturing() -> bool:
        return torch.cuda.is_current_stream_capturing()

    def recv(self, rows: int) -> tuple[torch.Tensor, torch.Tensor]:
        if not self._capturing():
            self.pre_replay(rows)
        return self.h_in[:rows], self.r_in[:rows]

    def send(self, h: torch.Tensor, r: torch.Tensor) -> None:
        rows = h.shape[0]
        self.h_out[:rows].copy_(h)
        self.r_out[:rows].copy_(r)
        if not self._capturing():
            self.post_replay(rows)

    def pre_replay(self, rows: int) -> None:
        """Before a replay: this step's rows from the previous stage into h_in / r_in."""
        if not self.first:
            from . import comm
            comm.pp_recv_into([self.h_in[:rows], self.r_in[:rows]])

    def post_replay(self, rows: int) -> None:
        """After a replay: the rows the graph left in h_out / r_out to the next stage."""
        if not self.last:
            from . import comm
            comm.pp_send([self.h_out[:rows], self.r_out[:rows]])

    # point-to-point failures raise in the collective itself: nothing sticky to read
    def enqueue_err_read(self):
        return None

    def raise_if_failed(self, slot=None) -> None:
        return None

    def check(self) -> None:
        return None

    def close(self) -> None:
        return None


def init_pp_link(ps, device: torch.device, max_rows: int, hidden: int, dtype: torch.dtype,
                 nnodes: int):
    """The stage link of PP decode graphs: the peer-memory kernels when every stage is on
    this node (one IPC domain), otherwise -- or with KGC_PP_LINK=host -- point-to-point
    sends between per-stage graph replays.  None: PP decode stays eager."""
    if ps.pp_size == 1:
        return None
    if nnodes == 1 and os.environ.get("KGC_PP_LINK", "ipc") != "host":
        return maybe_init_pp_handoff(ps, device, max_rows, hidden, dtype)
    return HostPipelineLink(ps, device, max_rows, hidden, dtype)


def maybe_init_pp_handoff(ps, device: torch.device, max_rows: int, hidden: int,
                          dtype: torch.dtype) -> Optional[PipelineHandoff]:
    """The peer-memory stage handoff for decode graphs, or None (eager PP steps only).
    Needs every stage on this node (one IPC domain): ``nnodes == 1``."""
    if os.environ.get("KGC_PP_IPC", "1") == "0" or ps.pp_size == 1:
        return None
    try:
        return PipelineHandoff(ps, device, max_rows, hidden, dtype)
    except Exception as e:  # noqa: BLE001
        log.warning("PP peer-memory handoff unavailable (%s); PP decode stays eager", e)
        return None
