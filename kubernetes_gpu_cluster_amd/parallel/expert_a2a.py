"""Expert-parallel all-to-all over xGMI peer memory (C7), graph-capturable.

The eager EP path (``models/moe.MoEBlock._forward_ep``) needs the per-rank counts on the
host for ``all_to_all_single``, so decode graphs could not capture Mixtral with
``--moe-parallel ep``.  Here the routing never leaves the device
(``csrc/kernels/ep_a2a.hip``): every EP rank maps its peers' IPC buffers, the source
writes each (token, expert) row straight into the owner's receive region (positions from
a device-side prefix scan), the owner runs the grouped expert MLP (K14) over what
arrived, and writes the results back into the source's return region; epoch flags in
device memory order the phases, so the whole block replays from a hipGraph.

Buffers are sized for ``max_pairs`` = tokens x top-k of one call (the largest decode
bucket); larger calls (prefill chunks) take the eager all-to-all.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..engine.health import AllReduceFailed
from .custom_allreduce import SUPPORTED_WORLD, _agree

log = logging.getLogger("kgc.ep")


class ExpertAllToAll:
    """Collective constructor over the EP (= TP) group's gloo ``cpu_group``."""

    def __init__(self, cpu_group, rank: int, world: int, device: torch.device, max_pairs: int,
                 hidden: int, dtype: torch.dtype):
        if world not in SUPPORTED_WORLD:
            raise ValueError(f"EP all-to-all supports {SUPPORTED_WORLD} ranks, not {world}")
        from .. import ops
        ops.load_extension(strict=True)
        k = torch.ops.kgc
        if max_pairs > int(k.ep_max_pairs()):
            raise ValueError(f"{max_pairs} pairs per call > kernel limit {int(k.ep_max_pairs())}")
        self.rank, self.world, self.device = rank, world, device
        self.C, self.H, self.dtype = int(max_pairs), int(hidden), dtype
        self._own, self._opened = 0, []
        self._err_host: Optional[torch.Tensor] = None
        handle, err = None, None
        try:
            with torch.cuda.device(device):
                self.sig_bytes = int(k.ep_signal_bytes())
                nbytes = self.sig_bytes + int(k.ep_region_bytes(world, self.C, self.H,
                                                                torch.finfo(dtype).bits // 8))
                self._own = int(k.ar_alloc(nbytes))       # uncached, zeroed
                handle = k.ar_get_handle(self._own).tolist()
        except Exception as e:  # noqa: BLE001
            err = e
        if not _agree(err is None, cpu_group):
            self.close()
            raise RuntimeError(f"EP buffer allocation failed: {err}")
        gathered: list = [None] * world
        dist.all_gather_object(gathered, handle, group=cpu_group)
        bases = []
        try:
            with torch.cuda.device(device):
                for r, h in enumerate(gathered):
                    if r == rank:
                        bases.append(self._own)
                    else:
                        p = int(k.ar_open_handle(torch.tensor(h, dtype=torch.uint8)))
                        self._opened.append(p)
                        bases.append(p)
        except Exception as e:  # noqa: BLE001
            err = e
        if not _agree(err is None, cpu_group):
            self.close()
            raise RuntimeError(f"EP peer mapping failed: {err}")
        self.sig = bases
        self.data = [b + self.sig_bytes for b in bases]

    def fits(self, x: torch.Tensor, topk_ids: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == self.dtype and x.shape[1] == self.H
                and topk_ids.numel() <= self.C)

    def forward(self, x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor,
                experts, E_local: int) -> torch.Tensor:
        """sum_j topk_w[t, j] * expert_{topk_ids[t, j]}(x[t]) with the experts spread over
        the EP ranks; ``experts(x_local, ones, ids, expert_offset)`` is the owner's grouped
        MLP: one row per receive slot ([NR * C, H] in x's dtype) or fp32 split-K slices of
        it ([S, >= NR * C, H], summed by ep_return); rows of empty slots are never read."""
        k = torch.ops.kgc
        ids = topk_ids.to(torch.int32).contiguous()
        k.ep_dispatch(x.contiguous(), ids, self.data, self.sig, self.rank, E_local, self.C)
        slots = self.world * self.C
        x_local = torch.empty(slots, self.H, dtype=x.dtype, device=x.device)
        sids = torch.empty(slots, dtype=torch.int32, device=x.device)
        route = torch.empty(slots, dtype=torch.int32, device=x.device)
        k.ep_receive(x_local, sids, route, self.data, self.sig, self.rank, E_local, self.C)
        ones = torch.ones(slots, 1, dtype=torch.float32, device=x.device)
        y = experts(x_local, ones, sids.view(slots, 1), self.rank * E_local)
        k.ep_return(y.contiguous(), route, self.data, self.sig, self.rank, self.C, x.dtype)
        out = torch.empty_like(x)
        k.ep_combine(out, topk_w.float().contiguous(), self.data, self.sig, self.rank, self.C)
        return out

    def check(self) -> None:
        err = int(torch.ops.kgc.ep_read_err(self.sig[self.rank]))
        if err:
            raise AllReduceFailed(f"EP all-to-all: peers {bin(err)} never arrived")

    def enqueue_err_read(self) -> None:
        """Queue an async copy of the sticky error word behind the current step."""
        if self._err_host is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        torch.ops.kgc.ep_err_copy_async(self.sig[self.rank], self._err_host)

    def raise_if_failed(self, slot=None) -> None:
        h = self._err_host
        if h is not None and int(h[0]):
            raise AllReduceFailed(f"EP all-to-all: peers {bin(int(h[0]))} never arrived "
                                  f"(an EP rank is dead or wedged); the engine stops")

    def close(self) -> None:
        if self._own or self._opened:
            torch.cuda.synchronize(self.device)
            for p in self._opened:
                torch.ops.kgc.ar_close_handle(p)
            if self._own:
                torch.ops.kgc.ar_free(self._own)
            self._own = 0
            self._opened = []


class PhantomExpertAllToAll(ExpertAllToAll):
    """The device-side EP all-to-all of rank ``rank`` of an EP = ``world`` group whose peers
    do not exist (KGC_TP_PHANTOM with ``--moe-parallel ep``, the analogue of
    ``PhantomAllReduce``): every peer buffer is a local allocation and the peers' arrival
    flags in this rank's signal are raised far ahead of any epoch
    (kgc.ep_raise_peer_flags), so dispatch / receive / grouped MLP / return / combine run
    their full per-rank sequence inside the captured decode graphs without waiting.  The
    rows this rank sends to its "peers" land in local HBM, not over xGMI, and the peers'
    receive regions stay empty (zero counts): the owner's grouped MLP sees this rank's own
    rows only and the combine reads zeros for the others -- per-rank TIMING of the EP
    decode step at its real shapes, never a model's outputs."""

    FLAG_VALUE = 1 << 30

    def __init__(self, rank: int, world: int, device: torch.device, max_pairs: int,
                 hidden: int, dtype: torch.dtype):
        if world not in SUPPORTED_WORLD:
            raise ValueError(f"EP all-to-all supports {SUPPORTED_WORLD} ranks, not {world}")
        from .. import ops
        ops.load_extension(strict=True)
        k = torch.ops.kgc
        if max_pairs > int(k.ep_max_pairs()):
            raise ValueError(f"{max_pairs} pairs per call > kernel limit {int(k.ep_max_pairs())}")
        self.rank, self.world, self.device = rank, world, device
        self.C, self.H, self.dtype = int(max_pairs), int(hidden), dtype
        self._err_host = None
        with torch.cuda.device(device):
            self.sig_bytes = int(k.ep_signal_bytes())
            nbytes = self.sig_bytes + int(k.ep_region_bytes(world, self.C, self.H,
                                                            torch.finfo(dtype).bits // 8))
            bases = [int(k.ar_alloc(nbytes)) for _ in range(world)]
            k.ep_raise_peer_flags(bases[rank], rank, world, self.FLAG_VALUE)
            torch.cuda.synchronize(device)
        self._own, self._opened = bases[rank], []
        self._peers = [b for r, b in enumerate(bases) if r != rank]
        self.sig = bases
        self.data = [b + self.sig_bytes for b in bases]

    def close(self) -> None:
        if self._own:
            torch.cuda.synchronize(self.device)
            for p in self._peers + [self._own]:
                torch.ops.kgc.ar_free(p)
            self._own, self._peers = 0, []


def maybe_init_expert_a2a(ps, device: torch.device, max_tokens: int, top_k: int, hidden: int,
                          dtype: torch.dtype) -> Optional[ExpertAllToAll]:
    """The device-side EP all-to-all for this rank's TP group, or None (eager all-to-all).
    A phantom TP rank (parallel/state.py init_phantom) gets ``PhantomExpertAllToAll``."""
    if os.environ.get("KGC_EP_IPC", "1") == "0" or ps.tp_size not in SUPPORTED_WORLD:
        return None
    if getattr(ps, "phantom", False):
        log.info("phantom EP rank %d of %d: device all-to-all against local peer buffers",
                 ps.tp_rank, ps.tp_size)
        return PhantomExpertAllToAll(ps.tp_rank, ps.tp_size, device, max_tokens * top_k,
                                     hidden, dtype)
    try:
        return ExpertAllToAll(ps.tp_cpu_group, ps.tp_rank, ps.tp_size, device,
                              max_tokens * top_k, hidden, dtype)
    except Exception as e:  # noqa: BLE001
        log.warning("device-side EP all-to-all unavailable (%s); using RCCL all_to_all", e)
        return None
