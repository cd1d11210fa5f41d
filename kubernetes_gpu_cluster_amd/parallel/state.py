"""Process-group topology for TP x PP (x EP) inside one serving pod.

One process per GPU (``torch.distributed``; backend ``nccl`` = RCCL on ROCm, over
xGMI within a node; ``gloo`` for CPU tests).  Rank layout is TP-fastest: ranks
``[pp_rank * tp, (pp_rank + 1) * tp)`` form one tensor-parallel group, so TP peers
are adjacent GPU ids (on an 8x MI355X node every pair has a direct xGMI link, so
any contiguous TP group is a full mesh).

Reference: the values files drive TP/PP through ``vllmConfig.tensorParallelSize``,
``pipelineParallelSize`` and ``extraArgs`` (``values-01-minimal-example4.yaml:17-18``,
``values-01-minimal-example8.yaml:35-38``); the reference delegates the groups to vLLM.
"""
from __future__ import annotations

import dataclasses
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


@dataclasses.dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    pp_size: int = 1
    pp_rank: int = 0
    tp_group: Optional[object] = None
    pp_group: Optional[object] = None
    cpu_group: Optional[object] = None      # gloo group over the model ranks (metadata)
    tp_cpu_group: Optional[object] = None
    backend: str = "none"
    device: torch.device = dataclasses.field(default_factory=lambda: torch.device("cpu"))
    # phantom TP rank (KGC_TP_PHANTOM=N, init_phantom): ONE process holds rank 0's shard
    # of a TP = N model; there are no peer processes and no process groups
    phantom: bool = False

    @property
    def is_first_pp(self) -> bool:
        return self.pp_rank == 0

    @property
    def is_last_pp(self) -> bool:
        return self.pp_rank == self.pp_size - 1

    @property
    def is_driver(self) -> bool:
        return self.rank == 0

    def pp_prev_rank(self) -> int:
        return self.rank - self.tp_size

    def pp_next_rank(self) -> int:
        return self.rank + self.tp_size


_STATE = ParallelState()


def get_state() -> ParallelState:
    return _STATE


def set_state(s: ParallelState) -> None:
    global _STATE
    _STATE = s


def init_parallel(tp: int = 1, pp: int = 1, backend: Optional[str] = None,
                  device: Optional[torch.device] = None, rank: Optional[int] = None,
                  world_size: Optional[int] = None, init_method: Optional[str] = None,
                  timeout_s: int = 600) -> ParallelState:
    """Initialise torch.distributed (if tp*pp > 1) and build the TP/PP groups."""
    ws = tp * pp
    if ws == 1 and not dist.is_initialized():
        s = ParallelState(device=device or torch.device("cpu"))
        set_state(s)
        return s
    if not dist.is_initialized():
        rank = int(os.environ.get("RANK", 0)) if rank is None else rank
        world_size = int(os.environ.get("WORLD_SIZE", ws)) if world_size is None else world_size
        if backend is None:
            # KGC_DIST_BACKEND=gloo lets several TP ranks share ONE GPU (RCCL refuses
            # duplicate devices): a correctness harness for the TP path on a 1-GPU box
            backend = os.environ.get("KGC_DIST_BACKEND") or (
                "nccl" if (device is not None and device.type == "cuda") else "gloo")
        if device is not None and device.type == "cuda":
            torch.cuda.set_device(device)
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = device
        dist.init_process_group(backend, init_method=init_method or "env://", rank=rank,
                                world_size=world_size,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    rank, world_size = dist.get_rank(), dist.get_world_size()
    assert world_size % ws == 0, f"world {world_size} not a multiple of tp*pp={ws}"
    backend = dist.get_backend()
    base = (rank // ws) * ws              # data-parallel replicas of the model, if any
    local = rank - base
    tp_rank, pp_rank = local % tp, local // tp
    tp_group = pp_group = tp_cpu = cpu_group = None
    # every rank must create every group in the same order
    for rep in range(world_size // ws):
        b = rep * ws
        for p in range(pp):
            ranks = list(range(b + p * tp, b + (p + 1) * tp))
            g = dist.new_group(ranks)
            gc = dist.new_group(ranks, backend="gloo")
            if rank in ranks:
                tp_group, tp_cpu = g, gc
        for t in range(tp):
            ranks = list(range(b + t, b + ws, tp))
            g = dist.new_group(ranks)
            if rank in ranks:
                pp_group = g
        ranks = list(range(b, b + ws))
        gc = dist.new_group(ranks, backend="gloo")
        if rank in ranks:
            cpu_group = gc
    s = ParallelState(world_size=ws, rank=local, tp_size=tp, tp_rank=tp_rank, pp_size=pp,
                      pp_rank=pp_rank, tp_group=tp_group, pp_group=pp_group,
                      cpu_group=cpu_group, tp_cpu_group=tp_cpu, backend=backend,
                      device=device or torch.device("cpu"))
    s.global_base = base  # type: ignore[attr-defined]
    set_state(s)
    return s


def init_phantom(tp: int, device: torch.device) -> ParallelState:
    """Rank 0 of a TP = ``tp`` model as a single process on one GPU (KGC_TP_PHANTOM=tp):
    every layer holds rank 0's shard (70B at TP = 8: nq 8, nkv 1, I / 8, vocab / 8), the
    row-parallel sums run the real xGMI kernels against peer buffers that never arrive
    with data (parallel/custom_allreduce.py PhantomAllReduce), and the other collectives
    are local stand-ins of the same shapes (parallel/comm.py).  It exercises -- and lets
    rocprof time -- one rank's decode step with its real kernel sequence inside the
    captured graphs, on a box with one GPU.  Outputs are not a TP = tp model's outputs
    (the peers contribute zeros): a measurement and capture harness, never a server."""
    assert tp in (2, 4, 8), f"phantom TP size {tp} not in (2, 4, 8)"
    s = ParallelState(world_size=1, rank=0, tp_size=tp, tp_rank=0, pp_size=1, pp_rank=0,
                      backend="phantom", device=device, phantom=True)
    set_state(s)
    return s


def phantom_tp() -> int:
    """KGC_TP_PHANTOM as an int (0: off)."""
    v = os.environ.get("KGC_TP_PHANTOM", "0") or "0"
    return int(v)


def destroy_parallel() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
    set_state(ParallelState())
