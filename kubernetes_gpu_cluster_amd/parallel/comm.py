"""Collectives used by the model (SURVEY.md §2.6 call sites C1-C8).

All TP collectives go through RCCL (``torch.distributed`` backend ``nccl``) on the
TP group, except decode-size all-reduces, which use the one-shot xGMI all-reduce
(``parallel.custom_allreduce``) when it is registered for the group and the
message fits its buffer; ``--disable-custom-all-reduce`` (reference
``values-01-minimal-example8.yaml:32``) keeps everything on RCCL.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .state import get_state

_custom_ar = None   # parallel.custom_allreduce.CustomAllReduce or None


def set_custom_allreduce(car) -> None:
    global _custom_ar
    _custom_ar = car


def get_custom_allreduce():
    return _custom_ar


def _gloo_half(x: torch.Tensor, group) -> bool:
    """gloo reduces bf16 / fp16 in that dtype, rounding after every rank's add (7 roundings
    of the running sum at TP = 8: the 8-rank engine on one GPU drifted from TP = 1 on the
    first token).  Those sums go through fp32 and round once, like the xGMI kernel's."""
    return (x.dtype in (torch.bfloat16, torch.float16)
            and dist.get_backend(group) == dist.Backend.GLOO)


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    """C1/C2/C3: sum over the TP group (in place when possible)."""
    s = get_state()
    if s.tp_size == 1:
        return x
    car = _custom_ar
    if car is not None and car.should_use(x):
        return car.all_reduce(x)
    if s.phantom:
        return x            # RCCL-size message of a phantom rank: no peers to sum
    if _gloo_half(x, s.tp_group):
        acc = x.float()
        dist.all_reduce(acc, group=s.tp_group)
        x.copy_(acc)
        return x
    dist.all_reduce(x, group=s.tp_group)
    return x


class _Done:
    def wait(self) -> None:
        pass


class _Fp32Back:
    """Async fp32 sum of a half-precision tensor: wait() rounds it back into the tensor."""

    def __init__(self, work, acc: torch.Tensor, x: torch.Tensor):
        self.work, self.acc, self.x = work, acc, x

    def wait(self) -> None:
        self.work.wait()
        self.x.copy_(self.acc)


def tp_all_reduce_async(x: torch.Tensor):
    """In-place TP sum launched WITHOUT ordering the caller's later work behind it:
    returns a handle whose ``wait()`` orders the current stream after the collective
    (RCCL: a stream wait on the communicator's stream, no host block; gloo: blocks).
    Used by the two-half prefill overlap (models/llama.py ``_forward_tp_overlap``), where
    one half's GEMMs run while the other half's all-reduce is on the links.  Always
    RCCL/gloo: the xGMI kernel would run on the compute stream and overlap nothing."""
    s = get_state()
    if s.tp_size == 1 or s.phantom:
        return _Done()
    if _gloo_half(x, s.tp_group):
        acc = x.float()
        return _Fp32Back(dist.all_reduce(acc, group=s.tp_group, async_op=True), acc, x)
    return dist.all_reduce(x, group=s.tp_group, async_op=True)


def tp_all_reduce_add_rms(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                          eps: float) -> tuple[torch.Tensor, torch.Tensor]:
    """Row-parallel projection output -> (rms_norm(residual + sum_ranks x) * w, residual),
    residual updated in place: the fused xGMI kernel when the rows fit its one-shot
    size, else all-reduce + fused_add_rms_norm (identical rounding either way)."""
    from .. import ops
    car = _custom_ar
    if car is not None and get_state().tp_size > 1 and car.can_fuse(x):
        return car.all_reduce_add_rms(x, residual, w, eps)
    return ops.fused_add_rms_norm(tp_all_reduce(x), residual, w, eps)


def tp_all_reduce_max(x: torch.Tensor) -> torch.Tensor:
    """In-place MAX over the TP group (vocab-parallel sampling: 8 bytes per row)."""
    s = get_state()
    if s.tp_size > 1 and not s.phantom:
        dist.all_reduce(x, op=dist.ReduceOp.MAX, group=s.tp_group)
    return x


def tp_all_gather(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    s = get_state()
    if s.tp_size == 1:
        return x
    dim = dim % x.dim()
    x = x.contiguous()
    out = torch.empty((s.tp_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype,
                      device=x.device)
    if s.phantom:
        # the peers' shards stand in as copies of this rank's (same bytes moved locally)
        out.view((s.tp_size,) + tuple(x.shape)).copy_(x.unsqueeze(0).expand(
            (s.tp_size,) + tuple(x.shape)))
    else:
        dist.all_gather_into_tensor(out, x, group=s.tp_group)
    if dim == 0:
        return out
    return torch.cat(out.view((s.tp_size,) + tuple(x.shape)).unbind(0), dim=dim)


def tp_gather(x: torch.Tensor, dim: int = -1) -> Optional[torch.Tensor]:
    """C4: gather vocab shards of the logits onto TP rank 0 (None elsewhere).
    On RCCL a gather is an all-gather's cost; all ranks receive (cheap, and lets
    every rank run the same sampler when needed)."""
    return tp_all_gather(x, dim)


def tp_broadcast(x: torch.Tensor, src_local: int = 0) -> torch.Tensor:
    """C6: broadcast from a TP-local rank."""
    s = get_state()
    if s.tp_size == 1 or s.phantom:
        return x
    base = getattr(s, "global_base", 0) + s.pp_rank * s.tp_size
    dist.broadcast(x, src=base + src_local, group=s.tp_group)
    return x


def _host_staged() -> bool:
    """gloo point-to-point moves host memory only: GPU tensors are staged through the
    host (the KGC_DIST_BACKEND=gloo harness that puts several ranks on one GPU)."""
    return dist.get_backend() == "gloo"


def pp_send(tensors: list[torch.Tensor]) -> None:
    """C5: stage boundary, hidden + residual to the next stage."""
    s = get_state()
    dst = getattr(s, "global_base", 0) + s.rank + s.tp_size
    for t in tensors:
        t = t.contiguous()
        dist.send(t.cpu() if t.is_cuda and _host_staged() else t, dst=dst)


def pp_recv(shapes: list[tuple], dtype: torch.dtype, device) -> list[torch.Tensor]:
    s = get_state()
    src = getattr(s, "global_base", 0) + s.rank - s.tp_size
    out = []
    for shp in shapes:
        t = torch.empty(shp, dtype=dtype, device=device)
        if t.is_cuda and _host_staged():
            h = torch.empty(shp, dtype=dtype)
            dist.recv(h, src=src)
            t.copy_(h)
        else:
            dist.recv(t, src=src)
        out.append(t)
    return out


def pp_recv_into(out: list[torch.Tensor]) -> None:
    """C5 receive into existing (static) tensors -- the per-stage graph's input rows."""
    s = get_state()
    src = getattr(s, "global_base", 0) + s.rank - s.tp_size
    for t in out:
        if t.is_cuda and _host_staged():
            h = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(h, src=src)
            t.copy_(h)
        elif t.is_contiguous():
            dist.recv(t, src=src)
        else:
            tmp = torch.empty_like(t, memory_format=torch.contiguous_format)
            dist.recv(tmp, src=src)
            t.copy_(tmp)


def all_reduce_min_scalar(v: int) -> int:
    """C8: agree on the KV block count across all model ranks."""
    s = get_state()
    if s.world_size == 1 or not dist.is_initialized():
        return v
    t = torch.tensor([v], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=s.cpu_group)
    return int(t.item())
