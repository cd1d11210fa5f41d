"""Tensor-parallel layers (Megatron column/row sharding) over the TP group.

GEMMs are ``ops.gemm.linear``: hipBLASLt, or the K9 skinny GEMM for the small-batch
decode shapes where the engine-start tuner measured it faster, on weights stored
[out, in] so the reduction dim is contiguous for both.  Sharding:

* ColumnParallelLinear     weight rows split; no communication.
* MergedColumnParallelLinear  fused gate_up: each logical output split separately
                              so rank r holds [gate_r; up_r] contiguous (silu_mul
                              then works on the local half-split).
* QKVParallelLinear        q heads split; kv heads split, or replicated when
                           nkv < tp (each rank holds kv head rank*nkv//tp).
* RowParallelLinear        weight cols split; all-reduce (C1/C2); bias after reduce.
* VocabParallelEmbedding   vocab rows split; masked lookup + all-reduce (C3).
* ParallelLMHead           vocab rows split; all-gather of logit shards (C4).

Every parameter carries ``weight_loader(param, full_tensor, shard_id=None)`` which
slices an unsharded checkpoint tensor for this rank.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.gemm import linear
from . import comm
from .state import get_state


def _tp():
    s = get_state()
    return s.tp_size, s.tp_rank


def _param(shape, dtype, device, loader):
    p = nn.Parameter(torch.empty(shape, dtype=dtype, device=device), requires_grad=False)
    p.weight_loader = loader  # type: ignore[attr-defined]
    return p


def _default_loader(param: torch.Tensor, w: torch.Tensor, shard_id=None) -> None:
    assert param.shape == w.shape, f"{tuple(param.shape)} vs {tuple(w.shape)}"
    param.data.copy_(w)


class ReplicatedLinear(nn.Module):
    def __init__(self, in_f: int, out_f: int, bias: bool = False, dtype=torch.bfloat16,
                 device=None):
        super().__init__()
        self.weight = _param((out_f, in_f), dtype, device, _default_loader)
        self.bias = _param((out_f,), dtype, device, _default_loader) if bias else None

    def forward(self, x):
        return linear(x, self.weight, self.bias)


class ColumnParallelLinear(nn.Module):
    def __init__(self, in_f: int, out_f: int, bias: bool = False, dtype=torch.bfloat16,
                 device=None, gather_output: bool = False):
        super().__init__()
        tp, _ = _tp()
        assert out_f % tp == 0, f"out {out_f} not divisible by tp {tp}"
        self.out_per = out_f // tp
        self.gather_output = gather_output
        self.weight = _param((self.out_per, in_f), dtype, device, self._load)
        self.bias = _param((self.out_per,), dtype, device, self._load) if bias else None

    def _load(self, param, w, shard_id=None):
        _, r = _tp()
        param.data.copy_(w.narrow(0, r * self.out_per, self.out_per))

    def forward(self, x):
        y = linear(x, self.weight, self.bias)
        return comm.tp_all_gather(y, -1) if self.gather_output else y


class MergedColumnParallelLinear(nn.Module):
    def __init__(self, in_f: int, out_sizes: list[int], bias: bool = False,
                 dtype=torch.bfloat16, device=None):
        super().__init__()
        tp, _ = _tp()
        for o in out_sizes:
            assert o % tp == 0
        self.per = [o // tp for o in out_sizes]
        self.offsets = [sum(self.per[:i]) for i in range(len(self.per))]
        self.weight = _param((sum(self.per), in_f), dtype, device, self._load)
        self.bias = _param((sum(self.per),), dtype, device, self._load) if bias else None

    def _load(self, param, w, shard_id: int):
        _, r = _tp()
        n = self.per[shard_id]
        param.data.narrow(0, self.offsets[shard_id], n).copy_(w.narrow(0, r * n, n))

    def forward(self, x):
        return linear(x, self.weight, self.bias)


class QKVParallelLinear(nn.Module):
    def __init__(self, hidden: int, head_dim: int, num_heads: int, num_kv_heads: int,
                 bias: bool = False, dtype=torch.bfloat16, device=None):
        super().__init__()
        tp, r = _tp()
        assert num_heads % tp == 0, f"num_heads {num_heads} % tp {tp}"
        self.head_dim = head_dim
        self.nq = num_heads // tp
        if num_kv_heads >= tp:
            assert num_kv_heads % tp == 0
            self.nkv = num_kv_heads // tp
            self.kv_start = r * self.nkv
        else:
            assert tp % num_kv_heads == 0
            self.nkv = 1
            self.kv_start = r * num_kv_heads // tp
        self.q_size = self.nq * head_dim
        self.kv_size = self.nkv * head_dim
        out = self.q_size + 2 * self.kv_size
        self.weight = _param((out, hidden), dtype, device, self._load)
        self.bias = _param((out,), dtype, device, self._load) if bias else None

    def _load(self, param, w, shard_id: str):
        _, r = _tp()
        d = self.head_dim
        if shard_id == "q":
            param.data.narrow(0, 0, self.q_size).copy_(w.narrow(0, r * self.q_size, self.q_size))
        else:
            off = self.q_size + (0 if shard_id == "k" else self.kv_size)
            param.data.narrow(0, off, self.kv_size).copy_(
                w.narrow(0, self.kv_start * d, self.kv_size))

    def forward(self, x):
        return linear(x, self.weight, self.bias)


class RowParallelLinear(nn.Module):
    def __init__(self, in_f: int, out_f: int, bias: bool = False, dtype=torch.bfloat16,
                 device=None, reduce_results: bool = True):
        super().__init__()
        tp, _ = _tp()
        assert in_f % tp == 0
        self.in_per = in_f // tp
        self.reduce_results = reduce_results
        self.weight = _param((out_f, self.in_per), dtype, device, self._load)
        self.bias = _param((out_f,), dtype, device, _default_loader) if bias else None

    def _load(self, param, w, shard_id=None):
        _, r = _tp()
        param.data.copy_(w.narrow(1, r * self.in_per, self.in_per))

    def forward(self, x):
        y = linear(x, self.weight)
        if self.reduce_results:
            y = comm.tp_all_reduce(y)
        if self.bias is not None:
            y = y + self.bias
        return y


def _pad_vocab(v: int, tp: int, align: int = 64) -> int:
    m = align * tp
    return (v + m - 1) // m * m


class VocabParallelEmbedding(nn.Module):
    def __init__(self, vocab: int, hidden: int, dtype=torch.bfloat16, device=None):
        super().__init__()
        tp, r = _tp()
        self.vocab = vocab
        self.padded = _pad_vocab(vocab, tp) if tp > 1 else vocab
        self.per = self.padded // tp
        self.start = r * self.per
        self.weight = _param((self.per, hidden), dtype, device, self._load)

    def _load(self, param, w, shard_id=None):
        n = max(0, min(self.per, self.vocab - self.start))
        param.data.zero_()
        if n:
            param.data.narrow(0, 0, n).copy_(w.narrow(0, self.start, n))

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        tp, _ = _tp()
        if tp == 1:
            return F.embedding(ids, self.weight)
        local = ids - self.start
        mask = (local < 0) | (local >= self.per)
        y = F.embedding(local.masked_fill(mask, 0), self.weight)
        y.masked_fill_(mask[:, None], 0)
        return comm.tp_all_reduce(y)


class ParallelLMHead(nn.Module):
    """Vocab-sharded output projection; may share its weight with the embedding."""

    def __init__(self, vocab: int, hidden: int, dtype=torch.bfloat16, device=None,
                 tied: Optional[VocabParallelEmbedding] = None):
        super().__init__()
        tp, r = _tp()
        self.vocab = vocab
        if tied is not None:
            self.emb = tied
            self.per, self.start = tied.per, tied.start
            self.weight = None
        else:
            self.emb = None
            padded = _pad_vocab(vocab, tp) if tp > 1 else vocab
            self.per = padded // tp
            self.start = r * self.per
            self.weight = _param((self.per, hidden), dtype, device, self._load)

    def _load(self, param, w, shard_id=None):
        n = max(0, min(self.per, self.vocab - self.start))
        param.data.zero_()
        if n:
            param.data.narrow(0, 0, n).copy_(w.narrow(0, self.start, n))

    def get_weight(self):
        return self.emb.weight if self.emb is not None else self.weight

    def forward(self, h: torch.Tensor, gather: bool = True) -> torch.Tensor:
        """gather=False keeps this rank's shard [T, per] (padding columns included:
        the vocab-parallel sampler reads only the valid ones)."""
        logits = linear(h, self.get_weight())
        tp, _ = _tp()
        if not gather:
            return logits
        if tp > 1:
            logits = comm.tp_all_gather(logits, -1)
        return logits[:, : self.vocab]
