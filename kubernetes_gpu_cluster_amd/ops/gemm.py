"""Linear layers on the GPU: hipBLASLt (``F.linear``) or the hand-written K9 skinny
GEMM (``csrc/kernels/gemm_skinny.hip``) for small-batch decode.

Which one runs is a per-(M, N, K) decision made once at engine start by timing
both on the model's own weights (``tune_skinny``), never guessed: at M <= 64 the GEMM
is a weight stream, where hipBLASLt leaves the 4096-wide projections at 2-4 TB/s,
while at M >= 128 hipBLASLt's MFMA tiles win.  The table is consulted on every call;
graph capture bakes the chosen kernel into each decode bucket's graph.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Iterable, Optional

import torch
import torch.nn.functional as F

log = logging.getLogger("kgc.gemm")

SKINNY_MAX_M = 64
# (mt, nt, nw, ntl) configurations the tuner tries; mt = 16-row batch tiles.
_CONFIGS = [(mt, nt, nw, ntl) for mt in (1, 2, 4) for nt in (1, 2) for nw in (4, 8, 16)
            for ntl in (True, False)]

_plan: dict[tuple[int, int, int], tuple[int, int, int, bool]] = {}
_enabled = os.environ.get("KGC_SKINNY_GEMM", "1") != "0"


def skinny_ok(M: int, N: int, K: int, cfg) -> bool:
    mt, nt, nw, _ = cfg
    return 1 <= M <= 16 * mt and N % (16 * nt) == 0 and K % (32 * nw) == 0


def skinny_gemm(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], cfg,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    from . import _k
    mt, nt, nw, ntl = cfg
    if out is None:
        out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
    _k().skinny_gemm(out, x, w, bias, mt, nt, nw, ntl)
    return out


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    if x.is_cuda and x.dim() == 2 and x.shape[0] <= SKINNY_MAX_M and _plan:
        cfg = _plan.get((x.shape[0], w.shape[0], w.shape[1]))
        if cfg is not None and x.stride(1) == 1:
            return skinny_gemm(x, w, bias, cfg)
    return F.linear(x, w, bias)


def clear_plan() -> None:
    _plan.clear()


def plan() -> dict:
    return dict(_plan)


def _time(fn, reps: int) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


@torch.inference_mode()
def tune_skinny(weights: Iterable[torch.Tensor], ms: Iterable[int], margin: float = 0.97,
                reps: int = 3) -> dict:
    """Time hipBLASLt against every skinny configuration for each weight shape and
    batch size M (decode buckets <= SKINNY_MAX_M) and record the skinny kernel where it
    is faster by more than ``1 - margin``.  Each timing sweeps ALL weights of the shape
    (every layer's copy) so the weights stream from HBM as in a real decode step,
    not from the 256 MB Infinity Cache.  Returns {(M, N, K): (chosen cfg or None,
    hipBLASLt us, best skinny us, best skinny cfg)}, times per GEMM call."""
    if not _enabled:
        return {}
    by_shape: dict[tuple[int, int], list[torch.Tensor]] = {}
    for w in weights:
        if w.is_cuda and w.dim() == 2 and w.dtype in (torch.bfloat16, torch.float16):
            by_shape.setdefault((w.shape[0], w.shape[1]), []).append(w)
    res = {}
    t0 = time.time()
    for (N, K), ws in sorted(by_shape.items()):
        for M in sorted(set(m for m in ms if 1 <= m <= SKINNY_MAX_M)):
            x = torch.randn(M, K, dtype=ws[0].dtype, device=ws[0].device)
            out = torch.empty(M, N, dtype=x.dtype, device=x.device)

            def lib():
                for w in ws:
                    F.linear(x, w)
            lib_t = _time(lib, reps)
            sk_t, sk_cfg = float("inf"), None
            for cfg in _CONFIGS:
                # the smallest batch tile that holds M
                if not skinny_ok(M, N, K, cfg) or (cfg[0] > 1 and M <= 16 * (cfg[0] // 2)):
                    continue

                def sk(cfg=cfg):
                    for w in ws:
                        skinny_gemm(x, w, None, cfg, out)
                t = _time(sk, reps)
                if t < sk_t:
                    sk_t, sk_cfg = t, cfg
            best = sk_cfg if sk_t < lib_t * margin else None
            n = len(ws)
            res[(M, N, K)] = (best, lib_t * 1e3 / n, sk_t * 1e3 / n, sk_cfg)
            if best is not None:
                _plan[(M, N, K)] = best
            log.info("gemm M=%d N=%d K=%d: hipBLASLt %.1f us, skinny %s %.1f us -> %s", M, N, K,
                     lib_t * 1e3 / n, sk_cfg, sk_t * 1e3 / n, "skinny" if best else "hipBLASLt")
    log.info("skinny GEMM tuning: %d shapes in %.1f s", len(res), time.time() - t0)
    return res
