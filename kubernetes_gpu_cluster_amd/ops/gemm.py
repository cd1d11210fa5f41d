"""Linear layers on the GPU: hipBLASLt (``F.linear``), the hand-written K9 skinny
GEMM (``csrc/kernels/gemm_skinny.hip``) for small-batch decode, or the dense split-K
MFMA GEMM (``dense_gemm_splitk`` in ``csrc/kernels/moe.hip``: the K14 tiles with one
K-slice per XCD, fp32 slices summed by ``splitk_reduce``) for mid-size decode batches,
where hipBLASLt's few output tiles leave the long-K projections (the MLP down
projection, K = 14336) at ~1.8 TB/s.

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
# (M, N, K) -> (cfg, us) of the fastest SK_NORM variant, and (M, N, K) -> us of the path
# the plain plan runs (hipBLASLt or skinny); (M, K) -> us of a separate rms_norm.
_plan_norm: dict[tuple[int, int, int], tuple[tuple, float]] = {}
_chosen_us: dict[tuple[int, int, int], float] = {}
_rms_us: dict[tuple[int, int], float] = {}
_enabled = os.environ.get("KGC_SKINNY_GEMM", "1") != "0"

# dense split-K: (M, N, K) -> (bm, S) where it measured faster than hipBLASLt
SPLITK_MAX_M = 512
_SK_CONFIGS = [(bm, S) for bm in (64, 128) for S in (2, 4, 8)]
_plan_sk: dict[tuple[int, int, int], tuple[int, int]] = {}
_sk_enabled = os.environ.get("KGC_SPLITK_GEMM", "1") != "0"


def splitk_ok(M: int, N: int, K: int, cfg) -> bool:
    bm, S = cfg
    return 1 <= M <= SPLITK_MAX_M and N % 128 == 0 and K % 64 == 0 and K // 64 >= S


def splitk_gemm(x: torch.Tensor, w: torch.Tensor, cfg,
                out: Optional[torch.Tensor] = None,
                ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x W^T as S fp32 K-slices (one per XCD group) plus a reduction to x's dtype."""
    from . import _k
    bm, S = cfg
    M, N = x.shape[0], w.shape[0]
    if ws is None:
        ws = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    k = _k()
    k.dense_gemm_splitk(ws, x, w, bm)
    k.splitk_reduce(out, ws)
    return out


def splitk_gemm_silu(x: torch.Tensor, w: torch.Tensor, cfg,
                     out: Optional[torch.Tensor] = None,
                     ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(x Wg^T) * (x Wu^T) for a merged [gate; up] weight: the split-K slices are
    summed and activated in one pass (``splitk_reduce_silu``), so the [M, 2I] gate_up
    output is never materialised and no separate silu_mul runs."""
    from . import _k
    bm, S = cfg
    M, N = x.shape[0], w.shape[0]
    if ws is None:
        ws = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
    if out is None:
        out = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
    k = _k()
    k.dense_gemm_splitk(ws, x, w, bm)
    k.splitk_reduce_silu(out, ws)
    return out


def linear_silu(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu_mul(linear(x, w, bias)) over a merged gate_up weight, with the activation
    folded into the split-K reduction where the plan runs split-K at this (M, N, K)."""
    from . import silu_mul
    if (_plan_sk and bias is None and x.is_cuda and x.dim() == 2 and x.stride(1) == 1
            and x.stride(0) % 8 == 0 and w.shape[0] % 16 == 0):
        cfg = _plan_sk.get((x.shape[0], w.shape[0], w.shape[1]))
        if cfg is not None:
            return splitk_gemm_silu(x, w, cfg)
    return silu_mul(linear(x, w, bias))


def linear_add_rms(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor,
                   gamma: torch.Tensor, eps: float) -> tuple[torch.Tensor, torch.Tensor]:
    """residual += x W^T; returns (rms_norm(residual) * gamma, residual) -- a row-parallel
    projection (o / down, TP = 1) and the fused add + RMSNorm that consumes it.  Where the
    plan runs split-K at this (M, N, K), the slice reduction, residual add and norm are one
    kernel (``splitk_add_rms_norm``); otherwise the GEMM and ``fused_add_rms_norm`` run."""
    from . import _k, fused_add_rms_norm
    if (_plan_sk and x.is_cuda and x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and w.shape[0] <= 8192 and residual.is_contiguous()):
        cfg = _plan_sk.get((x.shape[0], w.shape[0], w.shape[1]))
        if cfg is not None:
            bm, S = cfg
            ws = torch.empty(S, x.shape[0], w.shape[0], dtype=torch.float32, device=x.device)
            out = torch.empty_like(residual)
            k = _k()
            k.dense_gemm_splitk(ws, x, w, bm)
            k.splitk_add_rms_norm(out, ws, residual, gamma, eps)
            return out, residual
    return fused_add_rms_norm(linear(x, w), residual, gamma, eps)


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
    if (_plan_sk and bias is None and x.is_cuda and x.dim() == 2 and x.stride(1) == 1
            and x.stride(0) % 8 == 0):
        cfg = _plan_sk.get((x.shape[0], w.shape[0], w.shape[1]))
        if cfg is not None:
            return splitk_gemm(x, w, cfg)
    return F.linear(x, w, bias)


def skinny_cfg(M: int, N: int, K: int):
    """The tuned skinny configuration for (M, N, K), or None where hipBLASLt runs."""
    return _plan.get((M, N, K))


def skinny_norm(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor],
                gamma: torch.Tensor, eps: float, cfg) -> torch.Tensor:
    """rms_norm(x) * gamma, then the GEMM, in one launch (K9 SK_NORM epilogue)."""
    from . import _k
    out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
    _k().skinny_gemm(out, x, w, bias, *cfg, 1, gamma, eps)
    return out


def skinny_accum(out: torch.Tensor, x: torch.Tensor, w: torch.Tensor,
                 bias: Optional[torch.Tensor], cfg) -> torch.Tensor:
    """out += x W^T (+ bias) in one launch (K9 SK_ACC epilogue: the residual add)."""
    from . import _k
    _k().skinny_gemm(out, x, w, bias, *cfg, 2, None, 1e-6)
    return out


def fused_norm_plan(M: int, norm_shapes, acc_shapes):
    """Configurations for a decoder layer whose RMSNorms run inside the GEMMs that
    consume them (SK_NORM on ``norm_shapes``) and whose residual adds run in the GEMMs
    that produce them (SK_ACC on ``acc_shapes``) -- or None unless tuning measured the
    SK_NORM GEMMs to cost less than the plain GEMMs plus the separate norm launches."""
    try:
        norm = [_plan_norm[(M, N, K)] for N, K in norm_shapes]
        acc = [_plan[(M, N, K)] for N, K in acc_shapes]
        plain = sum(_chosen_us[(M, N, K)] + _rms_us[(M, K)] for N, K in norm_shapes)
    except KeyError:
        return None
    if sum(t for _, t in norm) >= 0.98 * plain:
        return None
    return [c for c, _ in norm], acc


def clear_plan() -> None:
    _plan_sk.clear()
    _plan_norm.clear()
    _chosen_us.clear()
    _rms_us.clear()
    _plan.clear()


def plan() -> dict:
    return dict(_plan)


def splitk_plan() -> dict:
    return dict(_plan_sk)


def splitk_plan_has_m(M: int) -> bool:
    return _sk_enabled and any(k[0] == M for k in _plan_sk)


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
                reps: int = 3, norm_shapes=(), norm_max_m: int = 16, silu_shapes=(),
                tail_shapes=()) -> dict:
    """Time hipBLASLt against every skinny configuration for each weight shape and
    batch size M (decode buckets <= SKINNY_MAX_M) and record the skinny kernel where it
    is faster by more than ``1 - margin``.  Each timing sweeps ALL weights of the shape
    (every layer's copy) so the weights stream from HBM as in a real decode step,
    not from the 256 MB Infinity Cache.  Returns {(M, N, K): (chosen cfg or None,
    hipBLASLt us, best skinny us, best skinny cfg)}, times per GEMM call.
    ``silu_shapes``: (N, K) of merged gate_up weights, whose split-K candidates are timed
    with the fused SiLU reduction against hipBLASLt + silu_mul (``linear_silu``).
    ``tail_shapes``: (N, K) of row-parallel projections feeding a residual add + RMSNorm
    (``linear_add_rms``), timed with that norm on both sides."""
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
            _chosen_us[(M, N, K)] = (sk_t if best is not None else lib_t) * 1e3 / n
            if best is not None:
                _plan[(M, N, K)] = best
            if (N, K) in norm_shapes and M <= norm_max_m:
                _tune_norm(ws, x, out, M, N, K, reps)
            log.info("gemm M=%d N=%d K=%d: hipBLASLt %.1f us, skinny %s %.1f us -> %s", M, N, K,
                     lib_t * 1e3 / n, sk_cfg, sk_t * 1e3 / n, "skinny" if best else "hipBLASLt")
        if _sk_enabled:
            _tune_splitk(ws, N, K, [m for m in ms if SKINNY_MAX_M < m <= SPLITK_MAX_M], margin,
                         reps, res, silu=(N, K) in silu_shapes, tail=(N, K) in tail_shapes)
    log.info("GEMM tuning: %d shapes in %.1f s", len(res), time.time() - t0)
    return res


def _tune_splitk(ws, N: int, K: int, ms, margin: float, reps: int, res: dict,
                 silu: bool = False, tail: bool = False) -> None:
    """hipBLASLt vs every dense split-K configuration at each M in ``ms``, over all
    weights of the shape (HBM-resident, as in a decode step).  ``silu``: both sides
    include the SiLU-and-mul that follows a gate_up projection; ``tail``: both sides
    include the residual add + RMSNorm that consumes an o / down projection."""
    from . import _k, fused_add_rms_norm, silu_mul
    for M in sorted(set(ms)):
        if not splitk_ok(M, N, K, (64, 1)):
            continue
        x = torch.randn(M, K, dtype=ws[0].dtype, device=ws[0].device)
        out = torch.empty(M, N // 2 if silu else N, dtype=x.dtype, device=x.device)
        act = torch.empty(M, N // 2, dtype=x.dtype, device=x.device) if silu else None
        tail = tail and not silu and N <= 8192
        res_t = torch.zeros(M, N, dtype=x.dtype, device=x.device) if tail else None
        gamma = torch.ones(N, dtype=x.dtype, device=x.device) if tail else None

        def lib():
            for w in ws:
                y = F.linear(x, w)
                if silu:
                    silu_mul(y, act)
                elif tail:
                    fused_add_rms_norm(y, res_t, gamma, 1e-6)
        lib_t = _time(lib, reps)
        best_t, best_cfg = float("inf"), None

        def sk_tail(x, w, cfg, out, buf):
            _k().dense_gemm_splitk(buf, x, w, cfg[0])
            _k().splitk_add_rms_norm(out, buf, res_t, gamma, 1e-6)
        sk_fn = splitk_gemm_silu if silu else (sk_tail if tail else splitk_gemm)
        for cfg in _SK_CONFIGS:
            if not splitk_ok(M, N, K, cfg) or (cfg[0] == 128 and M <= 64):
                continue
            buf = torch.empty(cfg[1], M, N, dtype=torch.float32, device=x.device)

            def sk(cfg=cfg, buf=buf):
                for w in ws:
                    sk_fn(x, w, cfg, out, buf)
            t = _time(sk, reps)
            if t < best_t:
                best_t, best_cfg = t, cfg
        n = len(ws)
        chosen = best_cfg if best_t < lib_t * margin else None
        if chosen is not None:
            _plan_sk[(M, N, K)] = chosen
        res[(M, N, K)] = (chosen, lib_t * 1e3 / n, best_t * 1e3 / n, best_cfg)
        log.info("gemm M=%d N=%d K=%d%s: hipBLASLt %.1f us, split-K %s %.1f us -> %s", M, N, K,
                 " +silu" if silu else (" +add_rms" if tail else ""), lib_t * 1e3 / n,
                 best_cfg, best_t * 1e3 / n, "split-K" if chosen else "hipBLASLt")


def _tune_norm(ws, x, out, M: int, N: int, K: int, reps: int) -> None:
    """Time the SK_NORM variants (one m-tile) and a separate rms_norm launch at (M, K)."""
    from . import _k, rms_norm
    gamma = torch.ones(K, dtype=x.dtype, device=x.device)
    best_t, best_cfg = float("inf"), None
    for cfg in _CONFIGS:
        if cfg[0] != 1 or not skinny_ok(M, N, K, cfg):
            continue

        def fn(cfg=cfg):
            for w in ws:
                _k().skinny_gemm(out, x, w, None, *cfg, 1, gamma, 1e-6)
        t = _time(fn, reps)
        if t < best_t:
            best_t, best_cfg = t, cfg
    if best_cfg is not None:
        _plan_norm[(M, N, K)] = (best_cfg, best_t * 1e3 / len(ws))
    if (M, K) not in _rms_us:
        # inside a graph, as in the decode step: eager launches of a ~2 us kernel would
        # time the host's launch rate instead
        xn = torch.empty_like(x)
        rms_norm(x, gamma, 1e-6, xn)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(32):
                rms_norm(x, gamma, 1e-6, xn)
        _rms_us[(M, K)] = _time(g.replay, reps) * 1e3 / 32
