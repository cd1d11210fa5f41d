"""Linear layers on the GPU: hipBLASLt (``F.linear``), the hand-written K9 skinny
GEMM (``csrc/kernels/gemm_skinny.hip``) for small-batch decode (M <= 64), or the K9m
mid-batch decode GEMM (``csrc/kernels/gemm_decode.hip``: LDS-DMA ring, packed weight
tiles, XCD-mapped split-K with the K-slice reduction fused into the consumer) for
M = 65..512, where hipBLASLt leaves the long-K projections (the MLP down projection,
K = 14336) at ~1.8 TB/s.

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
import weakref
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
# merged gate_up (M, 2I, K) -> cfg of the SK_SILU skinny variant, where it measured faster
# than the plain plan + a silu_mul launch
_plan_silu: dict[tuple[int, int, int], tuple[int, int, int, bool]] = {}
# row-parallel (o / down) (M, N, K) -> cfg of the SK_ACC_NORM skinny variant (residual add
# and the consuming RMSNorm inside the GEMM launch), where it measured faster than the
# plain plan + fused_add_rms_norm; and the per-device tickets that variant draws
_plan_accnorm: dict[tuple[int, int, int], tuple[int, int, int, bool]] = {}
_tickets: dict[torch.device, torch.Tensor] = {}
# (M, N, K) -> the fastest skinny configuration, chosen over hipBLASLt or not: the
# norm-free small-M layer (skinny_acc_ss / skinny_rscale) runs every projection on K9
_best_sk: dict[tuple[int, int, int], tuple] = {}
_best_silu: dict[tuple[int, int, int], tuple] = {}     # the same for the SiLU epilogue
# norm-free layer (rs_plan): the fastest configuration of each epilogue AS IT RUNS there --
# ("ss" | "rs" | "rss", M, N, K) for SK_ACC_SS / SK_RSCALE / SK_RSCALE_SILU (the plain
# GEMM's ranking does not carry over: the epilogues cost differently per tile shape)
_best_rs: dict[tuple, tuple] = {}
_enabled = os.environ.get("KGC_SKINNY_GEMM", "1") != "0"

# K9m mid-batch decode GEMM (csrc/kernels/gemm_decode.hip), M in (SKINNY_MAX_M, DG_MAX_M]:
# (M, N, K, kind) -> (cfg, S) where it measured faster than hipBLASLt (+ the same consumer).
# kind: "plain" (qkv / lm_head / any linear), "silu" (merged gate_up -> silu_mul),
# "tail" (o / down -> residual add + RMSNorm).  S > 1: fp32 K-slices summed by the consumer.
DG_MAX_M = 512
_plan_dg: dict[tuple[int, int, int, str], tuple[int, int]] = {}
_dg_enabled = os.environ.get("KGC_DGEMM", "1") != "0"
# packed weight copies for the packed K9m tiles: (data_ptr, silu) -> [N/128, K/64, 8192]
# (data_ptr, silu) -> (weakref to the source weight, packed copy).  The weakref drops the
# entry when the weight dies: a later tensor allocated at the same address (the next
# engine in the same process, a test) must never pick up this weight's packed copy.
_packed: dict[tuple[int, bool], tuple] = {}


def _packed_get(w: torch.Tensor, silu: bool) -> Optional[torch.Tensor]:
    key = (w.data_ptr(), silu)
    e = _packed.get(key)
    if e is None:
        return None
    src = e[0]()
    if src is None:
        _packed.pop(key, None)
        return None
    if src.data_ptr() != w.data_ptr() or src.shape != w.shape:
        return None
    return e[1]


def _packed_put(w: torch.Tensor, silu: bool, p: torch.Tensor) -> None:
    key = (w.data_ptr(), silu)

    def drop(ref, key=key):
        e = _packed.get(key)
        if e is not None and e[0] is ref:
            del _packed[key]
    _packed[key] = (weakref.ref(w, drop), p)
_PACK_FRACTION = float(os.environ.get("KGC_DGEMM_PACK_FRACTION", "0.25"))


def _dg_info(cfg: int):
    from . import _k
    bm, bn, pk = _k().dgemm_cfg_info(cfg)
    return bm, bn, bool(pk)


def dgemm_ok(M: int, N: int, K: int) -> bool:
    return SKINNY_MAX_M < M <= DG_MAX_M and N % 128 == 0 and K % 64 == 0


def pack_decode_weights(plain: Iterable[torch.Tensor], silu: Iterable[torch.Tensor]) -> int:
    """Packed copies ([N/128][K/64][128 x 64] tiles, swizzle baked in: one contiguous 16 KB
    block per K-step of a column tile) of the decode-GEMM weights, made once at load time so
    the K9m weight stream reads HBM in whole blocks (~5.8 vs ~4.4 TB/s for the row-major
    tile walk, tools/dma_probe.hip).  ``silu``: merged gate_up weights, packed with gate and
    up 16-row groups interleaved for the fused SiLU epilogue.  Skipped (row-major K9m tiles
    only) when the copies would exceed KGC_DGEMM_PACK_FRACTION of device memory, e.g. a
    70B model on one GPU.  Call BEFORE the KV cache is sized.  Returns bytes packed."""
    if not _dg_enabled:
        return 0
    from . import _k
    todo = []
    for w, sl in [(w, False) for w in plain] + [(w, True) for w in silu]:
        if (w.is_cuda and w.dim() == 2 and w.dtype in (torch.bfloat16, torch.float16)
                and w.is_contiguous() and w.shape[0] % 128 == 0 and w.shape[1] % 64 == 0
                and _packed_get(w, sl) is None):
            todo.append((w, sl))
    need = sum(w.numel() * w.element_size() for w, _ in todo)
    if not todo:
        return 0
    free, total = torch.cuda.mem_get_info(todo[0][0].device)
    if need > _PACK_FRACTION * total or need > free - (8 << 30):
        log.info("K9m: %.1f GB of packed weights exceeds the budget; row-major tiles only",
                 need / 1e9)
        return 0
    for w, sl in todo:
        N, K = w.shape
        p = torch.empty(N // 128, K // 64, 8192, dtype=w.dtype, device=w.device)
        _k().dgemm_pack(p, w, sl)
        _packed_put(w, sl, p)
    log.info("K9m: packed %d decode weights (%.1f GB)", len(todo), need / 1e9)
    return need


def packed_weight(w: torch.Tensor, silu: bool = False) -> Optional[torch.Tensor]:
    return _packed_get(w, silu)


def cfg_packed(cfg: int) -> bool:
    return _dg_info(cfg)[2]


def _dg_weight(w: torch.Tensor, cfg: int, silu: bool) -> Optional[torch.Tensor]:
    return packed_weight(w, silu) if _dg_info(cfg)[2] else w


def dgemm(x: torch.Tensor, w: torch.Tensor, cfg: int, S: int, epi: int = 1,
          out: Optional[torch.Tensor] = None, silu_w: bool = False,
          rscale: Optional[torch.Tensor] = None, wk: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K9m: S == 1 -> x W^T in x's dtype (epi 1) or silu-paired [M, N/2] (epi 2);
    S > 1 -> the [S, M, N] fp32 K-slices (the caller's consumer sums them).  silu_w: a
    merged gate_up weight's slices from its SiLU-packed copy (packed cfgs: gate / up
    16-column groups interleaved per tile, ``splitk_reduce_silu(interleaved=True)``).
    rscale [M] fp32 (S == 1): output row m scaled by rscale[m] (before the SiLU).  wk: the
    weight in the layout ``cfg`` streams (default: ``w``'s packed copy or ``w``) -- the
    norm-free layer's gamma-folded copies."""
    from . import _k
    M, N = x.shape[0], w.shape[0]
    if wk is None:
        wk = _dg_weight(w, cfg, epi == 2 or silu_w)
    if wk is None:
        raise RuntimeError("K9m plan names a packed tile but the weight was not packed")
    if S > 1:
        out = torch.empty(S, M, N, dtype=torch.float32, device=x.device) if out is None else out
        _k().dgemm(out, x, wk, cfg, 0)
    else:
        if out is None:
            out = torch.empty(M, N // 2 if epi == 2 else N, dtype=x.dtype, device=x.device)
        _k().dgemm(out, x, wk, cfg, epi, rscale)
    return out


def _dg_plan(x: torch.Tensor, w: torch.Tensor, kind: str):
    if not _plan_dg or not x.is_cuda or x.dim() != 2 or x.stride(1) != 1 or x.stride(0) % 8:
        return None
    return _plan_dg.get((x.shape[0], w.shape[0], w.shape[1], kind))


def linear_silu(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu_mul(linear(x, w, bias)) over a merged gate_up weight: where the plan runs K9m
    at this (M, N, K) the activation is the GEMM's epilogue (S = 1) or rides the split-K
    reduction (``splitk_reduce_silu``), so the [M, 2I] gate_up output never exists."""
    from . import _k, silu_mul
    if bias is None and x.is_cuda and x.dim() == 2 and x.stride(1) == 1 and _plan_silu:
        cfg = _plan_silu.get((x.shape[0], w.shape[0], w.shape[1]))
        if cfg is not None:
            return skinny_silu(x, w, cfg)
    if bias is None:
        p = _dg_plan(x, w, "silu")
        if p is not None:
            cfg, S = p
            if S == 1:
                return dgemm(x, w, cfg, 1, epi=2)
            ws = dgemm(x, w, cfg, S, silu_w=True)
            out = torch.empty(x.shape[0], w.shape[0] // 2, dtype=x.dtype, device=x.device)
            _k().splitk_reduce_silu(out, ws, _dg_info(cfg)[2])
            return out
    return silu_mul(linear(x, w, bias))


def linear_qkv(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """The QKV projection for the fused RoPE / KV-write kernel: x W^T, or -- where the plan
    runs K9m split-K at this (M, N, K) -- its fp32 K-slices [S, M, N], which that kernel
    sums (``ops.rope_kv_write``), so the reduction needs no launch of its own."""
    p = _dg_plan(x, w, "qkv")
    if p is not None:
        cfg, S = p
        return dgemm(x, w, cfg, S)
    return linear(x, w)


def linear_add_rms(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor,
                   gamma: torch.Tensor, eps: float) -> tuple[torch.Tensor, torch.Tensor]:
    """residual += x W^T; returns (rms_norm(residual) * gamma, residual) -- a row-parallel
    projection (o / down, TP = 1) and the fused add + RMSNorm that consumes it.  Where the
    plan runs K9m split-K at this (M, N, K), the slice reduction, residual add and norm are
    one kernel (``splitk_add_rms_norm``); otherwise the GEMM and ``fused_add_rms_norm``."""
    from . import _k, fused_add_rms_norm
    if _plan_accnorm and x.is_cuda and x.dim() == 2 and x.stride(1) == 1:
        cfg = _plan_accnorm.get((x.shape[0], w.shape[0], w.shape[1]))
        if cfg is not None and residual.is_contiguous():
            out = torch.empty_like(residual)
            skinny_acc_norm(residual, x, w, gamma, eps, cfg, out)
            return out, residual
    p = _dg_plan(x, w, "tail")
    if p is not None and w.shape[0] <= 8192 and residual.is_contiguous():
        cfg, S = p
        if S > 1:
            ws = dgemm(x, w, cfg, S)
            out = torch.empty_like(residual)
            _k().splitk_add_rms_norm(out, ws, residual, gamma, eps)
            return out, residual
        return fused_add_rms_norm(dgemm(x, w, cfg, 1), residual, gamma, eps)
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
    if bias is None:
        p = _dg_plan(x, w, "plain")
        if p is not None:
            cfg, S = p
            if S == 1:
                return dgemm(x, w, cfg, 1)
            from . import _k
            ws = dgemm(x, w, cfg, S)
            out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
            _k().splitk_reduce(out, ws)
            return out
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


def skinny_silu(x: torch.Tensor, w: torch.Tensor, cfg,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(x Wg^T) * (x Wu^T) over the merged [gate; up] weight in one launch (K9
    SK_SILU epilogue): out [M, I]."""
    from . import _k
    if out is None:
        out = torch.empty(x.shape[0], w.shape[0] // 2, dtype=x.dtype, device=x.device)
    _k().skinny_gemm(out, x, w, None, *cfg, 3, None, 1e-6)
    return out


def _ticket(device: torch.device) -> torch.Tensor:
    t = _tickets.get(device)
    if t is None:
        t = _tickets[device] = torch.zeros(16, dtype=torch.int32, device=device)
    return t


def skinny_acc_norm(residual: torch.Tensor, x: torch.Tensor, w: torch.Tensor,
                    gamma: torch.Tensor, eps: float, cfg, out: torch.Tensor) -> torch.Tensor:
    """residual += x W^T; out = rms_norm(residual) * gamma -- one launch (K9 SK_ACC_NORM:
    the last workgroup of the grid normalises the finished rows)."""
    from . import _k
    _k().skinny_gemm(residual, x, w, None, *cfg, 4, gamma, eps, out, _ticket(x.device))
    return out


def fold_norm_weight(w: torch.Tensor, gamma: torch.Tensor) -> torch.Tensor:
    """W' = W diag(gamma) in W's dtype: rms_norm(x) W^T == rsqrt(mean(x^2) + eps) * x W'^T
    up to where the bf16 roundings fall (the norm-free small-M layer)."""
    return (w.float() * gamma.float()[None, :]).to(w.dtype).contiguous()


# the norm-free layer's sum-of-squares partials: a [16 * 256] fp32 buffer per producer,
# and at most 256 partials per row for the consumer (gemm_skinny.hip ssl[16][256])
RS_MAX_NSS = 256
RS_SSP_FLOATS = 16 * 256


def rs_plan(M: int, shapes) -> Optional[list]:
    """Skinny configurations of (qkv, o, gate_up, down) at this M for the norm-free layer
    (``LlamaForCausalLM._forward_rs``), or None: every projection needs a timed skinny
    configuration, gate_up its SiLU one, and the row scale holds M <= 4 * NW rows."""
    if M > 16:
        return None
    (nq, kq), (no, ko), (ng, kg), (nd, kd) = shapes
    try:
        c = [_best_rs.get(("rs", M, nq, kq)) or _best_sk[(M, nq, kq)],
             _best_rs.get(("ss", M, no, ko)) or _best_sk[(M, no, ko)],
             _best_rs.get(("rss", M, ng, kg)) or _best_silu[(M, ng, kg)],
             _best_rs.get(("ss", M, nd, kd)) or _best_sk[(M, nd, kd)]]
    except KeyError:
        return None
    if any(cfg[0] != 1 or M > 4 * cfg[2] for cfg in c):
        return None
    # the producers (o / down, SK_ACC_SS) leave N / (16 nt) partials per row: they must fit
    # the [16 * 256] ssp buffer, and the consumer (SK_RSCALE, ssl[16][256] in LDS) sums at
    # most 256 per row (kgc.skinny_gemm checks it at launch: fail here, at plan time)
    for cfg, n in ((c[1], no), (c[3], nd)):
        nss = n // (16 * cfg[1])
        if nss > RS_MAX_NSS or M * nss > RS_SSP_FLOATS:
            return None
    return c


def skinny_acc_ss(residual: torch.Tensor, x: torch.Tensor, w: torch.Tensor, cfg,
                  ssp: torch.Tensor) -> int:
    """residual += x W^T, and ssp[m, j] = sum over workgroup j's columns of the new
    residual row m squared (K9 SK_ACC_SS).  Returns the partials per row."""
    from . import _k
    _k().skinny_gemm(residual, x, w, None, *cfg, 5, None, 1e-6, None, None, ssp, 0)
    return w.shape[0] // (16 * cfg[1])


def skinny_rscale(x: torch.Tensor, w_folded: torch.Tensor, cfg, ssp: torch.Tensor, nss: int,
                  eps: float, out: torch.Tensor, silu: bool = False) -> torch.Tensor:
    """out = rsqrt(sum_j ssp[m, j] / K + eps) * x W'^T (K9 SK_RSCALE; silu: the SiLU pairs of
    a folded merged gate_up, SK_RSCALE_SILU) -- rms_norm(x) and the GEMM in one launch."""
    from . import _k
    _k().skinny_gemm(out, x, w_folded, None, *cfg, 7 if silu else 6, None, eps, None, None,
                     ssp, nss)
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


def norm_fused_cfg(M: int, N: int, K: int):
    """The SK_NORM configuration of a GEMM that can absorb its input RMSNorm at this M,
    where tuning measured it cheaper than the plain GEMM plus the norm launch; else None."""
    try:
        cfg, t = _plan_norm[(M, N, K)]
        plain = _chosen_us[(M, N, K)] + _rms_us[(M, K)]
    except KeyError:
        return None
    return cfg if t < 0.98 * plain else None


# offline K9m selections (tools/tune_dgemm_table.py): (M, N, K, kind) -> (cfg, S), or None
# where hipBLASLt won.  Start-up tuning skips these: its short interleaved timing picked
# configurations up to ~0.35 ms per batch-256 decode step apart from one engine start to
# the next; the offline table is the median of many more rounds, and makes the chosen
# kernels the same in every run.  Empty unless ``load_dg_table`` found a table.
_dg_table: dict[tuple[int, int, int, str], Optional[tuple[int, int]]] = {}


def dg_table_path(model: str, tp: int = 1) -> str:
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return os.path.join(root, "profiles", "tunableop", f"k9m_{model}_tp{tp}_gfx950.json")


def dg_fingerprint() -> dict:
    """What an offline K9m table's (cfg, S) picks depend on: the GPU architecture and its
    compute-unit count, and the id -> tile map of the loaded kernel library (ids index kCfg
    in gemm_decode.hip; a renumbered or retiled id would silently mean another kernel).
    The marketing name is recorded (``device``) but not compared: it comes from libdrm's
    amdgpu.ids, which the same MI355X resolves differently with and without rocprofv3
    preloaded ("AMD Radeon Graphics" vs the product name), and a run under the profiler
    then dropped the table and profiled other kernels than the service runs."""
    from . import _k
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    n = int(_k().dgemm_num_cfgs())
    return {"arch": str(getattr(props, "gcnArchName", "")).split(":")[0], "device": props.name,
            "cus": int(props.multi_processor_count),
            "num_cfgs": n, "cfgs": [list(_dg_info(c)[:2]) + [int(_dg_info(c)[2])]
                                    for c in range(n)]}


# fingerprint keys that must match (``device`` is informational, see dg_fingerprint)
_DG_FP_KEYS = ("arch", "cus", "num_cfgs", "cfgs")


def load_dg_table(model: str, tp: int = 1) -> int:
    """Read the offline K9m table of this model / TP degree (KGC_DGEMM_TABLE: another file;
    "0": none).  Returns the entries loaded.  The table's fingerprint (``dg_fingerprint``)
    must match the running GPU and kernel library, or the whole table is dropped and
    start-up tuning runs; each entry must also fit its shape (N % BN == 0,
    S <= K / 64) or it is dropped alone."""
    import json
    _dg_table.clear()
    path = os.environ.get("KGC_DGEMM_TABLE") or dg_table_path(model, tp)
    if path == "0" or not os.path.exists(path):
        return 0
    with open(path) as f:
        t = json.load(f)
    fp = t.get("fingerprint")
    cur = dg_fingerprint()
    if fp is None:
        log.warning("K9m: %s has no fingerprint; ignored (start-up tuning runs)", path)
        return 0
    diff = sorted(k for k in _DG_FP_KEYS if fp.get(k) != cur.get(k))
    if diff:
        log.warning("K9m: %s was tuned for another GPU or kernel library (%s differ); "
                    "ignored, start-up tuning runs", path, ", ".join(diff))
        return 0
    dropped = 0
    for e in t.get("entries", []):
        key = (int(e["M"]), int(e["N"]), int(e["K"]), str(e["kind"]))
        if e.get("cfg") is None:
            _dg_table[key] = None
            continue
        cfg, S = int(e["cfg"]), int(e["S"])
        if not (0 <= cfg < cur["num_cfgs"]) or key[1] % cur["cfgs"][cfg][1] or not (
                1 <= S <= key[2] // 64):
            dropped += 1
            continue
        _dg_table[key] = (cfg, S)
    if dropped:
        log.warning("K9m: %d entries of %s do not fit their shapes; dropped", dropped, path)
    log.info("K9m: %d offline selections from %s", len(_dg_table), path)
    return len(_dg_table)


def save_dg_table(path: str, res: dict, meta: dict) -> int:
    """Write the K9m decisions of a tuner run (``tune_skinny``'s result dict), with the
    fingerprint ``load_dg_table`` checks."""
    import json
    ent = []
    for key, v in sorted(res.items()):
        if len(key) != 4 or key[3] not in ("plain", "silu", "tail", "qkv"):
            continue
        M, N, K, kind = key
        chosen, lib_us, best_us, best = v
        ent.append({"M": M, "N": N, "K": K, "kind": kind,
                    "cfg": None if chosen is None else chosen[0],
                    "S": None if chosen is None else chosen[1],
                    "k9m_us": round(best_us, 2), "hipblaslt_us": round(lib_us, 2),
                    "best_k9m": list(best) if best else None})
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(dict(meta, fingerprint=dg_fingerprint(), entries=ent), f, indent=1)
    return len(ent)


def clear_plan() -> None:
    _dg_table.clear()
    _best_sk.clear()
    _best_silu.clear()
    _best_rs.clear()
    _plan_accnorm.clear()
    _plan_silu.clear()
    _plan_dg.clear()
    _plan_norm.clear()
    _chosen_us.clear()
    _rms_us.clear()
    _plan.clear()


def plan() -> dict:
    return dict(_plan)


def silu_plan() -> dict:
    return dict(_plan_silu)


def dgemm_plan() -> dict:
    return dict(_plan_dg)


def dgemm_plan_has_m(M: int, kind: str) -> bool:
    return _dg_enabled and any(k[0] == M and k[3] == kind for k in _plan_dg)


def tail_plan_has_m(M: int) -> bool:
    """A fused projection-tail plan at this M: K9m split-K (M > 64) or SK_ACC_NORM."""
    return dgemm_plan_has_m(M, "tail") or any(k[0] == M for k in _plan_accnorm)


def accnorm_plan() -> dict:
    return dict(_plan_accnorm)


def _tune_rs(ws, x, M: int, N: int, K: int, reps: int, kind: str) -> None:
    """Time the norm-free layer's epilogue ``kind`` on every configuration it can run
    (one m-tile, M <= 4 * NW; SiLU pairs: NT = 2) and record the fastest in _best_rs."""
    ssp = torch.zeros(RS_SSP_FLOATS, dtype=torch.float32, device=x.device)
    best_t, best = float("inf"), None
    for cfg in _CONFIGS:
        mt, nt, nw, _ = cfg
        if mt != 1 or M > 4 * nw or not skinny_ok(M, N, K, cfg) or (kind == "rss" and nt != 2):
            continue
        if kind == "ss":
            # a consumer sums at most RS_MAX_NSS partials per row (rs_plan checks it again)
            if N // (16 * nt) > RS_MAX_NSS or M * (N // (16 * nt)) > ssp.numel():
                continue
            res = torch.zeros(M, N, dtype=x.dtype, device=x.device)

            def fn(cfg=cfg, res=res):
                for w in ws:
                    skinny_acc_ss(res, x, w, cfg, ssp)
        else:
            out = torch.empty(M, N // 2 if kind == "rss" else N, dtype=x.dtype, device=x.device)

            def fn(cfg=cfg, out=out):
                for w in ws:
                    skinny_rscale(x, w, cfg, ssp, 256, 1e-6, out, silu=kind == "rss")
        t = _time_graphed(fn, reps)
        if t < best_t:
            best_t, best = t, cfg
    if best is not None:
        _best_rs[(kind, M, N, K)] = best
        log.info("gemm M=%d N=%d K=%d norm-free %s: %s %.1f us", M, N, K, kind, best,
                 best_t * 1e3 / len(ws))


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


def _graph_of(body):
    """``body`` captured once into a hipGraph; returns its replay."""
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    return g.replay


def _time_graphed(body, reps: int) -> float:
    """``_time`` of ``body`` captured in one hipGraph: candidates that differ in launch
    count are compared as a decode graph replays them (eager timing would add the host's
    launch rate to the side with more launches, or hide the in-graph kernel boundaries)."""
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    return _time(g.replay, reps)


@torch.inference_mode()
def tune_skinny(weights: Iterable[torch.Tensor], ms: Iterable[int], margin: float = 0.97,
                reps: int = 3, norm_shapes=(), norm_max_m: int = 16, silu_shapes=(),
                tail_shapes=(), qkv_dims=None, rs_shapes: bool = False) -> dict:
    """Time hipBLASLt against every skinny configuration for each weight shape and
    batch size M (decode buckets <= SKINNY_MAX_M) and record the skinny kernel where it
    is faster by more than ``1 - margin``.  Each timing sweeps ALL weights of the shape
    (every layer's copy) so the weights stream from HBM as in a real decode step,
    not from the 256 MB Infinity Cache.  Returns {(M, N, K): (chosen cfg or None,
    hipBLASLt us, best skinny us, best skinny cfg)}, times per GEMM call.
    ``silu_shapes``: (N, K) of merged gate_up weights, whose split-K candidates are timed
    with the fused SiLU reduction against hipBLASLt + silu_mul (``linear_silu``).
    ``tail_shapes``: (N, K) of row-parallel projections feeding a residual add + RMSNorm
    (``linear_add_rms``), timed with that norm on both sides.  ``rs_shapes``: also time the
    norm-free layer's epilogues at M <= 16 (tail -> SK_ACC_SS, norm -> SK_RSCALE, silu ->
    SK_RSCALE_SILU) for ``rs_plan``."""
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
            # graph-replayed, as a decode step runs them: timed eagerly, a sweep of 8-us
            # kernels measures the host's launch rate and ranks the configurations by it
            lib_t = _time_graphed(lib, reps)
            sk_t, sk_cfg = float("inf"), None
            for cfg in _CONFIGS:
                # the smallest batch tile that holds M
                if not skinny_ok(M, N, K, cfg) or (cfg[0] > 1 and M <= 16 * (cfg[0] // 2)):
                    continue

                def sk(cfg=cfg):
                    for w in ws:
                        skinny_gemm(x, w, None, cfg, out)
                t = _time_graphed(sk, reps)
                if t < sk_t:
                    sk_t, sk_cfg = t, cfg
            best = sk_cfg if sk_t < lib_t * margin else None
            if sk_cfg is not None:
                _best_sk[(M, N, K)] = sk_cfg
            n = len(ws)
            res[(M, N, K)] = (best, lib_t * 1e3 / n, sk_t * 1e3 / n, sk_cfg)
            _chosen_us[(M, N, K)] = (sk_t if best is not None else lib_t) * 1e3 / n
            if best is not None:
                _plan[(M, N, K)] = best
            if (N, K) in norm_shapes and M <= norm_max_m:
                _tune_norm(ws, x, out, M, N, K, reps)
            if (N, K) in silu_shapes:
                _tune_silu(ws, x, M, N, K, reps, margin)
            if (N, K) in tail_shapes and N % 512 == 0 and N <= 8192:
                _tune_accnorm(ws, x, M, N, K, reps, margin)
            if M <= 16 and rs_shapes:
                kind = ("rss" if (N, K) in silu_shapes else "ss" if (N, K) in tail_shapes
                        else "rs" if (N, K) in norm_shapes else None)
                if kind is not None:
                    _tune_rs(ws, x, M, N, K, reps, kind)
            log.info("gemm M=%d N=%d K=%d: hipBLASLt %.1f us, skinny %s %.1f us -> %s", M, N, K,
                     lib_t * 1e3 / n, sk_cfg, sk_t * 1e3 / n, "skinny" if best else "hipBLASLt")
        if _dg_enabled:
            qd = (qkv_dims or {}).get((N, K))
            kind = ("silu" if (N, K) in silu_shapes else
                    "tail" if (N, K) in tail_shapes else "qkv" if qd else "plain")
            _tune_dgemm(ws, N, K, [m for m in ms if SKINNY_MAX_M < m <= DG_MAX_M], margin,
                        reps, res, kind, qd)
    log.info("GEMM tuning: %d shapes in %.1f s", len(res), time.time() - t0)
    return res


# K9m candidates per M range: (cfg ids, split factors).  Packed tiles only when the weight
# was packed; 4 loader waves (6, 7), split loaders (8, 9) and XCD-paired 128-row blocks (10)
# per tools/dgemm_bench.py.
_DG_SPLITS = tuple(int(v) for v in
                   os.environ.get("KGC_DGEMM_SPLITS", "1,2,3,4,5,6,8,12,16").split(","))
# a K9m launch runs ONE workgroup per CU: candidates whose grid exceeds the 256 CUs by more
# than this are a second round of workgroups behind the first and are not timed
_DG_MAX_GRID = 264
# the tuner's refinement: this many fastest K9m candidates re-timed (with hipBLASLt) in
# this many interleaved rounds, the median decides
_DG_REFINE = int(os.environ.get("KGC_DGEMM_REFINE", "3"))
_DG_REFINE_ROUNDS = int(os.environ.get("KGC_DGEMM_REFINE_ROUNDS", "5"))


def _dg_candidates(M: int, N: int, K: int, kind: str, packed: bool):
    # (K9v / K9r, measured slower than K9m on every M = 256 shape, are not in the engine's
    # library: tools/research/; profiles/README.md "Round 3: K9r" / "Round 3: K9v")
    from . import _k
    # 11-14: packed 64 / 80 / 112-wide column tiles (gemm_decode.hip kCfg) for the narrow
    # shards of a TP = 8 rank
    cfgs = [5, 7, 2, 14, 11] if M <= 128 else [6, 8, 4, 0, 10, 11, 12, 13, 14]
    out = []
    for c in range(_k().dgemm_num_cfgs()):
        if c not in cfgs:
            continue
        bm, bn, pk = _dg_info(c)
        if (pk and not packed) or N % bn:
            continue
        epis = int(_k().dgemm_cfg_epis(c))
        if kind == "silu" and not (epis >> 2) & 1 and ((M + bm - 1) // bm) * (N // bn) >= 192:
            continue            # S = 1 would need the SiLU epilogue this tile does not have
        # S = 3, 5, 6 fill the CUs where powers of two do not (qkv at M = 256: 48
        # column tiles x 5 = 240 workgroups vs 192 at S = 4); no XCD pairing for them.
        # gate_up + SiLU: the fused epilogue (S = 1) where its column tiles fill the chip,
        # split-K slices + the SiLU reduction where they do not (Llama-3-70B at TP = 8:
        # 56 tiles at M = 256, 73 us on hipBLASLt in the phantom-rank anatomy)
        tiles = ((M + bm - 1) // bm) * (N // bn)
        splits = (1,) if kind == "silu" and tiles >= 192 else _DG_SPLITS
        for S in splits:
            if S > K // 64 or (S > 1 and tiles * S > _DG_MAX_GRID):
                continue
            if S == 1 and kind == "silu" and not (epis >> 2) & 1:
                continue
            out.append((c, S))
    return out


def _tune_dgemm(ws, N: int, K: int, ms, margin: float, reps: int, res: dict,
                kind: str, qkv_dims=None) -> None:
    """hipBLASLt vs the K9m candidates at each M in ``ms``, over all weights of the shape
    (HBM-resident, as in a decode step), each side timed WITH its consumer: "silu" the
    SiLU-and-mul, "tail" the residual add + RMSNorm, "qkv" the fused RoPE / KV-write /
    decode-attention kernel (which sums the K-slices in its prologue), "plain" the split-K
    reduction."""
    from . import (_k, decode_partials, fused_add_rms_norm, paged_attention_decode_rope,
                   silu_mul)
    packed = all(packed_weight(w, kind == "silu") is not None for w in ws)
    for M in sorted(set(ms)):
        if not dgemm_ok(M, N, K) or (kind == "tail" and N > 8192):
            continue
        key = (M, N, K, kind)
        if key in _dg_table:
            fixed = _dg_table[key]
            if fixed is None or packed or not _dg_info(fixed[0])[2]:
                if fixed is not None:
                    _plan_dg[key] = fixed
                res[key] = (fixed, float("nan"), float("nan"), fixed)
                continue
        dev, dt = ws[0].device, ws[0].dtype
        x = torch.randn(M, K, dtype=dt, device=dev)
        res_t = torch.zeros(M, N, dtype=dt, device=dev) if kind == "tail" else None
        gamma = torch.ones(N, dtype=dt, device=dev) if kind == "tail" else None
        act = torch.empty(M, N // 2, dtype=dt, device=dev) if kind == "silu" else None
        if kind == "qkv":
            # the decode step's real consumer: the fused RoPE / KV-write / attention kernel,
            # whose prologue sums the K-slices -- over a one-token context per row, so what
            # it adds per split factor is that prologue, not the attention itself (the
            # earlier rope_kv_write stand-in read the slices differently)
            nq, nkv, hd = qkv_dims
            pos = torch.zeros(M, dtype=torch.int64, device=dev)
            slots = (torch.arange(M, dtype=torch.int64, device=dev) + 1) * 32
            cs = torch.zeros(1, hd, dtype=torch.float32, device=dev)
            kc = torch.zeros(M + 1, nkv, 32, hd, dtype=dt, device=dev)
            vc = torch.zeros(M + 1, nkv, 4, hd, 8, dtype=dt, device=dev)
            bt = (torch.arange(M, dtype=torch.int32, device=dev) + 1).view(M, 1)
            cl = torch.ones(M, dtype=torch.int32, device=dev)
            wsp = decode_partials(M, nq, hd, 1, 32, dev)

            def consume(y):
                paged_attention_decode_rope(y, pos, cs, kc, vc, slots, nq, nkv, hd, bt, cl,
                                            hd ** -0.5, workspace=wsp, grid_z=1, dtype=dt)

        def lib():
            for w in ws:
                y = F.linear(x, w)
                if kind == "silu":
                    silu_mul(y, act)
                elif kind == "tail":
                    fused_add_rms_norm(y, res_t, gamma, 1e-6)
                elif kind == "qkv":
                    consume(y)
        lib_t = _time(lib, reps)
        best_t, best_cfg = float("inf"), None
        timed = []                  # (t, (cfg, S), run) of every candidate
        for cfg, S in _dg_candidates(M, N, K, kind, packed):
            wl = [_dg_weight(w, cfg, kind == "silu") for w in ws]
            il = kind == "silu" and _dg_info(cfg)[2]      # packed SiLU tiles: interleaved
            buf = (torch.empty(S, M, N, dtype=torch.float32, device=x.device) if S > 1 else
                   torch.empty(M, N // 2 if kind == "silu" else N, dtype=x.dtype,
                               device=x.device))
            red = torch.empty(M, N // 2 if kind == "silu" else N, dtype=x.dtype, device=x.device)

            def run(cfg=cfg, S=S, wl=wl, buf=buf, red=red, il=il):
                for w in wl:
                    if S == 1:
                        _k().dgemm(buf, x, w, cfg, 2 if kind == "silu" else 1)
                        if kind == "tail":
                            fused_add_rms_norm(buf, res_t, gamma, 1e-6)
                        elif kind == "qkv":
                            consume(buf)
                    else:
                        _k().dgemm(buf, x, w, cfg, 0)
                        if kind == "qkv":
                            consume(buf)
                        elif kind == "silu":
                            _k().splitk_reduce_silu(red, buf, il)
                        elif kind == "tail":
                            _k().splitk_add_rms_norm(red, buf, res_t, gamma, 1e-6)
                        else:
                            _k().splitk_reduce(red, buf)
            t = _time(run, reps)
            timed.append((t, (cfg, S), run))
        # refine: the few fastest candidates and the library re-timed in interleaved
        # rounds, median of each -- one short pass ranked near-ties by clock noise (the
        # same tree picked configurations 1-3 us per call apart from one engine start to
        # the next: ~0.25 ms of a batch-256 decode step).  The rounds replay each side
        # captured in a hipGraph, as the decode step runs it: eagerly timed, Llama-3-8B's
        # down_proj ranked S = 6 ahead of S = 8, which runs 41.5 vs 33.4 us in the engine's
        # graphs (profiles/k9m_tuner_eager_vs_graph_r5.txt)
        timed.sort(key=lambda e: e[0])
        top = timed[:_DG_REFINE]
        if top:
            rounds: dict = {c: [] for _, c, _ in top}
            lib_r = []
            lib_g = _graph_of(lib)
            graphs = [(c, _graph_of(fn)) for _, c, fn in top]
            for _ in range(_DG_REFINE_ROUNDS):
                lib_r.append(_time(lib_g, reps))
                for c, g in graphs:
                    rounds[c].append(_time(g, reps))
            del graphs, lib_g
            med = {c: sorted(v)[len(v) // 2] for c, v in rounds.items()}
            best_cfg = min(med, key=med.get)
            best_t = med[best_cfg]
            lib_t = sorted(lib_r)[len(lib_r) // 2]
        n = len(ws)
        chosen = best_cfg if best_t < lib_t * margin else None
        if chosen is not None:
            _plan_dg[(M, N, K, kind)] = chosen
        res[(M, N, K, kind)] = (chosen, lib_t * 1e3 / n, best_t * 1e3 / n, best_cfg)
        log.info("gemm M=%d N=%d K=%d %s: hipBLASLt %.1f us, K9m %s %.1f us -> %s", M, N, K,
                 kind, lib_t * 1e3 / n, best_cfg, best_t * 1e3 / n,
                 "K9m" if chosen else "hipBLASLt")


def _tune_silu(ws, x, M: int, N: int, K: int, reps: int, margin: float) -> None:
    """Time the SK_SILU variants against the plain plan (skinny or hipBLASLt, as just
    chosen) followed by silu_mul, over every layer's gate_up weight, both in a graph
    (eager timing called M = 1-4 a tie; in the decode graph the separate silu_mul launch
    costs ~4.7 us per layer)."""
    from . import silu_mul
    if os.environ.get("KGC_SKINNY_SILU", "1") == "0":
        return
    act = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)

    def sep():
        for w in ws:
            silu_mul(linear(x, w), act)
    sep_t = _time_graphed(sep, reps)
    best_t, best_cfg = float("inf"), None
    for cfg in _CONFIGS:
        if cfg[1] != 2 or not skinny_ok(M, N, K, cfg) or (cfg[0] > 1 and M <= 16 * (cfg[0] // 2)):
            continue

        def fn(cfg=cfg):
            for w in ws:
                skinny_silu(x, w, cfg, act)
        t = _time_graphed(fn, reps)
        if t < best_t:
            best_t, best_cfg = t, cfg
    n = len(ws)
    # both sides are our kernels timed the same way (graphed): the fused one wins when it
    # is faster at all (the margin guards the custom-vs-library choices; here it kept a
    # 42.4 vs 43.7 us / layer SK_SILU out at M = 1)
    if best_cfg is not None:
        _best_silu[(M, N, K)] = best_cfg
    if best_cfg is not None and best_t < sep_t:
        _plan_silu[(M, N, K)] = best_cfg
    log.info("gemm M=%d N=%d K=%d silu: plan + silu_mul %.1f us, SK_SILU %s %.1f us -> %s",
             M, N, K, sep_t * 1e3 / n, best_cfg, best_t * 1e3 / n,
             "SK_SILU" if (M, N, K) in _plan_silu else "separate")


def _tune_accnorm(ws, x, M: int, N: int, K: int, reps: int, margin: float) -> None:
    """Time SK_ACC_NORM against the plain plan + fused_add_rms_norm, both captured in a
    graph (the separate side is two launches per layer: eager timing would measure the
    host's launch rate)."""
    from . import fused_add_rms_norm
    if os.environ.get("KGC_SKINNY_ACC_NORM", "1") == "0":
        return
    gamma = torch.ones(N, dtype=x.dtype, device=x.device)
    res = torch.zeros(M, N, dtype=x.dtype, device=x.device)
    out = torch.empty_like(res)

    def sep():
        for w in ws:
            fused_add_rms_norm(linear(x, w), res, gamma, 1e-6)
    sep_t = _time_graphed(sep, reps)
    best_t, best_cfg = float("inf"), None
    for cfg in _CONFIGS:
        if not skinny_ok(M, N, K, cfg) or (cfg[0] > 1 and M <= 16 * (cfg[0] // 2)):
            continue

        def fn(cfg=cfg):
            for w in ws:
                skinny_acc_norm(res, x, w, gamma, 1e-6, cfg, out)
        t = _time_graphed(fn, reps)
        if t < best_t:
            best_t, best_cfg = t, cfg
    n = len(ws)
    if best_cfg is not None and best_t < sep_t * margin:
        _plan_accnorm[(M, N, K)] = best_cfg
    log.info("gemm M=%d N=%d K=%d tail: plan + add_rms_norm %.1f us, SK_ACC_NORM %s %.1f us "
             "-> %s", M, N, K, sep_t * 1e3 / n, best_cfg, best_t * 1e3 / n,
             "SK_ACC_NORM" if (M, N, K) in _plan_accnorm else "separate")


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
        t = _time_graphed(fn, reps)
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
