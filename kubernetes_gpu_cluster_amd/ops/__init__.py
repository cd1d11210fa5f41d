"""Fused ops: gfx950 HIP kernels (``torch.ops.kgc``) for GPU tensors, the
pure-PyTorch reference (``ops.reference``) for CPU tensors.

There is exactly one GPU implementation per op.  If a GPU tensor reaches an op
and the in-tree extension ``_kgc_ops.so`` is not loadable, the op raises: there
is no silent eager fallback on the GPU path.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import reference as ref

# KGC_HIP_DEBUG=1: the bounds-checking build (``KGC_HIP_DEBUG=1 python csrc/build.py``)
DEBUG = os.environ.get("KGC_HIP_DEBUG", "0") not in ("", "0")
_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "_kgc_ops_debug.so" if DEBUG else "_kgc_ops.so")
# KGC_OPS_SO=path: another build of the same library (same-box A/B of two kernel builds)
_SO = os.environ.get("KGC_OPS_SO") or _SO
_loaded: Optional[bool] = None
_load_err: Optional[str] = None


def load_extension(strict: bool = False) -> bool:
    """Load the HIP kernel library once.  strict=True raises if unavailable."""
    global _loaded, _load_err
    if _loaded is None:
        try:
            if not os.path.exists(_SO):
                raise FileNotFoundError(f"{_SO} not built (run `python csrc/build.py`)")
            torch.ops.load_library(_SO)
            _loaded = True
        except Exception as e:  # noqa: BLE001 - report reason on use
            _loaded, _load_err = False, f"{type(e).__name__}: {e}"
    if strict and not _loaded:
        raise RuntimeError(f"kgc HIP extension unavailable: {_load_err}")
    return bool(_loaded)


def extension_path() -> str:
    return _SO


class KernelDebugCheckFailed(RuntimeError):
    """A debug-build kernel read an out-of-range block-table entry, slot or length."""


def debug_check() -> None:
    """Debug build: raise if any K1/K2/K3 bounds check tripped since the last call (the
    kernel printed the offending value and clamped it).  No-op in release builds."""
    if not DEBUG or not load_extension():
        return
    torch.cuda.synchronize()
    err = int(torch.ops.kgc.debug_errors())
    if err:
        which = [n for b, n in ((1, "paged decode (K1)"), (2, "prefill attention (K2)"),
                                (4, "rope / KV write (K3)")) if err & b]
        raise KernelDebugCheckFailed(f"device bounds check failed in {', '.join(which)}; "
                                     f"see the kernel's printf above")


def _k():
    load_extension(strict=True)
    return torch.ops.kgc


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def fused_small_m_enabled() -> bool:
    """KGC_FUSED_SMALL_M=0 turns off the fused small-batch decoder layer (models/llama.py)."""
    return os.environ.get("KGC_FUSED_SMALL_M", "1") != "0"


# ------------------------------------------------------------------ norms
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(x):
        r = ref.rms_norm(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    x2 = x.reshape(-1, x.shape[-1]) if x.is_contiguous() else x
    out = torch.empty(x2.shape, dtype=x.dtype, device=x.device) if out is None else out
    _k().rms_norm(out.view(x2.shape), x2, None, w, eps)
    return out.view(x.shape)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                       eps: float) -> tuple[torch.Tensor, torch.Tensor]:
    """In place: residual += x; x = rms_norm(residual) * w.  Returns (x, residual)."""
    if not _gpu(x):
        o, r = ref.fused_add_rms_norm(x, residual, w, eps)
        x.copy_(o)
        residual.copy_(r)
        return x, residual
    x2 = x.view(-1, x.shape[-1])
    _k().rms_norm(x2, x2, residual.view(-1, x.shape[-1]), w, eps)
    return x, residual


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5):
    if not _gpu(x):
        return ref.layer_norm(x, w, b, eps)
    x2 = x.reshape(-1, x.shape[-1]).contiguous()
    out = torch.empty_like(x2)
    _k().layer_norm(out, x2, w, b, eps)
    return out.view(x.shape)


def silu_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(x):
        return ref.silu_mul(x)
    I = x.shape[-1] // 2
    x2 = x.view(-1, x.shape[-1])
    if out is None:
        out = torch.empty(x2.shape[0], I, dtype=x.dtype, device=x.device)
    _k().silu_mul(out, x2)
    return out.view(*x.shape[:-1], I)


# ------------------------------------------------------------------ rope + kv cache
def rope_kv_write(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                  num_heads: int, num_kv_heads: int, head_dim: int,
                  q_norm_w: Optional[torch.Tensor] = None,
                  k_norm_w: Optional[torch.Tensor] = None, eps: float = 1e-6,
                  use_rope: bool = True, k_scale: float = 1.0,
                  v_scale: float = 1.0, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """k_cache / v_cache may be fp8 (torch.float8_e4m3fn): values are stored as
    fp8(x / scale).  On the GPU ``qkv`` may also be the K9m split-K slices of the QKV
    projection (fp32 [S, T, N], ops/gemm.py linear_qkv): the kernel sums them, and
    ``dtype`` names the activation dtype of q."""
    if not _gpu(qkv):
        return ref.rope_qk_kv_write(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping,
                                    num_heads, num_kv_heads, head_dim, q_norm_w, k_norm_w, eps,
                                    use_rope, k_scale, v_scale)
    sl = qkv.dim() == 3
    T = qkv.shape[1] if sl else qkv.shape[0]
    q = torch.empty(T, num_heads, head_dim, dtype=(dtype or qkv.dtype) if sl else qkv.dtype,
                    device=qkv.device)
    _k().rope_kv_write(qkv, positions, cos_sin, q, k_cache, v_cache, slot_mapping, q_norm_w,
                       k_norm_w, num_heads, num_kv_heads, head_dim, eps, use_rope, k_scale,
                       v_scale)
    return q


def kv_write_rope(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                  num_heads: int, num_kv_heads: int, head_dim: int,
                  k_norm_w: Optional[torch.Tensor] = None, eps: float = 1e-6,
                  k_scale: float = 1.0, v_scale: float = 1.0) -> None:
    """rope_kv_write for k / v only (GPU, bf16 / f16 qkv [T, N]): the q part is left to
    ``prefill_attention_rope``, which rotates it as it loads it."""
    q = torch.empty(0, dtype=qkv.dtype, device=qkv.device)
    _k().rope_kv_write(qkv, positions, cos_sin, q, k_cache, v_cache, slot_mapping,
                       k_norm_w, k_norm_w, num_heads, num_kv_heads, head_dim, eps, True,
                       k_scale, v_scale)


# ------------------------------------------------------------------ attention
DECODE_PARTITION = 64        # tokens per wave-iteration of the 4-wave decode kernel
DECODE_CHUNK = 32            # tokens per pipelined step of K1w
DECODE_TARGET_WAVES = 2048   # K1w: 8 resident waves per CU (2 per SIMD at 256 VGPRs)
DECODE_WAVE_MIN_PAIRS = 64   # attention_decode.hip DEC_WAVE_MIN_PAIRS
DECODE_LONG_PAIRS = 256      # attention_decode.hip DEC_LONG_PAIRS
DECODE_LONG_TARGET_WAVES = 1024
PREFILL_BLOCK_M = 128


def decode_wave_kernel() -> bool:
    """K1w (one wave per (seq, kv-head, z-slice), csrc/kernels/attention_decode.hip) unless
    KGC_DECODE_WAVE=0 selects the 4-wave workgroup kernel; the C++ launcher reads the same
    variable, so the Z chosen here and the kernel that runs always agree."""
    return os.environ.get("KGC_DECODE_WAVE", "1") != "0"


def decode_uses_wave(batch: int, num_kv_heads: int) -> bool:
    """The kernel a launch of this grid takes: K1w from DECODE_WAVE_MIN_PAIRS (seq, kv-head)
    pairs up (at B = 1 the 4-wave kernel's 4x finer context split wins: 9.3 vs 12.3 us)."""
    lim = int(os.environ.get("KGC_DECODE_WAVE_MIN_PAIRS", DECODE_WAVE_MIN_PAIRS))
    return decode_wave_kernel() and batch * num_kv_heads >= lim


def decode_max_z(max_blocks: int, block_size: int) -> int:
    """The largest Z either kernel picks for this context capacity."""
    ctx = max_blocks * block_size
    wave = math.ceil(math.ceil(ctx / DECODE_CHUNK) / 2)     # >= 2 chunks per K1w slice
    four = math.ceil(math.ceil(ctx / DECODE_PARTITION) / 4)
    return max(1, min(1024, max(wave if decode_wave_kernel() else 1, four)))


def decode_partials(batch: int, num_heads: int, head_dim: int, max_blocks: int,
                    block_size: int, device) -> tuple:
    """Per-z-slice (max, sum, O) partials of the split-context decode kernels (static:
    graph-capturable), flat: row (seq, q-head) * Z + z, for every Z ``decode_grid_z`` picks
    at any batch <= ``batch`` (Z <= decode_max_z, and B * Z bounded by the wave targets:
    K1w B * nkv * Z <= 2 x 2048, the 4-wave kernel B * nkv * 4 * Z <= 2 x 4096).  Unused
    when the grid has a single z-slice."""
    Z = decode_max_z(max_blocks, block_size)
    rows = min(batch * Z, 2 * 4096 + batch)
    ml = torch.empty(rows * num_heads, dtype=torch.float32, device=device)
    es = torch.empty(rows * num_heads, dtype=torch.float32, device=device)
    tmp = torch.empty(rows * num_heads, head_dim, dtype=torch.float32, device=device)
    return ml, es, tmp


def _decode_z_cap(ws, B: int, nq: int) -> int:
    """Largest Z the workspace holds for a batch of B rows of nq heads."""
    return max(1, min(1024, ws[0].numel() // max(1, B * nq)))


def decode_grid_z(batch: int, num_kv_heads: int, max_ctx: int, target_waves: int = 0) -> int:
    """z-slices of the decode grid: enough waves to fill 256 CUs, bounded by the
    context (K1w: two 32-token chunks per wave; 4-wave kernel: 64-token partitions) and by
    the 1024 slices the reduce kernel merges.  Z == 1 (large batches) lets the kernel
    write its output directly."""
    pairs = max(1, batch * num_kv_heads)
    if decode_uses_wave(batch, num_kv_heads):
        chunks = max(1, math.ceil(max_ctx / DECODE_CHUNK))
        # from DECODE_LONG_PAIRS pairs up: ~4 waves per CU of longer slices (the kernel
        # also keeps those slices >= 10 chunks, attention_decode.hip DEC_LONG_MIN_CHUNKS)
        tgt = target_waves or (DECODE_LONG_TARGET_WAVES if pairs >= DECODE_LONG_PAIRS
                               else DECODE_TARGET_WAVES)
        want = math.ceil(tgt / pairs)
        return max(1, min(want, math.ceil(chunks / 2), 1024))
    parts = max(1, math.ceil(max_ctx / DECODE_PARTITION))
    want = math.ceil((target_waves or 4096) / (pairs * 4))
    return max(1, min(want, math.ceil(parts / 4), 1024))


def paged_attention_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, context_lens: torch.Tensor, scale: float,
                           workspace=None, grid_z: int = 1,
                           out: Optional[torch.Tensor] = None, k_scale: float = 1.0,
                           v_scale: float = 1.0) -> torch.Tensor:
    if not _gpu(q):
        return ref.paged_attention_decode(q, k_cache, v_cache, block_tables, context_lens, scale,
                                          k_scale, v_scale)
    B, nq, d = q.shape
    if out is None:
        out = torch.empty_like(q)
    if workspace is None:
        workspace = decode_partials(B, nq, d, block_tables.shape[1], k_cache.shape[2], q.device)
    ml, es, tmp = workspace
    grid_z = min(grid_z, _decode_z_cap(workspace, B, nq))
    _k().paged_decode(out, q, k_cache, v_cache, block_tables, context_lens, ml, es, tmp,
                      grid_z, scale, k_scale, v_scale)
    return out


def paged_attention_decode_rope(qkv: torch.Tensor, positions: torch.Tensor,
                                cos_sin: torch.Tensor, k_cache: torch.Tensor,
                                v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                                num_heads: int, num_kv_heads: int, head_dim: int,
                                block_tables: torch.Tensor, context_lens: torch.Tensor,
                                scale: float, q_norm_w: Optional[torch.Tensor] = None,
                                k_norm_w: Optional[torch.Tensor] = None, eps: float = 1e-6,
                                use_rope: bool = True, workspace=None, grid_z: int = 1,
                                k_scale: float = 1.0, v_scale: float = 1.0,
                                dtype: Optional[torch.dtype] = None,
                                row_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``rope_kv_write`` + ``paged_attention_decode`` of a decode-only batch in ONE
    launch (K1 with K3/K5/K6 as its prologue): q is built in registers from the QKV
    projection (or its K9m fp32 split-K slices [S, B, N]), the new token's k / v are
    written to the cache by the workgroup that reads them back.  -> [B, nq, d].
    ``row_scale`` [B] fp32: projection row b is scaled by it before its rounding (the
    norm-free layer's rsqrt(mean(x^2) + eps) over a gamma-folded QKV weight)."""
    if not _gpu(qkv):
        if row_scale is not None:
            qkv = (qkv.float().sum(0) if qkv.dim() == 3 else qkv.float()) * row_scale[:, None]
            qkv = qkv.to(dtype or torch.float32)
        q = ref.rope_qk_kv_write(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping,
                                 num_heads, num_kv_heads, head_dim, q_norm_w, k_norm_w, eps,
                                 use_rope, k_scale, v_scale)
        return ref.paged_attention_decode(q, k_cache, v_cache, block_tables, context_lens, scale,
                                          k_scale, v_scale)
    sl = qkv.dim() == 3
    B = qkv.shape[1] if sl else qkv.shape[0]
    out = torch.empty(B, num_heads, head_dim, dtype=(dtype or qkv.dtype) if sl else qkv.dtype,
                      device=qkv.device)
    if workspace is None:
        workspace = decode_partials(B, num_heads, head_dim, block_tables.shape[1],
                                    k_cache.shape[2], qkv.device)
    ml, es, tmp = workspace
    grid_z = min(grid_z, _decode_z_cap(workspace, B, num_heads))
    _k().paged_decode_rope(out, qkv, positions, cos_sin, k_cache, v_cache, slot_mapping,
                           q_norm_w, k_norm_w, block_tables, context_lens, ml, es, tmp,
                           num_heads, grid_z, scale, eps, use_rope, k_scale, v_scale,
                           row_scale)
    return out


def prefill_work_list(query_lens: list[int], seq_lens: list[int]) -> tuple[list[int], list[int]]:
    """(seq, 128-row block) work items, heaviest (most keys) first."""
    items = []
    for i, (ql, sl) in enumerate(zip(query_lens, seq_lens)):
        ctx0 = sl - ql
        for mb in range((ql + PREFILL_BLOCK_M - 1) // PREFILL_BLOCK_M):
            last = ctx0 + min((mb + 1) * PREFILL_BLOCK_M, ql)
            items.append((-last, i, mb))
    items.sort()
    return [i for _, i, _ in items], [m for _, _, m in items]


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                      block_tables: torch.Tensor, query_start_loc: torch.Tensor,
                      seq_lens: torch.Tensor, scale: float, work_seq: torch.Tensor = None,
                      work_mblk: torch.Tensor = None,
                      out: Optional[torch.Tensor] = None, k_scale: float = 1.0,
                      v_scale: float = 1.0) -> torch.Tensor:
    if not _gpu(q):
        return ref.prefill_attention(q, k_cache, v_cache, block_tables, query_start_loc,
                                     seq_lens, scale, k_scale, v_scale)
    if work_seq is None:
        qsl = query_start_loc.tolist()
        ws, wm = prefill_work_list([qsl[i + 1] - qsl[i] for i in range(len(qsl) - 1)],
                                   seq_lens.tolist())
        work_seq = torch.tensor(ws, dtype=torch.int32, device=q.device)
        work_mblk = torch.tensor(wm, dtype=torch.int32, device=q.device)
    if out is None:
        out = torch.empty_like(q)
    _k().prefill_attention(out, q, k_cache, v_cache, block_tables, query_start_loc, seq_lens,
                           work_seq, work_mblk, scale, k_scale, v_scale)
    return out


def prefill_attention_rope(qkv: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor,
                           v_cache: torch.Tensor, block_tables: torch.Tensor,
                           query_start_loc: torch.Tensor, seq_lens: torch.Tensor, scale: float,
                           num_heads: int, head_dim: int, work_seq: Optional[torch.Tensor] = None,
                           work_mblk: Optional[torch.Tensor] = None,
                           out: Optional[torch.Tensor] = None,
                           k_scale: float = 1.0, v_scale: float = 1.0) -> torch.Tensor:
    """K2 on a prefill-only step whose q is still the unrotated QKV projection row: NeoX
    RoPE (position = context start + row, as the engine numbers tokens) is applied as the
    kernel loads q, so q is never written or re-read (k / v: ``kv_write_rope``)."""
    T = qkv.shape[0]
    if work_seq is None:
        qsl = query_start_loc.tolist()
        ws, wm = prefill_work_list([qsl[i + 1] - qsl[i] for i in range(len(qsl) - 1)],
                                   seq_lens.tolist())
        work_seq = torch.tensor(ws, dtype=torch.int32, device=qkv.device)
        work_mblk = torch.tensor(wm, dtype=torch.int32, device=qkv.device)
    if out is None:
        out = torch.empty(T, num_heads, head_dim, dtype=qkv.dtype, device=qkv.device)
    _k().prefill_attention_rope(out, qkv, cos_sin, k_cache, v_cache, block_tables,
                                query_start_loc, seq_lens, work_seq, work_mblk, num_heads, scale,
                                k_scale, v_scale)
    return out


# ------------------------------------------------------------------ sampling
def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
           top_p: torch.Tensor, seeds: torch.Tensor,
           out: Optional[torch.Tensor] = None, thresholds: bool = True) -> torch.Tensor:
    """K10.  ``thresholds=False`` promises that no row uses top-k / top-p (the caller
    knows from the host-side plan): the single-pass kernel then runs; otherwise the
    cooperative kernel splits each row's threshold passes over its workgroups."""
    if not _gpu(logits):
        return ref.sample(logits, temperature, top_k, top_p, seeds)
    B = logits.shape[0]
    if out is None:
        out = torch.empty(B, dtype=torch.int64, device=logits.device)
    _k().sample(out, logits, temperature, top_k, top_p, seeds, thresholds)
    return out


class SamplerFailed(RuntimeError):
    """The cooperative top-k / top-p sampler's row barrier timed out: the step's
    thresholds (and tokens) are invalid."""


class SamplerHealth:
    """The cooperative sampler's sticky error word (sampling.hip ``g_smp_err``), checked
    like the peer-memory collectives' words: ``enqueue_err_read`` queues a copy into a
    pinned host slot and a clear of the device word behind the step, and returns the slot;
    ``raise_if_failed(slot)`` (after that step completed) raises instead of letting its
    tokens be served.  Every in-flight step copies into its OWN slot (a ring): with async
    scheduling step N + 1 is launched before N's tokens are read, and N + 1's copy of the
    just-cleared word must not overwrite N's flag."""

    SLOTS = 8      # > steps in flight (async: 2; PP: one per stage, <= 8)

    def __init__(self, device: torch.device):
        with torch.cuda.device(device):
            self.addr = int(_k().sample_err_addr())
        self.host = torch.zeros(self.SLOTS, dtype=torch.int32, pin_memory=True)
        self._next = 0

    def enqueue_err_read(self) -> int:
        slot = self._next
        self._next = (slot + 1) % self.SLOTS
        self.host[slot] = 0
        _k().u32_copy_async(self.addr, self.host, slot)
        _k().u32_clear_async(self.addr)
        return slot

    def failed(self, slot: int) -> bool:
        """The flag of `slot` (its step must have completed)."""
        return bool(int(self.host[slot]))

    def raise_if_failed(self, slot: Optional[int] = None) -> None:
        if slot is None:
            slot = (self._next - 1) % self.SLOTS
        if int(self.host[slot]):
            self.host[slot] = 0
            raise SamplerFailed("top-k / top-p sampler: a row's workgroups were not co-resident "
                                "and its barrier timed out; the step's tokens are invalid")


def sample_vp_partial(logits: torch.Tensor, V: int, temperature: torch.Tensor,
                      seeds: torch.Tensor, vocab_off: int,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Vocab-parallel K10 (rows without top-k / top-p): this rank's packed (value,
    global index) candidate per row over its shard ``logits[:, :V]`` (columns
    ``vocab_off ..``), as int64 ordered for a MAX all-reduce over the TP group; then
    ``sample_vp_finish``.  The result equals ``sample`` on the unsharded logits."""
    B = logits.shape[0]
    if not _gpu(logits):
        return ref.sample_vp_partial(logits[:, :V], temperature[:B], seeds[:B], vocab_off)
    if out is None:
        out = torch.empty(B, dtype=torch.int64, device=logits.device)
    _k().sample_vp(out, logits, V, temperature, seeds, vocab_off)
    return out


def sample_vp_finish(packed: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Token ids from the all-reduced packed candidates."""
    if not _gpu(packed):
        return ref.sample_vp_unpack(packed)
    if out is None:
        out = torch.empty_like(packed)
    _k().sample_vp_unpack(out, packed)
    return out


__all__ = ["load_extension", "rms_norm", "fused_add_rms_norm", "layer_norm", "silu_mul",
           "rope_kv_write", "paged_attention_decode", "paged_attention_decode_rope", "prefill_attention", "sample", "sample_vp_partial", "sample_vp_finish",
           "decode_partials", "decode_grid_z", "moe_pack", "moe_packable", "prefill_work_list", "ref"]


# ------------------------------------------------------------------ MoE (K13 / K14)
MOE_GATE_FUSED_MAX_T = 1024  # tokens up to which the router GEMM runs inside the top-k kernel
MOE_NATIVE_MAX_ROWS = 128   # mean rows per expert above which hipBLASLt per expert wins


def moe_supported(n: int, k: int) -> bool:
    """Shapes the grouped GEMM tiles cover: N % 128 == 0 and K % 64 == 0."""
    return n % 128 == 0 and k % 64 == 0


def moe_topk_softmax(router_logits: torch.Tensor, k: int, renormalize: bool = True):
    """K13: (weights fp32 [T, k], expert ids int32 [T, k])."""
    if not _gpu(router_logits):
        return ref.moe_topk_softmax(router_logits, k, renormalize)
    T = router_logits.shape[0]
    w = torch.empty(T, k, dtype=torch.float32, device=router_logits.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=router_logits.device)
    _k().moe_route(w, ids, router_logits, renormalize)
    return w, ids


def moe_gate_topk(x: torch.Tensor, wg: torch.Tensor, k: int,
                  renormalize: bool = True) -> Optional[tuple]:
    """K13 with the router GEMM folded in: (weights fp32 [T, k], expert ids int32 [T, k])
    of x [T, H] . wg [E, H]^T in one launch, or None where the fused kernel does not apply
    (CPU, E > 16, H % 512 != 0): the caller then runs the GEMM and ``moe_topk_softmax``."""
    if (not _gpu(x) or x.dim() != 2 or wg.shape[0] > 16 or x.shape[1] % 512
            or x.dtype not in (torch.bfloat16, torch.float16) or wg.dtype != x.dtype
            or x.stride(1) != 1 or x.stride(0) % 8):
        return None
    T = x.shape[0]
    w = torch.empty(T, k, dtype=torch.float32, device=x.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=x.device)
    _k().moe_gate_route(w, ids, x, wg.contiguous(), renormalize)
    return w, ids


def moe_splitk(npairs: int, E: int, N: int, K: int, bm: int) -> int:
    """K-slices for the down projection: enough workgroups to fill 256 CUs twice over,
    each slice still >= 16 K-tiles of 64.  The row-block count is bounded without a host
    sync (at most npairs/bm + E blocks carry rows)."""
    if os.environ.get("KGC_MOE_SPLITK") is not None:
        return max(1, int(os.environ["KGC_MOE_SPLITK"]))
    wgs = min((npairs + bm - 1) // bm + E, npairs) * (N // 128)
    S = 1
    while S < 8 and wgs * S < 1024 and K // 64 // (2 * S) >= 16:
        S *= 2
    return S


def moe_pack(w: torch.Tensor, silu: bool) -> torch.Tensor:
    """Per-expert K9m packed copy [E, N/128, K/64, 8192] of an expert weight stack
    [E, N, K] (``dgemm_pack`` per expert; w13 SiLU-packed: gate / up 16-row groups
    interleaved per 128-row tile), the operand of ``moe_dgemm`` (K14m)."""
    E, N, K = w.shape
    p = torch.empty(E, N // 128, K // 64, 8192, dtype=w.dtype, device=w.device)
    for e in range(E):
        _k().dgemm_pack(p[e], w[e], silu)
    return p


def moe_packable(w13: torch.Tensor, w2: torch.Tensor) -> bool:
    """Shapes K14m's packed tiles cover: 2I % 128, I % 64, H % 128, K % 64."""
    I2, H = w13.shape[1], w13.shape[2]
    return I2 % 128 == 0 and (I2 // 2) % 64 == 0 and H % 128 == 0 and w2.shape[2] % 64 == 0


def moe_k14m_bm(npairs: int, E: int) -> int:
    """K14m row block for a call of ``npairs`` (token, expert) pairs over E local experts:
    the smallest of 64 / 96 / 128 that holds a typical expert's pairs in ONE block (an
    expert with more rows than a block streams its weights once per block): routed
    uniformly, a bucket is ~npairs / E +- 3 sd (Mixtral 8x7B decode at batch 256: 64 per
    expert, max ~80 -> 96)."""
    mean = npairs / max(1, E)
    if mean <= 44:
        return 64
    return 96 if mean <= 72 else 128


def moe_k14m_bn() -> int:
    """K14m column tile: 256 (KGC_MOE_BN=128 for A/B)."""
    return 128 if os.environ.get("KGC_MOE_BN") == "128" else 256


def moe_dgemm_splitk(npairs: int, E: int, N: int, K: int, bm: int, bn: int = 128) -> int:
    """K-slices of K14m's down projection: the used row blocks (at most npairs/bm + E)
    times N/bn column tiles times S near one workgroup per CU, each slice >= 8 K-steps
    (KGC_MOE_SPLITK overrides, as for the register-staged kernel)."""
    if os.environ.get("KGC_MOE_SPLITK") is not None:
        return max(1, int(os.environ["KGC_MOE_SPLITK"]))
    blocks = min((npairs + bm - 1) // bm + E, max(1, npairs))
    wgs = blocks * (N // bn)
    S = 1
    while S < 16 and wgs * S * 2 <= 320 and K // 64 // (2 * S) >= 8:
        S *= 2
    return S


def fused_moe(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
              topk_ids: torch.Tensor, expert_offset: int = 0,
              all_local: bool = True, w13p: Optional[torch.Tensor] = None,
              w2p: Optional[torch.Tensor] = None, rows_hint: Optional[int] = None,
              combine: bool = True) -> torch.Tensor:
    """K14: sum_j topk_w[t, j] * MLP_{topk_ids[t, j]}(x[t]) for the experts held here
    (global ids ``expert_offset .. expert_offset + w13.shape[0]``).  x [T, H];
    w13 [E, 2I, H] (gate rows then up rows); w2 [E, H, I].  No host synchronisation:
    bucket sizes stay on the device, so the block is captured in decode graphs.
    ``w13p`` / ``w2p`` (``moe_pack``): K14m -- both projections on the K9m LDS-DMA
    pipeline over packed per-expert tiles, the SiLU in the gate_up epilogue (no [rows, 2I]
    intermediate, no silu_mul launch); else the register-staged grouped GEMM.

    ``rows_hint``: the number of pairs expected to carry rows when ``topk_ids`` has room
    for more (the EP owner's receive slots: NR x C slots, ~T x k of them used); it sizes
    the row block and the down projection's split-K.  ``combine=False`` returns the down
    projection's output per pair instead of the weighted sum -- [npairs, H] in x's dtype,
    or its fp32 split-K slices [S, npairs, H] -- for a consumer that sums the slices
    itself (``ep_return``)."""
    if not _gpu(x):
        return ref.moe_mlp_local(x, w13, w2, topk_w, topk_ids, expert_offset)
    k = _k()
    T, H = x.shape
    E, I2 = w13.shape[0], w13.shape[1]
    topk = topk_ids.shape[1]
    npairs = T * topk
    used = min(npairs, rows_hint) if rows_hint else npairs
    packed = w13p is not None and w2p is not None
    bm = int(os.environ.get("KGC_MOE_BM", 0)) or (moe_k14m_bm(used, E) if packed else
                                                  (64 if used <= 40 * E else 128))
    if bm == 96 and not packed:
        bm = 128                    # the register-staged kernel has 64 / 128-row tiles only
    rows = (npairs + E * (bm - 1) + bm - 1) // bm * bm
    dev = x.device
    sorted_ids = torch.empty(rows, dtype=torch.int32, device=dev)
    block_expert = torch.empty(rows // bm, dtype=torch.int32, device=dev)
    meta = torch.empty(1, dtype=torch.int32, device=dev)
    ids = topk_ids.contiguous()
    k.moe_align(sorted_ids, block_expert, meta, ids, expert_offset, E, bm)
    if packed:
        bn = moe_k14m_bn()
        act = torch.empty(rows, I2 // 2, dtype=x.dtype, device=dev)
        k.moe_dgemm(act, x.contiguous(), w13p, sorted_ids, block_expert, meta, npairs, topk,
                    bm, 1, bn if I2 % bn == 0 else 128)
        bn2 = bn if H % bn == 0 else 128
        S = moe_dgemm_splitk(used, E, H, I2 // 2, bm, bn2)
        alloc = torch.empty if all_local else torch.zeros
        if S > 1:
            y = alloc(S, npairs, H, dtype=torch.float32, device=dev)
        else:
            y = alloc(npairs, H, dtype=x.dtype, device=dev)
        k.moe_dgemm(y, act, w2p, sorted_ids, block_expert, meta, npairs, topk, bm, 2, bn2)
        if not combine:
            return y
        out = torch.empty(T, H, dtype=x.dtype, device=dev)
        k.moe_combine(out, y, topk_w.contiguous().float())
        return out
    inter = torch.empty(rows, I2, dtype=x.dtype, device=dev)
    k.moe_gemm(inter, x.contiguous(), w13, sorted_ids, block_expert, meta, npairs, topk, bm,
               True, False)
    act = silu_mul(inter)
    S = moe_splitk(used, E, H, w2.shape[2], bm)
    alloc = torch.empty if all_local else torch.zeros   # EP: pairs of remote experts add 0
    if S > 1:
        y = alloc(S, npairs, H, dtype=torch.float32, device=dev)
    else:
        y = alloc(npairs, H, dtype=x.dtype, device=dev)
    k.moe_gemm(y, act, w2, sorted_ids, block_expert, meta, npairs, topk, bm, False, True, S)
    if not combine:
        return y
    out = torch.empty(T, H, dtype=x.dtype, device=dev)
    k.moe_combine(out, y, topk_w.contiguous().float())
    return out
