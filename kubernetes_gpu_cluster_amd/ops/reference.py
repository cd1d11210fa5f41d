"""Pure-PyTorch reference implementations of every fused op.

These are the numerics oracles for the HIP kernels in ``csrc/kernels`` and the
CPU execution path (tiny models, the OPT-125m CPU plumbing pod).  They are
written for clarity, in fp32, not speed.

KV-cache layout (shared with the HIP kernels, chosen for CDNA4 MFMA operand
loads, see csrc/kernels/attention_decode.hip):
  k_cache: [num_blocks, num_kv_heads, block_size, head_dim]   (key rows contiguous)
  v_cache: [num_blocks, num_kv_heads, block_size/8, head_dim, 8]
           (V^T in 8-key groups: the 8 consecutive keys of one dim are 16 contiguous
            bytes -- the MFMA A-operand fragment of O^T = V^T.P^T -- and the 16 dims
            of one 16-row tile are 256 contiguous bytes)
"""
from __future__ import annotations

import math
import struct
from typing import Optional

import torch


# ---------------------------------------------------------------- norms / act
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return (xf * torch.rsqrt(var + eps) * w.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                       eps: float) -> tuple[torch.Tensor, torch.Tensor]:
    """residual' = x + residual ; out = rms_norm(residual') * w.  Returns (out, residual')."""
    r = (x.float() + residual.float()).to(residual.dtype)
    return rms_norm(r, w, eps), r


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5):
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(),
                                          eps).to(x.dtype)


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    d = x.shape[-1] // 2
    xf = x.float()
    return (torch.nn.functional.silu(xf[..., :d]) * xf[..., d:]).to(x.dtype)


# ---------------------------------------------------------------- rope
def _llama3_inv_freq(inv_freq: torch.Tensor, sc: dict) -> torch.Tensor:
    factor = sc["factor"]
    lo, hi = sc.get("low_freq_factor", 1.0), sc.get("high_freq_factor", 4.0)
    old = sc.get("original_max_position_embeddings", 8192)
    lo_wl, hi_wl = old / lo, old / hi
    wl = 2 * math.pi / inv_freq
    smooth = (old / wl - lo) / (hi - lo)
    scaled = torch.where(wl > lo_wl, inv_freq / factor, inv_freq)
    mid = (1 - smooth) * inv_freq / factor + smooth * inv_freq
    is_mid = (wl <= lo_wl) & (wl >= hi_wl)
    return torch.where(is_mid, mid, scaled)


def rope_cos_sin_cache(head_dim: int, max_pos: int, theta: float,
                       scaling: Optional[dict] = None) -> torch.Tensor:
    """[max_pos, head_dim] fp32: first half cos, second half sin (NeoX layout)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        inv = _llama3_inv_freq(inv, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv)
    return torch.cat([freqs.cos(), freqs.sin()], dim=-1).float()


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, n, d]; NeoX rotate-half."""
    d = x.shape[-1]
    cs = cos_sin[positions.long()]                 # [T, d]
    cos = cs[:, None, : d // 2]
    sin = cs[:, None, d // 2:]
    xf = x.float()
    x1, x2 = xf[..., : d // 2], xf[..., d // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def rope_qk_kv_write(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor,
                     k_cache: torch.Tensor, v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                     num_heads: int, num_kv_heads: int, head_dim: int,
                     q_norm_w: Optional[torch.Tensor] = None,
                     k_norm_w: Optional[torch.Tensor] = None, eps: float = 1e-6,
                     use_rope: bool = True, k_scale: float = 1.0,
                     v_scale: float = 1.0) -> torch.Tensor:
    """K3+K5(+K6): split fused qkv [T, (nq+2nkv)*d], optional per-head q/k RMSNorm,
    RoPE on q,k, scatter k,v into the paged cache at slot_mapping (-1 = skip).
    Returns rotated q as a contiguous [T, nq, d] tensor."""
    T = qkv.shape[0]
    qs, ks = num_heads * head_dim, num_kv_heads * head_dim
    q = qkv[:, :qs].reshape(T, num_heads, head_dim)
    k = qkv[:, qs:qs + ks].reshape(T, num_kv_heads, head_dim)
    v = qkv[:, qs + ks:qs + 2 * ks].reshape(T, num_kv_heads, head_dim)
    if q_norm_w is not None:
        q = rms_norm(q, q_norm_w, eps)
        k = rms_norm(k, k_norm_w, eps)
    if use_rope:
        q = apply_rope(q, positions, cos_sin)
        k = apply_rope(k, positions, cos_sin)
    kv_cache_write(k, v, k_cache, v_cache, slot_mapping, k_scale, v_scale)
    return q.contiguous()


FP8_MAX = 448.0


def to_cache(x: torch.Tensor, cache_dtype: torch.dtype, scale: float = 1.0) -> torch.Tensor:
    """Value -> cache element: the cache dtype itself, or fp8 e4m3 of (x / scale) with
    saturation (the kernels clamp to +-448 before the hardware conversion)."""
    if cache_dtype == torch.float8_e4m3fn:
        return (x.float() / scale).clamp(-FP8_MAX, FP8_MAX).to(cache_dtype)
    return x.to(cache_dtype)


def kv_cache_write(k: torch.Tensor, v: torch.Tensor, k_cache: torch.Tensor,
                   v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                   k_scale: float = 1.0, v_scale: float = 1.0) -> None:
    bs = k_cache.shape[2]
    sm = slot_mapping.long()
    valid = sm >= 0
    if not bool(valid.any()):
        return
    sm = sm[valid]
    blk, off = sm // bs, sm % bs
    # an fp8 cache stores the activation-dtype-rounded value, quantised
    k_cache[blk, :, off, :] = to_cache(k[valid].to(k.dtype), k_cache.dtype, k_scale)
    v_cache[blk, :, off // 8, :, off % 8] = to_cache(v[valid].to(v.dtype), v_cache.dtype, v_scale)


# ---------------------------------------------------------------- attention
def _gather_kv(k_cache, v_cache, block_table, ctx_len, k_scale=1.0, v_scale=1.0):
    bs = k_cache.shape[2]
    nb = (ctx_len + bs - 1) // bs
    blocks = block_table[:nb].long()
    k = k_cache[blocks]                                   # [nb, nkv, bs, d]
    k = k.permute(0, 2, 1, 3).reshape(nb * bs, k.shape[1], k.shape[3])[:ctx_len]
    v = v_cache[blocks]                                   # [nb, nkv, bs/8, d, 8]
    v = v.permute(0, 2, 4, 1, 3).reshape(nb * bs, v.shape[1], v.shape[3])[:ctx_len]
    return k.float() * k_scale, v.float() * v_scale      # [ctx, nkv, d]


def paged_attention_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, context_lens: torch.Tensor,
                           scale: float, k_scale: float = 1.0, v_scale: float = 1.0) -> torch.Tensor:
    """K1: q [B, nq, d] -> out [B, nq, d], one query token per sequence."""
    B, nq, d = q.shape
    nkv = k_cache.shape[1]
    g = nq // nkv
    out = torch.empty_like(q)
    for b in range(B):
        L = int(context_lens[b])
        k, v = _gather_kv(k_cache, v_cache, block_tables[b], L, k_scale, v_scale)
        qb = q[b].float().view(nkv, g, d)
        s = torch.einsum("hgd,lhd->hgl", qb, k) * scale
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgl,lhd->hgd", p, v)
        out[b] = o.reshape(nq, d).to(q.dtype)
    return out


def prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                      block_tables: torch.Tensor, query_start_loc: torch.Tensor,
                      seq_lens: torch.Tensor, scale: float, k_scale: float = 1.0,
                      v_scale: float = 1.0) -> torch.Tensor:
    """K2: varlen causal attention for packed prompt chunks.  Sequence i owns query
    rows [qsl[i], qsl[i+1]); its keys are cache positions [0, seq_lens[i]) and its
    queries sit at absolute positions seq_lens[i]-qlen .. seq_lens[i]-1."""
    T, nq, d = q.shape
    nkv = k_cache.shape[1]
    g = nq // nkv
    out = torch.empty_like(q)
    for i in range(len(seq_lens)):
        a, b = int(query_start_loc[i]), int(query_start_loc[i + 1])
        ql, L = b - a, int(seq_lens[i])
        if ql == 0:
            continue
        k, v = _gather_kv(k_cache, v_cache, block_tables[i], L, k_scale, v_scale)
        qi = q[a:b].float().view(ql, nkv, g, d)
        s = torch.einsum("qhgd,lhd->hgql", qi, k) * scale
        qpos = torch.arange(L - ql, L)[:, None]
        kpos = torch.arange(L)[None, :]
        s = s.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgql,lhd->qhgd", p, v)
        out[a:b] = o.reshape(ql, nq, d).to(q.dtype)
    return out


def dense_causal_attention(q, k, v, scale):
    """Plain causal attention over one sequence: q [S, nq, d], k/v [S, nkv, d]."""
    S, nq, d = q.shape
    g = nq // k.shape[1]
    k = k.float().repeat_interleave(g, dim=1)
    v = v.float().repeat_interleave(g, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), k) * scale
    mask = torch.triu(torch.ones(S, S, dtype=torch.bool), 1)
    s = s.masked_fill(mask, float("-inf"))
    return torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).to(q.dtype)


# ---------------------------------------------------------------- sampling
_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 integer hash on int64 tensors holding uint32 values."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def _row_key(seeds: torch.Tensor) -> torch.Tensor:
    """Per-row stream key from both halves of the int64 seed (sampling.hip row_key)."""
    s = seeds.long()
    hi = _mix32(((s >> 32) + 0x632BE5AB) & _M32)
    return _mix32((s & _M32) ^ hi)


def uniform_noise(seeds: torch.Tensor, vocab: int) -> torch.Tensor:
    """Counter-based uniform(0,1) noise, identical to the HIP sampler's generator.
    seeds: [B] int64 (per-row stream key) -> [B, V] fp32."""
    return uniform_noise_cols(seeds, 0, vocab)


def uniform_noise_cols(seeds: torch.Tensor, col0: int, n: int) -> torch.Tensor:
    """``uniform_noise`` restricted to the global columns col0 .. col0 + n - 1."""
    col = torch.arange(col0, col0 + n, dtype=torch.int64)
    h = _mix32(_row_key(seeds)[:, None] ^ ((col[None, :] * 0x9E3779B9) & _M32))
    return ((h >> 9).double() + 0.5).float() * (1.0 / 8388608.0)    # 23 bits: u < 1 exactly


_LN2 = 0.69314718


def gumbel(u: torch.Tensor) -> torch.Tensor:
    """-ln(-ln u) as sampling.hip gumbel computes it (fp32): -ln2 * log2(-ln2 * log2 u)."""
    ln2 = torch.tensor(_LN2, dtype=torch.float32)
    return -(ln2 * torch.log2(-(ln2 * torch.log2(u.float()))))


_VP_BIAS = 1 << 63


def _ord_key(v: float) -> int:
    b = struct.unpack("<I", struct.pack("<f", v))[0]
    return (~b & 0xFFFFFFFF) if b & 0x80000000 else (b | 0x80000000)


def sample_vp_partial(logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor,
                      vocab_off: int) -> torch.Tensor:
    """Vocab-parallel sampler, one shard: per row the packed (ord(value) << 32 | ~global
    index) of the shard's (Gumbel-)argmax, biased to a signed int64 so that a MAX
    all-reduce over the shards yields the unsharded sampler's pick (ties -> lower
    index).  Rows must not use top-k / top-p."""
    B, V = logits.shape
    x = logits.float().cpu()
    u = uniform_noise_cols(seeds.cpu(), vocab_off, V)
    out = torch.empty(B, dtype=torch.int64)
    for b in range(B):
        t = float(temperature[b])
        row = x[b] if t <= 1e-5 else x[b] / t + gumbel(u[b])
        i = int(torch.argmax(row))                       # first index on ties
        packed = (_ord_key(float(row[i])) << 32) | (~(i + vocab_off) & 0xFFFFFFFF)
        out[b] = packed - _VP_BIAS                       # == (packed ^ bias) as int64
    return out.to(logits.device)


def sample_vp_unpack(packed: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(packed)
    for b, v in enumerate(packed.tolist()):
        u64 = v + _VP_BIAS
        idx = ~u64 & 0xFFFFFFFF
        out[b] = 0 if (u64 == 0 or idx >= 0x7FFFFFFF) else idx
    return out


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
           top_p: torch.Tensor, seeds: torch.Tensor) -> torch.Tensor:
    """K10: greedy when temperature==0, else Gumbel-max over the top-k/top-p support.
    Returns int64 token ids [B]."""
    B, V = logits.shape
    x = logits.float()
    out = torch.empty(B, dtype=torch.int64)
    u = uniform_noise(seeds.cpu(), V)
    for b in range(B):
        row = x[b].cpu()
        t = float(temperature[b])
        if t <= 1e-5:
            out[b] = int(torch.argmax(row))
            continue
        row = row / t
        drop = torch.zeros(V, dtype=torch.bool)
        k = int(top_k[b])
        if 0 < k < V:
            kth = torch.topk(row, k).values[-1]
            drop |= row < kth
        p = float(top_p[b])
        if p < 1.0:
            probs = torch.softmax(row.masked_fill(drop, float("-inf")), -1)
            sp, idx = torch.sort(probs, descending=True)
            cum = torch.cumsum(sp, 0)
            keep = (cum - sp) < p
            thr = sp[keep][-1]
            drop |= probs < thr
        # noise first, then the mask: a dropped column is -inf whatever its noise
        out[b] = int(torch.argmax((row + gumbel(u[b])).masked_fill(drop, float("-inf"))))
    return out.to(logits.device)


# ---------------------------------------------------------------- MoE
def moe_topk_softmax(router_logits: torch.Tensor, k: int, renormalize: bool = True):
    """K13: softmax over experts, top-k; returns (weights fp32 [T,k], ids int32 [T,k])."""
    p = torch.softmax(router_logits.float(), dim=-1)
    w, ids = torch.topk(p, k, dim=-1)
    if renormalize:
        w = w / w.sum(-1, keepdim=True)
    return w, ids.to(torch.int32)


def moe_mlp_local(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
                  topk_ids: torch.Tensor, expert_offset: int = 0) -> torch.Tensor:
    """K14 over the experts held locally (global ids offset by ``expert_offset``); pairs
    routed elsewhere contribute nothing.  Expert outputs are rounded to x.dtype before
    the fp32 weighted combine, like the kernel."""
    T, H = x.shape
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    for e in range(w13.shape[0]):
        tok, slot = torch.nonzero(topk_ids == e + expert_offset, as_tuple=True)
        if tok.numel() == 0:
            continue
        h = silu_mul((x[tok].float() @ w13[e].float().t()).to(x.dtype).float())
        y = (h.to(x.dtype).float() @ w2[e].float().t()).to(x.dtype)
        out.index_add_(0, tok, y.float() * topk_w[tok, slot, None].float())
    return out.to(x.dtype)


def moe_mlp(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
            topk_ids: torch.Tensor) -> torch.Tensor:
    """K14: per-expert SwiGLU MLP, weighted combine.  w13 [E, 2I, H], w2 [E, H, I]."""
    T, H = x.shape
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    for e in range(w13.shape[0]):
        tok, slot = torch.nonzero(topk_ids == e, as_tuple=True)
        if tok.numel() == 0:
            continue
        h = x[tok].float() @ w13[e].float().t()
        h = silu_mul(h)
        y = h @ w2[e].float().t()
        out.index_add_(0, tok, y * topk_w[tok, slot, None].float())
    return out.to(x.dtype)
