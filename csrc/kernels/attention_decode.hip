// K1 paged-attention decode for gfx950 (CDNA4), bf16/f16, head_dim 64/128.
//
// Work decomposition: grid (num_seqs, num_kv_heads, Z).  A 256-thread workgroup is
// four waves; the 64-token partitions of the context are dealt round-robin to the
// 4*Z waves of a (seq, kv-head): wave w of z-slice z owns p = z*4 + w, + 4Z, ...
// Each wave carries an online softmax (m, l, O) across its partitions; the four
// waves merge through LDS.  With Z == 1 (large batches: the host picks Z so the
// grid fills the 256 CUs) the workgroup writes the normalised output directly --
// no partials, no second kernel.  With Z > 1 it writes one (max, sum, O) partial per
// z-slice and paged_decode_reduce_kernel merges the Z partials.  Z is a host choice
// that does not depend on the batch's actual lengths, so the launch is hipGraph-static.
//
// Per 32-key chunk a wave runs two MFMA products, both v_mfma_f32_16x16x32:
//   S^T[key][head] = K[key][:] . Q^T[:][head]       A = K rows straight from HBM
//                                                   B = the GQA group's Q (<= 16 heads
//                                                       packed in the MFMA N dim)
//   O^T[d][head]  += V^T[d][key] . P^T[key][head]   A = V^T rows straight from HBM
//                                                   B = P, taken from S^T's accumulator
// The two S^T tiles of a chunk use the row->key map  key(m) = 8*(m>>2) + (m&3) (+4 for
// the second tile), so after QK^T lane l holds keys 8*(l>>4) + 0..7 of head l&15 --
// exactly the B-operand fragment of the P.V MFMA: no LDS, no lane shuffles for P.
// The head of every accumulator element is lane&15, so the softmax statistics and
// the O rescale are lane-local up to a 4-lane (xor 16/32) reduction.
// Scores are kept in the log2 domain (scale * log2(e) folded in), exp2.
//
// FUSE (decode-only steps, launch_paged_decode_rope): the RoPE / q-k-norm / KV-write
// kernel (rope_cache.hip) runs as this kernel's prologue: one thread per NeoX chunk
// pair of the GQA group's heads builds q (split-K slice sum, q-norm, RoPE) into LDS,
// where every wave picks up its MFMA B fragments, while wave 3 of the z-slice whose
// last wave owns the final context token writes that token's k / v (workgroup fence +
// barrier, then the normal loads see it through the CU's own L1).  Measured first
// with every wave building its own q in registers (4 dependent slice round trips
// each): 149 vs 137 us for rope_kv + decode at B = 256, S = 4.
#include "common.h"
#include "launch.h"
#include <cstdlib>
#include <type_traits>

namespace kgc {

constexpr int DEC_PART = 64;     // tokens per partition (one wave-iteration)
constexpr int DEC_CHUNKS = DEC_PART / 32;
constexpr int DEC_MAX_Z = 1024;  // z-slices the reduce kernel merges (host-checked)
// K1w runs where the grid has at least this many (seq, kv-head) pairs; smaller batches
// take the 4-wave kernel (B = 1: 9.3 vs 12.3 us at ctx 640; ops/__init__.py mirrors it)
constexpr int DEC_WAVE_MIN_PAIRS = 64;
// ... and from this many pairs up a z-slice holds at least DEC_LONG_MIN_CHUNKS chunks
// (ops/__init__.py also aims such grids at ~4 waves per CU instead of 8): with the KV
// streamed from HBM (tools/attn_bench.py cycles copies past the Infinity Cache), fewer,
// longer slices won at every many-pairs shape measured -- B = 256 nq 8 / nkv 1 ctx 640:
// 23.2 us at 2 slices of 10 chunks vs 26.9 at 7 of 3; B = 128 nq 32 / nkv 8: 65.0 vs
// 68.8 us at one slice; B = 32 ctx 2300: 61.9 vs 66.5 (profiles/attn_decode_r5.jsonl)
constexpr int DEC_LONG_PAIRS = 256;
constexpr int DEC_LONG_MIN_CHUNKS = 10;

// K1w: 32-token chunks per z-slice (>= min_per, at least 2: the pipeline depth); slices
// past the context are empty and the reduce stops at decode_used_slices.  min_per is a
// per-launch host choice (decode_min_chunks): the graph's Z is sized for max_model_len,
// so at short contexts many-pairs grids would otherwise cut each context into slices of
// 2-3 chunks, each paying the q prologue and a partial write for little streaming.
__host__ __device__ __forceinline__ int decode_slice_chunks(int nchunk, int Z, int min_per) {
  const int per = (nchunk + Z - 1) / Z;
  return per < min_per ? min_per : per;
}
__host__ __device__ __forceinline__ int decode_used_slices(int nchunk, int Z, int min_per) {
  const int per = decode_slice_chunks(nchunk, Z, min_per);
  const int n = (nchunk + per - 1) / per;
  return n < Z ? n : Z;
}

// max of x over lanes l and l ^ 16 / l ^ 32: the gfx950 permlane swaps hand each lane its
// partner's value in the second register (VALU, no LDS round trip)
__device__ __forceinline__ float max_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ u32x4 ld16(const void* p) {
  return *reinterpret_cast<const u32x4*>(p);
}

// ---- FUSE prologue helpers (rope_cache.hip computes the same values for the general
// case; the roundings to T match it: summed slices, normed values and rotated outputs)
template <typename T>
__device__ __forceinline__ void qkv_row8(const DecodeRope& rp, int64_t e, float* x, float sc) {
  if (rp.S == 0) {
    Pack8<T> p;
    p.u = ld16(reinterpret_cast<const T*>(rp.qkv) + e);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = rp.row_scale ? to_f(from_f<T>(to_f(p.h[j]) * sc)) : to_f(p.h[j]);
    return;
  }
  // SB = 8 slices' loads in flight per round trip (clamped duplicates are not added: the
  // tuner picks S <= 8, so every split is ONE round trip -- at SB = 4 the S = 5 qkv of
  // Llama-3-8B at M = 256 took two, 132 vs 127 us per layer);
  // summed z = 0, 1, ... from 0 as rope_cache.hip does: bit-identical
  const float* src = reinterpret_cast<const float*>(rp.qkv) + e;
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
  constexpr int SB = 8;
  for (int z0 = 0; z0 < rp.S; z0 += SB) {
    f32x4 ta[SB], tb[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int64_t z = min(z0 + j, rp.S - 1);
      ta[j] = *reinterpret_cast<const f32x4*>(src + z * rp.slice_stride);
      tb[j] = *reinterpret_cast<const f32x4*>(src + z * rp.slice_stride + 4);
    }
#pragma unroll
    for (int j = 0; j < SB; ++j)
      if (z0 + j < rp.S) { a += ta[j]; b += tb[j]; }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    x[q] = to_f(from_f<T>(a[q] * sc));
    x[4 + q] = to_f(from_f<T>(b[q] * sc));
  }
}

// The pair (xa at e_a, xb at e_b) of one lane's NeoX chunks in ONE round trip: with the
// slice count a compile-time constant every slice load of both chunks is issued before the
// first add -- 4 S loads, no clamped duplicates (qkv_row8's batches of SB re-load slice
// S - 1 to fill a batch) -- summed in slice order from 0, bit-identical to qkv_row8.
template <typename T, int S>
__device__ __forceinline__ void qkv_pair8_s(const DecodeRope& rp, int64_t ea, int64_t eb,
                                            float* xa, float* xb, float sc) {
  const float* pa = reinterpret_cast<const float*>(rp.qkv) + ea;
  const float* pb = reinterpret_cast<const float*>(rp.qkv) + eb;
  f32x4 t[S][4];
#pragma unroll
  for (int z = 0; z < S; ++z) {
    t[z][0] = *reinterpret_cast<const f32x4*>(pa + z * rp.slice_stride);
    t[z][1] = *reinterpret_cast<const f32x4*>(pa + z * rp.slice_stride + 4);
    t[z][2] = *reinterpret_cast<const f32x4*>(pb + z * rp.slice_stride);
    t[z][3] = *reinterpret_cast<const f32x4*>(pb + z * rp.slice_stride + 4);
  }
  f32x4 a0 = t[0][0], a1 = t[0][1], b0 = t[0][2], b1 = t[0][3];
#pragma unroll
  for (int z = 1; z < S; ++z) {
    a0 += t[z][0];
    a1 += t[z][1];
    b0 += t[z][2];
    b1 += t[z][3];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    xa[q] = to_f(from_f<T>(a0[q] * sc));
    xa[4 + q] = to_f(from_f<T>(a1[q] * sc));
    xb[q] = to_f(from_f<T>(b0[q] * sc));
    xb[4 + q] = to_f(from_f<T>(b1[q] * sc));
  }
}

template <typename T>
__device__ __forceinline__ void qkv_pair8(const DecodeRope& rp, int64_t ea, int64_t eb,
                                          float* xa, float* xb, float sc) {
  switch (rp.S) {        // wave-uniform: the K9m split factors the tuner picks
    case 2: qkv_pair8_s<T, 2>(rp, ea, eb, xa, xb, sc); return;
    case 3: qkv_pair8_s<T, 3>(rp, ea, eb, xa, xb, sc); return;
    case 4: qkv_pair8_s<T, 4>(rp, ea, eb, xa, xb, sc); return;
    case 5: qkv_pair8_s<T, 5>(rp, ea, eb, xa, xb, sc); return;
    case 6: qkv_pair8_s<T, 6>(rp, ea, eb, xa, xb, sc); return;
    case 8: qkv_pair8_s<T, 8>(rp, ea, eb, xa, xb, sc); return;
    default:
      qkv_row8<T>(rp, ea, xa, sc);
      qkv_row8<T>(rp, eb, xb, sc);
  }
}

// the projection row's scale (1 unless the norm-free layer runs)
__device__ __forceinline__ float qkv_row_scale(const DecodeRope& rp, int b) {
  return rp.row_scale ? rp.row_scale[b] : 1.f;
}

// x * inv * w[col..col+7], rounded through T
template <typename T>
__device__ __forceinline__ void norm8(float* x, float inv, const void* w, int col) {
  Pack8<T> wv;
  wv.u = ld16(reinterpret_cast<const T*>(w) + col);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = to_f(from_f<T>(x[j] * inv * to_f(wv.h[j])));
}

// NeoX rotation of the chunk pair (a at col, b at col + D/2); cs = cos_sin row
__device__ __forceinline__ void rope8(float* a, float* b, const float* cs, int col, int half) {
  const float4 c0 = *reinterpret_cast<const float4*>(cs + col);
  const float4 c1 = *reinterpret_cast<const float4*>(cs + col + 4);
  const float4 s0 = *reinterpret_cast<const float4*>(cs + half + col);
  const float4 s1 = *reinterpret_cast<const float4*>(cs + half + col + 4);
  const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    neox_rot(a[j], b[j], cc[j], sn[j], a[j], b[j]);
  }
}

// The new token's k (rotated) and v of kv-head h into the paged cache: lanes
// 0 .. D/16-1 own a k chunk pair (their D/16 lanes reduce the k-norm sum), lanes
// 16 .. 16+D/8-1 one v chunk (8 two-byte stores into the V^T 8-key group).
template <typename T, int D, bool KV8>
__device__ __forceinline__ void decode_kv_write(const DecodeRope& rp, int b, int h, int nq,
                                                int nkv, int bs_log2, int num_blocks,
                                                void* kc_, void* vc_, int lane) {
  int64_t slot = rp.slots[b];
  KGC_DCHECK_RANGE(slot, -1, (int64_t)num_blocks << bs_log2, "decode KV slot");
  if (slot < 0) return;
  constexpr int TPH = D / 16, half = D / 2;
  const int64_t blk = slot >> bs_log2;
  const int off = (int)(slot & ((1 << bs_log2) - 1));
  const int64_t row = (int64_t)b * rp.qkv_stride;
  if (lane < TPH) {
    const int c = lane;
    float xa[8], xb[8];
    qkv_pair8<T>(rp, row + (int64_t)(nq + h) * D + c * 8, row + (int64_t)(nq + h) * D + half + c * 8,
                 xa, xb, qkv_row_scale(rp, b));
    if (rp.k_norm_w) {
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += xa[j] * xa[j] + xb[j] * xb[j];
#pragma unroll
      for (int o = 1; o < TPH; o <<= 1) ss += __shfl_xor(ss, o, 64);
      const float inv = rsqrtf(ss / (float)D + rp.eps);
      norm8<T>(xa, inv, rp.k_norm_w, c * 8);
      norm8<T>(xb, inv, rp.k_norm_w, half + c * 8);
    }
    if (rp.use_rope) rope8(xa, xb, rp.cos_sin + rp.positions[b] * D, c * 8, half);
    Pack8<T> oa, ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) { oa.h[j] = from_f<T>(xa[j]); ob.h[j] = from_f<T>(xb[j]); }
    const int64_t e = ((blk * nkv + h) << bs_log2 | off) * D;
    if constexpr (KV8) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(kc_) + e;
      float fa[8], fb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { fa[j] = to_f(oa.h[j]) * rp.k_inv; fb[j] = to_f(ob.h[j]) * rp.k_inv; }
      *reinterpret_cast<u32x2*>(dst + c * 8) =
          u32x2{fp8x4(fa[0], fa[1], fa[2], fa[3]), fp8x4(fa[4], fa[5], fa[6], fa[7])};
      *reinterpret_cast<u32x2*>(dst + half + c * 8) =
          u32x2{fp8x4(fb[0], fb[1], fb[2], fb[3]), fp8x4(fb[4], fb[5], fb[6], fb[7])};
    } else {
      T* dst = reinterpret_cast<T*>(kc_) + e;
      *reinterpret_cast<u32x4*>(dst + c * 8) = oa.u;
      *reinterpret_cast<u32x4*>(dst + half + c * 8) = ob.u;
    }
  } else if (lane >= 16 && lane < 16 + D / 8) {
    const int c = lane - 16;
    float xv[8];
    qkv_row8<T>(rp, row + (int64_t)(nq + nkv + h) * D + c * 8, xv, qkv_row_scale(rp, b));
    const int64_t e = ((blk * nkv + h) << bs_log2) * D + ((int64_t)(off >> 3) * D + c * 8) * 8 +
                      (off & 7);
    if constexpr (KV8) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(vc_) + e;
      const uint32_t w0 = fp8x4(xv[0] * rp.v_inv, xv[1] * rp.v_inv, xv[2] * rp.v_inv, xv[3] * rp.v_inv);
      const uint32_t w1 = fp8x4(xv[4] * rp.v_inv, xv[5] * rp.v_inv, xv[6] * rp.v_inv, xv[7] * rp.v_inv);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dst[j * 8] = (uint8_t)(w0 >> (8 * j));
        dst[(j + 4) * 8] = (uint8_t)(w1 >> (8 * j));
      }
    } else {
      T* dst = reinterpret_cast<T*>(vc_) + e;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j * 8] = from_f<T>(xv[j]);
    }
  }
}

// PREF: true = issue all K and V loads of a wave-iteration before its first MFMA;
// false = load each fragment right before its MFMA.  NCH = 32-token chunks per
// wave-iteration, OCC = waves per SIMD.  Shipped: PREF, NCH = 1, OCC = 4 (<= 128 VGPR).
// Measured (tools/attn_bench.py, profiles/attn_decode_microbench.jsonl) against the
// previous PREF/NCH=2/OCC=3 (134 VGPR): +4 % at B=256 ctx 640 (5.36 vs 5.14 TB/s),
// +9 % at B=32 ctx 2600 (Z=4), +4 % at B=64 (Z=2); the per-fragment-load form at
// OCC 4 is 3-8 % slower than both.  At B=256 the grid is 2048 workgroups: OCC 4 runs
// them in 2 full rounds of 1024 instead of 2.67 rounds of 768.  Non-temporal K/V loads
// and an MFMA-tiled K layout (1 KB contiguous per load) were measured too: -7 % and
// +3 %, neither kept.
// KV8: fp8 e4m3 cache (8-byte fragment loads widened in registers); the K scale is
// folded into scale_log2 by the launcher, the V scale (v_scale) into the output.
// FUSE: q comes from the QKV projection row through the rope prologue (rp) and the
// workgroup holding the last context token writes that token's k / v first -- through
// kc_ / vc_ themselves (const_cast), so every store and load of the cache is based on
// the same __restrict__ pointer and the workgroup fence orders them.
template <typename T, int D, bool PREF, bool KV8, int OCC = 3, int NCH = DEC_CHUNKS,
          bool FUSE = false>
__global__ __launch_bounds__(256, OCC) void paged_decode_kernel(
    T* __restrict__ out, const T* __restrict__ q, const void* __restrict__ kc_,
    const void* __restrict__ vc_, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ctx_lens, float* __restrict__ max_logits,
    float* __restrict__ exp_sums, float* __restrict__ tmp_out, int nq, int nkv, int bs_log2,
    int Zmax, float scale_log2, float v_scale, int num_blocks, DecodeRope rp) {
  typedef typename Vec8<T>::type V8;
  typedef std::conditional_t<KV8, uint8_t, T> C;   // cache element
  const C* __restrict__ kc = reinterpret_cast<const C*>(kc_);
  const C* __restrict__ vc = reinterpret_cast<const C*>(vc_);
  auto ldf = [](const C* p) -> u32x4 {
    if constexpr (KV8) return fp8x8_widen<T>(*reinterpret_cast<const u32x2*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
  };
  constexpr int KS = D / 32;      // k-steps of the QK^T product
  constexpr int DT = D / 16;      // 16-row d-tiles of O^T
  // rows padded by 4 floats: the b128 stores of lanes (head r16, qd) land in (r16 + qd) mod 16
  // bank groups, 4 lanes each (the b128 minimum), instead of 16 heads on one group
  __shared__ __attribute__((aligned(16))) float lds_o[4][16][D + 4];
  __shared__ float lds_m[4][16], lds_l[4][16];
  // q rows padded by 8 elements: unpadded, the 256-B rows put the 16 heads a b128 read
  // gathers on the same 4 banks (393K bank-conflict cycles per dispatch at B = 256)
  __shared__ __attribute__((aligned(16))) T lds_q[FUSE ? 16 : 1][FUSE ? D + 8 : 8];
  const int b = blockIdx.x, h = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, qd = lane >> 4;
  const int G = nq / nkv;
  // clamp to the block-table capacity: a bad length gives wrong output, never a fault
  int ctx_in = ctx_lens[b];
  KGC_DCHECK_RANGE(ctx_in, 0, (bt_stride << bs_log2) + 1, "decode ctx_len");
  const int ctx = min(ctx_in, bt_stride << bs_log2);
  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int bsm = (1 << bs_log2) - 1;
  const int64_t head_stride = (int64_t)D << bs_log2;   // elements per (block, kv-head)
  const C* kbase = kc + h * head_stride;
  const C* vbase = vc + h * head_stride;
  const int64_t blk_stride = (int64_t)nkv * head_stride;

  const int keyA = 8 * (r16 >> 2) + (r16 & 3);
  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Balanced split: the ctx's 32-token chunks are divided evenly over the Z x 4 waves
  // (sizes differ by at most one chunk), so no wave of a workgroup idles while a
  // sibling processes one more 64-token partition (whole-partition round-robin left
  // up to 25 % of wave time idle at ctx ~ 600).  A wave's last step may hold one
  // chunk; the other chunk's loads clamp to the wave's last token (cache hits) and
  // its scores are masked.
  const int nchunk = (ctx + 31) >> 5;
  const int nwk = gridDim.z * 4, wk = blockIdx.z * 4 + wave;
  const int c0 = (int)(((int64_t)nchunk * wk) / nwk);
  const int c1 = (int)(((int64_t)nchunk * (wk + 1)) / nwk);
  const int end = min(ctx, c1 << 5);       // this wave's token range is [c0*32, end)
  Pack8<T> kf[NCH][2][KS];
  Pack8<T> vf[NCH][DT];
  static_assert(PREF, "the per-fragment-load form (measured 3-8 % slower) was removed");
  // K / V fragments of the wave-iteration starting at chunk ci (PREF: all up front)
  auto load_k = [&](int ci) {
    const int base = ci << 5;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ta = min(base + c * 32 + keyA, end - 1);
      const int tb = min(base + c * 32 + keyA + 4, end - 1);
      const C* ka = kbase + kgc_bt(bt, ta >> bs_log2, bt_stride, num_blocks) * blk_stride + (int64_t)(ta & bsm) * D + 8 * qd;
      const C* kb = kbase + kgc_bt(bt, tb >> bs_log2, bt_stride, num_blocks) * blk_stride + (int64_t)(tb & bsm) * D + 8 * qd;
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        kf[c][0][s2].u = ldf(ka + 32 * s2);
        kf[c][1][s2].u = ldf(kb + 32 * s2);
      }
    }
  };
  auto load_v = [&](int ci) {
    const int base = ci << 5;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      // V^T 8-key group of keys t0..t0+7: [(t0 & bsm) / 8][d][8]; 16 lanes = 256 B
      const int t0 = min(base + c * 32 + 8 * qd, end - 1) & ~7;
      const C* va = vbase + kgc_bt(bt, t0 >> bs_log2, bt_stride, num_blocks) * blk_stride + ((t0 & bsm) >> 3) * (D * 8) + r16 * 8;
#pragma unroll
      for (int t = 0; t < DT; ++t) vf[c][t].u = ldf(va + 16 * t * 8);
    }
  };
  // FUSE: the first iteration's K loads go out before the q prologue (whose slice
  // reads and barrier they then overlap), unless that iteration holds the new token
  // this workgroup is about to write.  (K and V both in flight spilled at 128 VGPRs.)
  const bool prefetched = FUSE && c0 < c1 && c0 != nchunk - 1;
  if (prefetched) load_k(c0);
  V8 qf[KS];
  if constexpr (FUSE) {
    // q of the GQA group staged through LDS: thread i < G * D/16 owns the NeoX chunk
    // pair (c, c + D/2) of head i / (D/16) (its head's D/16 threads are an aligned lane
    // group for the q-norm sum); wave 3 of the z-slice holding the last context token
    // writes that token's k / v meanwhile.  One barrier publishes both.
    constexpr int TPH = D / 16;
    const int tid = threadIdx.x;
    if (tid < G * TPH) {
      const int g = tid / TPH, c = tid % TPH;
      const int64_t qe = (int64_t)b * rp.qkv_stride + (int64_t)(h * G + g) * D;
      float xa[8], xb[8];
      const float sc = qkv_row_scale(rp, b);
      qkv_row8<T>(rp, qe + c * 8, xa, sc);
      qkv_row8<T>(rp, qe + D / 2 + c * 8, xb, sc);
      if (rp.q_norm_w) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += xa[j] * xa[j] + xb[j] * xb[j];
#pragma unroll
        for (int o = 1; o < TPH; o <<= 1) ss += __shfl_xor(ss, o, 64);
        const float inv = rsqrtf(ss / (float)D + rp.eps);
        norm8<T>(xa, inv, rp.q_norm_w, c * 8);
        norm8<T>(xb, inv, rp.q_norm_w, D / 2 + c * 8);
      }
      if (rp.use_rope) rope8(xa, xb, rp.cos_sin + rp.positions[b] * D, c * 8, D / 2);
      Pack8<T> oa, ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) { oa.h[j] = from_f<T>(xa[j]); ob.h[j] = from_f<T>(xb[j]); }
      *reinterpret_cast<u32x4*>(&lds_q[g][c * 8]) = oa.u;
      *reinterpret_cast<u32x4*>(&lds_q[g][D / 2 + c * 8]) = ob.u;
    }
    if (wave == 3 && blockIdx.z == gridDim.z - 1 && ctx > 0)
      decode_kv_write<T, D, KV8>(rp, b, h, nq, nkv, bs_log2, num_blocks,
                                 const_cast<void*>(kc_), const_cast<void*>(vc_), lane);
    // release the k / v stores to the workgroup (same CU, same L1) and the LDS q
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const bool valid = r16 < G;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      Pack8<T> t;
      t.u = *reinterpret_cast<const u32x4*>(&lds_q[valid ? r16 : 0][32 * s + 8 * qd]);
      if (!valid) t.u = u32x4{0, 0, 0, 0};
      qf[s] = t.v;
    }
  } else {
    const bool valid = r16 < G;
    const T* qrow = q + ((int64_t)b * nq + h * G + (valid ? r16 : 0)) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      Pack8<T> t;
      t.u = *reinterpret_cast<const u32x4*>(qrow + 32 * s + 8 * qd);
      if (!valid) t.u = u32x4{0, 0, 0, 0};
      qf[s] = t.v;
    }
  }
  for (int ci = c0; ci < c1; ci += NCH) {
    const int base = ci << 5;
    if (!(prefetched && ci == c0)) load_k(ci);
    load_v(ci);
    f32x4 sa[NCH], sb[NCH];
    // ---- S^T = K . Q^T
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      f32x4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        accA = mfma16x16x32(kf[c][0][s2].v, qf[s2], accA);
        accB = mfma16x16x32(kf[c][1][s2].v, qf[s2], accB);
      }
      sa[c] = accA;
      sb[c] = accB;
    }
    // ---- mask + partition max (log2 domain) + online rescale of the carry
    float m = m_run;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tok = base + c * 32 + 8 * qd + i;
        sa[c][i] = tok < end ? sa[c][i] * scale_log2 : -INFINITY;
        sb[c][i] = tok + 4 < end ? sb[c][i] * scale_log2 : -INFINITY;
        m = fmaxf(m, fmaxf(sa[c][i], sb[c][i]));
      }
    }
    m = max_xor16(m);
    m = max_xor32(m);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m);     // 0 on the first partition
    m_run = m;
    l_run *= alpha;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= alpha;
    // ---- P = exp2(S - m), O^T += V^T . P^T
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      Pack8<T> pf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pa = __builtin_amdgcn_exp2f(sa[c][i] - m);
        const float pb = __builtin_amdgcn_exp2f(sb[c][i] - m);
        l_run += pa + pb;
        pf.h[i] = from_f<T>(pa);
        pf.h[4 + i] = from_f<T>(pb);
      }
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        o[t] = mfma16x16x32(vf[c][t].v, pf.v, o[t]);
      }
    }
  }
  // ---- merge the 4 waves through LDS: lane (r16 = head, qd) holds O^T[16t+4qd+i][r16]
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
#pragma unroll
  for (int t = 0; t < DT; ++t)
    *reinterpret_cast<f32x4*>(&lds_o[wave][r16][16 * t + 4 * qd]) = o[t];
  if (qd == 0) {
    lds_m[wave][r16] = m_run;
    lds_l[wave][r16] = l_run;
  }
  __syncthreads();
  const bool direct = gridDim.z == 1;
  for (int e = threadIdx.x; e < G * D; e += 256) {
    const int hh = e / D, d = e % D;
    float M = fmaxf(fmaxf(lds_m[0][hh], lds_m[1][hh]), fmaxf(lds_m[2][hh], lds_m[3][hh]));
    float acc = 0.f, L = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float f = exp2f(lds_m[w][hh] - M);
        acc += f * lds_o[w][hh][d];
        L += f * lds_l[w][hh];
      }
    }
    const int64_t row = (int64_t)b * nq + h * G + hh;
    if (direct) {
      out[row * D + d] = from_f<T>(L > 0.f ? acc / L * v_scale : 0.f);
    } else {
      const int64_t prow = row * Zmax + blockIdx.z;
      tmp_out[prow * D + d] = acc * v_scale;
      if (d == 0) {
        max_logits[prow] = M;
        exp_sums[prow] = L;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// K1w: ONE WAVE per (seq, kv-head, z-slice), a 64-thread workgroup, its 32-key chunks
// software-pipelined two deep (chunk c + 1's K and V loads are in flight while chunk c's
// MFMAs and softmax run).  Why (round 4, profiles/README.md "K1w"): the 4-wave workgroup
// above runs equal-length workgroups in lock-step rounds; every round starts with all
// waves of a CU in their q / rope prologue and ends with all of them in the LDS merge, so
// the CU's memory pipe idles twice per round (~10-15 % of a 125 us dispatch at B = 256),
// and each wave's own loads stop while it computes.  Here a wave streams its whole
// context share (B = 256: one wave per (seq, kv-head), 20 chunks at ctx 640) with the
// next chunk always in flight; prologue and epilogue come once per wave, there is no
// cross-wave merge and no barrier.  256 VGPRs at 2 waves per SIMD hold both chunk
// buffers (2 x 64), O^T (32) and q (16).  Same math as paged_decode_kernel: S^T tiles
// with the row->key map key(m) = 8*(m>>2) + (m&3), P taken from S^T's accumulator as the
// P.V B operand, log2-domain online softmax.
// Block ids come from wave-uniform scalar loads (one or two per chunk), never from a
// vector load the chunk pipeline would have to wait behind.
// Z > 1: slice z writes (max, sum, O) partials at row-major slot row * Z + z (the reduce
// kernel runs with Zmax = Z).
// (A four-deep variant -- four named chunk buffers at one wave per SIMD -- measured slower
// at every shape, e.g. 21.5 vs 17.5 us at B = 256, nq 8 / nkv 1, one slice: removed.)
template <typename T, int D, bool KV8, bool FUSE>
__global__ __launch_bounds__(64, 2) void paged_decode_wave_kernel(
    T* __restrict__ out, const T* __restrict__ q, const void* __restrict__ kc_,
    const void* __restrict__ vc_, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ctx_lens, float* __restrict__ max_logits,
    float* __restrict__ exp_sums, float* __restrict__ tmp_out, int nq, int nkv, int bs_log2,
    float scale_log2, float v_scale, int num_blocks, DecodeRope rp, int min_per) {
  typedef typename Vec8<T>::type V8;
  typedef std::conditional_t<KV8, uint8_t, T> C;
  const C* __restrict__ kc = reinterpret_cast<const C*>(kc_);
  const C* __restrict__ vc = reinterpret_cast<const C*>(vc_);
  auto ldf = [](const C* p) -> u32x4 {
    if constexpr (KV8) return fp8x8_widen<T>(*reinterpret_cast<const u32x2*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
  };
  constexpr int KS = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) T lds_q[FUSE ? 16 : 1][FUSE ? D + 8 : 8];
  const int b = blockIdx.x, h = blockIdx.y, z = blockIdx.z, Z = gridDim.z;
  const int lane = threadIdx.x;
  const int r16 = lane & 15, qd = lane >> 4;
  const int G = nq / nkv;
  int ctx_in = ctx_lens[b];
  KGC_DCHECK_RANGE(ctx_in, 0, (bt_stride << bs_log2) + 1, "decode ctx_len");
  const int ctx = min(ctx_in, bt_stride << bs_log2);
  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int bsm = (1 << bs_log2) - 1;
  const int64_t head_stride = (int64_t)D << bs_log2;
  const C* kbase = kc + h * head_stride;
  const C* vbase = vc + h * head_stride;
  const int64_t blk_stride = (int64_t)nkv * head_stride;
  const int keyA = 8 * (r16 >> 2) + (r16 & 3);

  // slice z owns chunks [z * per, (z + 1) * per) with per >= 2 (the pipeline depth): the
  // non-empty slices come first and the reduce merges only those (a graph captured with
  // Z sized for max_model_len meets short contexts: most slices are then empty)
  const int nchunk = (ctx + 31) >> 5;
  const int per = decode_slice_chunks(nchunk, Z, min_per);
  const int nused = decode_used_slices(nchunk, Z, min_per);
  const int c0 = min(nchunk, z * per);
  const int c1 = min(nchunk, c0 + per);
  const int end = min(ctx, c1 << 5);          // this wave's tokens: [c0*32, end)
  const int last_blk = max(0, (end - 1) >> bs_log2);

  struct Frag {
    Pack8<T> k[2][KS];
    Pack8<T> v[DT];
  };
  // A 32-token chunk spans one block (bs >= 32) or two (bs = 16; the host keeps bs >= 16):
  // their ids are wave-uniform scalar loads (lgkmcnt), so looking them up never waits on
  // the vector loads in flight (a lane-shuffled register window did: its rare reload
  // branch made the wait-count pass drain vmcnt at every chunk).
  auto issue_part = [&](Frag& f, int ci, bool dok, bool dov) {
    const int base = ci << 5;
    const int blo = base >> bs_log2, bhi = min((base + 31) >> bs_log2, last_blk);
    const int64_t plo = kgc_bt(bt, blo, bt_stride, num_blocks);
    const int64_t phi = kgc_bt(bt, bhi, bt_stride, num_blocks);
    auto blk_of = [&](int tok) -> int64_t { return (tok >> bs_log2) == blo ? plo : phi; };
    const int ta = min(base + keyA, end - 1), tb = min(base + keyA + 4, end - 1);
    const C* ka = kbase + blk_of(ta) * blk_stride + (int64_t)(ta & bsm) * D + 8 * qd;
    const C* kb = kbase + blk_of(tb) * blk_stride + (int64_t)(tb & bsm) * D + 8 * qd;
    if (dok) {
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        f.k[0][s2].u = ldf(ka + 32 * s2);
        f.k[1][s2].u = ldf(kb + 32 * s2);
      }
    }
    const int t0 = min(base + 8 * qd, end - 1) & ~7;
    const C* va = vbase + blk_of(t0) * blk_stride + ((t0 & bsm) >> 3) * (D * 8) + r16 * 8;
    if (dov) {
#pragma unroll
      for (int t = 0; t < DT; ++t) f.v[t].u = ldf(va + 16 * t * 8);
    }
  };
  auto issue = [&](Frag& f, int ci) { issue_part(f, ci, true, true); };

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  V8 qf[KS];

  auto compute = [&](const Frag& f, int ci) {
    const int base = ci << 5;
    f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      sa = mfma16x16x32(f.k[0][s2].v, qf[s2], sa);
      sb = mfma16x16x32(f.k[1][s2].v, qf[s2], sb);
    }
    float m = m_run;
    if (base + 32 <= end) {
      // a whole chunk inside the slice (every chunk but the context's last): no mask
      // (wave-uniform branch with VALU only: it moves no load across the pipeline)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sa[i] *= scale_log2;
        sb[i] *= scale_log2;
        m = fmaxf(m, fmaxf(sa[i], sb[i]));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tok = base + 8 * qd + i;
        sa[i] = tok < end ? sa[i] * scale_log2 : -INFINITY;
        sb[i] = tok + 4 < end ? sb[i] * scale_log2 : -INFINITY;
        m = fmaxf(m, fmaxf(sa[i], sb[i]));
      }
    }
    // row max over the 4 key groups (lanes xor 16 / 32): permlane swaps on the VALU, not
    // two ds_bpermute round trips on the chunk's critical path
    m = max_xor16(m);
    m = max_xor32(m);
    // v_exp_f32 directly (exp2f adds a denormal range fix-up: compare, two selects and a
    // ldexp per call, ~35 % of the loop's VALU); exponents here are <= 0 and results that
    // would be denormal only ever weight a probability by ~0
    const float alpha = __builtin_amdgcn_exp2f(m_run - m);
    m_run = m;
    l_run *= alpha;
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] *= alpha;
    Pack8<T> pf;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pa = __builtin_amdgcn_exp2f(sa[i] - m), pb = __builtin_amdgcn_exp2f(sb[i] - m);
      l_run += pa + pb;
      pf.h[i] = from_f<T>(pa);
      pf.h[4 + i] = from_f<T>(pb);
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] = mfma16x16x32(f.v[t].v, pf.v, o[t]);
  };

  Frag fa, fb;
  // the slice's first chunk and the second one's keys go out before the q prologue (unless
  // one of them holds the new token this wave is about to write): every wave of the grid starts
  // with its prologue, so the K / V stream must already be in flight beside the prologue's
  // split-K slice reads (Llama-3-8B at B = 256: 31.5 MB of fp32 q/k/v slices per layer)
  const bool pre_a = c0 < c1 && !(FUSE && c0 == nchunk - 1);
  const bool pre_b = pre_a && !(FUSE && min(c0 + 1, c1 - 1) == nchunk - 1);
  if (pre_a) issue(fa, c0);
  if (pre_b) issue_part(fb, min(c0 + 1, c1 - 1), true, false);
  if constexpr (FUSE) {
    constexpr int TPH = D / 16;
    // the new token's k / v: written by the slice that reads the context's last chunk
    // (slices are compact: that is slice nz - 1, not Z - 1)
    const bool has_kv = ctx > 0 && z == nused - 1;
    if (G * TPH <= 32) {
      // ONE pass, every lane its own role, so the q, k and v slice loads are all in
      // flight together (as separate branches they were three dependent round trips):
      // lanes [0, G*TPH) a q chunk pair, [32, 32+TPH) a k chunk pair, [48, 48+D/8) a v
      // chunk of the new token (k / v only on the wave that owns it)
      const int kind = lane < G * TPH ? 0 : (has_kv && lane >= 32 && lane < 32 + TPH) ? 1
                     : (has_kv && lane >= 48 && lane < 48 + D / 8) ? 2 : 3;
      const int c = kind == 0 ? lane % TPH : kind == 1 ? lane - 32 : kind == 2 ? lane - 48 : 0;
      const int g = kind == 0 ? lane / TPH : 0;
      const int64_t row = (int64_t)b * rp.qkv_stride;
      const int64_t col = kind == 0 ? (int64_t)(h * G + g) * D : kind == 1 ? (int64_t)(nq + h) * D
                        : (int64_t)(nq + nkv + h) * D;
      float xa[8], xb[8];
      qkv_pair8<T>(rp, row + col + c * 8, row + col + (kind == 2 ? 0 : D / 2) + c * 8, xa,
                   xb, qkv_row_scale(rp, b));                   // v: xb a dummy reload
      const void* nw = kind == 0 ? rp.q_norm_w : rp.k_norm_w;
      if (nw) {                    // q / k norm over the head's TPH lanes (aligned groups)
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += xa[j] * xa[j] + xb[j] * xb[j];
#pragma unroll
        for (int o2 = 1; o2 < TPH; o2 <<= 1) ss += __shfl_xor(ss, o2, 64);
        if (kind < 2) {
          const float inv = rsqrtf(ss / (float)D + rp.eps);
          norm8<T>(xa, inv, nw, c * 8);
          norm8<T>(xb, inv, nw, D / 2 + c * 8);
        }
      }
      if (rp.use_rope && kind < 2) rope8(xa, xb, rp.cos_sin + rp.positions[b] * D, c * 8, D / 2);
      Pack8<T> oa, ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) { oa.h[j] = from_f<T>(xa[j]); ob.h[j] = from_f<T>(xb[j]); }
      if (kind == 0) {
        *reinterpret_cast<u32x4*>(&lds_q[g][c * 8]) = oa.u;
        *reinterpret_cast<u32x4*>(&lds_q[g][D / 2 + c * 8]) = ob.u;
      } else if (kind < 3) {
        int64_t slot = rp.slots[b];
        KGC_DCHECK_RANGE(slot, -1, (int64_t)num_blocks << bs_log2, "decode KV slot");
        if (slot >= 0) {
          const int64_t blk = slot >> bs_log2;
          const int off = (int)(slot & ((1 << bs_log2) - 1));
          if (kind == 1) {
            const int64_t e = ((blk * nkv + h) << bs_log2 | off) * D;
            if constexpr (KV8) {
              uint8_t* dst = const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(kc_)) + e;
              float fa[8], fb[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                fa[j] = to_f(oa.h[j]) * rp.k_inv;
                fb[j] = to_f(ob.h[j]) * rp.k_inv;
              }
              *reinterpret_cast<u32x2*>(dst + c * 8) =
                  u32x2{fp8x4(fa[0], fa[1], fa[2], fa[3]), fp8x4(fa[4], fa[5], fa[6], fa[7])};
              *reinterpret_cast<u32x2*>(dst + D / 2 + c * 8) =
                  u32x2{fp8x4(fb[0], fb[1], fb[2], fb[3]), fp8x4(fb[4], fb[5], fb[6], fb[7])};
            } else {
              T* dst = const_cast<T*>(reinterpret_cast<const T*>(kc_)) + e;
              *reinterpret_cast<u32x4*>(dst + c * 8) = oa.u;
              *reinterpret_cast<u32x4*>(dst + D / 2 + c * 8) = ob.u;
            }
          } else {
            // v: the un-normed, un-rotated value row chunk into the V^T 8-key group
            const int64_t e = ((blk * nkv + h) << bs_log2) * D +
                              ((int64_t)(off >> 3) * D + c * 8) * 8 + (off & 7);
            if constexpr (KV8) {
              uint8_t* dst = const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(vc_)) + e;
              const uint32_t w0 = fp8x4(xa[0] * rp.v_inv, xa[1] * rp.v_inv, xa[2] * rp.v_inv,
                                        xa[3] * rp.v_inv);
              const uint32_t w1 = fp8x4(xa[4] * rp.v_inv, xa[5] * rp.v_inv, xa[6] * rp.v_inv,
                                        xa[7] * rp.v_inv);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                dst[j * 8] = (uint8_t)(w0 >> (8 * j));
                dst[(j + 4) * 8] = (uint8_t)(w1 >> (8 * j));
              }
            } else {
              T* dst = const_cast<T*>(reinterpret_cast<const T*>(vc_)) + e;
#pragma unroll
              for (int j = 0; j < 8; ++j) dst[j * 8] = from_f<T>(xa[j]);
            }
          }
        }
      }
    } else {
      for (int i = lane; i < G * TPH; i += 64) {
        const int g = i / TPH, c = i % TPH;
        const int64_t qe = (int64_t)b * rp.qkv_stride + (int64_t)(h * G + g) * D;
        float xa[8], xb[8];
        qkv_pair8<T>(rp, qe + c * 8, qe + D / 2 + c * 8, xa, xb, qkv_row_scale(rp, b));
        if (rp.q_norm_w) {
          float ss = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += xa[j] * xa[j] + xb[j] * xb[j];
#pragma unroll
          for (int o2 = 1; o2 < TPH; o2 <<= 1) ss += __shfl_xor(ss, o2, 64);
          const float inv = rsqrtf(ss / (float)D + rp.eps);
          norm8<T>(xa, inv, rp.q_norm_w, c * 8);
          norm8<T>(xb, inv, rp.q_norm_w, D / 2 + c * 8);
        }
        if (rp.use_rope) rope8(xa, xb, rp.cos_sin + rp.positions[b] * D, c * 8, D / 2);
        Pack8<T> oa, ob;
#pragma unroll
        for (int j = 0; j < 8; ++j) { oa.h[j] = from_f<T>(xa[j]); ob.h[j] = from_f<T>(xb[j]); }
        *reinterpret_cast<u32x4*>(&lds_q[g][c * 8]) = oa.u;
        *reinterpret_cast<u32x4*>(&lds_q[g][D / 2 + c * 8]) = ob.u;
      }
      if (has_kv)
        decode_kv_write<T, D, KV8>(rp, b, h, nq, nkv, bs_log2, num_blocks,
                                   const_cast<void*>(kc_), const_cast<void*>(vc_), lane);
    }
    // the k / v stores complete before any later load of the chunk that holds them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const bool valid = r16 < G;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      Pack8<T> t;
      t.u = *reinterpret_cast<const u32x4*>(&lds_q[valid ? r16 : 0][32 * s + 8 * qd]);
      if (!valid) t.u = u32x4{0, 0, 0, 0};
      qf[s] = t.v;
    }
  } else {
    const bool valid = r16 < G;
    const T* qrow = q + ((int64_t)b * nq + h * G + (valid ? r16 : 0)) * D;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      Pack8<T> t;
      t.u = *reinterpret_cast<const u32x4*>(qrow + 32 * s + 8 * qd);
      if (!valid) t.u = u32x4{0, 0, 0, 0};
      qf[s] = t.v;
    }
  }
  if (!pre_a && c0 < c1) issue(fa, c0);
  if (c0 < c1) issue_part(fb, min(c0 + 1, c1 - 1), !pre_b, true);
  // two-deep pipeline over named buffers (a runtime-indexed buffer pair would live in
  // scratch): while one chunk computes, the next one's loads are in flight.  The loop
  // body is straight-line -- unconditional issues (past the range they re-load the wave's
  // last chunk: cache hits) and, for an odd chunk count, one final chunk computed fully
  // masked (its tokens are >= end: p = 0, alpha = 1) -- because any branch between an
  // issue and its use makes the compiler's wait-count pass merge the paths and wait for
  // the younger buffer too (measured in the .s: vmcnt(15) instead of (31) before the
  // first MFMA, i.e. the pipeline serialised).  The two buffers' first chunks were issued
  // above, so each iteration computes one buffer and refills it two chunks ahead.
  for (int ci = c0; ci < c1; ci += 2) {
    compute(fa, ci);
    issue(fa, min(ci + 2, c1 - 1));
    compute(fb, ci + 1);
    issue(fb, min(ci + 3, c1 - 1));
  }

  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  const int64_t row = (int64_t)b * nq + h * G + r16;
  // one slice covers the whole context (Z == 1, or min_per >= the context's chunks): the
  // normalised output directly -- the reduce skips such a row
  if (Z == 1 || nused == 1) {
    if (z > 0) return;
    if (r16 >= G) return;
    const float inv = l_run > 0.f ? v_scale / l_run : 0.f;
    T* orow = out + row * D + 4 * qd;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      Pack4<T> pk;
#pragma unroll
      for (int i = 0; i < 4; ++i) pk.h[i] = from_f<T>(o[t][i] * inv);
      *reinterpret_cast<u32x2*>(orow + 16 * t) = pk.u;
    }
    return;
  }
  // Z > 1: the used slices write (max, sum, O) partials at row * Z + z; slices past the
  // context write nothing (paged_decode_reduce_kernel merges slices 0 .. nz - 1 only).
  // (A merge by the last-arriving slice inside this launch -- sc1 partials, a ticket per
  // (seq, kv-head) -- measured slower than the reduce launch at every Z > 1 shape: B = 32
  // 59.2 vs 52.8 us, B = 1 12.9 vs 12.3 us; one wave merging G heads serialises what the
  // reduce spreads over B * nq waves.  profiles/README.md "K1w".)
  if (z >= nused || r16 >= G) return;
  const int64_t prow = row * Z + z;
  float* dst = tmp_out + prow * D + 4 * qd;
#pragma unroll
  for (int t = 0; t < DT; ++t)
    *reinterpret_cast<f32x4*>(dst + 16 * t) = o[t] * v_scale;
  if (qd == 0) {
    max_logits[prow] = m_run;
    exp_sums[prow] = l_run;
  }
}

// Merge the z-slice partials: one 64-thread wave per (seq, q-head).  WAVE (K1w): only the
// sequence's used slices wrote a partial (decode_used_slices); the 4-wave kernel writes
// all Z (empty ones with weight 0).
template <typename T, int D, bool WAVE>
__global__ __launch_bounds__(64) void paged_decode_reduce_kernel(
    T* __restrict__ out, const float* __restrict__ max_logits,
    const float* __restrict__ exp_sums, const float* __restrict__ tmp_out,
    const int* __restrict__ ctx_lens, int nq, int Zg, int Zmax, int ctx_cap, int min_per) {
  // The slice statistics are read in parallel (lane z), the weights staged in LDS,
  // and the partial rows loaded 8 slices at a time: the previous per-slice loop was a
  // chain of dependent L2 round trips (~7 us per call at B = 1; decode + reduce for
  // B = 1, ctx 565, Z = 16 went 13.0 -> 9.3 us).
  __shared__ float wz[DEC_MAX_Z];
  const int b = blockIdx.x, hq = blockIdx.y, tid = threadIdx.x;
  // the context the decode kernel covered: clamped to the block table's capacity exactly
  // as it clamps it (ctx_cap = bt_stride << bs_log2), so a ctx_len past the table never
  // makes this merge read slices that kernel did not write this step
  const int ctx = min(max(ctx_lens[b], 0), ctx_cap);
  const int Z = WAVE ? decode_used_slices((ctx + 31) >> 5, Zg, min_per) : Zg;
  if (WAVE && Z == 1 && ctx > 0) return;     // the decode kernel wrote this row itself
  T* orow = out + ((int64_t)b * nq + hq) * D;
  constexpr int EPT = D / 64;
  const int64_t base = ((int64_t)b * nq + hq) * Zmax;
  if (Z <= 0) {
    // no slice wrote a partial (an empty context: the graphs' idle rows): zeros, and no
    // partial row is read (the clamped loads below would index slice -1)
#pragma unroll
    for (int e = 0; e < EPT; ++e) orow[tid * EPT + e] = from_f<T>(0.f);
    return;
  }
  if (Z <= 64) {
    // one round trip: lane z's (max, sum) and the first 16 slices' partial rows are all
    // loaded before any of them is used; the weights travel by lane shuffles, not LDS (the
    // batch-1 step ran this merge as ~4 dependent round trips: 4.8 us x 32 layers)
    const float mz = tid < Z ? max_logits[base + tid] : -INFINITY;
    const float ez = tid < Z ? exp_sums[base + tid] : 0.f;
    constexpr int ZB = 16;
    float v[ZB][EPT];
#pragma unroll
    for (int j = 0; j < ZB; ++j) {
      const float* src = tmp_out + (base + min(j, Z - 1)) * D + tid * EPT;
#pragma unroll
      for (int e = 0; e < EPT; ++e) v[j][e] = src[e];
    }
    const float m = wave_max(mz);
    const bool live = ctx > 0 && m != -INFINITY;
    const float wl = live && tid < Z ? exp2f(mz - m) : 0.f;
    const float tot = wave_sum(wl * ez);
    float acc[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) acc[e] = 0.f;
#pragma unroll
    for (int j = 0; j < ZB; ++j) {
      const float w = __shfl(wl, j, 64);          // 0 past Z: lane j >= Z holds wl = 0
#pragma unroll
      for (int e = 0; e < EPT; ++e) acc[e] += w * v[j][e];
    }
    for (int z0 = ZB; z0 < Z; z0 += ZB) {
#pragma unroll
      for (int j = 0; j < ZB; ++j) {
        const float* src = tmp_out + (base + min(z0 + j, Z - 1)) * D + tid * EPT;
#pragma unroll
        for (int e = 0; e < EPT; ++e) v[j][e] = src[e];
      }
#pragma unroll
      for (int j = 0; j < ZB; ++j) {
        const float w = __shfl(wl, z0 + j, 64);
#pragma unroll
        for (int e = 0; e < EPT; ++e) acc[e] += w * v[j][e];
      }
    }
    const float inv = tot > 0.f ? 1.f / tot : 0.f;
#pragma unroll
    for (int e = 0; e < EPT; ++e) orow[tid * EPT + e] = from_f<T>(acc[e] * inv);
    return;
  }
  float m = -INFINITY;
  for (int z = tid; z < Z; z += 64) m = fmaxf(m, max_logits[base + z]);
  m = wave_max(m);
  float acc[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) acc[e] = 0.f;
  float tot = 0.f;
  if (ctx > 0 && m != -INFINITY) {
    for (int z = tid; z < Z; z += 64) {
      const float w = exp2f(max_logits[base + z] - m);
      wz[z] = w;
      tot += w * exp_sums[base + z];
    }
    tot = wave_sum(tot);
    __syncthreads();
    // 8 slices' partial rows in flight per step (every slice wrote its row, empty
    // ones with weight 0), instead of one dependent L2 round trip per slice
    for (int z0 = 0; z0 < Z; z0 += 8) {
      float v[8][EPT], wv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int z = min(z0 + j, Z - 1);
        wv[j] = z0 + j < Z ? wz[z] : 0.f;
        const float* src = tmp_out + (base + z) * D + tid * EPT;
#pragma unroll
        for (int e = 0; e < EPT; ++e) v[j][e] = src[e];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < EPT; ++e) acc[e] += wv[j] * v[j][e];
    }
  }
  const float inv = tot > 0.f ? 1.f / tot : 0.f;
#pragma unroll
  for (int e = 0; e < EPT; ++e) orow[tid * EPT + e] = from_f<T>(acc[e] * inv);
}

// KGC_DECODE_WAVE=0: the 4-wave workgroup kernel (A/B); default: K1w
bool decode_wave_enabled() {
  static const bool v = [] {
    const char* e = getenv("KGC_DECODE_WAVE");
    return !(e && e[0] == '0');
  }();
  return v;
}

// K1w for grids of >= DEC_WAVE_MIN_PAIRS (seq, kv-head) pairs (unless KGC_DECODE_WAVE=0),
// else the 4-wave kernel; both write partial rows Z apart (Zmax = Z)
// (KGC_DECODE_WAVE_MIN_PAIRS overrides the threshold: the tests run both kernels on every
// shape; ops/__init__.py reads the same variable)
static int decode_wave_min_pairs() {
  const char* e = getenv("KGC_DECODE_WAVE_MIN_PAIRS");
  return e ? atoi(e) : DEC_WAVE_MIN_PAIRS;
}
bool decode_use_wave(int B, int nkv) {
  return decode_wave_enabled() && (int64_t)B * nkv >= decode_wave_min_pairs();
}

// K1w's minimum 32-token chunks per z-slice for a launch of B x nkv pairs: from
// DEC_LONG_PAIRS pairs up the chip is filled by the pairs themselves, so a context of up to
// DEC_LONG_MIN_CHUNKS chunks stays one slice (no partials, no merge); below it slices of 2
// (KGC_DECODE_MIN_CHUNKS overrides for every launch).
static int decode_min_chunks(int B, int nkv) {
  const char* e = getenv("KGC_DECODE_MIN_CHUNKS");
  if (e) return atoi(e) < 2 ? 2 : atoi(e);
  return (int64_t)B * nkv >= DEC_LONG_PAIRS ? DEC_LONG_MIN_CHUNKS : 2;
}

template <typename T, int D, bool KV8, bool FUSE>
static void decode_dispatch(void* out, const void* q, const void* kc, const void* vc,
                            const int* bt, int bt_stride, const int* ctx, float* ml, float* es,
                            float* tmp, int B, int nq, int nkv, int bs_log2, int Z,
                            float scale_log2, float v_scale, int num_blocks,
                            const DecodeRope& rp, hipStream_t s) {
  const bool wave = decode_use_wave(B, nkv);
  // ONE min_per value feeds both launches below: the decode kernel and its merge derive the
  // same slice plan from it (decode_used_slices), and the merge trusts the decode kernel to
  // have written exactly the rows that plan names -- a single-slice row directly (nused ==
  // 1), the others as partials (tests/test_kernels_gpu.py
  // ::test_paged_decode_single_slice_rows_many_pairs)
  const int min_per = decode_min_chunks(B, nkv);
  if (wave) {
    paged_decode_wave_kernel<T, D, KV8, FUSE><<<dim3(B, nkv, Z), 64, 0, s>>>(
        (T*)out, (const T*)q, kc, vc, bt, bt_stride, ctx, ml, es, tmp, nq, nkv, bs_log2,
        scale_log2, v_scale, num_blocks, rp, min_per);
  } else {
    paged_decode_kernel<T, D, true, KV8, 4, 1, FUSE><<<dim3(B, nkv, Z), 256, 0, s>>>(
        (T*)out, (const T*)q, kc, vc, bt, bt_stride, ctx, ml, es, tmp, nq, nkv, bs_log2, Z,
        scale_log2, v_scale, num_blocks, rp);
  }
  if (Z == 1) return;
  if (wave)
    paged_decode_reduce_kernel<T, D, true><<<dim3(B, nq), 64, 0, s>>>((T*)out, ml, es, tmp, ctx,
                                                                      nq, Z, Z,
                                                                      bt_stride << bs_log2,
                                                                      min_per);
  else
    paged_decode_reduce_kernel<T, D, false><<<dim3(B, nq), 64, 0, s>>>((T*)out, ml, es, tmp,
                                                                       ctx, nq, Z, Z,
                                                                       bt_stride << bs_log2,
                                                                       min_per);
}

template <bool FUSE>
static void decode_launch(int dtype, void* out, const void* q, const void* k_cache,
                          const void* v_cache, const int* block_tables, int bt_stride,
                          const int* ctx_lens, float* max_logits, float* exp_sums,
                          float* tmp_out, int B, int nq, int nkv, int D, int bs_log2, int Z,
                          float scale, bool kv_fp8, float k_scale, float v_scale, int num_blocks,
                          const DecodeRope& rp, hipStream_t s) {
  if (B == 0) return;
  const float sl2 = scale * k_scale * 1.4426950408889634f;
#define KGC_DEC(TT, DD, K8)                                                                 \
  decode_dispatch<TT, DD, K8, FUSE>(out, q, k_cache, v_cache, block_tables, bt_stride,       \
                                    ctx_lens, max_logits, exp_sums, tmp_out, B, nq, nkv,    \
                                    bs_log2, Z, sl2, v_scale, num_blocks, rp, s)
#define KGC_DEC_D(TT, K8) \
  if (D == 128) KGC_DEC(TT, 128, K8); else KGC_DEC(TT, 64, K8)
  if (dtype == DT_BF16) {
    if (kv_fp8) { KGC_DEC_D(bf16, true); } else { KGC_DEC_D(bf16, false); }
  } else {
    if (kv_fp8) { KGC_DEC_D(f16, true); } else { KGC_DEC_D(f16, false); }
  }
#undef KGC_DEC_D
#undef KGC_DEC
}

void launch_paged_decode(int dtype, void* out, const void* q, const void* k_cache,
                         const void* v_cache, const int* block_tables, int bt_stride,
                         const int* ctx_lens, float* max_logits, float* exp_sums,
                         float* tmp_out, int B, int nq, int nkv, int D, int bs_log2, int Z,
                         float scale, bool kv_fp8, float k_scale, float v_scale, int num_blocks,
                         hipStream_t s) {
  const DecodeRope none{};
  decode_launch<false>(dtype, out, q, k_cache, v_cache, block_tables, bt_stride, ctx_lens,
                       max_logits, exp_sums, tmp_out, B, nq, nkv, D, bs_log2, Z, scale, kv_fp8,
                       k_scale, v_scale, num_blocks, none, s);
}

void launch_paged_decode_rope(int dtype, const DecodeRope& rp, void* out, void* k_cache,
                              void* v_cache, const int* block_tables, int bt_stride,
                              const int* ctx_lens, float* max_logits, float* exp_sums,
                              float* tmp_out, int B, int nq, int nkv, int D, int bs_log2,
                              int Z, float scale, bool kv_fp8, float k_scale, float v_scale,
                              int num_blocks, hipStream_t s) {
  decode_launch<true>(dtype, out, nullptr, k_cache, v_cache, block_tables, bt_stride, ctx_lens,
                      max_logits, exp_sums, tmp_out, B, nq, nkv, D, bs_log2, Z, scale, kv_fp8,
                      k_scale, v_scale, num_blocks, rp, s);
}

int paged_decode_wave_min_pairs() { return decode_wave_enabled() ? decode_wave_min_pairs() : -1; }

KGC_DEBUG_TU(attention_decode)

}  // namespace kgc
