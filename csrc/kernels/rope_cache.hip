// K3 + K5 + K6 fused: split the fused QKV projection row, optional per-head q/k
// RMSNorm (Qwen3), NeoX RoPE on q and k, write rotated q contiguous and scatter
// k / v into the paged cache.  grid (tokens, item groups); one thread owns the pair
// of 16-byte chunks (c, c + d/2) of one head so the rotation needs no exchange;
// the head's TPH = d/16 threads are an aligned lane group for the q/k-norm sum.
//
// SL: the QKV projection arrives as S fp32 split-K slices [S, T, N] of the K9m decode
// GEMM (gemm_decode.hip) and is summed here (rounded to T as the unfused GEMM output
// would be), so the slice reduction costs no kernel of its own.
// Cache layouts (see ops/reference.py):
//   k_cache [nb, nkv, bs, d]    v_cache [nb, nkv, bs/8, d, 8]  (V^T in 8-key groups)
// KV8: the cache holds fp8 e4m3 of (value / scale) (--kv-cache-dtype fp8); the value
// quantised is the T-rounded one, exactly what a T cache would store.
#include "common.h"
#include "launch.h"
#include <cstdlib>

namespace kgc {

constexpr int ROPE_NT = 128;
constexpr int ROPE_HG = 8;       // heads per q/k item (shared cos / sin)
// split-K slices (decode shapes): one head per item -- 8 heads x S slices of loads per
// thread made the small-T launch latency bound (161.7 vs 137 us, rope + decode at B = 256)
template <bool SL> constexpr int rope_hg() { return SL ? 1 : ROPE_HG; }

// 8 consecutive elements of the QKV row: T storage, or the sum of S fp32 slices
template <typename T, bool SL>
__device__ __forceinline__ u32x4 qkv8(const void* qkv, int64_t row_elem, int col, int S,
                                      int64_t slice_stride) {
  if constexpr (!SL) {
    return *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(qkv) + row_elem + col);
  } else {
    const float* p = reinterpret_cast<const float*>(qkv) + row_elem + col;
    f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
    for (int z = 1; z < S; ++z) {
      a += *reinterpret_cast<const f32x4*>(p + z * slice_stride);
      b += *reinterpret_cast<const f32x4*>(p + z * slice_stride + 4);
    }
    Pack8<T> o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o.h[q] = from_f<T>(a[q]);
      o.h[4 + q] = from_f<T>(b[q]);
    }
    return o.u;
  }
}

// KVO: k / v only (q_out unused): the prefill attention kernel rotates q itself as it
// loads it from the QKV row, so a prefill-only step never writes or re-reads q
template <typename T, bool NORM, bool ROPE, bool KV8, bool SL, bool KVO>
__global__ __launch_bounds__(ROPE_NT) void rope_kv_kernel(
    const void* __restrict__ qkv, int64_t qkv_stride, int S, int64_t slice_stride,
    const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, T* __restrict__ q_out, void* __restrict__ k_cache,
    void* __restrict__ v_cache, const int64_t* __restrict__ slot_mapping,
    const T* __restrict__ qn_w, const T* __restrict__ kn_w, int nq, int nkv, int d, int bs,
    float eps, float k_inv, float v_inv, int num_blocks) {
  // item space of one token: [q/k rotation items, padded to a wave] [v scatter items];
  // gridDim.y workgroups of ROPE_NT items share a token (fills the CUs at decode).
  // A q/k item is one chunk pair (c, c + d/2) of a group of ROPE_HG heads: the position's
  // cos / sin are loaded once for all of them and the heads' loads are all in flight
  // together (one item per head re-read the same 64 B of cos / sin per head, ~20 KB of
  // L2 reads per token at 40 heads).
  const int t = blockIdx.x;
  const int tph = d >> 4;               // threads per head group (pairs of 8-elem chunks)
  const int half = d >> 1;
  const int nheads = KVO ? nkv : nq + nkv;
  const int h_off = KVO ? nq : 0;       // 0..nq-1 = q, nq.. = k
  constexpr int HG = rope_hg<SL>();
  const int n_qk = (nheads + HG - 1) / HG * tph;
  const int n_qk_pad = (n_qk + 63) & ~63;
  const int it = blockIdx.y * ROPE_NT + threadIdx.x;
  int64_t slot = slot_mapping[t];
  KGC_DCHECK_RANGE(slot, -1, (int64_t)num_blocks * bs, "KV slot");   // -1: no KV write
  const int64_t row = (int64_t)t * qkv_stride;   // element offset of this token's row
  const int64_t blk = slot >= 0 ? slot / bs : 0;
  const int off = slot >= 0 ? (int)(slot % bs) : 0;
  if (it < n_qk_pad) {                  // whole waves take this branch together
    const bool active = it < n_qk;
    const int h0 = (active ? it / tph : 0) * HG;
    const int nh = min(HG, nheads - h0);   // the same for the tph lanes of a group
    const int c = it % tph;                     // chunk index within the first half
    Pack8<T> a[HG], b[HG];
#pragma unroll
    for (int k = 0; k < HG; ++k) {              // tail heads re-load the group's last head
      const int head = h_off + h0 + min(k, nh - 1);
      a[k].u = qkv8<T, SL>(qkv, row + head * d, c * 8, S, slice_stride);
      b[k].u = qkv8<T, SL>(qkv, row + head * d, half + c * 8, S, slice_stride);
    }
    float cc[8], sn[8];
    if (ROPE) {
      const float* cs = cos_sin + positions[t] * d;
      const float4 c0 = *reinterpret_cast<const float4*>(cs + c * 8);
      const float4 c1 = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(cs + half + c * 8);
      const float4 s1 = *reinterpret_cast<const float4*>(cs + half + c * 8 + 4);
      cc[0] = c0.x; cc[1] = c0.y; cc[2] = c0.z; cc[3] = c0.w;
      cc[4] = c1.x; cc[5] = c1.y; cc[6] = c1.z; cc[7] = c1.w;
      sn[0] = s0.x; sn[1] = s0.y; sn[2] = s0.z; sn[3] = s0.w;
      sn[4] = s1.x; sn[5] = s1.y; sn[6] = s1.z; sn[7] = s1.w;
    }
    Pack8<T> qwa, qwb, kwa, kwb;
    if (NORM) {
      qwa.u = *reinterpret_cast<const u32x4*>(qn_w + c * 8);
      qwb.u = *reinterpret_cast<const u32x4*>(qn_w + half + c * 8);
      kwa.u = *reinterpret_cast<const u32x4*>(kn_w + c * 8);
      kwb.u = *reinterpret_cast<const u32x4*>(kn_w + half + c * 8);
    }
#pragma unroll
    for (int k = 0; k < HG; ++k) {
      if (k >= nh) break;                       // uniform within the lane group
      const int head = h_off + h0 + k;
      float xa[8], xb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { xa[j] = to_f(a[k].h[j]); xb[j] = to_f(b[k].h[j]); }
      if (NORM) {
        const Pack8<T>& wa = head < nq ? qwa : kwa;
        const Pack8<T>& wb = head < nq ? qwb : kwb;
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += xa[j] * xa[j] + xb[j] * xb[j];
        for (int o = 1; o < tph; o <<= 1) ss += __shfl_xor(ss, o, 64);
        const float inv = rsqrtf(ss / (float)d + eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // round through T like the unfused reference (norm output is stored in T)
          xa[j] = to_f(from_f<T>(xa[j] * inv * to_f(wa.h[j])));
          xb[j] = to_f(from_f<T>(xb[j] * inv * to_f(wb.h[j])));
        }
      }
      if (!active) continue;
      Pack8<T> oa, ob;
      if (ROPE) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float ra, rb;
          neox_rot(xa[j], xb[j], cc[j], sn[j], ra, rb);
          oa.h[j] = from_f<T>(ra);
          ob.h[j] = from_f<T>(rb);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { oa.h[j] = from_f<T>(xa[j]); ob.h[j] = from_f<T>(xb[j]); }
      }
      if (!KVO && head < nq) {
        T* dst = q_out + ((int64_t)t * nq + head) * d;
        *reinterpret_cast<u32x4*>(dst + c * 8) = oa.u;
        *reinterpret_cast<u32x4*>(dst + half + c * 8) = ob.u;
      } else if (slot >= 0) {
        const int kh = head - nq;
        const int64_t e = ((blk * nkv + kh) * bs + off) * d;
        if constexpr (KV8) {
          uint8_t* dst = reinterpret_cast<uint8_t*>(k_cache) + e;
          float fa[8], fb[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) { fa[j] = to_f(oa.h[j]) * k_inv; fb[j] = to_f(ob.h[j]) * k_inv; }
          *reinterpret_cast<u32x2*>(dst + c * 8) =
              u32x2{fp8x4(fa[0], fa[1], fa[2], fa[3]), fp8x4(fa[4], fa[5], fa[6], fa[7])};
          *reinterpret_cast<u32x2*>(dst + half + c * 8) =
              u32x2{fp8x4(fb[0], fb[1], fb[2], fb[3]), fp8x4(fb[4], fb[5], fb[6], fb[7])};
        } else {
          T* dst = reinterpret_cast<T*>(k_cache) + e;
          *reinterpret_cast<u32x4*>(dst + c * 8) = oa.u;
          *reinterpret_cast<u32x4*>(dst + half + c * 8) = ob.u;
        }
      }
    }
    return;
  }
  // v heads: transposed scatter into the 8-key group of this token (2-byte stores at
  // a 16-byte stride: the 8 stores of a thread share one 128-byte line)
  const int iv = it - n_qk_pad;
  if (slot < 0 || iv >= nkv * (d >> 3)) return;
  const int h = iv / (d >> 3), c = iv % (d >> 3);
  Pack8<T> v;
  v.u = qkv8<T, SL>(qkv, row + (nq + nkv) * d + h * d, c * 8, S, slice_stride);
  const int64_t e = (blk * nkv + h) * (int64_t)bs * d + ((int64_t)(off >> 3) * d + c * 8) * 8 +
                    (off & 7);
  if constexpr (KV8) {
    uint8_t* dst = reinterpret_cast<uint8_t*>(v_cache) + e;
    const uint32_t w0 = fp8x4(to_f(v.h[0]) * v_inv, to_f(v.h[1]) * v_inv, to_f(v.h[2]) * v_inv,
                              to_f(v.h[3]) * v_inv);
    const uint32_t w1 = fp8x4(to_f(v.h[4]) * v_inv, to_f(v.h[5]) * v_inv, to_f(v.h[6]) * v_inv,
                              to_f(v.h[7]) * v_inv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dst[j * 8] = (uint8_t)(w0 >> (8 * j));
      dst[(j + 4) * 8] = (uint8_t)(w1 >> (8 * j));
    }
  } else {
    T* dst = reinterpret_cast<T*>(v_cache) + e;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j * 8] = v.h[j];
  }
}

// Prefill K / V write (KVO, RoPE, no k-norm, T cache): one 256-thread workgroup per
// 8-token group.  The per-token grid above gives a token 8 K threads in a 64-lane wave
// and 128 V threads that each issue eight 2-byte stores; at a 16K-token chunk that kernel
// took 137 us per layer for 134 MB of traffic.  Here a group whose 8 tokens fill one
// 8-key group of the cache (consecutive slots, the first a multiple of 8 -- every group
// of a sequence's aligned prefill) is written as:
//   K: every (token, head, chunk pair) item rotated and stored as two 16-byte rows;
//   V: thread (head, chunk) loads the chunk of all 8 tokens and writes the 8 x 8 block
//      transposed, eight 16-byte stores (whole V^T rows of the group).
// Other groups (sequence boundaries inside the group, padding slots) take 2-byte V stores.
constexpr int KVG_NT = 256;
template <typename T>
__global__ __launch_bounds__(KVG_NT) void kv_group_kernel(
    const T* __restrict__ qkv, int64_t qkv_stride, const int64_t* __restrict__ positions,
    const float* __restrict__ cos_sin, T* __restrict__ k_cache, T* __restrict__ v_cache,
    const int64_t* __restrict__ slot_mapping, int T_, int nq, int nkv, int d, int bs,
    int num_blocks) {
  const int t0 = blockIdx.x * 8, nt = min(8, T_ - t0);
  const int tph = d >> 4, half = d >> 1, cpr = d >> 3;
  __shared__ int64_t s_slot[8];
  __shared__ int s_full;
  if (threadIdx.x < 8) {
    int64_t s = threadIdx.x < nt ? slot_mapping[t0 + threadIdx.x] : -1;
    KGC_DCHECK_RANGE(s, -1, (int64_t)num_blocks * bs, "KV slot");
    s_slot[threadIdx.x] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bool full = nt == 8 && s_slot[0] >= 0 && (s_slot[0] & 7) == 0;
    for (int k = 1; k < 8; ++k) full = full && s_slot[k] == s_slot[0] + k;
    s_full = full;
  }
  // K: items (token k, head h, chunk pair c), two per thread with both loads in flight
  const int nk_items = nt * nkv * tph;
  for (int base = 0; base < nk_items; base += 2 * KVG_NT) {
    Pack8<T> a[2], b[2];
    int kk[2], hh[2], cc_[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = min(base + u * KVG_NT + (int)threadIdx.x, nk_items - 1);
      kk[u] = it / (nkv * tph);
      hh[u] = (it / tph) % nkv;
      cc_[u] = it % tph;
      const T* src = qkv + (int64_t)(t0 + kk[u]) * qkv_stride + (int64_t)(nq + hh[u]) * d;
      a[u].u = *reinterpret_cast<const u32x4*>(src + cc_[u] * 8);
      b[u].u = *reinterpret_cast<const u32x4*>(src + half + cc_[u] * 8);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int it = base + u * KVG_NT + (int)threadIdx.x;
      const int64_t slot = s_slot[kk[u]];
      if (it >= nk_items || slot < 0) continue;
      const float* cs = cos_sin + positions[t0 + kk[u]] * d;
      const int c = cc_[u];
      const float4 c0 = *reinterpret_cast<const float4*>(cs + c * 8);
      const float4 c1 = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(cs + half + c * 8);
      const float4 s1 = *reinterpret_cast<const float4*>(cs + half + c * 8 + 4);
      const float co[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float si[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      Pack8<T> oa, ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float ra, rb;
        neox_rot(to_f(a[u].h[j]), to_f(b[u].h[j]), co[j], si[j], ra, rb);
        oa.h[j] = from_f<T>(ra);
        ob.h[j] = from_f<T>(rb);
      }
      T* dst = k_cache + (((slot / bs) * nkv + hh[u]) * bs + slot % bs) * (int64_t)d;
      *reinterpret_cast<u32x4*>(dst + c * 8) = oa.u;
      *reinterpret_cast<u32x4*>(dst + half + c * 8) = ob.u;
    }
  }
  // V: item (head h, chunk c) over the group's tokens
  __syncthreads();
  const bool full = s_full;
  for (int iv = threadIdx.x; iv < nkv * cpr; iv += KVG_NT) {
    const int h = iv / cpr, c = iv % cpr;
    const T* src = qkv + (int64_t)t0 * qkv_stride + (int64_t)(nq + nkv + h) * d + c * 8;
    if (full) {
      Pack8<T> vv[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) vv[k].u = *reinterpret_cast<const u32x4*>(src + k * qkv_stride);
      const int64_t slot = s_slot[0];
      const int off = (int)(slot % bs);
      T* dst = v_cache + ((slot / bs) * nkv + h) * (int64_t)bs * d +
               ((int64_t)(off >> 3) * d + c * 8) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Pack8<T> o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o.h[k] = vv[k].h[j];
        *reinterpret_cast<u32x4*>(dst + j * 8) = o.u;
      }
    } else {
      for (int k = 0; k < nt; ++k) {
        const int64_t slot = s_slot[k];
        if (slot < 0) continue;
        Pack8<T> v;
        v.u = *reinterpret_cast<const u32x4*>(src + k * qkv_stride);
        const int off = (int)(slot % bs);
        T* dst = v_cache + ((slot / bs) * nkv + h) * (int64_t)bs * d +
                 ((int64_t)(off >> 3) * d + c * 8) * 8 + (off & 7);
#pragma unroll
        for (int j = 0; j < 8; ++j) dst[j * 8] = v.h[j];
      }
    }
  }
}

// KGC_ROPE_KVG=0: prefill K / V writes on the per-token kernel (A/B)
static bool rope_kvg() {
  const char* e = getenv("KGC_ROPE_KVG");
  return !(e && atoi(e) == 0);
}

// (A whole-8-key-group V^T store by the group's first token -- KGC_ROPE_VGROUP, round 3 --
// measured slower at 16K-token prefill chunks, 152 -> 173 us: removed in round 6; the
// 8-token-group kernel below is the prefill K / V writer)

template <typename T, bool KV8, bool SL>
static void rope_dispatch(const void* qkv, int64_t qkv_stride, int S, int64_t ss,
                          const int64_t* pos,
                          const float* cs, void* q_out, void* kc, void* vc,
                          const int64_t* slots, const void* qn, const void* kn, int T_,
                          int nq, int nkv, int d, int bs, float eps, bool rope, float k_inv,
                          float v_inv, int num_blocks, hipStream_t s) {
  if (T_ == 0) return;
  const bool kvo = q_out == nullptr;
  constexpr int HG = rope_hg<SL>();
  const int n_items = (((((kvo ? 0 : nq) + nkv) + HG - 1) / HG * (d >> 4) + 63) & ~63) +
                      nkv * (d >> 3);
  const dim3 grid(T_, (n_items + ROPE_NT - 1) / ROPE_NT);
#define KGC_ROPE_LAUNCH(N, R, O)                                                            \
  rope_kv_kernel<T, N, R, KV8, SL, O><<<grid, ROPE_NT, 0, s>>>(                             \
      qkv, qkv_stride, S, ss, pos, cs, (T*)q_out, kc, vc, slots, (const T*)qn,               \
      (const T*)kn, nq, nkv, d, bs, eps, k_inv, v_inv, num_blocks)
  const bool norm = qn != nullptr;
  if constexpr (!KV8 && !SL) {
    if (kvo && rope && !norm && rope_kvg() && (d & 15) == 0 && (bs & 7) == 0) {
      kv_group_kernel<T><<<(T_ + 7) / 8, KVG_NT, 0, s>>>(
          (const T*)qkv, qkv_stride, pos, cs, (T*)kc, (T*)vc, slots, T_, nq, nkv, d, bs,
          num_blocks);
      return;
    }
  }
  if (kvo) {                    // prefill-only steps of RoPE models without q/k norm
    if (rope && !norm) KGC_ROPE_LAUNCH(false, true, true);
    else if (rope) KGC_ROPE_LAUNCH(true, true, true);
    else KGC_ROPE_LAUNCH(false, false, true);
  } else if (norm && rope) KGC_ROPE_LAUNCH(true, true, false);
  else if (norm) KGC_ROPE_LAUNCH(true, false, false);
  else if (rope) KGC_ROPE_LAUNCH(false, true, false);
  else KGC_ROPE_LAUNCH(false, false, false);
#undef KGC_ROPE_LAUNCH
}

template <typename T, bool KV8>
static void rope_dispatch_sl(const void* qkv, int64_t qkv_stride, int S, int64_t ss,
                             const int64_t* pos, const float* cs, void* q_out, void* kc, void* vc,
                             const int64_t* slots, const void* qn, const void* kn, int T_,
                             int nq, int nkv, int d, int bs, float eps, bool rope, float k_inv,
                             float v_inv, int num_blocks, hipStream_t s) {
  if (S > 0)
    rope_dispatch<T, KV8, true>(qkv, qkv_stride, S, ss, pos, cs, q_out, kc, vc, slots, qn, kn,
                                T_, nq, nkv, d, bs, eps, rope, k_inv, v_inv, num_blocks, s);
  else
    rope_dispatch<T, KV8, false>(qkv, qkv_stride, 0, 0, pos, cs, q_out, kc, vc, slots, qn, kn,
                                 T_, nq, nkv, d, bs, eps, rope, k_inv, v_inv, num_blocks, s);
}

void launch_rope_kv_write(int dtype, const void* qkv, int64_t qkv_stride, int S,
                          int64_t slice_stride, const int64_t* positions, const float* cos_sin,
                          void* q_out, void* k_cache, void* v_cache,
                          const int64_t* slot_mapping, const void* q_norm_w,
                          const void* k_norm_w, int T, int nq, int nkv, int d, int bs,
                          float eps, bool use_rope, bool kv_fp8, float k_scale, float v_scale,
                          int num_blocks, hipStream_t s) {
  const float ki = 1.f / k_scale, vi = 1.f / v_scale;
  if (dtype == DT_BF16) {
    if (kv_fp8)
      rope_dispatch_sl<bf16, true>(qkv, qkv_stride, S, slice_stride, positions, cos_sin, q_out,
                                   k_cache, v_cache, slot_mapping, q_norm_w, k_norm_w, T, nq,
                                   nkv, d, bs, eps, use_rope, ki, vi, num_blocks, s);
    else
      rope_dispatch_sl<bf16, false>(qkv, qkv_stride, S, slice_stride, positions, cos_sin, q_out,
                                    k_cache, v_cache, slot_mapping, q_norm_w, k_norm_w, T, nq,
                                    nkv, d, bs, eps, use_rope, ki, vi, num_blocks, s);
  } else {
    if (kv_fp8)
      rope_dispatch_sl<f16, true>(qkv, qkv_stride, S, slice_stride, positions, cos_sin, q_out,
                                  k_cache, v_cache, slot_mapping, q_norm_w, k_norm_w, T, nq,
                                  nkv, d, bs, eps, use_rope, ki, vi, num_blocks, s);
    else
      rope_dispatch_sl<f16, false>(qkv, qkv_stride, S, slice_stride, positions, cos_sin, q_out,
                                   k_cache, v_cache, slot_mapping, q_norm_w, k_norm_w, T, nq,
                                   nkv, d, bs, eps, use_rope, ki, vi, num_blocks, s);
  }
}

KGC_DEBUG_TU(rope_cache)

}  // namespace kgc
