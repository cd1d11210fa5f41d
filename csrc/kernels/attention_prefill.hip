// K2 varlen causal prefill attention over the paged KV cache (gfx950, bf16/f16).
//
// Each sequence contributes query rows [qsl[i], qsl[i+1]) at absolute positions
// seq_len-qlen .. seq_len-1 and attends causally to cache positions [0, seq_len):
// fresh prompts and chunked-prefill continuations run the same code.  The new
// tokens' K/V were already scattered into the cache by rope_kv_write.
//
// Grid: (work items, q-heads); a work item = (sequence, 128-row query block), listed
// heaviest-first by the host.  Workgroup = 4 waves x 32 query rows (two 16-row
// q-tiles per wave).  K/V advance in 64-key tiles staged global->VGPR->LDS,
// double-buffered, loads issued before the tile's MFMAs and written after them
// (one barrier per tile).
//
// MFMA orientation (v_mfma_f32_16x16x32): S^T = K.Q^T and O^T = V^T.P^T, so the
// query index is lane&15 in every accumulator: the online-softmax max/sum/rescale
// are lane-local (+ xor 16/32), and S^T's accumulator is already the B operand of
// the P.V product (row->key map key(m) = 8*(m>>2)+(m&3), +4 for the second tile of
// each 32-key pair).
// LDS images (16-byte chunk swizzles, conflict-free for the ds_read_b128 groups):
//   K   [64 keys][D]   chunk c of key k stored at c ^ f(k), f(k) = (k&3)|((k>>3)&3)<<2
//   V^T [D][64 keys]   chunk c of dim d stored at c ^ ((d>>1)&7)
#include "common.h"
#include "launch.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace kgc {

constexpr int PF_BM = 128;
constexpr int PF_BN = 64;

__device__ __forceinline__ int kswz(int k) { return (k & 3) | (((k >> 3) & 3) << 2); }

// q fragments of one 16-row q-tile: lane (r16, qd) holds dims 32 s + 8 qd .. + 7 of its
// row.  cos_sin != nullptr: the row is the unrotated q of the fused QKV projection and
// gets NeoX RoPE at position pos here -- dims i and i + D/2 sit in fragments s and
// s + KS/2 of the same lane, so the rotation is lane-local -- rounded to T exactly as
// rope_cache.hip rounds it.  (Prefill-only steps: rope_kv_write then writes only k / v,
// and q is neither stored nor re-read.)
template <typename T, int D>
__device__ __forceinline__ void pf_load_q(const T* qrow, const float* __restrict__ cos_sin,
                                          int cs_rows, int pos, int qd,
                                          typename Vec8<T>::type (&qf)[D / 32]) {
  constexpr int KS = D / 32;
  Pack8<T> t[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) t[s].u = *reinterpret_cast<const u32x4*>(qrow + 32 * s + 8 * qd);
  if (cos_sin != nullptr) {
    // clamped: a bad sequence length gives wrong output, never a fault
    const float* cs = cos_sin + (int64_t)min(pos, cs_rows - 1) * D;
#pragma unroll
    for (int s = 0; s < KS / 2; ++s) {
      const int col = 32 * s + 8 * qd;
      const float4 c0 = *reinterpret_cast<const float4*>(cs + col);
      const float4 c1 = *reinterpret_cast<const float4*>(cs + col + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(cs + D / 2 + col);
      const float4 s1 = *reinterpret_cast<const float4*>(cs + D / 2 + col + 4);
      const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float ra, rb;
        neox_rot(to_f(t[s].h[j]), to_f(t[s + KS / 2].h[j]), cc[j], sn[j], ra, rb);
        t[s].h[j] = from_f<T>(ra);
        t[s + KS / 2].h[j] = from_f<T>(rb);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = t[s].v;
}

// pf_load_q in two halves, so the loads can be issued early and the rotation done later:
// the persistent walk issues the next item's q (and cos / sin) loads BEFORE the current
// item's output stores -- on gfx9 stores count in vmcnt too, so loads issued after the
// stores would wait for the stores' completion at their first use.
template <typename T, int D>
struct PfQRaw {
  Pack8<T> t[D / 32];
  float4 c[D / 64][4];       // per rotated fragment pair: cos lo / hi, sin lo / hi
};
// cs_row: the row's cos / sin (always a readable row -- the caller passes a dummy one
// without RoPE -- so every register of r is written here and none stays live across the
// caller's loop)
template <typename T, int D>
__device__ __forceinline__ void pf_issue_q(const T* qrow, const float* __restrict__ cs_row,
                                           int qd, PfQRaw<T, D>& r) {
  constexpr int KS = D / 32;
#pragma unroll
  for (int s = 0; s < KS; ++s) r.t[s].u = *reinterpret_cast<const u32x4*>(qrow + 32 * s + 8 * qd);
#pragma unroll
  for (int s = 0; s < KS / 2; ++s) {
    const int col = 32 * s + 8 * qd;
    r.c[s][0] = *reinterpret_cast<const float4*>(cs_row + col);
    r.c[s][1] = *reinterpret_cast<const float4*>(cs_row + col + 4);
    r.c[s][2] = *reinterpret_cast<const float4*>(cs_row + D / 2 + col);
    r.c[s][3] = *reinterpret_cast<const float4*>(cs_row + D / 2 + col + 4);
  }
}
template <typename T, int D>
__device__ __forceinline__ void pf_finish_q(PfQRaw<T, D>& r, bool rope,
                                            typename Vec8<T>::type (&qf)[D / 32]) {
  constexpr int KS = D / 32;
  if (rope) {
#pragma unroll
    for (int s = 0; s < KS / 2; ++s) {
      const float cc[8] = {r.c[s][0].x, r.c[s][0].y, r.c[s][0].z, r.c[s][0].w,
                           r.c[s][1].x, r.c[s][1].y, r.c[s][1].z, r.c[s][1].w};
      const float sn[8] = {r.c[s][2].x, r.c[s][2].y, r.c[s][2].z, r.c[s][2].w,
                           r.c[s][3].x, r.c[s][3].y, r.c[s][3].z, r.c[s][3].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float ra, rb;
        neox_rot(to_f(r.t[s].h[j]), to_f(r.t[s + KS / 2].h[j]), cc[j], sn[j], ra, rb);
        r.t[s].h[j] = from_f<T>(ra);
        r.t[s + KS / 2].h[j] = from_f<T>(rb);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = r.t[s].v;
}

// Lazy O rescale (log2 units): the running max m only moves when some row's tile max
// exceeds it by more than this, so P = exp2(s - m) stays <= 2^8 and the O / l rescale
// (DT*8 + 2 VALU per lane) runs on a few tiles per row instead of on every tile.  The
// decision covers the tile BEFORE its P is exponentiated and after the previous tile's
// P.V is complete, and O, l and m move together (no P at the old scale is pending).
constexpr float PF_RESCALE_THR = 8.f;

// One 64-key tile for a wave's 32 query rows (two 16-row q-tiles), shared by both
// kernels.  K / V are the staged LDS images; key0 = the tile's first key.  Scores stay
// raw through the max (scale_log2 > 0 commutes with max) and enter the exponent as
// fma(s, scale_log2, -m): one VALU per score instead of a multiply and a subtract.
// exp2 is the bare v_exp_f32 (inputs <= PF_RESCALE_THR, -inf -> 0; no denormal
// range fix-up: exp2f() lowered to ~6 VALU per call).  MASK = the causal diagonal
// crosses this tile for some row of the wave; off-diagonal tiles skip the per-element
// key compare entirely.
template <typename T, int D, bool MASK>
__device__ __forceinline__ void pf_wave_tile(const T* __restrict__ K, const T* __restrict__ V,
                                             const typename Vec8<T>::type (&qf)[2][D / 32],
                                             f32x4 (&o)[2][D / 16], float (&m)[2], float (&l)[2],
                                             const int (&qpos)[2], int key0, float c, int r16,
                                             int qd) {
  typedef typename Vec8<T>::type V8;
  constexpr int NCH = D / 8, KS = D / 32, DT = D / 16;
  const int keyA = 8 * (r16 >> 2) + (r16 & 3);
  // ---- S^T tiles: [qt][a0, b0, a1, b1]
  f32x4 s[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int key = (j >> 1) * 32 + keyA + 4 * (j & 1);
    const T* krow = K + key * D;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      Pack8<T> f;
      f.u = *reinterpret_cast<const u32x4*>(krow + (((4 * ks + qd) ^ (r16 & (NCH - 1))) * 8));
      a0 = mfma16x16x32(f.v, qf[0][ks], a0);
      a1 = mfma16x16x32(f.v, qf[1][ks], a1);
    }
    s[0][j] = a0;
    s[1][j] = a1;
  }
  // ---- causal mask + lazy online softmax (query = lane&15: lane-local stats)
  V8 pf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    if constexpr (MASK) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (key0 + (j >> 1) * 32 + 8 * qd + 4 * (j & 1) + i > qpos[qt]) s[qt][j][i] = -INFINITY;
    }
    float tmax = fmaxf(fmaxf(s[qt][0][0], s[qt][0][1]), fmaxf(s[qt][0][2], s[qt][0][3]));
#pragma unroll
    for (int j = 1; j < 4; ++j)
      tmax = fmaxf(tmax, fmaxf(fmaxf(s[qt][j][0], s[qt][j][1]), fmaxf(s[qt][j][2], s[qt][j][3])));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    tmax *= c;                              // -inf stays -inf (a fully masked row)
    if (__any(tmax > m[qt] + PF_RESCALE_THR)) {
      const float mn = fmaxf(m[qt], tmax);
      const float alpha = __builtin_amdgcn_exp2f(m[qt] - mn);   // 0 on the first tile
      m[qt] = mn;
      l[qt] *= alpha;
#pragma unroll
      for (int t = 0; t < DT; ++t) o[qt][t] *= alpha;
    }
    const float nm = -m[qt];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Pack8<T> pk;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pa = __builtin_amdgcn_exp2f(__builtin_fmaf(s[qt][2 * kk][i], c, nm));
        const float pb = __builtin_amdgcn_exp2f(__builtin_fmaf(s[qt][2 * kk + 1][i], c, nm));
        l[qt] += pa + pb;
        pk.h[i] = from_f<T>(pa);
        pk.h[4 + i] = from_f<T>(pb);
      }
      pf[qt][kk] = pk.v;
    }
  }
  // ---- O^T += V^T . P^T
#pragma unroll
  for (int t = 0; t < DT; ++t) {
    const int d = 16 * t + r16;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      Pack8<T> f;
      f.u = *reinterpret_cast<const u32x4*>(V + d * PF_BN + (((4 * kk + qd) ^ ((d >> 1) & 7)) * 8));
      o[0][t] = mfma16x16x32(f.v, pf[0][kk], o[0][t]);
      o[1][t] = mfma16x16x32(f.v, pf[1][kk], o[1][t]);
    }
  }
}

// KV8: fp8 e4m3 cache; staged as 8-byte loads, widened to T on the way into LDS (the
// LDS image and everything after it is unchanged).  K scale folded into scale_log2,
// V scale applied in the epilogue.
template <typename T, int D, bool KV8>
__global__ __launch_bounds__(256, 2) void prefill_attn_kernel(
    const T* __restrict__ q, T* __restrict__ out, const void* __restrict__ kc_,
    const void* __restrict__ vc_, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ qsl, const int* __restrict__ seq_lens,
    const int* __restrict__ work_seq, const int* __restrict__ work_mblk, int nq, int nkv,
    int bs_log2, float scale_log2, float v_scale, int num_blocks, int64_t q_stride,
    const float* __restrict__ cos_sin, int cs_rows) {
  typedef typename Vec8<T>::type V8;
  typedef std::conditional_t<KV8, uint8_t, T> C;   // cache element
  typedef std::conditional_t<KV8, u32x2, u32x4> R; // staged raw fragment (8 elements)
  const C* __restrict__ kc = reinterpret_cast<const C*>(kc_);
  const C* __restrict__ vc = reinterpret_cast<const C*>(vc_);
  auto widen = [](R r) -> u32x4 {
    if constexpr (KV8) return fp8x8_widen<T>(r);
    else return r;
  };
  constexpr int NCH = D / 8;                 // 16-byte chunks per K row
  constexpr int KS = D / 32;                 // k-steps of QK^T
  constexpr int DT = D / 16;                 // d-tiles of O^T
  constexpr int KPT = PF_BN * NCH / 256;     // K chunks staged per thread
  constexpr int VPT = D * (PF_BN / 8) / 256; // V chunks staged per thread
  constexpr int TILE = PF_BN * D;            // elements per K (or V) image
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* lds = reinterpret_cast<T*>(smem);

  const int seq = work_seq[blockIdx.x], mb = work_mblk[blockIdx.x];
  const int hq = blockIdx.y;
  const int h = hq / (nq / nkv);
  const int q0 = qsl[seq];
  const int qlen = qsl[seq + 1] - q0;
  int L_in = seq_lens[seq];
  KGC_DCHECK_RANGE(L_in, 0, (bt_stride << bs_log2) + 1, "prefill seq_len");
  const int L = min(L_in, bt_stride << bs_log2);  // never index past the table
  const int ctx0 = L - qlen;
  if (qlen <= 0 || ctx0 < 0) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, qd = lane >> 4;
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int bsm = (1 << bs_log2) - 1;
  const int64_t hs = (int64_t)D << bs_log2;  // elements per (block, kv-head)

  V8 qf[2][KS];
  int qpos[2];
  // q is loaded (and, with cos_sin, rotated) AFTER the first K/V tile's loads are issued:
  // the rotation waits for q, and vmcnt retires in order, so q loaded first put its
  // latency in series with the block-table -> K/V chain of every workgroup's first tile
  auto load_q = [&]() {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = mb * PF_BM + wave * 32 + qt * 16 + r16;
      const int qc = min(qi, qlen - 1);
      qpos[qt] = ctx0 + qc;
      pf_load_q<T, D>(q + (int64_t)(q0 + qc) * q_stride + (int64_t)hq * D, cos_sin, cs_rows,
                      qpos[qt], qd, qf[qt]);
    }
  };
  const int last_q = ctx0 + min((mb + 1) * PF_BM, qlen) - 1;
  const int n_tiles = last_q / PF_BN + 1;

  // Block ids of a tile's chunks are fetched one tile AHEAD of its K/V loads: the
  // dependent block-table load would otherwise stall every tile's load issue for an
  // L2 round trip before the compute it is meant to overlap.
  R kreg[KPT], vreg[VPT];
  int kblk[KPT], vblk[VPT];
  auto fetch_bt = [&](int kt) {
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int key = (threadIdx.x + 256 * u) / NCH;
      kblk[u] = kgc_bt(bt, min(kt * PF_BN + key, L - 1) >> bs_log2, bt_stride, num_blocks);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int c = (threadIdx.x + 256 * u) / D;
      vblk[u] = kgc_bt(bt, (min(kt * PF_BN + 8 * c, L - 1) & ~7) >> bs_log2, bt_stride, num_blocks);
    }
  };
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int ci = threadIdx.x + 256 * u;
      const int key = ci / NCH, c = ci % NCH;
      const int ka = min(kt * PF_BN + key, L - 1);
      const C* src = kc + ((int64_t)kblk[u] * nkv + h) * hs + (int64_t)(ka & bsm) * D + c * 8;
      kreg[u] = *reinterpret_cast<const R*>(src);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {       // 8-key group c of dim d: contiguous in d
      const int ci = threadIdx.x + 256 * u;
      const int c = ci / D, d = ci % D;
      const int ka = min(kt * PF_BN + 8 * c, L - 1) & ~7;
      const C* src = vc + ((int64_t)vblk[u] * nkv + h) * hs + ((ka & bsm) >> 3) * (D * 8) + d * 8;
      vreg[u] = *reinterpret_cast<const R*>(src);
    }
  };
  auto store_tile = [&](int buf) {
    T* K = lds + buf * 2 * TILE;
    T* V = K + TILE;
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int ci = threadIdx.x + 256 * u;
      const int key = ci / NCH, c = ci % NCH;
      *reinterpret_cast<u32x4*>(K + key * D + ((c ^ (kswz(key) & (NCH - 1))) * 8)) = widen(kreg[u]);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int ci = threadIdx.x + 256 * u;
      const int c = ci / D, d = ci % D;
      *reinterpret_cast<u32x4*>(V + d * PF_BN + ((c ^ ((d >> 1) & 7)) * 8)) = widen(vreg[u]);
    }
  };

  f32x4 o[2][DT];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int t = 0; t < DT; ++t) o[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};

  fetch_bt(0);
  load_tile(0);
  load_q();
  if (n_tiles > 1) fetch_bt(1);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < n_tiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < n_tiles) {
      load_tile(kt + 1);
      fetch_bt(min(kt + 2, n_tiles - 1));   // unconditional: static vmcnt below
    }
    const T* K = lds + buf * 2 * TILE;
    const T* V = K + TILE;
    if ((kt + 1) * PF_BN - 1 > ctx0 + mb * PF_BM + wave * 32)
      pf_wave_tile<T, D, true>(K, V, qf, o, m, l, qpos, kt * PF_BN, scale_log2, r16, qd);
    else
      pf_wave_tile<T, D, false>(K, V, qf, o, m, l, qpos, kt * PF_BN, scale_log2, r16, qd);
    if (kt + 1 < n_tiles) store_tile(buf ^ 1);
    __syncthreads();
  }
  // ---- epilogue: O / l; lane holds O[query r16][16t + 4qd + i]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float tot = l[qt];
    tot += __shfl_xor(tot, 16, 64);
    tot += __shfl_xor(tot, 32, 64);
    const float inv = v_scale / tot;
    const int qi = mb * PF_BM + wave * 32 + qt * 16 + r16;
    if (qi < qlen) {
      T* orow = out + ((int64_t)(q0 + qi) * nq + hq) * D + 4 * qd;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        Pack4<T> pk;
#pragma unroll
        for (int i = 0; i < 4; ++i) pk.h[i] = from_f<T>(o[qt][t][i] * inv);
        *reinterpret_cast<u32x2*>(orow + 16 * t) = pk.u;
      }
    }
  }
}

// GQA-shared variant (G = nq / nkv >= 4): one workgroup = GH q-heads of ONE kv head x
// QB = 256 / GH queries, 8 waves of 32 query rows (wave w: head w % GH, rows
// 32 * (w / GH) ..).  Every K/V tile staged into LDS feeds 256 query rows of four or
// eight heads instead of 128 rows of one head: half the K/V staging per FLOP, and one
// staging pass per kv head instead of one per q-head.  The 128-row work items of the
// engine's work list split into 128 / QB sub-blocks (grid.z); the per-wave math is the
// single-head kernel's.
template <typename T, int D, bool KV8, int GH>
__global__ __launch_bounds__(512, 1) void prefill_attn_gqa_kernel(
    const T* __restrict__ q, T* __restrict__ out, const void* __restrict__ kc_,
    const void* __restrict__ vc_, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ qsl, const int* __restrict__ seq_lens,
    const int* __restrict__ work_seq, const int* __restrict__ work_mblk, int nq, int nkv,
    int bs_log2, float scale_log2, float v_scale, int num_blocks, int64_t q_stride,
    const float* __restrict__ cos_sin, int cs_rows) {
  typedef typename Vec8<T>::type V8;
  typedef std::conditional_t<KV8, uint8_t, T> C;
  typedef std::conditional_t<KV8, u32x2, u32x4> R;
  const C* __restrict__ kc = reinterpret_cast<const C*>(kc_);
  const C* __restrict__ vc = reinterpret_cast<const C*>(vc_);
  auto widen = [](R r) -> u32x4 {
    if constexpr (KV8) return fp8x8_widen<T>(r);
    else return r;
  };
  constexpr int NT_ = 512;
  constexpr int QB = 256 / GH;               // queries per workgroup
  static_assert(QB <= PF_BM && PF_BM % QB == 0, "sub-blocks of the 128-row work item");
  constexpr int NCH = D / 8, KS = D / 32, DT = D / 16;
  constexpr int KPT = PF_BN * NCH / NT_;
  constexpr int VPT = D * (PF_BN / 8) / NT_;
  constexpr int TILE = PF_BN * D;
  static_assert(KPT * NT_ == PF_BN * NCH && VPT * NT_ == D * (PF_BN / 8), "staging split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* lds = reinterpret_cast<T*>(smem);

  const int seq = work_seq[blockIdx.x], mb = work_mblk[blockIdx.x];
  const int G = nq / nkv;
  const int h = blockIdx.y / (G / GH);                 // kv head
  const int hg0 = h * G + (blockIdx.y % (G / GH)) * GH; // first q-head of this workgroup
  const int q0 = qsl[seq];
  const int qlen = qsl[seq + 1] - q0;
  int L_in = seq_lens[seq];
  KGC_DCHECK_RANGE(L_in, 0, (bt_stride << bs_log2) + 1, "prefill seq_len");
  const int L = min(L_in, bt_stride << bs_log2);
  const int ctx0 = L - qlen;
  const int qbase = mb * PF_BM + blockIdx.z * QB;      // first query row of the workgroup
  if (qlen <= 0 || ctx0 < 0 || qbase >= qlen) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int hq = hg0 + wave % GH;
  const int wq0 = qbase + (wave / GH) * 32;            // first query row of this wave
  const int r16 = lane & 15, qd = lane >> 4;
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int bsm = (1 << bs_log2) - 1;
  const int64_t hs = (int64_t)D << bs_log2;

  V8 qf[2][KS];
  int qpos[2];
  // q is loaded (and, with cos_sin, rotated) AFTER the first K/V tile's loads are issued:
  // the rotation waits for q, and vmcnt retires in order, so q loaded first put its
  // latency in series with the block-table -> K/V chain of every workgroup's first tile
  auto load_q = [&]() {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = wq0 + qt * 16 + r16;
      const int qc = min(qi, qlen - 1);
      qpos[qt] = ctx0 + qc;
      pf_load_q<T, D>(q + (int64_t)(q0 + qc) * q_stride + (int64_t)hq * D, cos_sin, cs_rows,
                      qpos[qt], qd, qf[qt]);
    }
  };
  const int last_q = ctx0 + min(qbase + QB, qlen) - 1;
  const int n_tiles = last_q / PF_BN + 1;

  // Block ids of a tile's chunks are fetched one tile AHEAD of its K/V loads: the
  // dependent block-table load would otherwise stall every tile's load issue for an
  // L2 round trip before the compute it is meant to overlap.
  R kreg[KPT], vreg[VPT];
  int kblk[KPT], vblk[VPT];
  auto fetch_bt = [&](int kt) {
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int key = (threadIdx.x + NT_ * u) / NCH;
      kblk[u] = kgc_bt(bt, min(kt * PF_BN + key, L - 1) >> bs_log2, bt_stride, num_blocks);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int c = (threadIdx.x + NT_ * u) / D;
      vblk[u] = kgc_bt(bt, (min(kt * PF_BN + 8 * c, L - 1) & ~7) >> bs_log2, bt_stride, num_blocks);
    }
  };
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int ci = threadIdx.x + NT_ * u;
      const int key = ci / NCH, c = ci % NCH;
      const int ka = min(kt * PF_BN + key, L - 1);
      const C* src = kc + ((int64_t)kblk[u] * nkv + h) * hs + (int64_t)(ka & bsm) * D + c * 8;
      kreg[u] = *reinterpret_cast<const R*>(src);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {       // 8-key group c of dim d: contiguous in d
      const int ci = threadIdx.x + NT_ * u;
      const int c = ci / D, d = ci % D;
      const int ka = min(kt * PF_BN + 8 * c, L - 1) & ~7;
      const C* src = vc + ((int64_t)vblk[u] * nkv + h) * hs + ((ka & bsm) >> 3) * (D * 8) + d * 8;
      vreg[u] = *reinterpret_cast<const R*>(src);
    }
  };
  auto store_tile = [&](int buf) {
    T* K = lds + buf * 2 * TILE;
    T* V = K + TILE;
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int ci = threadIdx.x + NT_ * u;
      const int key = ci / NCH, c = ci % NCH;
      *reinterpret_cast<u32x4*>(K + key * D + ((c ^ (kswz(key) & (NCH - 1))) * 8)) = widen(kreg[u]);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int ci = threadIdx.x + NT_ * u;
      const int c = ci / D, d = ci % D;
      *reinterpret_cast<u32x4*>(V + d * PF_BN + ((c ^ ((d >> 1) & 7)) * 8)) = widen(vreg[u]);
    }
  };

  f32x4 o[2][DT];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int t = 0; t < DT; ++t) o[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  // this wave's own last key tile (its rows end before the workgroup's last row)
  const int wave_tiles = (ctx0 + min(wq0 + 31, qlen - 1)) / PF_BN + 1;

  fetch_bt(0);
  load_tile(0);
  load_q();
  if (n_tiles > 1) fetch_bt(1);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < n_tiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < n_tiles) {
      load_tile(kt + 1);
      fetch_bt(min(kt + 2, n_tiles - 1));   // unconditional: static vmcnt below
    }
    if (kt < wave_tiles) {
      const T* K = lds + buf * 2 * TILE;
      const T* V = K + TILE;
      if ((kt + 1) * PF_BN - 1 > ctx0 + wq0)
        pf_wave_tile<T, D, true>(K, V, qf, o, m, l, qpos, kt * PF_BN, scale_log2, r16, qd);
      else
        pf_wave_tile<T, D, false>(K, V, qf, o, m, l, qpos, kt * PF_BN, scale_log2, r16, qd);
    }
    if (kt + 1 < n_tiles) store_tile(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float tot = l[qt];
    tot += __shfl_xor(tot, 16, 64);
    tot += __shfl_xor(tot, 32, 64);
    const float inv = v_scale / tot;
    const int qi = wq0 + qt * 16 + r16;
    if (qi < qlen && qi < qbase + QB) {
      T* orow = out + ((int64_t)(q0 + qi) * nq + hq) * D + 4 * qd;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        Pack4<T> pk;
#pragma unroll
        for (int i = 0; i < 4; ++i) pk.h[i] = from_f<T>(o[qt][t][i] * inv);
        *reinterpret_cast<u32x2*>(orow + 16 * t) = pk.u;
      }
    }
  }
}

// Persistent GQA variant: ONE workgroup per CU walks the work list (items = (128-row work
// item, kv-head group, QB-row sub-block), heaviest first, dealt round-robin), with the K / V
// tile stream running ACROSS items: the last tile of an item loads the next item's first
// tile into the free LDS buffer, so a new item starts with its tile already staged.
// Per-wave math, tile order and rounding are those of prefill_attn_gqa_kernel (results are
// bit-identical).  Why: at short prompts every workgroup of the one-shot grid paid its own
// pipeline fill -- the work_seq -> qsl / seq_lens -> block table -> K / V chain of dependent
// loads, the q load and the first LDS store, ~10 us -- against 1-8 tiles of ~2.5 us of
// work each (32 x 512 causal: 8 workgroups per CU, 0.40 PF/s against 0.84 PF/s at 16K).
template <typename T, int D, bool KV8, int GH>
__global__ __launch_bounds__(512, 1) void prefill_attn_gqa_persist_kernel(
    const T* __restrict__ q, T* __restrict__ out, const void* __restrict__ kc_,
    const void* __restrict__ vc_, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ qsl, const int* __restrict__ seq_lens,
    const int* __restrict__ work_seq, const int* __restrict__ work_mblk, int nq, int nkv,
    int bs_log2, float scale_log2, float v_scale, int num_blocks, int64_t q_stride,
    const float* __restrict__ cos_sin, int cs_rows, int n_items) {
  typedef typename Vec8<T>::type V8;
  typedef std::conditional_t<KV8, uint8_t, T> C;
  typedef std::conditional_t<KV8, u32x2, u32x4> R;
  const C* __restrict__ kc = reinterpret_cast<const C*>(kc_);
  const C* __restrict__ vc = reinterpret_cast<const C*>(vc_);
  auto widen = [](R r) -> u32x4 {
    if constexpr (KV8) return fp8x8_widen<T>(r);
    else return r;
  };
  constexpr int NT_ = 512;
  constexpr int QB = 256 / GH;
  constexpr int ZS = PF_BM / QB;                       // sub-blocks per 128-row work item
  constexpr int NCH = D / 8, KS = D / 32, DT = D / 16;
  constexpr int KPT = PF_BN * NCH / NT_;
  constexpr int VPT = D * (PF_BN / 8) / NT_;
  constexpr int TILE = PF_BN * D;
  static_assert(KPT * NT_ == PF_BN * NCH && VPT * NT_ == D * (PF_BN / 8), "staging split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* lds = reinterpret_cast<T*>(smem);

  const int G = nq / nkv;
  const int Y = nkv * (G / GH);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, qd = lane >> 4;
  const int bsm = (1 << bs_log2) - 1;
  const int64_t hs = (int64_t)D << bs_log2;
  const int cap = bt_stride << bs_log2;

  // an item's workgroup-uniform geometry (scalar registers); the per-wave values (q-head,
  // first row, last tile) are derived for the current item only (VGPRs are the limit
  // here: 256 at one workgroup of 8 waves per CU)
  struct Item {
    int q0, qlen, L, ctx0, qbase, hg0, h, n_tiles;
    const int* bt;
  };
  // item idx -> its geometry; false: nothing to do (empty / out-of-range sub-block)
  auto decode = [&](int idx, Item& I) -> bool {
    const int w = idx / (Y * ZS), r = idx - w * (Y * ZS);
    const int y = r / ZS, z = r - y * ZS;
    const int seq = work_seq[w], mb = work_mblk[w];
    I.h = y / (G / GH);
    I.hg0 = I.h * G + (y % (G / GH)) * GH;
    I.q0 = qsl[seq];
    I.qlen = qsl[seq + 1] - I.q0;
    int L_in = seq_lens[seq];
    KGC_DCHECK_RANGE(L_in, 0, cap + 1, "prefill seq_len");
    I.L = min(L_in, cap);
    I.ctx0 = I.L - I.qlen;
    I.qbase = mb * PF_BM + z * QB;
    if (I.qlen <= 0 || I.ctx0 < 0 || I.qbase >= I.qlen) return false;
    I.n_tiles = (I.ctx0 + min(I.qbase + QB, I.qlen) - 1) / PF_BN + 1;
    I.bt = block_tables + (int64_t)seq * bt_stride;
    return true;
  };
  // Items are dealt in rounds of gridDim.x, heaviest first (the host's work-list order),
  // alternating direction round to round: workgroup b takes item r * G + b in even rounds
  // and r * G + G - 1 - b in odd ones, so the workgroup dealt a round's heaviest item gets
  // the next round's lightest (plain round-robin left long prompts ~10 % imbalanced).
  const int G_ = gridDim.x, b_ = blockIdx.x;
  auto item_of = [&](int r) -> int { return r * G_ + ((r & 1) ? G_ - 1 - b_ : b_); };
  // the first round >= r whose item this workgroup has work in (its item in `I`), or a
  // round past the list
  auto next_valid = [&](int r, Item& I) -> int {
    while (r * G_ < n_items) {
      const int idx = item_of(r);
      if (idx < n_items && decode(idx, I)) break;
      ++r;
    }
    return r;
  };

  V8 qf[2][KS];
  int qpos[2];
  const int wrow = (wave / GH) * 32, whead = wave % GH;    // this wave's rows / head
  auto load_q = [&](const Item& I) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = I.qbase + wrow + qt * 16 + r16;
      const int qc = min(qi, I.qlen - 1);
      qpos[qt] = I.ctx0 + qc;
      pf_load_q<T, D>(q + (int64_t)(I.q0 + qc) * q_stride + (int64_t)(I.hg0 + whead) * D,
                      cos_sin, cs_rows, qpos[qt], qd, qf[qt]);
    }
  };
  PfQRaw<T, D> qraw[2];
  int qpos_n[2];
  auto issue_q = [&](const Item& I) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qi = I.qbase + wrow + qt * 16 + r16;
      const int qc = min(qi, I.qlen - 1);
      qpos_n[qt] = I.ctx0 + qc;
      // without RoPE the (unused) cos / sin come from a fixed readable row: q's first
      const float* csr = cos_sin != nullptr
                             ? cos_sin + (int64_t)min(qpos_n[qt], cs_rows - 1) * D
                             : reinterpret_cast<const float*>(q);
      pf_issue_q<T, D>(q + (int64_t)(I.q0 + qc) * q_stride + (int64_t)(I.hg0 + whead) * D,
                       csr, qd, qraw[qt]);
    }
  };
  auto finish_q = [&]() {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      qpos[qt] = qpos_n[qt];
      pf_finish_q<T, D>(qraw[qt], cos_sin != nullptr, qf[qt]);
    }
  };
  R kreg[KPT], vreg[VPT];
  int kblk[KPT], vblk[VPT];
  auto fetch_bt = [&](const int* bt, int L, int kt) {
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int key = (threadIdx.x + NT_ * u) / NCH;
      kblk[u] = kgc_bt(bt, min(kt * PF_BN + key, L - 1) >> bs_log2, bt_stride, num_blocks);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int c = (threadIdx.x + NT_ * u) / D;
      vblk[u] = kgc_bt(bt, (min(kt * PF_BN + 8 * c, L - 1) & ~7) >> bs_log2, bt_stride, num_blocks);
    }
  };
  auto load_tile = [&](int L, int h, int kt) {
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int ci = threadIdx.x + NT_ * u;
      const int key = ci / NCH, c = ci % NCH;
      const int ka = min(kt * PF_BN + key, L - 1);
      const C* src = kc + ((int64_t)kblk[u] * nkv + h) * hs + (int64_t)(ka & bsm) * D + c * 8;
      kreg[u] = *reinterpret_cast<const R*>(src);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int ci = threadIdx.x + NT_ * u;
      const int c = ci / D, d = ci % D;
      const int ka = min(kt * PF_BN + 8 * c, L - 1) & ~7;
      const C* src = vc + ((int64_t)vblk[u] * nkv + h) * hs + ((ka & bsm) >> 3) * (D * 8) + d * 8;
      vreg[u] = *reinterpret_cast<const R*>(src);
    }
  };
  auto store_tile = [&](int buf) {
    T* K = lds + buf * 2 * TILE;
    T* V = K + TILE;
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int ci = threadIdx.x + NT_ * u;
      const int key = ci / NCH, c = ci % NCH;
      *reinterpret_cast<u32x4*>(K + key * D + ((c ^ (kswz(key) & (NCH - 1))) * 8)) = widen(kreg[u]);
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int ci = threadIdx.x + NT_ * u;
      const int c = ci / D, d = ci % D;
      *reinterpret_cast<u32x4*>(V + d * PF_BN + ((c ^ ((d >> 1) & 7)) * 8)) = widen(vreg[u]);
    }
  };

  Item cur, nxt;
  int it = next_valid(0, cur);                    // `it`: the current item's round
  if (it * G_ >= n_items) return;                 // uniform: the whole workgroup leaves
  fetch_bt(cur.bt, cur.L, 0);
  load_tile(cur.L, cur.h, 0);
  load_q(cur);
  store_tile(0);
  __syncthreads();
  int buf = 0;
  bool kb_ready = false;     // kblk / vblk already hold the block ids of this item's tile 1
  for (;;) {
    const int nit = next_valid(it + 1, nxt);
    const bool has_next = nit * G_ < n_items;
    // the block ids of the tile loaded next: this item's tile 1, or the next item's tile 0
    if (!kb_ready) {
      if (cur.n_tiles > 1) fetch_bt(cur.bt, cur.L, 1);
      else if (has_next) fetch_bt(nxt.bt, nxt.L, 0);
    }
    kb_ready = false;
    const int wq0 = cur.qbase + wrow;
    const int wave_tiles = (cur.ctx0 + min(wq0 + 31, cur.qlen - 1)) / PF_BN + 1;
    f32x4 o[2][DT];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int t = 0; t < DT; ++t) o[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
    for (int kt = 0; kt < cur.n_tiles; ++kt) {
      // the tile after this one in the stream (this item's kt + 1, else the next item's
      // tile 0) is loaded while this one computes; then the block ids of the one after it
      bool loaded = false;
      if (kt + 1 < cur.n_tiles) {
        load_tile(cur.L, cur.h, kt + 1);
        if (kt + 2 < cur.n_tiles) fetch_bt(cur.bt, cur.L, kt + 2);
        else if (has_next) fetch_bt(nxt.bt, nxt.L, 0);
        loaded = true;
      } else if (has_next) {
        load_tile(nxt.L, nxt.h, 0);
        if (nxt.n_tiles > 1) {
          fetch_bt(nxt.bt, nxt.L, 1);
          kb_ready = true;
        }
        loaded = true;
      }
      if (kt < wave_tiles) {
        const T* K = lds + buf * 2 * TILE;
        const T* V = K + TILE;
        if ((kt + 1) * PF_BN - 1 > cur.ctx0 + wq0)
          pf_wave_tile<T, D, true>(K, V, qf, o, m, l, qpos, kt * PF_BN, scale_log2, r16, qd);
        else
          pf_wave_tile<T, D, false>(K, V, qf, o, m, l, qpos, kt * PF_BN, scale_log2, r16, qd);
      }
      if (loaded) store_tile(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
    // the next item's q loads go out before this item's output stores (see PfQRaw);
    // unconditional (the current item's rows again at the end of the walk) so the raw
    // registers are written every iteration and not kept live around the loop
    issue_q(has_next ? nxt : cur);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float tot = l[qt];
      tot += __shfl_xor(tot, 16, 64);
      tot += __shfl_xor(tot, 32, 64);
      const float inv = v_scale / tot;
      const int qi = wq0 + qt * 16 + r16;
      if (qi < cur.qlen && qi < cur.qbase + QB) {
        T* orow = out + ((int64_t)(cur.q0 + qi) * nq + cur.hg0 + whead) * D + 4 * qd;
#pragma unroll
        for (int t = 0; t < DT; ++t) {
          Pack4<T> pk;
#pragma unroll
          for (int i = 0; i < 4; ++i) pk.h[i] = from_f<T>(o[qt][t][i] * inv);
          *reinterpret_cast<u32x2*>(orow + 16 * t) = pk.u;
        }
      }
    }
    if (!has_next) break;
    // the next item's first tile is already staged in LDS buffer `buf`
    cur = nxt;
    it = nit;
    finish_q();
  }
}

// KGC_PREFILL_GQA=0: the one-head-per-workgroup kernel everywhere (A/B and tests)
static int prefill_gqa_enabled() {
  const char* e = getenv("KGC_PREFILL_GQA");
  return e ? atoi(e) : 1;
}

// KGC_PREFILL_PERSIST=0: the one-shot GQA grid instead of the persistent walk (A/B, tests)
static int prefill_persist_enabled() {
  const char* e = getenv("KGC_PREFILL_PERSIST");
  return e ? atoi(e) : 1;
}

template <typename T, int D, bool KV8, int GH>
static void prefill_gqa_dispatch(const void* q, void* out, const void* kc, const void* vc,
                                 const int* bt, int bt_stride, const int* qsl, const int* sl,
                                 const int* ws, const int* wm, int n_work, int nq, int nkv,
                                 int bs_log2, float scale_log2, float v_scale, int num_blocks,
                                 int64_t q_stride, const float* cos_sin, int cs_rows, hipStream_t s) {
  const size_t lds = 2 * 2 * PF_BN * D * sizeof(T);
  const int G = nq / nkv;
  const dim3 grid(n_work, nkv * (G / GH), PF_BM / (256 / GH));
  const int64_t n_items = (int64_t)grid.x * grid.y * grid.z;
  if (prefill_persist_enabled() && n_items < ((int64_t)1 << 30)) {
    // one workgroup per CU (launch_bounds(512, 1), 64 KB of LDS), never more than items
    static const int n_cu = [] {
      int dev = 0, cu = 256;
      if (hipGetDevice(&dev) == hipSuccess)
        hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
      return cu > 0 ? cu : 256;
    }();
    const int g = (int)std::min<int64_t>(n_items, n_cu);
    prefill_attn_gqa_persist_kernel<T, D, KV8, GH><<<g, 512, lds, s>>>(
        (const T*)q, (T*)out, kc, vc, bt, bt_stride, qsl, sl, ws, wm, nq, nkv, bs_log2,
        scale_log2, v_scale, num_blocks, q_stride, cos_sin, cs_rows, (int)n_items);
    return;
  }
  prefill_attn_gqa_kernel<T, D, KV8, GH><<<grid, 512, lds, s>>>(
      (const T*)q, (T*)out, kc, vc, bt, bt_stride, qsl, sl, ws, wm, nq, nkv, bs_log2,
      scale_log2, v_scale, num_blocks, q_stride, cos_sin, cs_rows);
}

template <typename T, int D, bool KV8>
static void prefill_dispatch(const void* q, void* out, const void* kc, const void* vc,
                             const int* bt, int bt_stride, const int* qsl, const int* sl,
                             const int* ws, const int* wm, int n_work, int nq, int nkv,
                             int bs_log2, float scale_log2, float v_scale, int num_blocks,
                             int64_t q_stride, const float* cos_sin, int cs_rows, hipStream_t s) {
  const int G = nkv > 0 ? nq / nkv : 1;
  if (D == 128 && prefill_gqa_enabled() && nq % nkv == 0 && (G == 4 || G % 8 == 0)) {
    if (G == 4)
      prefill_gqa_dispatch<T, D, KV8, 4>(q, out, kc, vc, bt, bt_stride, qsl, sl, ws, wm, n_work,
                                         nq, nkv, bs_log2, scale_log2, v_scale, num_blocks,
                                         q_stride, cos_sin, cs_rows, s);
    else
      prefill_gqa_dispatch<T, D, KV8, 8>(q, out, kc, vc, bt, bt_stride, qsl, sl, ws, wm, n_work,
                                         nq, nkv, bs_log2, scale_log2, v_scale, num_blocks,
                                         q_stride, cos_sin, cs_rows, s);
    return;
  }
  const size_t lds = 2 * 2 * PF_BN * D * sizeof(T);
  prefill_attn_kernel<T, D, KV8><<<dim3(n_work, nq), 256, lds, s>>>(
      (const T*)q, (T*)out, kc, vc, bt, bt_stride, qsl, sl, ws, wm, nq,
      nkv, bs_log2, scale_log2, v_scale, num_blocks, q_stride, cos_sin, cs_rows);
}

void launch_prefill_attention(int dtype, const void* q, void* out, const void* k_cache,
                              const void* v_cache, const int* block_tables, int bt_stride,
                              const int* query_start_loc, const int* seq_lens,
                              const int* work_seq, const int* work_mblk, int n_work, int nq,
                              int nkv, int D, int bs_log2, float scale, bool kv_fp8,
                              float k_scale, float v_scale, int num_blocks, int64_t q_stride,
                              const float* cos_sin, int cs_rows, hipStream_t s) {
  if (n_work == 0) return;
  const float sl2 = scale * k_scale * 1.4426950408889634f;
#define KGC_PF(TT, DD, K8)                                                                 \
  prefill_dispatch<TT, DD, K8>(q, out, k_cache, v_cache, block_tables, bt_stride,          \
                               query_start_loc, seq_lens, work_seq, work_mblk, n_work, nq, \
                               nkv, bs_log2, sl2, v_scale, num_blocks, q_stride, cos_sin, cs_rows, s)
#define KGC_PF_D(TT, K8) \
  if (D == 128) KGC_PF(TT, 128, K8); else KGC_PF(TT, 64, K8)
  if (dtype == DT_BF16) {
    if (kv_fp8) { KGC_PF_D(bf16, true); } else { KGC_PF_D(bf16, false); }
  } else {
    if (kv_fp8) { KGC_PF_D(f16, true); } else { KGC_PF_D(f16, false); }
  }
#undef KGC_PF_D
#undef KGC_PF
}

int prefill_block_m() { return PF_BM; }

KGC_DEBUG_TU(attention_prefill)

}  // namespace kgc
