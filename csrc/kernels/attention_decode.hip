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
#include "common.h"
#include "launch.h"
#include <type_traits>

namespace kgc {

constexpr int DEC_PART = 64;     // tokens per partition (one wave-iteration)
constexpr int DEC_CHUNKS = DEC_PART / 32;
constexpr int DEC_MAX_Z = 1024;  // z-slices the reduce kernel merges (host-checked)

__device__ __forceinline__ u32x4 ld16(const void* p) {
  return *reinterpret_cast<const u32x4*>(p);
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
template <typename T, int D, bool PREF, bool KV8, int OCC = 3, int NCH = DEC_CHUNKS>
__global__ __launch_bounds__(256, OCC) void paged_decode_kernel(
    T* __restrict__ out, const T* __restrict__ q, const void* __restrict__ kc_,
    const void* __restrict__ vc_, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ ctx_lens, float* __restrict__ max_logits,
    float* __restrict__ exp_sums, float* __restrict__ tmp_out, int nq, int nkv, int bs_log2,
    int Zmax, float scale_log2, float v_scale, int num_blocks) {
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

  V8 qf[KS];
  {
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
  for (int ci = c0; ci < c1; ci += NCH) {
    const int base = ci << 5;
    const C* kaddr[NCH][2];
    const C* vaddr[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ta = min(base + c * 32 + keyA, end - 1);
      const int tb = min(base + c * 32 + keyA + 4, end - 1);
      kaddr[c][0] = kbase + kgc_bt(bt, ta >> bs_log2, bt_stride, num_blocks) * blk_stride + (int64_t)(ta & bsm) * D + 8 * qd;
      kaddr[c][1] = kbase + kgc_bt(bt, tb >> bs_log2, bt_stride, num_blocks) * blk_stride + (int64_t)(tb & bsm) * D + 8 * qd;
      // V^T 8-key group of keys t0..t0+7: [(t0 & bsm) / 8][d][8]; 16 lanes = 256 B
      const int t0 = min(base + c * 32 + 8 * qd, end - 1) & ~7;
      vaddr[c] = vbase + kgc_bt(bt, t0 >> bs_log2, bt_stride, num_blocks) * blk_stride + ((t0 & bsm) >> 3) * (D * 8) + r16 * 8;
    }
    Pack8<T> kf[NCH][2][KS];
    Pack8<T> vf[PREF ? NCH : 1][DT];
    if constexpr (PREF) {
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          kf[c][0][s2].u = ldf(kaddr[c][0] + 32 * s2);
          kf[c][1][s2].u = ldf(kaddr[c][1] + 32 * s2);
        }
    }
    if constexpr (PREF) {
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int t = 0; t < DT; ++t) vf[PREF ? c : 0][t].u = ldf(vaddr[c] + 16 * t * 8);
    }
    f32x4 sa[NCH], sb[NCH];
    // ---- S^T = K . Q^T
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      f32x4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        if constexpr (!PREF) {
          kf[c][0][s2].u = ldf(kaddr[c][0] + 32 * s2);
          kf[c][1][s2].u = ldf(kaddr[c][1] + 32 * s2);
        }
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
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float alpha = exp2f(m_run - m);     // 0 on the first partition
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
        const float pa = exp2f(sa[c][i] - m), pb = exp2f(sb[c][i] - m);
        l_run += pa + pb;
        pf.h[i] = from_f<T>(pa);
        pf.h[4 + i] = from_f<T>(pb);
      }
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        Pack8<T> v;
        if constexpr (PREF) v = vf[PREF ? c : 0][t];
        else v.u = ldf(vaddr[c] + 16 * t * 8);
        o[t] = mfma16x16x32(v.v, pf.v, o[t]);
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

// Merge the Z z-slice partials: one 64-thread wave per (seq, q-head).
template <typename T, int D>
__global__ __launch_bounds__(64) void paged_decode_reduce_kernel(
    T* __restrict__ out, const float* __restrict__ max_logits,
    const float* __restrict__ exp_sums, const float* __restrict__ tmp_out,
    const int* __restrict__ ctx_lens, int nq, int Z, int Zmax) {
  // The slice statistics are read in parallel (lane z), the weights staged in LDS,
  // and the partial rows loaded 8 slices at a time: the previous per-slice loop was a
  // chain of dependent L2 round trips (~7 us per call at B = 1; decode + reduce for
  // B = 1, ctx 565, Z = 16 went 13.0 -> 9.3 us).
  __shared__ float wz[DEC_MAX_Z];
  const int b = blockIdx.x, hq = blockIdx.y, tid = threadIdx.x;
  T* orow = out + ((int64_t)b * nq + hq) * D;
  constexpr int EPT = D / 64;
  const int64_t base = ((int64_t)b * nq + hq) * Zmax;
  float m = -INFINITY;
  for (int z = tid; z < Z; z += 64) m = fmaxf(m, max_logits[base + z]);
  m = wave_max(m);
  float acc[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) acc[e] = 0.f;
  float tot = 0.f;
  if (ctx_lens[b] > 0 && m != -INFINITY) {
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

template <typename T, int D, bool KV8>
static void decode_dispatch(void* out, const void* q, const void* kc, const void* vc,
                            const int* bt, int bt_stride, const int* ctx, float* ml, float* es,
                            float* tmp, int B, int nq, int nkv, int bs_log2, int Zmax, int Z,
                            float scale_log2, float v_scale, int num_blocks, hipStream_t s) {
  auto kern = paged_decode_kernel<T, D, true, KV8, 4, 1>;
  kern<<<dim3(B, nkv, Z), 256, 0, s>>>(
      (T*)out, (const T*)q, kc, vc, bt, bt_stride, ctx, ml, es, tmp, nq,
      nkv, bs_log2, Zmax, scale_log2, v_scale, num_blocks);
  if (Z > 1)
    paged_decode_reduce_kernel<T, D><<<dim3(B, nq), 64, 0, s>>>((T*)out, ml, es, tmp, ctx, nq,
                                                                Z, Zmax);
}

void launch_paged_decode(int dtype, void* out, const void* q, const void* k_cache,
                         const void* v_cache, const int* block_tables, int bt_stride,
                         const int* ctx_lens, float* max_logits, float* exp_sums,
                         float* tmp_out, int B, int nq, int nkv, int D, int bs_log2,
                         int Zmax, int Z, float scale, bool kv_fp8, float k_scale,
                         float v_scale, int num_blocks, hipStream_t s) {
  if (B == 0) return;
  const float sl2 = scale * k_scale * 1.4426950408889634f;
#define KGC_DEC(TT, DD, K8)                                                               \
  decode_dispatch<TT, DD, K8>(out, q, k_cache, v_cache, block_tables, bt_stride, ctx_lens, \
                              max_logits, exp_sums, tmp_out, B, nq, nkv, bs_log2, Zmax, Z, \
                              sl2, v_scale, num_blocks, s)
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

int paged_decode_partition_size() { return DEC_PART; }

KGC_DEBUG_TU(attention_decode)

}  // namespace kgc
