// K13 / K14: Mixtral sparse-MoE on gfx950 (reference model deployed
// through values files, BASELINE config 4 "Mixtral 8x7B pod (MoE grouped GEMM ...)").
//
//   moe_route   : router logits [T, E] -> softmax -> top-k (renormalised) weights/ids.
//                 One wave per token, experts on lanes (E <= 64).
//   moe_align   : bucket the T*k (token, slot) pairs by expert, each bucket padded to
//                 BM rows; emits sorted pair ids, the expert of every BM-row block
//                 and the block count.  One workgroup, LDS counters -- all on device,
//                 so the whole MoE block is hipGraph-capturable (no host sync).
//   moe_gemm    : grouped GEMM over those row blocks.  Block (mb, nb) multiplies
//                 BM rows of one expert by a MG_BN-column slice of that expert's
//                 weight [N, K] on MFMA 16x16x32; A rows are gathered from the token
//                 matrix (first GEMM) or read contiguously (second GEMM); the second
//                 GEMM scatters rows back to pair order.  M-blocks run fastest in the
//                 grid so the blocks sharing a weight slice run together (L2/MALL reuse).
//   moe_combine : out[t] = sum_j w[t, j] * y[t*k + j]   (fp32 accumulation).
#include "common.h"
#include "launch.h"

namespace kgc {

constexpr int MG_BN = 128, MG_BK = 64, MG_THREADS = 256;
// Row-block height: 64 or 128, chosen per call so that a decode step's typical bucket
// (T*k/E rows) fits ONE block -- every extra block of an expert re-streams its weights.

// ---------------------------------------------------------------------------- route
template <typename T>
__global__ __launch_bounds__(256) void moe_route_kernel(const T* __restrict__ logits,
                                                        int64_t stride, int ntok, int E, int k,
                                                        int renorm, float* __restrict__ topk_w,
                                                        int* __restrict__ topk_ids) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= ntok) return;
  float v = lane < E ? to_f<T>(logits[(int64_t)t * stride + lane]) : -INFINITY;
  const float m = wave_max(v);
  float p = lane < E ? __expf(v - m) : 0.f;
  const float s = wave_sum(p);
  p = lane < E ? p / s : -1.f;
  float wsel = 0.f, wsum = 0.f;
  int isel = 0;
  for (int j = 0; j < k; ++j) {
    const float best = wave_max(p);
    // lowest expert index among the maxima (torch.topk order for ties is unspecified;
    // lowest-index is deterministic)
    const uint64_t hit = __ballot(p == best);
    const int e = __ffsll((unsigned long long)hit) - 1;
    if (lane == j) {
      wsel = best;
      isel = e;
    }
    wsum += best;
    if (lane == e) p = -1.f;
  }
  if (lane < k) {
    topk_w[(int64_t)t * k + lane] = renorm ? wsel / wsum : wsel;
    topk_ids[(int64_t)t * k + lane] = isel;
  }
}

// ---------------------------------------------------------------------------- gate + route
// The router GEMM (x [T, H] . Wg [E, H]^T, E <= 16) fused with moe_route: one workgroup
// per token, each lane a 16-byte column chunk of H per pass (every expert's dot product in
// registers, the 64 KB gate weight an L2 hit), a butterfly sum, then the logits -- rounded
// to T, as the GEMM's output would be -- go through the same softmax / top-k as
// moe_route_kernel.  At decode sizes this replaces a hipBLASLt launch that ran a 256 x 8
// output on a handful of workgroups (13.8 us at T = 256 in the Mixtral anatomy).
template <typename T, int E>
__global__ __launch_bounds__(256) void moe_gate_route_kernel(const T* __restrict__ x,
                                                             int64_t ldx,
                                                             const T* __restrict__ wg, int H,
                                                             int Er, int ntok, int k,
                                                             int renorm,
                                                             float* __restrict__ topk_w,
                                                             int* __restrict__ topk_ids) {
  // one workgroup per token: the 4 waves split the H dot product (interleaved 512-element
  // strips, so each wave keeps both of its strips' loads in flight at H = 4096) and meet in
  // LDS; wave 0 does the softmax / top-k.  One wave per token left 3/4 of the CUs idle at
  // decode batch 256 and ran 8 dependent strips per wave.
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = blockIdx.x;
  if (t >= ntok) return;                                  // workgroup-uniform
  __shared__ float red[4][E];
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  const T* xr = x + (int64_t)t * ldx;
  for (int c = (wave * 64 + lane) * 8; c < H; c += 2048) {
    Pack8<T> xv;
    xv.u = *reinterpret_cast<const u32x4*>(xr + c);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (e >= Er) break;                               // wave-uniform: only the real rows
      Pack8<T> wv;
      wv.u = *reinterpret_cast<const u32x4*>(wg + (int64_t)e * H + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[e] += to_f(xv.h[j]) * to_f(wv.h[j]);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = wave_sum(acc[e]);
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < E; ++e) red[wave][e] = acc[e];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
  float v = -INFINITY;
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (lane == e && e < Er) v = to_f(from_f<T>(acc[e]));   // rounded as the GEMM stores it
  const float m = wave_max(v);
  float p = lane < Er ? __expf(v - m) : 0.f;
  const float s = wave_sum(p);
  p = lane < Er ? p / s : -1.f;
  float wsel = 0.f, wsum = 0.f;
  int isel = 0;
  for (int j = 0; j < k; ++j) {
    const float best = wave_max(p);
    const uint64_t hit = __ballot(p == best);
    const int e = __ffsll((unsigned long long)hit) - 1;
    if (lane == j) {
      wsel = best;
      isel = e;
    }
    wsum += best;
    if (lane == e) p = -1.f;
  }
  if (lane < k) {
    topk_w[(int64_t)t * k + lane] = renorm ? wsel / wsum : wsel;
    topk_ids[(int64_t)t * k + lane] = isel;
  }
}

// ---------------------------------------------------------------------------- align
// sorted_ids: [max_rows] pair ids (padding = npairs); block_expert: [max_rows / bm]
// local expert per row block; meta[0] = number of row blocks in use.
__global__ __launch_bounds__(1024) void moe_align_kernel(const int* __restrict__ topk_ids,
                                                         int npairs, int e0, int E_local, int bm,
                                                         int max_rows, int* __restrict__ sorted_ids,
                                                         int* __restrict__ block_expert,
                                                         int* __restrict__ meta) {
  __shared__ int cnt[256], off[257], cur[256];
  const int tid = threadIdx.x;
  for (int e = tid; e < E_local; e += blockDim.x) {
    cnt[e] = 0;
    cur[e] = 0;
  }
  for (int r = tid; r < max_rows; r += blockDim.x) sorted_ids[r] = npairs;
  __syncthreads();
  for (int p = tid; p < npairs; p += blockDim.x) {
    const int e = topk_ids[p] - e0;
    if (e >= 0 && e < E_local) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int e = 0; e < E_local; ++e) {
      off[e] = acc;
      acc += (cnt[e] + bm - 1) / bm * bm;
    }
    off[E_local] = acc;
    meta[0] = acc / bm;
  }
  __syncthreads();
  const int nblk = off[E_local] / bm;
  for (int b = tid; b < max_rows / bm; b += blockDim.x) {
    int e = -1;
    if (b < nblk) {
      const int row = b * bm;
      for (int q = 0; q < E_local; ++q)
        if (row >= off[q] && row < off[q + 1]) e = q;
    }
    block_expert[b] = e;
  }
  __syncthreads();
  for (int p = tid; p < npairs; p += blockDim.x) {
    const int e = topk_ids[p] - e0;
    if (e >= 0 && e < E_local) sorted_ids[off[e] + atomicAdd(&cur[e], 1)] = p;
  }
}

// ---------------------------------------------------------------------------- grouped GEMM
__device__ __forceinline__ int mg_swz(int row, int chunk) {   // 16-B chunk index in LDS row
  return row * (MG_BK / 8) + (chunk ^ (row & 7));
}

// GATHER: A row r = x[sorted_ids[r] / topk]  (else A row r = A[r]);
// SCATTER: C row sorted_ids[r] (skip padding)  (else C row r).
// PARTIAL (split-K, with SCATTER): grid z = S slices of K; slice z writes its fp32 sum
// to Cf[z][row][:] and moe_combine adds the S slices.  At decode sizes the down
// projection has only (experts x N/128) = 256 workgroups, each walking K = 14336 alone;
// splitting K 4 ways fills the chip.
// DENSE (dense split-K decode GEMM, one weight matrix, no row maps): a 1-D grid of
// MB * NB * S workgroups, slice z = linear id % S.  Workgroups are dispatched round-robin
// over the 8 XCDs, so with S = 8 every XCD owns one K-slice: its [M, K/8] activation slice
// stays in that XCD's L2 for all N-tiles while the weights stream from HBM once, and the
// M-blocks sharing an N-tile run back to back on the same XCD.
template <typename T, int BM, bool GATHER, bool SCATTER, bool PARTIAL, bool DENSE = false>
__global__ __launch_bounds__(MG_THREADS, 2) void moe_gemm_kernel(
    void* __restrict__ Cv, const T* __restrict__ A, const T* __restrict__ W,
    const int* __restrict__ sorted_ids, const int* __restrict__ block_expert,
    const int* __restrict__ meta, int npairs, int topk, int N, int K, int64_t lda,
    int64_t ldc, int64_t slice_stride, int dense_m) {
  int mb, nb, z, S, e;
  if constexpr (DENSE) {
    // npairs = number of M-blocks, topk = number of K-slices (reused scalar args);
    // rows >= dense_m of the last M-block load row dense_m - 1 and store nothing
    S = topk;
    const int L = blockIdx.x;
    z = L % S;
    const int j = L / S;
    mb = j % npairs;
    nb = j / npairs;
    e = 0;
  } else {
    mb = blockIdx.x;
    nb = blockIdx.y;
    z = blockIdx.z;
    S = gridDim.z;
    if (mb >= meta[0]) return;
    e = block_expert[mb];
    if (e < 0) return;
  }
  constexpr int AC = BM / 32;     // A chunks per thread; also 16-row M tiles per wave
  __shared__ u32x4 lds[2 * (BM + MG_BN) * (MG_BK / 8)];
  u32x4* As = lds;                                   // [2][BM * 8]
  u32x4* Bs = lds + 2 * BM * (MG_BK / 8);            // [2][MG_BN * 8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q4 = lane >> 4;

  // global -> register staging assignment: A AC chunks/thread, B 4 chunks/thread
  const int chunk = tid & 7;
  const T* a_ptr[AC];
#pragma unroll
  for (int i = 0; i < AC; ++i) {
    const int row = (tid >> 3) + 32 * i;
    const int r = mb * BM + row;
    int64_t arow;
    if constexpr (GATHER) {
      const int p = sorted_ids[r];
      arow = p < npairs ? p / topk : 0;
    } else if constexpr (DENSE) {
      arow = r < dense_m ? r : dense_m - 1;
    } else {
      arow = r;
    }
    a_ptr[i] = A + arow * lda + chunk * 8;
  }
  const T* w_ptr = W + ((int64_t)e * N + (int64_t)nb * MG_BN + (tid >> 3)) * K + chunk * 8;
  u32x4 ra[AC], rb[4];
  auto gload = [&](int kb) {
    const int ko = kb * MG_BK;
#pragma unroll
    for (int i = 0; i < AC; ++i) ra[i] = *reinterpret_cast<const u32x4*>(a_ptr[i] + ko);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      rb[i] = *reinterpret_cast<const u32x4*>(w_ptr + (int64_t)32 * i * K + ko);
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AC; ++i) As[buf * BM * 8 + mg_swz((tid >> 3) + 32 * i, chunk)] = ra[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) Bs[buf * MG_BN * 8 + mg_swz((tid >> 3) + 32 * i, chunk)] = rb[i];
  };

  const int wm = wave >> 1, wn = wave & 1;   // wave tile: BM/2 rows x 64 cols
  f32x4 acc[AC][4];
#pragma unroll
  for (int i = 0; i < AC; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk_all = K / MG_BK;
  const int kb0 = (int)((int64_t)nk_all * z / S);
  const int nk = (int)((int64_t)nk_all * (z + 1) / S);
  gload(kb0);
  lstore(0);
  __syncthreads();
  for (int kb = kb0; kb < nk; ++kb) {
    const int buf = (kb - kb0) & 1;
    if (kb + 1 < nk) gload(kb + 1);
#pragma unroll
    for (int ks = 0; ks < MG_BK / 32; ++ks) {
      Pack8<T> af[AC], bf[4];
#pragma unroll
      for (int mt = 0; mt < AC; ++mt)
        af[mt].u = As[buf * BM * 8 + mg_swz(wm * (BM / 2) + mt * 16 + r16, ks * 4 + q4)];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        bf[nt].u = Bs[buf * MG_BN * 8 + mg_swz(wn * 64 + nt * 16 + r16, ks * 4 + q4)];
#pragma unroll
      for (int mt = 0; mt < AC; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16x16x32(af[mt].v, bf[nt].v, acc[mt][nt]);
    }
    if (kb + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds C[4*q4 + i][r16] of each 16x16 tile
#pragma unroll
  for (int mt = 0; mt < AC; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = mb * BM + wm * (BM / 2) + mt * 16 + 4 * q4 + i;
      int64_t crow = r;
      if constexpr (DENSE) {
        if (r >= dense_m) continue;
      }
      if constexpr (SCATTER) {
        const int p = sorted_ids[r];
        if (p >= npairs) continue;
        crow = p;
      }
      const int64_t off = crow * ldc + (int64_t)nb * MG_BN + wn * 64 + r16;
      if constexpr (PARTIAL) {
        float* cp = reinterpret_cast<float*>(Cv) + z * slice_stride + off;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) cp[nt * 16] = acc[mt][nt][i];
      } else {
        T* cp = reinterpret_cast<T*>(Cv) + off;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) cp[nt * 16] = from_f<T>(acc[mt][nt][i]);
      }
    }
  }
}

// out[m, n] = sum_z Cs[z, m, n]  (+ residual)  -- split-K reduction of the dense GEMM.
template <typename T, int SK>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(T* __restrict__ out,
                                                            const float* __restrict__ Cs, int S_,
                                                            int64_t n8, int64_t slice_stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const int S = SK > 0 ? SK : S_;     // SK > 0: all slice loads issued up front
  f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
#pragma unroll
  for (int z = 0; z < S; ++z) {
    const float* src = Cs + z * slice_stride + i * 8;
    a += *reinterpret_cast<const f32x4*>(src);
    b += *reinterpret_cast<const f32x4*>(src + 4);
  }
  Pack8<T> o;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o.h[q] = from_f<T>(a[q]);
    o.h[4 + q] = from_f<T>(b[q]);
  }
  *reinterpret_cast<u32x4*>(out + i * 8) = o.u;
}

// K7 fused into the gate_up split-K reduction: out[m, i] = silu(g) * u with
// g = sum_z Cs[z, m, i], u = sum_z Cs[z, m, I + i].  The [M, 2I] bf16 gate_up output
// is never written, and the separate silu_mul launch disappears from the decode step.
// grid (ceil(I/8/256), M): one 8-wide column group per thread, no index division.
// IL: the slices come from K9m's PACKED SiLU weights (gemm_decode.hip weight_row, EPI_SILU
// layout): in each 128-column tile, 16-column groups alternate gate / up, so output column
// c's gate is partial column (c / 64) * 128 + ((c % 64) / 16) * 32 + c % 16 and its up the
// 16 after it (the split-K form of the packed gate_up, used where S = 1 leaves most CUs
// idle: Llama-3-70B at TP = 8 has 56 column tiles at M = 256).
template <typename T, int SK, bool IL = false>
__global__ __launch_bounds__(256) void splitk_reduce_silu_kernel(T* __restrict__ out,
                                                                 const float* __restrict__ Cs,
                                                                 int S_, int I,
                                                                 int64_t slice_stride,
                                                                 const float* __restrict__ rsc) {
  const int S = SK > 0 ? SK : S_;
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= I) return;
  const int64_t m = blockIdx.y;
  // the norm-free layer: the row's rsqrt(mean(x^2) + eps) over a gamma-folded weight
  const float sc = rsc ? rsc[m] : 1.f;
  const int64_t gcol = IL ? (int64_t)(c >> 6) * 128 + ((c & 63) >> 4) * 32 + (c & 15) : c;
  const int64_t ucol = IL ? gcol + 16 : (int64_t)c + I;
  const float* row = Cs + m * 2 * I;
  f32x4 g0 = f32x4{0.f, 0.f, 0.f, 0.f}, g1 = g0, u0 = g0, u1 = g0;
#pragma unroll
  for (int z = 0; z < S; ++z) {
    const float* src = row + z * slice_stride;
    g0 += *reinterpret_cast<const f32x4*>(src + gcol);
    g1 += *reinterpret_cast<const f32x4*>(src + gcol + 4);
    u0 += *reinterpret_cast<const f32x4*>(src + ucol);
    u1 += *reinterpret_cast<const f32x4*>(src + ucol + 4);
  }
  g0 *= sc;
  g1 *= sc;
  u0 *= sc;
  u1 *= sc;
  Pack8<T> o;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o.h[q] = from_f<T>(g0[q] / (1.f + __expf(-g0[q])) * u0[q]);
    o.h[4 + q] = from_f<T>(g1[q] / (1.f + __expf(-g1[q])) * u1[q]);
  }
  *reinterpret_cast<u32x4*>(out + m * I + c) = o.u;
}

// ---------------------------------------------------------------------------- combine
// y: [T*k, H] in T, or (S > 0) S fp32 split-K slices [S][T*k, H] summed here.
template <typename T>
__global__ __launch_bounds__(256) void moe_combine_kernel(T* __restrict__ out,
                                                          const void* __restrict__ y,
                                                          const float* __restrict__ topk_w,
                                                          const int* __restrict__ row_map,
                                                          int64_t nrows, int k, int H, int S,
                                                          int64_t slice_stride) {
  const int t = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= H) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < k; ++j) {
    const float w = topk_w[(int64_t)t * k + j];
    // row_map: pair -> row of y (expert-sorted rows, no scatter back to pair order);
    // -1 = the pair has no row (expert not local) and contributes nothing; rows past y's
    // end are skipped the same way
    const int64_t pr = row_map ? (int64_t)row_map[(int64_t)t * k + j] : (int64_t)t * k + j;
    if (pr < 0 || pr >= nrows) continue;
    const int64_t row = pr * H + c;
    if (S == 0) {
      Pack8<T> v;
      v.u = *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(y) + row);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += w * to_f<T>(v.h[q]);
    } else {
      for (int z = 0; z < S; ++z) {
        const float* src = reinterpret_cast<const float*>(y) + z * slice_stride + row;
        const f32x4 a = *reinterpret_cast<const f32x4*>(src);
        const f32x4 b = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[q] += w * a[q];
          acc[4 + q] += w * b[q];
        }
      }
    }
  }
  Pack8<T> o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o.h[q] = from_f<T>(acc[q]);
  *reinterpret_cast<u32x4*>(out + (int64_t)t * H + c) = o.u;
}

// ---------------------------------------------------------------------------- launchers
int moe_block_n() { return MG_BN; }
int moe_block_k() { return MG_BK; }

void launch_moe_route(int dtype, const void* logits, int64_t stride, int ntok, int E, int k,
                      bool renorm, float* topk_w, int* topk_ids, hipStream_t s) {
  const dim3 grid((ntok + 3) / 4);
  if (dtype == DT_BF16)
    moe_route_kernel<bf16><<<grid, 256, 0, s>>>((const bf16*)logits, stride, ntok, E, k, renorm,
                                                topk_w, topk_ids);
  else if (dtype == DT_F16)
    moe_route_kernel<f16><<<grid, 256, 0, s>>>((const f16*)logits, stride, ntok, E, k, renorm,
                                               topk_w, topk_ids);
  else
    moe_route_kernel<float><<<grid, 256, 0, s>>>((const float*)logits, stride, ntok, E, k, renorm,
                                                 topk_w, topk_ids);
}

void launch_moe_gate_route(int dtype, const void* x, int64_t ldx, const void* wg, int H, int E,
                           int ntok, int k, bool renorm, float* topk_w, int* topk_ids,
                           hipStream_t s) {
  const dim3 grid(ntok);
#define GR(TT, EE)                                                                          \
  moe_gate_route_kernel<TT, EE><<<grid, 256, 0, s>>>((const TT*)x, ldx, (const TT*)wg, H, E, \
                                                      ntok, k, renorm, topk_w, topk_ids)
#define GR_E(TT)                                                                            \
  if (E <= 4) GR(TT, 4); else if (E <= 8) GR(TT, 8); else GR(TT, 16);
  // E below the template width: rows past E are never read (the loop stops at E) and
  // lanes >= E are masked out of the softmax
  if (dtype == DT_BF16) { GR_E(bf16) } else { GR_E(f16) }
#undef GR_E
#undef GR
}

void launch_moe_align(const int* topk_ids, int npairs, int e0, int E_local, int bm, int max_rows,
                      int* sorted_ids, int* block_expert, int* meta, hipStream_t s) {
  moe_align_kernel<<<1, 1024, 0, s>>>(topk_ids, npairs, e0, E_local, bm, max_rows, sorted_ids,
                                      block_expert, meta);
}

template <typename T, int BM>
static void moe_gemm_bm(void* C, const void* A, const void* W, const int* sorted_ids,
                        const int* block_expert, const int* meta, int npairs, int topk, int N,
                        int K, int64_t lda, int64_t ldc, int max_mblocks, bool gather,
                        bool scatter, int splitk, int64_t slice_stride, hipStream_t s) {
  const dim3 grid(max_mblocks, N / MG_BN, splitk);
#define MG_LAUNCH(G, S, P)                                                                   \
  moe_gemm_kernel<T, BM, G, S, P><<<grid, MG_THREADS, 0, s>>>(C, (const T*)A, (const T*)W,   \
                                                              sorted_ids, block_expert, meta, \
                                                              npairs, topk, N, K, lda, ldc,   \
                                                              slice_stride, 0)
  if (splitk > 1) MG_LAUNCH(false, true, true);          // host-checked: scatter, !gather
  else if (gather && !scatter) MG_LAUNCH(true, false, false);
  else if (!gather && scatter) MG_LAUNCH(false, true, false);
  else if (gather && scatter) MG_LAUNCH(true, true, false);
  else MG_LAUNCH(false, false, false);
#undef MG_LAUNCH
}

template <typename T>
static void moe_gemm_t(int bm, void* C, const void* A, const void* W, const int* sorted_ids,
                       const int* block_expert, const int* meta, int npairs, int topk, int N,
                       int K, int64_t lda, int64_t ldc, int max_mblocks, bool gather,
                       bool scatter, int splitk, int64_t slice_stride, hipStream_t s) {
  if (bm == 128)
    moe_gemm_bm<T, 128>(C, A, W, sorted_ids, block_expert, meta, npairs, topk, N, K, lda, ldc,
                        max_mblocks, gather, scatter, splitk, slice_stride, s);
  else
    moe_gemm_bm<T, 64>(C, A, W, sorted_ids, block_expert, meta, npairs, topk, N, K, lda, ldc,
                       max_mblocks, gather, scatter, splitk, slice_stride, s);
}

void launch_moe_gemm(int dtype, int bm, void* C, const void* A, const void* W,
                     const int* sorted_ids, const int* block_expert, const int* meta, int npairs,
                     int topk, int N, int K, int64_t lda, int64_t ldc, int max_mblocks,
                     bool gather, bool scatter, int splitk, int64_t slice_stride, hipStream_t s) {
  if (dtype == DT_BF16)
    moe_gemm_t<bf16>(bm, C, A, W, sorted_ids, block_expert, meta, npairs, topk, N, K, lda, ldc,
                     max_mblocks, gather, scatter, splitk, slice_stride, s);
  else
    moe_gemm_t<f16>(bm, C, A, W, sorted_ids, block_expert, meta, npairs, topk, N, K, lda, ldc,
                    max_mblocks, gather, scatter, splitk, slice_stride, s);
}

void launch_dense_gemm_splitk(int dtype, int bm, float* Cs, const void* A, const void* W, int M,
                              int N, int K, int64_t lda, int splitk, hipStream_t s) {
  const int MB = (M + bm - 1) / bm;
  const dim3 grid(MB * (N / MG_BN) * splitk);
  const int64_t ss = (int64_t)M * N;
#define DG_LAUNCH(T, BMV)                                                                     \
  moe_gemm_kernel<T, BMV, false, false, true, true><<<grid, MG_THREADS, 0, s>>>(             \
      Cs, (const T*)A, (const T*)W, nullptr, nullptr, nullptr, MB, splitk, N, K, lda, N, ss, M)
  if (dtype == DT_BF16) {
    if (bm == 128) DG_LAUNCH(bf16, 128);
    else DG_LAUNCH(bf16, 64);
  } else {
    if (bm == 128) DG_LAUNCH(f16, 128);
    else DG_LAUNCH(f16, 64);
  }
#undef DG_LAUNCH
}

template <typename T>
static void splitk_reduce_t(T* out, const float* Cs, int S, int64_t n8, int64_t ss,
                            hipStream_t s) {
  const dim3 grid((unsigned)((n8 + 255) / 256));
#define SKR(K) splitk_reduce_kernel<T, K><<<grid, 256, 0, s>>>(out, Cs, S, n8, ss)
  switch (S) {
    case 2: SKR(2); break;
    case 3: SKR(3); break;
    case 4: SKR(4); break;
    case 5: SKR(5); break;
    case 6: SKR(6); break;
    case 8: SKR(8); break;
    default: SKR(0); break;
  }
#undef SKR
}

void launch_splitk_reduce(int dtype, void* out, const float* Cs, int S, int64_t numel,
                          int64_t slice_stride, hipStream_t s) {
  const int64_t n8 = numel / 8;
  if (dtype == DT_BF16) splitk_reduce_t<bf16>((bf16*)out, Cs, S, n8, slice_stride, s);
  else splitk_reduce_t<f16>((f16*)out, Cs, S, n8, slice_stride, s);
}

template <typename T, bool IL>
static void splitk_reduce_silu_t(T* out, const float* Cs, int S, int n, int I, int64_t ss,
                                 const float* rsc, hipStream_t s) {
  const dim3 grid((unsigned)((I / 8 + 255) / 256), (unsigned)n);
#define SKS(K) splitk_reduce_silu_kernel<T, K, IL><<<grid, 256, 0, s>>>(out, Cs, S, I, ss, rsc)
  switch (S) {
    case 2: SKS(2); break;
    case 3: SKS(3); break;
    case 4: SKS(4); break;
    case 5: SKS(5); break;
    case 6: SKS(6); break;
    case 8: SKS(8); break;
    default: SKS(0); break;
  }
#undef SKS
}

void launch_splitk_reduce_silu(int dtype, void* out, const float* Cs, int S, int M, int I,
                               int64_t slice_stride, bool interleaved, const float* rsc,
                               hipStream_t s) {
  for (int m0 = 0; m0 < M; m0 += 65535) {   // gridDim.y <= 65535
    const int n = std::min(M - m0, 65535);
    const float* c = Cs + (int64_t)m0 * 2 * I;
    const float* r = rsc ? rsc + m0 : nullptr;
    if (dtype == DT_BF16) {
      if (interleaved)
        splitk_reduce_silu_t<bf16, true>((bf16*)out + (int64_t)m0 * I, c, S, n, I, slice_stride, r, s);
      else
        splitk_reduce_silu_t<bf16, false>((bf16*)out + (int64_t)m0 * I, c, S, n, I, slice_stride, r, s);
    } else {
      if (interleaved)
        splitk_reduce_silu_t<f16, true>((f16*)out + (int64_t)m0 * I, c, S, n, I, slice_stride, r, s);
      else
        splitk_reduce_silu_t<f16, false>((f16*)out + (int64_t)m0 * I, c, S, n, I, slice_stride, r, s);
    }
  }
}

void launch_moe_combine(int dtype, void* out, const void* y, const float* topk_w,
                        const int* row_map, int64_t nrows, int ntok, int k, int H,
                        int splitk, int64_t slice_stride, hipStream_t s) {
  const dim3 grid((H / 8 + 255) / 256, ntok);
  const int S = splitk > 1 ? splitk : 0;
  if (dtype == DT_BF16)
    moe_combine_kernel<bf16><<<grid, 256, 0, s>>>((bf16*)out, y, topk_w, row_map, nrows, k, H,
                                                   S, slice_stride);
  else
    moe_combine_kernel<f16><<<grid, 256, 0, s>>>((f16*)out, y, topk_w, row_map, nrows, k, H,
                                                  S, slice_stride);
}

}  // namespace kgc
