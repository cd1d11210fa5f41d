// K9w (round 4): the decode GEMM at M <= 256 with the weights PRIVATE per wave in a VGPR
// ring and only the activations shared through an LDS-DMA ring.  Research build
// (tools/research/build.py -> _kgc_research.so) until it beats K9m in the engine's tuner.
//
// Why: the K9m measurements fit a per-CU request-slot model (profiles/README.md, "what
// bounds the decode GEMMs at M = 256"): weight requests (HBM, ~2 us) and activation
// requests (L2, ~0.5 us) share one pool of outstanding requests per CU, and K9m's 256 x 128
// tile moves 2 activation bytes per weight byte, which caps the weight stream at ~4 TB/s.
// A 256 x 256 tile halves that ratio.  Its fp32 accumulator is 256 KB -- half of a CU's
// 512 KB register file, 128 registers per lane over 8 waves -- so the tile fits when the
// weights skip the LDS:
//   * workgroup = 8 waves, one per CU; wave w owns columns [32 w, 32 w + 32) of the tile
//     (two 16-column MFMA tiles) for ALL 256 rows (16 row tiles): 32 f32x4 accumulators;
//   * per 64-deep K-step each wave loads its own 32 x 64 weight block (4 KB, 4 x 16 B per
//     lane) from a packed layout where every load instruction reads 1 KB contiguous, into a
//     D + 1 deep register ring, and issues 1/8 of the 32 KB activation step by LDS-DMA into a
//     D + 1 slot ring (the K9m swizzle, so the A-fragment reads are conflict-free);
//   * every wave reads the whole activation slot (16 ds_read_b128 per 32-deep half-step),
//     so the LDS serves 256 KB per K-step per CU -- about the MFMA time of the step.
// Issue / wait discipline as K9v (gemm_vreg.hip): the ring's register loads are inline-asm
// loads the compiler does not track, every K-step issues one group of OPS memory ops (past
// the slice a filler group), and the wait before each step is "all but the D - 1 youngest
// groups", so neither the compiler nor a tail branch drains the pipeline.
#include "common.h"
#include "launch.h"
#include "research.h"
#include <cstdlib>

namespace kgc {

namespace {

constexpr int WV_BK = 64, WV_ROWB = 128, WV_BN = 256;
enum { EPI_PARTIAL = 0, EPI_OUT = 1, EPI_SILU = 2 };
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

template <int AUX>
__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_wave_base, 16, 0, AUX);
}
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }
__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }
__device__ __forceinline__ void store_partial(float* p, float v, int wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
static int partial_wt() {
  static const int v = [] {
    const char* e = getenv("KGC_PARTIAL_WT");
    return e ? atoi(e) : 1;
  }();
  return v;
}
// non-temporal 16-B weight load the compiler does not track (see the header)
__device__ __forceinline__ u32x4 ld_async16_nt(const void* p) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void wait_vm_b() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | 0x70 | 0xF00 | ((N >> 4) << 14));
}

// weight row of (column tile nb, wave w, n-tile n, column fr): EPI_SILU pairs gate row g
// (n = 0) with up row I + g (n = 1), g = nb * 128 + w * 16 + fr
template <int EPI>
__device__ __forceinline__ int64_t wv_row(int nb, int w, int n, int fr, int N) {
  if constexpr (EPI == EPI_SILU) return (int64_t)(n ? (N >> 1) : 0) + nb * 128 + w * 16 + fr;
  else return (int64_t)nb * WV_BN + w * 32 + n * 16 + fr;
}

template <typename T, int EPI, int D>
__global__ __launch_bounds__(512, 1) void dgemm_wv_kernel(
    void* __restrict__ Cv, const T* __restrict__ X, const T* __restrict__ Wp, int M, int N,
    int K, int64_t ldx, int S, int64_t slice_stride, int wt) {
  constexpr int NS = D + 1, MT = 16, NT = 2;
  constexpr int SLOT = 256 * WV_ROWB;             // 32 KB: 256 activation rows x 64 K
  constexpr int LA = 4, LW = 4, OPS = LA + LW;    // memory ops per K-step per wave
  constexpr int STEP_ELEMS = 8 * LW * 64 * 8;     // packed weight elements per K-step (32 KB)
  static_assert(NS * SLOT <= 163840, "LDS ring exceeds 160 KiB");
  __shared__ __attribute__((aligned(16))) char lds[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int z = blockIdx.x % S, nb = blockIdx.x / S;
  const int nk_all = K / WV_BK;
  const int kb0 = (int)((int64_t)nk_all * z / S);
  const int nk = (int)((int64_t)nk_all * (z + 1) / S) - kb0;
  const int rot = nk >= 4 ? (int)(((int64_t)nb * 37) % nk) : 0;

  // activation DMA: wave w fills rows 32 w .. 32 w + 31, instruction t rows 32 w + 8 t ..;
  // lane l fills 16-B slot l % 8 of row 8 t + l / 8 with global chunk (l % 8) ^ (row % 8)
  const int drow = lane >> 3, dchunk = (lane & 7) ^ drow;
  const T* a_src[LA];
#pragma unroll
  for (int t = 0; t < LA; ++t) {
    int r = wave * 32 + t * 8 + drow;
    r = r < M ? r : M - 1;                        // padded rows re-read the last row
    a_src[t] = X + (int64_t)r * ldx + dchunk * 8;
  }
  // packed weights: [nb][kb][wave][j][lane] 16-B chunks, j = k-half * 2 + n-tile
  const T* w_src = Wp + ((int64_t)nb * nk_all * 8 * LW + wave * LW) * 512 + lane * 8;

  u32x4 wreg[NS][LW];
  auto issue = [&](int step, int slot) {
    const bool real = step < nk;
    int st = step + rot;
    st = st >= nk ? st - nk : st;
    const int kb = kb0 + (real ? st : 0);
    char* dst = lds + slot * SLOT + wave * LA * 1024;
#pragma unroll
    for (int t = 0; t < LA; ++t) glds16<0>(real ? a_src[t] + kb * WV_BK : X, dst + t * 1024);
    const T* ws = w_src + (int64_t)kb * STEP_ELEMS;
#pragma unroll
    for (int j = 0; j < LW; ++j) wreg[slot][j] = ld_async16_nt(real ? ws + j * 512 : Wp);
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < D; ++p) issue(p, p);
  for (int it0 = 0; it0 < nk; it0 += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int it = it0 + u;
      if (it < nk) {
        // this step's group (and every older one) landed; the D - 1 younger ones fly
        wait_vm_b<OPS * (D - 1)>();
        __builtin_amdgcn_s_barrier();
        // slot (u + D) % NS held step it - 1, which every wave finished before the barrier
        issue(it + D, (u + D) % NS);
        const char* sa = lds + u * SLOT;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + fq;
          Pack8<T> wf[NT];
#pragma unroll
          for (int n = 0; n < NT; ++n) wf[n].u = wreg[u][ks * 2 + n];
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const int r = i * 16 + fr;
            Pack8<T> af;
            af.u = *reinterpret_cast<const u32x4*>(sa + r * WV_ROWB + (swz(r, c) << 4));
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[i][n] = mfma16x16x32(af.v, wf[n].v, acc[i][n]);
          }
        }
      }
    }
  }
  // the filler groups still fly: no LDS-DMA may land after this workgroup's LDS is gone,
  // and no ring register may be reused while its (filler) load is on the way
  wait_vm_b<0>();
#pragma unroll
  for (int sl = 0; sl < NS; ++sl)
#pragma unroll
    for (int j = 0; j < LW; ++j) asm volatile("" ::"v"(wreg[sl][j]));

  // ---- epilogue: lane holds C[16 i + 4 fq + e][column of (wave, n, fr)]
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = i * 16 + fq * 4 + e;
      if (row >= M) continue;
      if constexpr (EPI == EPI_PARTIAL) {
        float* cp = reinterpret_cast<float*>(Cv) + z * slice_stride + (int64_t)row * N +
                    nb * WV_BN + wave * 32 + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) store_partial(cp + n * 16, acc[i][n][e], wt);
      } else if constexpr (EPI == EPI_OUT) {
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * N + nb * WV_BN + wave * 32 + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) cp[n * 16] = from_f<T>(acc[i][n][e]);
      } else {
        const int I = N >> 1;
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * I + nb * 128 + wave * 16 + fr;
        *cp = from_f<T>(silu_f(acc[i][0][e]) * acc[i][1][e]);
      }
    }
  }
}

// P[nb][kb][w][j][lane] (16-B chunks) = W[wv_row(nb, w, j & 1, lane & 15)]
//                                        [kb * 64 + (j >> 1) * 32 + (lane >> 4) * 8 ..]
template <typename T, int EPI>
__global__ __launch_bounds__(256) void wv_pack_kernel(T* __restrict__ P, const T* __restrict__ W,
                                                      int N, int K) {
  const int nk_all = K / WV_BK;
  const int64_t ci = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (ci >= (int64_t)N * K / 8) return;
  const int lane = (int)(ci & 63), j = (int)((ci >> 6) & 3), w = (int)((ci >> 8) & 7);
  const int64_t t = ci >> 11;
  const int kb = (int)(t % nk_all);
  const int nb = (int)(t / nk_all);
  const int64_t src = wv_row<EPI>(nb, w, j & 1, lane & 15, N) * K + kb * WV_BK +
                      (j >> 1) * 32 + (lane >> 4) * 8;
  reinterpret_cast<u32x4*>(P)[ci] = *reinterpret_cast<const u32x4*>(W + src);
}

template <typename T, int D>
void dgemm_wv_cfg(int epi, void* C, const void* X, const void* W, int M, int N, int K,
                  int64_t ldx, int S, int64_t ss, hipStream_t s) {
  const dim3 grid((unsigned)((N / WV_BN) * S));
#define DG_W(E)                                                                       \
  dgemm_wv_kernel<T, E, D><<<grid, 512, 0, s>>>(C, (const T*)X, (const T*)W, M, N, K, \
                                                ldx, S, ss, partial_wt())
  if (epi == EPI_PARTIAL) DG_W(EPI_PARTIAL);
  else if (epi == EPI_OUT) DG_W(EPI_OUT);
  else DG_W(EPI_SILU);
#undef DG_W
}

}  // namespace

void launch_dgemm_wv(int depth, int epi, void* C, const void* X, const void* Wp, int M, int N,
                     int K, int64_t ldx, int S, int64_t ss, hipStream_t s) {
  switch (depth) {
    case 2: dgemm_wv_cfg<bf16, 2>(epi, C, X, Wp, M, N, K, ldx, S, ss, s); break;
    default: dgemm_wv_cfg<bf16, 3>(epi, C, X, Wp, M, N, K, ldx, S, ss, s); break;
  }
}

void launch_wv_pack(bool silu, void* P, const void* W, int N, int K, hipStream_t s) {
  const int64_t chunks = (int64_t)N * K / 8;
  const dim3 grid((unsigned)((chunks + 255) / 256));
  if (silu) wv_pack_kernel<bf16, EPI_SILU><<<grid, 256, 0, s>>>((bf16*)P, (const bf16*)W, N, K);
  else wv_pack_kernel<bf16, EPI_OUT><<<grid, 256, 0, s>>>((bf16*)P, (const bf16*)W, N, K);
}

}  // namespace kgc
