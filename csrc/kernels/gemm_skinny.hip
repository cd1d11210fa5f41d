// K9 skinny GEMM for small-batch decode on gfx950:  C[M, N] = X[M, K] . W[N, K]^T (+ bias)
// with M <= 64 (decode batch), W the [out, in] weight of a linear layer.
//
// At these M the GEMM is a weight stream: every W byte is read once from HBM, X is a
// few hundred KB that stays in L2.  hipBLASLt's tiles are built for M >= 128 and leave
// qkv / o-projection shapes at 2-4 TB/s (profiles/tunableop: N=4096 K=4096 M=1 takes
// 14.9 us = 2.2 TB/s).  Here:
//   * a workgroup owns 16*NT weight rows and ALL of K; its NW waves split K evenly,
//     so a 4096-row layer launches 4096/16/NT workgroups of NW waves (>= 2048 waves)
//     and every wave streams one contiguous K-range of its rows;
//   * W fragments go straight from HBM to VGPRs as the MFMA A operand (no LDS round
//     trip -- cdna_hip_programming.md §5, "GEMV / M <= 16 decode weights"); each wave
//     issues U k-steps of loads (W and X) before the first MFMA of the batch;
//   * X fragments (B operand, 16 batch rows per m-tile, rows >= M clamped to M-1 and
//     discarded) are L2 hits;
//   * v_mfma_f32_16x16x32: acc[m-tile][n-tile] holds C^T[n][m] -- lane l owns
//     n = 4*(l>>4)+i, m = l&15 -- so the NW per-wave partial sums are merged in LDS
//     and written as coalesced rows of C by the whole workgroup, bias added once.
//   * NTL: W loads carry the non-temporal hint (streamed once, never re-read).
// Shapes the kernel takes (checked on the host): N % (16*NT) == 0, K % (32*NW) == 0,
// 16-byte aligned rows.  Which (M, N, K) run here and which on hipBLASLt is decided at
// engine start by timing both on the model's own weights (ops/gemm.py).
#include "common.h"
#include "launch.h"

namespace kgc {

template <typename T, int MT, int NT, int NW, bool NTL>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(
    T* __restrict__ C, const T* __restrict__ X, const T* __restrict__ W,
    const T* __restrict__ bias, int M, int K, int64_t ldx, int64_t ldc) {
  typedef typename Vec8<T>::type V8;
  constexpr int U = (MT + NT) <= 2 ? 8 : 4;     // k-steps of loads in flight per batch
  __shared__ __attribute__((aligned(16))) float red[NW][MT][NT][64][4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, q4 = lane >> 4;
  const int64_t n0 = (int64_t)blockIdx.x * (16 * NT);
  const int kw = K / NW;
  const int kbeg = wave * kw, kend = kbeg + kw;

  const T* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wrow[nt] = W + (n0 + 16 * nt + r16) * (int64_t)K + 8 * q4;
  const T* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xrow[mt] = X + (int64_t)min(16 * mt + r16, M - 1) * ldx + 8 * q4;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto ldw = [](const T* p) -> u32x4 {
    if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
  };

  // Two register sets (A, B) of U k-steps each: batch b+1's loads are in flight while
  // batch b's MFMAs wait only for their own (counted vmcnt), so a wave always has one
  // to two batches of W outstanding instead of draining to zero between batches.
  typedef Pack8<T> WSet[U][NT];
  typedef Pack8<T> XSet[U][MT];
  auto load = [&](WSet& wf, XSet& xf, int k) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) wf[u][nt].u = ldw(wrow[nt] + k + 32 * u);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        xf[u][mt].u = *reinterpret_cast<const u32x4*>(xrow[mt] + k + 32 * u);
  };
  auto compute = [&](const WSet& wf, const XSet& xf) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = mfma16x16x32(wf[u][nt].v, xf[u][mt].v, acc[mt][nt]);
  };
  const int nb = (kend - kbeg) / (32 * U);
  int k = kbeg;
  WSet wa, wb;
  XSet xa, xb;
  if (nb > 0) load(wa, xa, k);
  for (int b = 0; b < nb; b += 2) {
    if (b + 1 < nb) load(wb, xb, k + 32 * U);
    compute(wa, xa);
    if (b + 1 < nb) {
      if (b + 2 < nb) load(wa, xa, k + 64 * U);
      compute(wb, xb);
    }
    k += 64 * U;
  }
  k = kbeg + nb * 32 * U;
  for (; k < kend; k += 32) {     // K-range not a multiple of 32*U
    Pack8<T> wf[NT], xf[MT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) wf[nt].u = ldw(wrow[nt] + k);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xf[mt].u = *reinterpret_cast<const u32x4*>(xrow[mt] + k);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(wf[nt].v, xf[mt].v, acc[mt][nt]);
  }

  // ---- merge the NW K-slices: lane (r16, q4) of wave w holds C^T[16nt+4q4+i][16mt+r16]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      *reinterpret_cast<f32x4*>(&red[wave][mt][nt][lane][0]) = acc[mt][nt];
  __syncthreads();
  constexpr int TN = 16 * NT;
  const int rows = min(M, 16 * MT);
  for (int e = threadIdx.x; e < rows * TN; e += NW * 64) {
    const int m = e / TN, n = e % TN;
    const int mt = m >> 4, nt = n >> 4, nn = n & 15;
    const int l = (nn >> 2) * 16 + (m & 15), i = nn & 3;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w][mt][nt][l][i];
    if (bias != nullptr) s += to_f<T>(bias[n0 + n]);
    C[(int64_t)m * ldc + n0 + n] = from_f<T>(s);
  }
}

template <typename T, int MT, int NT>
static void skinny_nw(int nw, bool ntl, void* C, const void* X, const void* W, const void* bias,
                      int M, int N, int K, int64_t ldx, int64_t ldc, hipStream_t s) {
  const dim3 grid(N / (16 * NT));
#define SK_LAUNCH(NW_, NTL_)                                                                  \
  skinny_gemm_kernel<T, MT, NT, NW_, NTL_><<<grid, NW_ * 64, 0, s>>>(                        \
      (T*)C, (const T*)X, (const T*)W, (const T*)bias, M, K, ldx, ldc)
  if (nw == 16) {
    if (ntl) SK_LAUNCH(16, true); else SK_LAUNCH(16, false);
  } else if (nw == 8) {
    if (ntl) SK_LAUNCH(8, true); else SK_LAUNCH(8, false);
  } else {
    if (ntl) SK_LAUNCH(4, true); else SK_LAUNCH(4, false);
  }
#undef SK_LAUNCH
}

template <typename T>
static void skinny_t(int mt, int nt, int nw, bool ntl, void* C, const void* X, const void* W,
                     const void* bias, int M, int N, int K, int64_t ldx, int64_t ldc,
                     hipStream_t s) {
#define SK_MT(MT_)                                                                            \
  if (nt == 2) skinny_nw<T, MT_, 2>(nw, ntl, C, X, W, bias, M, N, K, ldx, ldc, s);           \
  else skinny_nw<T, MT_, 1>(nw, ntl, C, X, W, bias, M, N, K, ldx, ldc, s)
  if (mt == 1) { SK_MT(1); }
  else if (mt == 2) { SK_MT(2); }
  else { SK_MT(4); }
#undef SK_MT
}

void launch_skinny_gemm(int dtype, int mt, int nt, int nw, bool ntl, void* C, const void* X,
                        const void* W, const void* bias, int M, int N, int K, int64_t ldx,
                        int64_t ldc, hipStream_t s) {
  if (M == 0 || N == 0) return;
  if (dtype == DT_BF16)
    skinny_t<bf16>(mt, nt, nw, ntl, C, X, W, bias, M, N, K, ldx, ldc, s);
  else
    skinny_t<f16>(mt, nt, nw, ntl, C, X, W, bias, M, N, K, ldx, ldc, s);
}

}  // namespace kgc
