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
//
// Fused epilogues for the decode layer at small M (the layer then runs no RMSNorm
// kernel: 2 of its ~10 launches at the ~4.7 us small-kernel floor disappear):
//   SK_NORM: X rows are RMS-normalised on the fly, C = rms(x)^-1 * ((x * gamma) W^T).
//            Each lane squares the X elements it loads anyway; the per-row sums of
//            squares meet in LDS with the partial products, and 1/rms scales the merged
//            row (one factor per row, so it commutes with the K-sum).  ~15 VALU cycles
//            per X element: only the one-m-tile (M <= 16) form is used by the model.
//   SK_ACC:  C += X W^T (+ bias) -- the residual add of o_proj / down_proj.
//   SK_SILU: W is the merged [gate; up] weight [2I, K] (row-major, as loaded); n-tile 0 of
//            a workgroup streams gate rows g0..g0+15 and n-tile 1 the matching up rows
//            I+g0.., so the merged sums of one lane pair give C[m, g0+n] = silu(g) * u with
//            C [M, I]: the [M, 2I] gate_up output and the silu_mul launch never exist.
//            NT = 2 only, no bias.
//   SK_ACC_NORM: SK_ACC, then the residual add + RMSNorm that consumes C inside the same
//            launch: every workgroup publishes its tile of C (write-through stores,
//            drained, no release fence) and draws a ticket; the last of the grid acquires and
//            writes NO[m, :] = C[m, :] * rsqrt(mean(C[m, :]^2) + eps) * gamma (one wave
//            per row, the rounding of fused_add_rms_norm), then re-arms the ticket.  The
//            separate norm launch and its kernel boundary disappear (o_proj -> post-
//            attention norm, down_proj -> next input norm at small M).  The ticket is
//            zeroed at allocation and by every last arriver; one ticket per stream.
//   SK_ACC_SS / SK_RSCALE(_SILU): the small-M decoder layer with NO RMSNorm launch.  The
//            norm's weight gamma is folded into the consuming weight once (W' = W diag(gamma),
//            ops/gemm.py fold_norm_weight), so rms_norm(x) W^T = rsqrt(mean(x^2) + eps) *
//            (x W'^T): a per-row scale of the plain GEMM.  The producer of x (o_proj /
//            down_proj, SK_ACC_SS) adds its output into the residual and writes each row's sum
//            of squares over ITS columns, rounded as stored, to SSP[row][workgroup]; the
//            consumer (qkv / gate_up, SK_RSCALE / SK_RSCALE_SILU) sums the NSS partials of its
//            rows -- loaded before its weight stream starts -- and scales them.  Two launches
//            per layer fewer than residual add + RMSNorm kernels at batch 1.
#include "common.h"
#include "launch.h"

namespace kgc {

enum { SK_PLAIN = 0, SK_NORM = 1, SK_ACC = 2, SK_SILU = 3, SK_ACC_NORM = 4, SK_ACC_SS = 5,
       SK_RSCALE = 6, SK_RSCALE_SILU = 7 };

// SK_RSCALE(_SILU) at MT = 1, NT = 2 (the shapes the model runs): held to the plain variant's 4 waves per SIMD (128 VGPRs);
// its few extra registers would otherwise cost a wave of occupancy on a weight stream
template <int MT, int NT, int EPI>
constexpr int sk_waves_per_eu() {
  return ((EPI == 6 || EPI == 7) && MT == 1 && NT == 2) ? 4 : 1;
}

// s_waitcnt immediate that waits for vmcnt <= n only (gfx9 encoding: vmcnt in bits 3:0 and
// 15:14, expcnt 6:4 and lgkmcnt 11:8 left at their maxima)
constexpr int sk_vmcnt(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

template <typename T, int MT, int NT, int NW, bool NTL, int EPI>
__global__ __launch_bounds__(NW * 64)
__attribute__((amdgpu_waves_per_eu(sk_waves_per_eu<MT, NT, EPI>()))) void skinny_gemm_kernel(
    T* __restrict__ C, const T* __restrict__ X, const T* __restrict__ W,
    const T* __restrict__ bias, const T* __restrict__ gamma, float eps, int M, int K,
    int64_t ldx, int64_t ldc, T* __restrict__ NO, uint32_t* __restrict__ ticket,
    float* __restrict__ SSP, int nss) {
  constexpr bool NORM = EPI == SK_NORM, ACCN = EPI == SK_ACC_NORM, ACCSS = EPI == SK_ACC_SS;
  constexpr bool RS = EPI == SK_RSCALE || EPI == SK_RSCALE_SILU;
  constexpr bool SILU = EPI == SK_SILU || EPI == SK_RSCALE_SILU;
  constexpr bool ACC = EPI == SK_ACC || ACCN || ACCSS;
  static_assert(!SILU || NT == 2, "SK_SILU pairs n-tile 0 (gate) with n-tile 1 (up)");
  // k-steps of loads in flight per batch (SK_NORM: gamma fragments ride along, so the
  // batch is halved to keep the register sets -- and the waves per SIMD -- as they were)
  constexpr int U = (!NORM && (MT + NT) <= 2) ? 8 : 4;
  __shared__ __attribute__((aligned(16))) float red[NW][MT][NT][64][4];
  __shared__ float ssr[NORM ? NW : 1][MT][64];  // per-lane partial sums of squares
  __shared__ float inv_s[16 * MT];
  __shared__ float ssl[RS ? 16 : 1][RS ? 256 : 1];  // SK_RSCALE: the rows' partials (LDS-DMA)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r16 = lane & 15, q4 = lane >> 4;
  // SK_SILU: gridDim.x = I / 16 workgroups over the I = 16 * gridDim.x output columns
  const int64_t n0 = (int64_t)blockIdx.x * (SILU ? 16 : 16 * NT);
  const int64_t n_half = SILU ? (int64_t)gridDim.x * 16 : 0;
  const int kw = K / NW;
  const int kbeg = wave * kw, kend = kbeg + kw;

  const T* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    wrow[nt] = W + (n0 + (SILU ? nt * n_half : 16 * nt) + r16) * (int64_t)K + 8 * q4;
  const T* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xrow[mt] = X + (int64_t)min(16 * mt + r16, M - 1) * ldx + 8 * q4;
  const T* grow = NORM ? gamma + 8 * q4 : nullptr;

  f32x4 acc[MT][NT];
  float ss[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    ss[mt] = 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  auto ldw = [](const T* p) -> u32x4 {
    if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
  };
  // one k-step of MFMAs; with NORM the X fragment is squared into ss and scaled by gamma
  auto step = [&](const Pack8<T>* wf, const Pack8<T>* xf, const Pack8<T>& gf) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      Pack8<T> xv = xf[mt];
      if constexpr (NORM) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = to_f<T>(xf[mt].h[j]);
          ss[mt] += a * a;
          xv.h[j] = from_f<T>(a * to_f<T>(gf.h[j]));
        }
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16x16x32(wf[nt].v, xv.v, acc[mt][nt]);
    }
  };

  // Two register sets (A, B) of U k-steps each: batch b+1's loads are in flight while
  // batch b's MFMAs wait only for their own (counted vmcnt), so a wave always has one
  // to two batches of W outstanding instead of draining to zero between batches.
  typedef Pack8<T> WSet[U][NT];
  typedef Pack8<T> XSet[U][MT];
  typedef Pack8<T> GSet[NORM ? U : 1];
  auto load = [&](WSet& wf, XSet& xf, GSet& gf, int k) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) wf[u][nt].u = ldw(wrow[nt] + k + 32 * u);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        xf[u][mt].u = *reinterpret_cast<const u32x4*>(xrow[mt] + k + 32 * u);
    if constexpr (NORM) {
#pragma unroll
      for (int u = 0; u < U; ++u) gf[u].u = *reinterpret_cast<const u32x4*>(grow + k + 32 * u);
    }
  };
  auto compute = [&](const WSet& wf, const XSet& xf, const GSet& gf) {
#pragma unroll
    for (int u = 0; u < U; ++u) step(wf[u], xf[u], gf[NORM ? u : 0]);
  };
  const int nb = (kend - kbeg) / (32 * U);
  int k = kbeg;
  WSet wa, wb;
  XSet xa, xb;
  GSet ga, gb;
  // SK_RSCALE: the sum-of-squares partials of this wave's rows (m = wave + r * NW) go out
  // ahead of the first weight batch straight into LDS (LDS-DMA, addresses dead before the
  // weight stream -- as register loads they cost a wave per SIMD of occupancy); the host
  // keeps nss <= 256 and M <= 16
  constexpr int RSR = (16 + NW - 1) / NW;
  if constexpr (RS) {
#pragma unroll
    for (int r = 0; r < RSR; ++r) {
      const int m = wave + r * NW;
      if (m >= M) break;                 // wave-uniform: rows past the batch load nothing
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (64 * i >= nss) break;        // uniform too: nss = 64 covers one DMA per row
        const int j = min(lane + 64 * i, nss - 1);
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(SSP + (int64_t)m * nss + j),
            (__attribute__((address_space(3))) void*)&ssl[wave + r * NW][64 * i], 4, 0, 0);
      }
    }
  }
  // Two register sets in flight; the compiler's wait-count pass places the waits.  The
  // SK_RSCALE forms issue both batches and then retire their (older) partial DMAs with a
  // compiler-visible wait: a DMA still counted at the loop header made every iteration
  // wait for vmcnt(0) (qkv at batch 1: 12.4 vs 12.9 us with the DMA retired first).
  // (A hand-placed in-order pipeline -- explicit vmcnt(loads per batch) waits fenced by
  // sched_barrier, one straight steady-state path -- was measured: down -2.9 us, but it
  // costs the NT = 2 forms a wave per SIMD and the decode step was no faster;
  // profiles/README.md "Norm-free small-M decoder layer".)
  constexpr int LB = U * (NT + MT + (NORM ? 1 : 0));   // vector loads per batch
  auto kb = [&](int bi) { return kbeg + bi * 32 * U; };
  if (nb > 0) load(wa, xa, ga, kb(0));
  if constexpr (RS) {
    if (nb > 1) {
      load(wb, xb, gb, kb(1));
      __builtin_amdgcn_s_waitcnt(sk_vmcnt(2 * LB));
    } else if (nb > 0) {
      __builtin_amdgcn_s_waitcnt(sk_vmcnt(LB));
    } else {
      __builtin_amdgcn_s_waitcnt(sk_vmcnt(0));
    }
  }
  for (int b = 0; b < nb; b += 2) {
    if (b + 1 < nb && !(RS && b == 0)) load(wb, xb, gb, kb(b + 1));
    compute(wa, xa, ga);
    if (b + 1 < nb) {
      if (b + 2 < nb) load(wa, xa, ga, kb(b + 2));
      compute(wb, xb, gb);
    }
  }
  k = kbeg + nb * 32 * U;
  for (; k < kend; k += 32) {     // K-range not a multiple of 32*U
    Pack8<T> wf[NT], xf[MT], gf;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) wf[nt].u = ldw(wrow[nt] + k);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xf[mt].u = *reinterpret_cast<const u32x4*>(xrow[mt] + k);
    if constexpr (NORM) gf.u = *reinterpret_cast<const u32x4*>(grow + k);
    step(wf, xf, gf);
  }

  // ---- merge the NW K-slices: lane (r16, q4) of wave w holds C^T[16nt+4q4+i][16mt+r16]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      *reinterpret_cast<f32x4*>(&red[wave][mt][nt][lane][0]) = acc[mt][nt];
    if constexpr (NORM) ssr[wave][mt][lane] = ss[mt];
  }
  if constexpr (RS) {
    // this wave's own partials landed (its LDS-DMAs are older than every weight load the
    // loop above waited for; vmcnt(0) for certainty) -- and only this wave reads them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the lane index re-derived behind an opaque move: nothing of this block is hoisted
    // into the weight loop, where it would hold registers (and cost a wave of occupancy)
    int ln = threadIdx.x & 63;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int r = 0; r < RSR; ++r) {
      const int m = wave + r * NW;
      if (m >= M) break;
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) t += ln + 64 * i < nss ? ssl[m < 16 ? m : 0][64 * i + ln] : 0.f;
      t = wave_sum(t);
      if (ln == 0 && m < M && m < 16 * MT) inv_s[m] = rsqrtf(t / (float)K + eps);
    }
  }
  __syncthreads();
  constexpr int TN = SILU ? 16 : 16 * NT;
  const int rows = min(M, 16 * MT);
  if constexpr (NORM) {
    // row m's sum of squares: its 4 lanes (q4) in each of the NW waves
    if (threadIdx.x < rows) {
      const int m = threadIdx.x, mt = m >> 4, r = m & 15;
      float t = 0.f;
      for (int w = 0; w < NW; ++w)
#pragma unroll
        for (int q = 0; q < 4; ++q) t += ssr[w][mt][q * 16 + r];
      inv_s[m] = rsqrtf(t / (float)K + eps);
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < rows * TN; e += NW * 64) {
    const int m = e / TN, n = e % TN;
    const int mt = m >> 4, nt = n >> 4, nn = n & 15;
    const int l = (nn >> 2) * 16 + (m & 15), i = nn & 3;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w][mt][nt][l][i];
    if constexpr (SILU) {
      float u = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) u += red[w][mt][1][l][i];
      if constexpr (RS) {
        s *= inv_s[m];
        u *= inv_s[m];
      }
      C[(int64_t)m * ldc + n0 + n] = from_f<T>(s / (1.f + __expf(-s)) * u);
      continue;
    }
    if constexpr (NORM || RS) s *= inv_s[m];
    if (bias != nullptr) s += to_f<T>(bias[n0 + n]);
    T* c = C + (int64_t)m * ldc + n0 + n;
    if constexpr (ACC) s += to_f<T>(*c);
    if constexpr (ACCN) {
      // write-through (sc1) store: the last workgroup reads it from another CU with no
      // release fence on this side
      const T v = from_f<T>(s);
      __hip_atomic_store(reinterpret_cast<uint16_t*>(c), __builtin_bit_cast(uint16_t, v),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (ACCSS) {
      // the TN lanes of a row's columns are one aligned lane group (stride NW * 64, and
      // 64 % TN == 0): their squares of the stored values sum over the group, fixed order
      const T v = from_f<T>(s);
      *c = v;
      float q = to_f<T>(v) * to_f<T>(v);
#pragma unroll
      for (int o = 1; o < TN; o <<= 1) q += __shfl_xor(q, o, 64);
      if (n == 0) SSP[(int64_t)m * gridDim.x + blockIdx.x] = q;
    } else {
      *c = from_f<T>(s);
    }
  }
  if constexpr (ACCN) {
    __shared__ uint32_t last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's C stores landed
    __syncthreads();
    if (threadIdx.x == 0) {
      // two-level fan-in: 8 sub-counters (blockIdx % 8, the XCD under round-robin
      // placement) of <= gridDim/8 arrivals each, then the 8 sub-last workgroups on the
      // top counter -- one device-scope counter took ~12 ns per arrival, ~3 us at 256
      // workgroups (MI355X_MICROARCH.md "fanin"), more than the separate norm launch
      const uint32_t sub = blockIdx.x & 7u;
      const uint32_t nsub = (gridDim.x - sub + 7u) >> 3;
      const uint32_t nact = min(gridDim.x, 8u);
      bool lst = false;
      const uint32_t t = __hip_atomic_fetch_add(ticket + 1 + sub, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      if (t == nsub - 1) {
        __hip_atomic_store(ticket + 1 + sub, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t t2 = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        lst = t2 == nact - 1;
      }
      last = lst;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (!last) return;
    // one wave per row; a lane holds its <= 16 chunks of 8 in registers, so a row costs ONE
    // load round trip (these lines were written by other CUs: L2 / HBM latency)
    const int N = gridDim.x * TN;                        // whole rows (host: 512 | N <= 8192)
    constexpr int CH = 16;
    for (int m = wave; m < M; m += NW) {
      const T* c = C + (int64_t)m * ldc;
      Pack8<T> v[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (j * 512 < N) v[j].u = *reinterpret_cast<const u32x4*>(c + j * 512 + lane * 8);
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (j * 512 < N) {
#pragma unroll
          for (int e = 0; e < 8; ++e) ss += to_f<T>(v[j].h[e]) * to_f<T>(v[j].h[e]);
        }
      const float inv = rsqrtf(wave_sum(ss) / (float)N + eps);
      T* o = NO + (int64_t)m * N;
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (j * 512 < N) {
          Pack8<T> g, r;
          g.u = *reinterpret_cast<const u32x4*>(gamma + j * 512 + lane * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) r.h[e] = from_f<T>(to_f<T>(v[j].h[e]) * inv * to_f<T>(g.h[e]));
          *reinterpret_cast<u32x4*>(o + j * 512 + lane * 8) = r.u;
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename T, int MT, int NT, int NW, bool NTL>
static void sk_launch(int epi, dim3 grid, hipStream_t s, void* C, const void* X, const void* W,
                      const void* bias, const void* gamma, float eps, int M, int K,
                      int64_t ldx, int64_t ldc, void* NO, uint32_t* ticket, float* ssp,
                      int nss) {
#define SK_GO(E)                                                                              \
  skinny_gemm_kernel<T, MT, NT, NW, NTL, E><<<grid, NW * 64, 0, s>>>(                        \
      (T*)C, (const T*)X, (const T*)W, (const T*)bias, (const T*)gamma, eps, M, K, ldx, ldc, \
      (T*)NO, ticket, ssp, nss)
  if (epi == SK_NORM) SK_GO(SK_NORM);
  else if (epi == SK_ACC) SK_GO(SK_ACC);
  else if (epi == SK_ACC_NORM) SK_GO(SK_ACC_NORM);
  else if (epi == SK_ACC_SS) SK_GO(SK_ACC_SS);
  else if (epi == SK_RSCALE) SK_GO(SK_RSCALE);
  else if constexpr (NT == 2) {
    if (epi == SK_SILU) SK_GO(SK_SILU);
    else if (epi == SK_RSCALE_SILU) SK_GO(SK_RSCALE_SILU);
    else SK_GO(SK_PLAIN);
  } else SK_GO(SK_PLAIN);
#undef SK_GO
}

template <typename T, int MT, int NT>
static void skinny_nw(int nw, bool ntl, int epi, void* C, const void* X, const void* W,
                      const void* bias, const void* gamma, float eps, int M, int N, int K,
                      int64_t ldx, int64_t ldc, void* NO, uint32_t* ticket, float* ssp, int nss,
                      hipStream_t s) {
  const bool silu = epi == SK_SILU || epi == SK_RSCALE_SILU;
  const dim3 grid(silu ? N / 32 : N / (16 * NT));   // silu epilogues: N = 2I
#define SK_NW(NW_)                                                                            \
  if (ntl) sk_launch<T, MT, NT, NW_, true>(epi, grid, s, C, X, W, bias, gamma, eps, M, K, ldx, ldc, \
                                           NO, ticket, ssp, nss);                            \
  else sk_launch<T, MT, NT, NW_, false>(epi, grid, s, C, X, W, bias, gamma, eps, M, K, ldx, ldc, \
                                        NO, ticket, ssp, nss)
  if (nw == 16) { SK_NW(16); }
  else if (nw == 8) { SK_NW(8); }
  else { SK_NW(4); }
#undef SK_NW
}

template <typename T>
static void skinny_t(int mt, int nt, int nw, bool ntl, int epi, void* C, const void* X,
                     const void* W, const void* bias, const void* gamma, float eps, int M, int N,
                     int K, int64_t ldx, int64_t ldc, void* NO, uint32_t* ticket, float* ssp,
                     int nss, hipStream_t s) {
#define SK_MT(MT_)                                                                            \
  if (nt == 2) skinny_nw<T, MT_, 2>(nw, ntl, epi, C, X, W, bias, gamma, eps, M, N, K, ldx, ldc, \
                                    NO, ticket, ssp, nss, s);                                 \
  else skinny_nw<T, MT_, 1>(nw, ntl, epi, C, X, W, bias, gamma, eps, M, N, K, ldx, ldc, NO,    \
                            ticket, ssp, nss, s)
  if (mt == 1) { SK_MT(1); }
  else if (mt == 2) { SK_MT(2); }
  else { SK_MT(4); }
#undef SK_MT
}

void launch_skinny_gemm(int dtype, int mt, int nt, int nw, bool ntl, int epi, void* C,
                        const void* X, const void* W, const void* bias, const void* gamma,
                        float eps, int M, int N, int K, int64_t ldx, int64_t ldc, void* NO,
                        uint32_t* ticket, float* ssp, int nss, hipStream_t s) {
  if (M == 0 || N == 0) return;
  if (dtype == DT_BF16)
    skinny_t<bf16>(mt, nt, nw, ntl, epi, C, X, W, bias, gamma, eps, M, N, K, ldx, ldc, NO, ticket,
                   ssp, nss, s);
  else
    skinny_t<f16>(mt, nt, nw, ntl, epi, C, X, W, bias, gamma, eps, M, N, K, ldx, ldc, NO, ticket,
                  ssp, nss, s);
}

}  // namespace kgc
