// K9v (round 3, measured slower than K9m on every M = 256 shape; profiles/README.md
// "Round 3: K9v"): the activation stream of the decode GEMM in a VGPR ring instead of
// LDS.  Research build only (tools/research/build.py -> _kgc_research.so); the engine's
// library does not contain it.
#include "common.h"
#include "launch.h"
#include "research.h"
#include <cstdlib>

namespace kgc {

namespace {

constexpr int DG_BK = 64, DG_ROWB = 128;
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

// The same waits as a real S_WAITCNT (the builtin, gfx9 encoding: vmcnt [3:0] + [15:14],
// expcnt and lgkmcnt left at their maxima) rather than opaque inline asm: the compiler's
// wait-count pass then knows how many loads are still outstanding and does not add a
// vmcnt(0) of its own before the first use of a register-ring load (K9v).
// A 16-B global load the compiler does not see as a load (inline asm): it adds no wait of
// its own before the register's first use -- the K9v ring waits with wait_vm_b, whose
// counts include these loads.  (As plain loads, the wait-count pass lost track of the
// ring across the loop back-edge and drained every load before each step's MFMAs.)
__device__ __forceinline__ u32x4 ld_async16(const void* p) {
  u32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}

template <int N>
__device__ __forceinline__ void wait_vm_b() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | 0x70 | 0xF00 | ((N >> 4) << 14));
}

// K9v: the activation stream goes into a VGPR ring instead of LDS.
// The K9m / K9r measurements fit an in-order intake model: a CU's vector-memory returns
// come back in issue order, so the L2-hit activation pieces wait behind the HBM-miss
// weight pieces and the per-CU rate is (bytes in flight) / (HBM latency), with the
// LDS ring (~96 KB in flight) as the cap -- two thirds of it activations at M = 256.
// Here each of the 8 waves owns a 32-row strip of the 256-row tile and loads its own MFMA
// A fragments straight from X (16 B per lane, no duplication across waves) into a
// D + 1 deep register ring (16 VGPRs per K-step), while the packed weights still stream
// through a D + 1 slot LDS-DMA ring (16 KB per K-step): D K-steps of both operands are in
// flight during every step's MFMAs (48 KB per step per CU: 144 KB at D = 3, 192 KB at
// D = 4), and the LDS holds only weights.  Every wave reads the whole weight slot
// (8 x 16 KB of ds_read_b128 per step, well inside the LDS rate).
// Tile 256 x 128 (M <= 256), packed weights, split-K over a 1-D grid as dgemm_kernel.
template <typename T, int EPI, int D>
__global__ __launch_bounds__(512, 1) void dgemm_vreg_kernel(
    void* __restrict__ Cv, const T* __restrict__ X, const T* __restrict__ W, int M, int N,
    int K, int64_t ldx, int S, int64_t slice_stride, int wt) {
  constexpr int BN = 128, NS = D + 1, MT = 2, NT = 8;
  constexpr int SLOT = BN * DG_ROWB;              // 16 KB of packed weights per K-step
  constexpr int OPS = MT * 2 + 2;                 // vm ops per K-step per wave
  static_assert(NS * SLOT <= 163840, "LDS ring exceeds 160 KiB");
  __shared__ __attribute__((aligned(16))) char lds[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int z = blockIdx.x % S, nb = blockIdx.x / S;
  const int nk_all = K / DG_BK;
  const int kb0 = (int)((int64_t)nk_all * z / S);
  const int nk = (int)((int64_t)nk_all * (z + 1) / S) - kb0;
  const int rot = nk >= 4 ? (int)(((int64_t)nb * 37) % nk) : 0;

  const T* a_src[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int r = wave * 32 + i * 16 + fr;
    r = r < M ? r : M - 1;                        // padded rows re-read the last row
    a_src[i] = X + (int64_t)r * ldx + fq * 8;
  }
  const T* b_src[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
    b_src[t] = W + (int64_t)nb * nk_all * (BN * DG_BK) + (wave * 2 + t) * 512 + lane * 8;

  // Every K-step issues one group of OPS loads, also past the end of the slice: a step
  // >= nk loads a filler group (every lane the same 16 B of X / W, one cached line per
  // instruction) into a slot nobody reads.  The wait before each step is then always
  // "all but the D - 1 youngest groups" -- an unconditional wait the compiler's count
  // tracks, where a tail-dependent one made it add a vmcnt(0) of its own every trip.
  u32x4 areg[NS][MT][2];
  auto issue = [&](int step, int slot) {
    const bool real = step < nk;
    int st = step + rot;
    st = st >= nk ? st - nk : st;
    const int kb = kb0 + (real ? st : 0);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const T* src = real ? a_src[i] + kb * DG_BK + s * 32 : X;
        areg[slot][i][s] = ld_async16(src);
      }
    char* dst = lds + slot * SLOT;
    const int64_t bo = (int64_t)kb * (BN * DG_BK);
#pragma unroll
    for (int t = 0; t < 2; ++t)
      glds16<2>(real ? b_src[t] + bo : W, dst + (wave * 2 + t) * 1024);
    // keep the groups in issue order (the scheduler hoisted the prologue's DMAs above its
    // register loads, and the counts above assume whole groups in order)
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
        // slot (it + D) % NS held step it - 1, which every wave finished before the barrier
        issue(it + D, (u + D) % NS);
        const char* sb = lds + u * SLOT;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + fq;
          Pack8<T> bfr[NT];
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            const int r = n * 16 + fr;
            bfr[n].u = *reinterpret_cast<const u32x4*>(sb + r * DG_ROWB + (swz(r, c) << 4));
          }
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            Pack8<T> af;
            af.u = areg[u][i][ks];
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[i][n] = mfma16x16x32(af.v, bfr[n].v, acc[i][n]);
          }
        }
      }
    }
  }
  // the filler groups still fly: no LDS-DMA may land after this workgroup's LDS is gone
  wait_vm_b<0>();
  // ... and no register load either: the compiler sees the ring's asm loads as finished
  // values, so a filler (never read) would be dead at once and its registers handed to
  // the epilogue's addresses while its data is still on the way.  Reading every slot
  // here keeps each one allocated until the wait above.
#pragma unroll
  for (int sl = 0; sl < NS; ++sl)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) asm volatile("" ::"v"(areg[sl][i][s]));

  // ---- epilogue: lane holds C[4*fq + e][fr] of every 16x16 tile
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = wave * 32 + i * 16 + fq * 4 + e;
      if (row >= M) continue;
      if constexpr (EPI == EPI_PARTIAL) {
        float* cp = reinterpret_cast<float*>(Cv) + z * slice_stride + (int64_t)row * N +
                    nb * BN + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) store_partial(cp + n * 16, acc[i][n][e], wt);
      } else if constexpr (EPI == EPI_OUT) {
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * N + nb * BN + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) cp[n * 16] = from_f<T>(acc[i][n][e]);
      } else {
        const int I = N >> 1;
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * I + nb * (BN / 2) + fr;
#pragma unroll
        for (int n = 0; n < NT; n += 2)
          cp[(n >> 1) * 16] = from_f<T>(silu_f(acc[i][n][e]) * acc[i][n + 1][e]);
      }
    }
  }
}

template <typename T, int D>
void dgemm_vreg_cfg(int epi, void* C, const void* X, const void* W, int M, int N, int K,
                    int64_t ldx, int S, int64_t ss, hipStream_t s) {
  const dim3 grid((unsigned)((N / 128) * S));
#define DG_V(E)                                                                       \
  dgemm_vreg_kernel<T, E, D><<<grid, 512, 0, s>>>(C, (const T*)X, (const T*)W, M, N, K, \
                                                  ldx, S, ss, partial_wt())
  if (epi == EPI_PARTIAL) DG_V(EPI_PARTIAL);
  else if (epi == EPI_OUT) DG_V(EPI_OUT);
  else DG_V(EPI_SILU);
#undef DG_V
}

}  // namespace

void launch_dgemm_vreg(int depth, int epi, void* C, const void* X, const void* W, int M, int N,
                       int K, int64_t ldx, int S, int64_t ss, hipStream_t s) {
  switch (depth) {
    case 2: dgemm_vreg_cfg<bf16, 2>(epi, C, X, W, M, N, K, ldx, S, ss, s); break;
    case 3: dgemm_vreg_cfg<bf16, 3>(epi, C, X, W, M, N, K, ldx, S, ss, s); break;
    default: dgemm_vreg_cfg<bf16, 4>(epi, C, X, W, M, N, K, ldx, S, ss, s); break;
  }
}

}  // namespace kgc
