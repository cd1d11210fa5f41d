// K9m: mid-batch decode GEMM for gfx950 (M = 65..512 rows, the batch-256 decode step).
//
//   C[M, N] = X[M, K] . W[N, K]^T      bf16 / f16 in, fp32 MFMA accumulation
//
// At M = 256 a decode projection sits at the HBM/MFMA ridge: every weight byte feeds 256
// MACs, so the weights (read once, from HBM), the activation tile (re-read from L2 by
// every column tile) and the MFMA pipe must all run near their rates at once.
//   * 512-thread workgroups (8 waves, 4 (M) x 2 (N)), one per CU, BM = 128 / 256 rows x
//     BN = 64 / 128 columns x BK = 64, mfma_f32_16x16x32 (the shape gfx950 clocks higher).
//   * Both operands go HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
//     instruction) into a 3-slot ring, two K-steps in flight behind the one consumed; the
//     ring is retired with a counted `s_waitcnt vmcnt(N)` and a raw s_barrier (never
//     __syncthreads(), whose implicit vmcnt(0) would drain the ring every step).
//   * LDS rows are 128 B (BK bf16) with a 16-B-chunk XOR swizzle (chunk ^ row % 8) applied
//     on the SOURCE address (the DMA writes lane-linear) and on the ds_read_b128 address:
//     conflict-free fragment reads for both operands.
//   * PACKED weights (PK): the weight matrix is re-laid out once at load time as
//     [N / BN][K / BK][BN x BK] tiles with the swizzle baked in, so each K-step of a
//     column tile is ONE contiguous 16 KB block.  Measured (tools/dma_probe.hip): the
//     row-major tile walk (128 rows x 128 B, rows 8 KB apart) streams HBM at ~4.4 TB/s,
//     contiguous blocks at ~5.8 TB/s.
//   * Each workgroup starts its K walk at its own step (wrapping), so the workgroups of an
//     XCD do not all fetch the same activation lines at once (-5..9 % time at S = 1).
//   * Split-K over a 1-D grid: workgroup L takes K-slice z = L % S, so with S | 8 every
//     XCD (workgroups L, L+8, ... share one) streams ONE K-slice of X, which stays in that
//     XCD's L2 for all its column tiles, while the weights stream from HBM exactly once.
//   * Epilogues: EPI_PARTIAL writes fp32 slice z of [S, M, N] (summed by the consumer:
//     splitk_add_rms_norm for o/down, splitk_reduce); EPI_OUT writes the tile in X's dtype
//     (S = 1); EPI_SILU (S = 1) takes a merged [gate; up] weight whose tile rows alternate
//     16-row groups of gate and up, so each lane holds gate and up of the same output
//     column and writes silu(g) * u: the [M, 2I] gate_up activation never exists.
// What did not pay (profiles/README.md, "K9m"): 32-deep K slots with a 6-slot ring (the
// per-step barrier costs more than the deeper ring buys), 256 x 256 tiles, and activations
// loaded straight into registers beside a 5-slot weight ring.
// Reference parity: SURVEY.md §2.5 K9 (decode GEMMs of the vLLM image the reference
// deploys, /root/reference/values-01-minimal-example2.yaml:6-7).
#include "common.h"
#include "launch.h"
#include <cstdlib>

namespace kgc {

namespace {

constexpr int DG_THREADS = 512;     // 8 waves: 4 along M x 2 along N
constexpr int DG_BK = 64, DG_NS = 3, DG_ROWB = 128;

enum { EPI_PARTIAL = 0, EPI_OUT = 1, EPI_SILU = 2 };
// ablation builds (tools/dgemm_bench.py --ablate): one K-step without its MFMAs, without
// its DMAs, or without one operand's DMAs
enum { ABL_NONE = 0, ABL_NO_MFMA = 1, ABL_NO_DMA = 2, ABL_NO_A = 3, ABL_NO_B = 4 };

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

// AUX = 2: non-temporal (the weight stream, read once by one CU, must not evict the
// activation slice every column tile of the XCD re-reads from L2)
template <int AUX>
__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_wave_base, 16, 0, AUX);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most min(D, younger) steps of L DMAs each are still in flight
template <int L, int D>
__device__ __forceinline__ void wait_younger(int younger) {
  if (younger >= D) { wait_vm<D * L>(); return; }
  if constexpr (D > 3) if (younger == 3) { wait_vm<3 * L>(); return; }
  if constexpr (D > 2) if (younger == 2) { wait_vm<2 * L>(); return; }
  if constexpr (D > 1) if (younger == 1) { wait_vm<L>(); return; }
  wait_vm<0>();
}

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// 16-B chunk position of (row, chunk) in a 128-B LDS row
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }

// weight row of B-tile row r (0..BN-1) for column tile nb; EPI_SILU interleaves gate / up
template <int BN, int EPI>
__device__ __forceinline__ int64_t weight_row(int nb, int r, int N) {
  if constexpr (EPI == EPI_SILU) {
    const int g = r >> 4;
    return (int64_t)((g & 1) ? (N >> 1) : 0) + nb * (BN / 2) + (g >> 1) * 16 + (r & 15);
  } else {
    return (int64_t)nb * BN + r;
  }
}

// Split-K partials are stored write-through (sc1, a relaxed agent-scope atomic store):
// no dirty L2 lines are left for the kernel boundary to write back (the boundary costs
// + B / 6 TB/s behind B dirty bytes: ~5.6 us behind the 33.5 MB of down_proj slices at
// M = 256, S = 8), the bytes leave during the GEMM instead.  wt = 0: plain stores
// (KGC_PARTIAL_WT=0, for A/B).
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

// LDW = 4: four extra loader waves issue every DMA and the 8 MFMA waves never stall on
// DMA issue (one s_barrier per step for all 12 waves); LDW = 0: the MFMA waves issue too.
// WN: MFMA waves along N (2: a 4 x 2 wave grid; 1: all 8 waves along M, each reading every
// column of the tile -- the narrow / odd column tiles (BN = 80, 112, 224) whose 16-column
// groups do not split in two, or whose SiLU gate / up pairs must stay in one wave).
// Column tiles of any multiple of 16 read the same packed [N/128][K/64][128 x 64] weight
// blocks: each 1-KiB DMA piece is 8 packed rows, which never straddle a 128-row block.
// A wave whose share of a step's pieces is short re-issues its last piece (the same bytes
// to the same LDS rows), so every issuing wave counts the same DMAs per step in vmcnt.
// MOE (K14m, launch_moe_dgemm): 1 = the grouped gate_up, A rows gathered from the tokens
// (sorted_ids[r] / topk), 2 = the grouped down, output rows scattered to pair order; the
// workgroup's row block names its expert (block_expert), whose packed weights it streams.
template <typename T, int BM, int BN, int EPI, bool PK, int ABL = ABL_NONE, int LDW = 0,
          int WN = 2, int MOE = 0, int NS = DG_NS>
__global__ __launch_bounds__(DG_THREADS + LDW * 64, 1) void dgemm_kernel(
    void* __restrict__ Cv, const T* __restrict__ X, const T* __restrict__ W, int M, int N,
    int K, int64_t ldx, int S, int MB, int64_t slice_stride, int xmap, int wt, DgAux aux) {
  static_assert(WN == 1 || WN == 2 || WN == 4, "waves along N");
  constexpr int WM = 8 / WN;                      // MFMA waves along M
  constexpr int MT = BM / WM / 16;                // 16-row MFMA tiles per wave
  constexpr int NT = BN / WN / 16;                // 16-col MFMA tiles per wave
  static_assert(MT * WM * 16 == BM && NT * WN * 16 == BN, "wave tiling");
  static_assert(EPI != EPI_SILU || NT % 2 == 0, "SiLU gate / up pairs inside one wave");
  constexpr int NIW = LDW > 0 ? LDW : 8;          // waves issuing DMAs
  constexpr int PA = BM / 8, PB = BN / 8;         // 1-KiB pieces per step
  constexpr int LA = (PA + NIW - 1) / NIW, LB = (PB + NIW - 1) / NIW;   // per issuing wave
  static_assert(PA % NIW == 0 && (PK || PB % NIW == 0), "DMA split");
  constexpr int L = LA + LB;
  constexpr int A_BYTES = BM * DG_ROWB, SLOT_BYTES = (BM + BN) * DG_ROWB;
  static_assert(NS >= 3 && NS <= 6 && NS * SLOT_BYTES <= 163840, "LDS ring: 3..6 slots, 160 KiB");
  // ONE shared array for the whole ring (a second __shared__ object can make hipcc emit a
  // vmcnt(0) before the first ds_read of every step)
  __shared__ __attribute__((aligned(16))) char lds[NS * SLOT_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool loader = LDW > 0 && wave >= 8;
  const bool consumer = LDW == 0 || wave < 8;
  const int iw = LDW > 0 ? wave - 8 : wave;       // index among the issuing waves
  // (WN = 4: a 2 x 4 wave grid, the 96-row K14m blocks: 48 rows x 32 columns per wave)
  const int wm = (wave & 7) / WN, wn = wave % WN;
  int z, j, mb, nb;
  if (xmap) {
    // XCD-paired row blocks (host: S | 8, (N / BN) % (8 / S) == 0): workgroups L and L + 8
    // -- one XCD under round-robin placement (speed only, never correctness) -- take the
    // row blocks of the SAME weight columns and K-slice, so the second read of each weight
    // tile is an L2 hit instead of an HBM (or Infinity Cache) read
    const int r8 = blockIdx.x & 7, q = blockIdx.x >> 3, cpg = 8 / S;
    z = r8 % S;
    mb = q % MB;
    nb = (q / MB) * cpg + r8 / S;
    j = nb * MB + mb;
  } else {
    z = blockIdx.x % S;
    j = blockIdx.x / S;
    mb = j % MB;
    nb = j / MB;
  }
  const int m0 = mb * BM;
  if constexpr (MOE != 0) {
    // row blocks past the ones moe_align filled, or of another rank's experts: no work
    // (workgroup-uniform, before any barrier)
    if (mb >= aux.meta[0]) return;
    const int e = aux.block_expert[mb];
    if (e < 0) return;
    W += (int64_t)e * aux.wexp;
  }

  // ---- DMA sources: lane l of instruction i fills LDS row 8i + l/8, 16-B slot l%8 with
  // global chunk (l%8) ^ (row%8)  (row%8 == l/8): the swizzle lives in the source address
  const int drow = lane >> 3, dchunk = (lane & 7) ^ drow;
  const T* a_src[LA];
#pragma unroll
  for (int t = 0; t < LA; ++t) {
    int r = m0 + (iw * LA + t) * 8 + drow;
    // padded rows re-read the last row; the MFMA waves of a loader-wave kernel (iw < 0)
    // never issue, their (clamped) rows are never read
    r = r < M ? (r < 0 ? 0 : r) : M - 1;
    if constexpr (MOE == 1) {
      // the token of sorted pair row r; a padding row (p == npairs) re-reads the block's
      // first pair's token (an L2 hit; its output row is never stored).  Only the waves
      // that issue DMAs read the row map.
      if (LDW == 0 || loader) {
        int p = aux.sorted_ids[r];
        if (p >= aux.npairs) p = aux.sorted_ids[m0];
        r = p / aux.topk;
      }
    }
    a_src[t] = X + (int64_t)r * ldx + dchunk * 8;
  }
  const int nk_all = K / DG_BK;
  const T* b_src[LB];
#pragma unroll
  for (int t = 0; t < LB; ++t) {
    if constexpr (PK) {
      // packed [N/128][K/BK][128*BK], swizzle baked in: piece p = 8 packed rows starting at
      // row n = nb * BN + 8p, inside 128-row block n / 128 (BN == 128: linear pieces)
      const int p = min(iw * LB + t, PB - 1);
      const int n = nb * BN + 8 * p;
      b_src[t] = W + (int64_t)(n >> 7) * nk_all * (128 * DG_BK) + (n & 127) * DG_BK + lane * 8;
    } else {
      const int r = (iw * LB + t) * 8 + drow;
      b_src[t] = W + weight_row<BN, EPI>(nb, r, N) * K + dchunk * 8;
    }
  }

  const int kb0 = (int)((int64_t)nk_all * z / S);
  const int nk = (int)((int64_t)nk_all * (z + 1) / S) - kb0;
  // each workgroup starts its walk at its own step
  const int rot = nk >= 4 ? (int)(((int64_t)j * 37) % nk) : 0;

  auto issue = [&](int slot, int step) {
    if constexpr (ABL == ABL_NO_DMA) return;
    if (LDW > 0 && !loader) return;
    char* sa = lds + slot * SLOT_BYTES;
    char* sb = sa + A_BYTES;
    int st = step + rot;
    st = st >= nk ? st - nk : st;
    const int kb = kb0 + st;
    if constexpr (ABL != ABL_NO_A) {
#pragma unroll
      for (int t = 0; t < LA; ++t)
        glds16<0>(a_src[t] + kb * DG_BK, sa + (iw * LA + t) * 1024);
    }
    if constexpr (ABL != ABL_NO_B) {
      const int64_t bo = PK ? (int64_t)kb * (128 * DG_BK) : (int64_t)kb * DG_BK;
#pragma unroll
      for (int t = 0; t < LB; ++t)
        glds16<2>(b_src[t] + bo, sb + min(iw * LB + t, PB - 1) * 1024);
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int a_row0 = wm * (BM / WM) + fr;
  const int b_row0 = wn * (BN / WN) + fr;
  // EPI_OUT / EPI_SILU with a row scale (the norm-free layer's rsqrt of the producer's
  // row norms): the lane's rows' scales, loaded before the K walk hides their latency
  float rsv[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) rsv[i][e] = 1.f;
  if constexpr (EPI == EPI_OUT || EPI == EPI_SILU) {
    if (aux.rsc != nullptr && consumer) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          rsv[i][e] = aux.rsc[min(m0 + wm * (BM / WM) + i * 16 + fq * 4 + e, M - 1)];
    }
  }

  // NS-slot ring: NS - 1 steps issued ahead, NS - 2 of them in flight behind the one read
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) issue(p, p);
  int slot = 0;
  for (int it = 0; it < nk; ++it) {
    // step `it` must have landed; the (up to NS - 2) younger steps may stay in flight
    if (LDW > 0 && !loader) {
      // MFMA waves have no DMAs of their own: the barrier below orders them after the
      // loaders' waits
    } else if constexpr (ABL == ABL_NO_A) {
      wait_younger<LB, NS - 2>(nk - 1 - it);
    } else if constexpr (ABL == ABL_NO_B) {
      wait_younger<LA, NS - 2>(nk - 1 - it);
    } else if constexpr (ABL != ABL_NO_DMA) {
      wait_younger<L, NS - 2>(nk - 1 - it);
    }
    __builtin_amdgcn_s_barrier();
    // the slot read in iteration it - 1 (every wave has passed the barrier since)
    if (it + NS - 1 < nk) issue(slot == 0 ? NS - 1 : slot - 1, it + NS - 1);
    const char* sa = lds + slot * SLOT_BYTES;
    const char* sb = sa + A_BYTES;
    slot = slot == NS - 1 ? 0 : slot + 1;
    if constexpr (ABL == ABL_NO_MFMA) continue;
    if (!consumer) continue;
#pragma unroll
    for (int ks = 0; ks < DG_BK / 32; ++ks) {
      const int c = ks * 4 + fq;
      Pack8<T> af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int r = a_row0 + i * 16;
        af[i].u = *reinterpret_cast<const u32x4*>(sa + r * DG_ROWB + (swz(r, c) << 4));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int r = b_row0 + n * 16;
        bfr[n].u = *reinterpret_cast<const u32x4*>(sb + r * DG_ROWB + (swz(r, c) << 4));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[i][n] = mfma16x16x32(af[i].v, bfr[n].v, acc[i][n]);
    }
  }

  // ---- epilogue: lane holds C[4*fq + e][fr] of every 16x16 tile
  if constexpr (EPI == EPI_OUT || EPI == EPI_SILU) {
    // one wait for the row scales here, unconditionally: waited for inside the per-row
    // branches below, each row's wait also drained the previous rows' stores
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(rsv[i][e]));
  }
  if (!consumer) return;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int row = m0 + wm * (BM / WM) + i * 16 + fq * 4 + e;
      if (row >= M) continue;
      if constexpr (MOE == 2) {
        row = aux.sorted_ids[row];                // scattered back to pair order
        if (row >= aux.npairs) continue;          // a padding row
      }
      if constexpr (EPI == EPI_PARTIAL) {
        float* cp = reinterpret_cast<float*>(Cv) + z * slice_stride + (int64_t)row * N +
                    nb * BN + wn * (BN / WN) + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) store_partial(cp + n * 16, acc[i][n][e], wt);
      } else if constexpr (EPI == EPI_OUT) {
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * N + nb * BN + wn * (BN / WN) + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) cp[n * 16] = from_f<T>(acc[i][n][e] * rsv[i][e]);
      } else {
        const int I = N >> 1;
        const float sc = rsv[i][e];
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * I + nb * (BN / 2) +
                wn * (BN / WN / 2) + fr;
#pragma unroll
        for (int n = 0; n < NT; n += 2)
          cp[(n >> 1) * 16] = from_f<T>(silu_f(acc[i][n][e] * sc) * (acc[i][n + 1][e] * sc));
      }
    }
  }
}

// Split-loader variant (packed weights only).  With every DMA of a step in one in-order
// queue, the activation pieces (L2 hits) wait behind the weight pieces (HBM misses), so a
// 3-slot ring of 48 KB caps the per-CU intake at ~96 KB per HBM latency (~48 GB/s, what
// the single-queue kernels measure).  Here the queues are separate waves:
//   waves 0-7   MFMA consumers (as dgemm_kernel),
//   waves 8-11  activation loaders: a 3-slot A ring (one step in flight behind the read),
//   waves 12-13 weight loaders: an NB-slot B ring (NB - 2 steps in flight: 32-48 KB of
//               HBM reads per CU at all times);
// each loader group waits only on its own vmcnt, and one s_barrier per step joins all 14.
template <typename T, int BM, int BN, int EPI, int NB, int NA = 3>
__global__ __launch_bounds__(896, 1) void dgemm_sl_kernel(
    void* __restrict__ Cv, const T* __restrict__ X, const T* __restrict__ W, int M, int N,
    int K, int64_t ldx, int S, int MB, int64_t slice_stride, int wt) {
  constexpr int MT = BM / 4 / 16, NT = BN / 2 / 16;
  static_assert(NA >= 2 && NB >= 2, "rings of at least two slots");
  constexpr int LA = BM / 8 / 4, LB = BN / 8 / 2;   // DMAs per A / B loader wave per step
  constexpr int A_SLOT = BM * DG_ROWB, B_SLOT = BN * DG_ROWB;
  static_assert(NA * A_SLOT + NB * B_SLOT <= 163840, "LDS rings exceed 160 KiB");
  __shared__ __attribute__((aligned(16))) char lds[NA * A_SLOT + NB * B_SLOT];
  char* const ring_a = lds;
  char* const ring_b = lds + NA * A_SLOT;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int z = blockIdx.x % S;
  const int j = blockIdx.x / S;
  const int mb = j % MB, nb = j / MB;
  const int m0 = mb * BM;
  const int nk_all = K / DG_BK;
  const int kb0 = (int)((int64_t)nk_all * z / S);
  const int nk = (int)((int64_t)nk_all * (z + 1) / S) - kb0;
  const int rot = nk >= 4 ? (int)(((int64_t)j * 37) % nk) : 0;
  auto kstep = [&](int step) {
    int st = step + rot;
    return kb0 + (st >= nk ? st - nk : st);
  };

  if (wave >= 8) {
    // ------------------------------------------------------------------ loaders
    const bool is_a = wave < 12;
    const int iw = is_a ? wave - 8 : wave - 12;
    const int drow = lane >> 3, dchunk = (lane & 7) ^ drow;
    const T* src[LA > LB ? LA : LB];
    if (is_a) {
#pragma unroll
      for (int t = 0; t < LA; ++t) {
        int r = m0 + (iw * LA + t) * 8 + drow;
        r = r < M ? r : M - 1;
        src[t] = X + (int64_t)r * ldx + dchunk * 8;
      }
    } else {
#pragma unroll
      for (int t = 0; t < LB; ++t)
        src[t] = W + (int64_t)nb * nk_all * (BN * DG_BK) + (iw * LB + t) * 512 + lane * 8;
    }
    auto issue_a = [&](int step) {
      char* d = ring_a + (step % NA) * A_SLOT + iw * LA * 1024;
      const int ko = kstep(step) * DG_BK;
#pragma unroll
      for (int t = 0; t < LA; ++t) glds16<0>(src[t] + ko, d + t * 1024);
    };
    auto issue_b = [&](int step) {
      char* d = ring_b + (step % NB) * B_SLOT + iw * LB * 1024;
      const int64_t bo = (int64_t)kstep(step) * (BN * DG_BK);
#pragma unroll
      for (int t = 0; t < LB; ++t) glds16<2>(src[t] + bo, d + t * 1024);
    };
    if (is_a) {
      for (int p = 0; p < NA - 1 && p < nk; ++p) issue_a(p);
    } else {
      for (int p = 0; p < NB - 1 && p < nk; ++p) issue_b(p);
    }
    for (int it = 0; it < nk; ++it) {
      if (is_a) {
        wait_younger<LA, NA - 2>(nk - 1 - it);
      } else {
        wait_younger<LB, NB - 2>(nk - 1 - it);
      }
      __builtin_amdgcn_s_barrier();
      if (is_a) {
        if (it + NA - 1 < nk) issue_a(it + NA - 1);
      } else {
        if (it + NB - 1 < nk) issue_b(it + NB - 1);
      }
    }
    return;
  }

  // -------------------------------------------------------------------- MFMA waves
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int a_row0 = wm * (BM / 4) + fr;
  const int b_row0 = wn * (BN / 2) + fr;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < nk; ++it) {
    __builtin_amdgcn_s_barrier();
    const char* sa = ring_a + (it % NA) * A_SLOT;
    const char* sb = ring_b + (it % NB) * B_SLOT;
#pragma unroll
    for (int ks = 0; ks < DG_BK / 32; ++ks) {
      const int c = ks * 4 + fq;
      Pack8<T> af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int r = a_row0 + i * 16;
        af[i].u = *reinterpret_cast<const u32x4*>(sa + r * DG_ROWB + (swz(r, c) << 4));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int r = b_row0 + n * 16;
        bfr[n].u = *reinterpret_cast<const u32x4*>(sb + r * DG_ROWB + (swz(r, c) << 4));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[i][n] = mfma16x16x32(af[i].v, bfr[n].v, acc[i][n]);
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = m0 + wm * (BM / 4) + i * 16 + fq * 4 + e;
      if (row >= M) continue;
      if constexpr (EPI == EPI_PARTIAL) {
        float* cp = reinterpret_cast<float*>(Cv) + z * slice_stride + (int64_t)row * N +
                    nb * BN + wn * (BN / 2) + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) store_partial(cp + n * 16, acc[i][n][e], wt);
      } else if constexpr (EPI == EPI_OUT) {
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * N + nb * BN + wn * (BN / 2) + fr;
#pragma unroll
        for (int n = 0; n < NT; ++n) cp[n * 16] = from_f<T>(acc[i][n][e]);
      } else {
        const int I = N >> 1;
        T* cp = reinterpret_cast<T*>(Cv) + (int64_t)row * I + nb * (BN / 2) + wn * (BN / 4) + fr;
#pragma unroll
        for (int n = 0; n < NT; n += 2)
          cp[(n >> 1) * 16] = from_f<T>(silu_f(acc[i][n][e]) * acc[i][n + 1][e]);
      }
    }
  }
}

template <typename T, int BM, int BN, int NB, int NA = 3>
void dgemm_sl_cfg(int epi, void* C, const void* X, const void* W, int M, int N, int K,
                  int64_t ldx, int S, int64_t ss, hipStream_t s) {
  const int MB = (M + BM - 1) / BM;
  const dim3 grid((unsigned)(MB * (N / BN) * S));
#define DG_SL(E)                                                                       \
  dgemm_sl_kernel<T, BM, BN, E, NB, NA><<<grid, 896, 0, s>>>(C, (const T*)X, (const T*)W, M, \
                                                              N, K, ldx, S, MB, ss, \
                                                              partial_wt())
  if (epi == EPI_PARTIAL) DG_SL(EPI_PARTIAL);
  else if (epi == EPI_OUT) DG_SL(EPI_OUT);
  else DG_SL(EPI_SILU);
#undef DG_SL
}

// Re-layout W [N, K] (EPI_SILU: merged [gate; up]) into the packed tiles the PK kernels
// stream: P[nb][kb][r][pos] (16-B chunks) = W[weight_row(nb, r)][kb*64 + (pos ^ r%8)*8 ..]
template <typename T, int BN, int EPI>
__global__ __launch_bounds__(256) void dgemm_pack_kernel(T* __restrict__ P,
                                                         const T* __restrict__ W, int N,
                                                         int K) {
  const int nk_all = K / DG_BK;
  const int64_t chunk = (int64_t)blockIdx.x * 256 + threadIdx.x;   // one 16-B chunk
  const int64_t total = (int64_t)N * K / 8;
  if (chunk >= total) return;
  const int pos = (int)(chunk & 7);
  const int64_t rowi = chunk >> 3;                 // (nb, kb, r) flattened
  const int r = (int)(rowi % BN);
  const int64_t t = rowi / BN;
  const int kb = (int)(t % nk_all);
  const int nb = (int)(t / nk_all);
  const int64_t src = weight_row<BN, EPI>(nb, r, N) * K + kb * DG_BK + swz(r, pos) * 8;
  reinterpret_cast<u32x4*>(P)[chunk] = *reinterpret_cast<const u32x4*>(W + src);
}

// Tile table: id -> (BM, BN, packed weights); ids 6, 7 = 4, 5 with 4 loader waves;
// ids 8, 9 = split loaders (dgemm_sl_kernel) 256 x 128 with a 4- / 128 x 128 with a 6-slot
// weight ring.  (A 2-slot activation ring with the LDS given to a 6- / 8-slot weight ring
// measured 5-10 % slower on every shape: profiles/k9m_dgemm_bench_r2_sweep.jsonl.)
// id 10 = 5 with XCD-paired row blocks (the two 128-row blocks of a column tile on one XCD:
// o_proj at M = 256, S = 4 17.4 vs 18.9 us).  128 x 256 tiles (weights packed 256 wide,
// 3-slot ring of 48 KB) measured 20-30 % slower than the split loaders on gate_up and
// down, with or without the pairing (profiles/k9m_dgemm_bench_r2_sweep.jsonl).
// K9v (activations in a VGPR ring, round 3) measured slower on every shape and lives in
// tools/research/ (its own library), out of the engine's.
// ids 11-14 (round 6): packed column tiles of 64 / 80 / 112 for the narrow shards of a
// TP = 8 rank (profiles/README.md "Round 6: full-grid K9m tiles"):
//   11  256 x  64, 8 issuing waves           70B TP = 8 o at S = 2 (128 tiles)
//   12  256 x  80, 4 loaders, WN = 1         70B TP = 8 qkv (N 1280: 16 tiles x S 16)
//   13  256 x 112, 4 loaders, WN = 1         70B TP = 8 gate_up slices (64 tiles x S 4)
//   14  128 x  64, 8 issuing waves, XCD      70B TP = 8 o at S = 1, ahead of its all-reduce
// Measured and not kept: 256 x 96 (Llama-3-8B qkv at S = 4, 256 workgroups), 128 x 224 with
// the SiLU epilogue (gate_up at S = 1, 256 workgroups) and 128 x 192: filling all 256 CUs
// did not beat the 192 / 224-workgroup 256 x 128 tiles at M = 256 (the extra activation
// re-reads of narrower tiles cost more than the idle CUs: profiles/k9m_full_grid_r6.jsonl).
// Also measured and not kept: 64-row blocks over the whole K (no split-K partials), the
// four row blocks of a column tile XCD-grouped, with a 3- or 6-slot ring (NS): 64 x 128 /
// 64 x 96 qkv 35.0 / 36.3 us against 28.0 us for 256 x 128 at S = 5 with its reduction,
// o 25.9-27.1 against 23.6, down 72-121 against 42.9 (profiles/k9m_64row_fullk_r6.jsonl):
// every workgroup then takes in a whole-K strip of weights AND activations, and the
// per-CU intake (bytes in flight / latency), not HBM, is what bounds K9m at M = 256.
struct DgCfg {
  int bm, bn, pk, ldw, wn, xmap, ns;
};
constexpr int kNumCfgs = 15;
static const DgCfg kCfg[kNumCfgs] = {
    {256, 128, 0, 0, 2, 0, 3}, {256, 64, 0, 0, 2, 0, 3}, {128, 128, 0, 0, 2, 0, 3},
    {128, 64, 0, 0, 2, 0, 3},  {256, 128, 1, 0, 2, 0, 3}, {128, 128, 1, 0, 2, 0, 3},
    {256, 128, 1, 4, 2, 0, 3}, {128, 128, 1, 4, 2, 0, 3}, {256, 128, 1, 0, 2, 0, 3},
    {128, 128, 1, 0, 2, 0, 3}, {128, 128, 1, 0, 2, 1, 3}, {256, 64, 1, 0, 2, 0, 3},
    {256, 80, 1, 4, 1, 0, 3},  {256, 112, 1, 4, 1, 0, 3}, {128, 64, 1, 0, 2, 1, 3}};

// epilogues a tile runs: bit EPI (PARTIAL / OUT always; SILU where each wave holds whole
// gate / up 16-column pairs)
template <int BN, int WN>
constexpr int dg_epis() {
  return (1 << EPI_PARTIAL) | (1 << EPI_OUT) |
         ((BN % 32 == 0 && (BN / WN / 16) % 2 == 0) ? (1 << EPI_SILU) : 0);
}

template <typename T, int BM, int BN, bool PK, int LDW = 0, int WN = 2, int NS = DG_NS>
void dgemm_cfg(int epi, void* C, const void* X, const void* W, int M, int N, int K, int64_t ldx,
               int S, int64_t ss, const DgAux& aux, hipStream_t s, int xmap = 0) {
  const int MB = (M + BM - 1) / BM;
  const dim3 grid((unsigned)(MB * (N / BN) * S));
  // the XCD pairing needs S | 8 and whole groups of 8 / S column tiles
  const int xm = (xmap && MB > 1 && 8 % S == 0 && (N / BN) % (8 / S) == 0) ? 1 : 0;
  constexpr int E = dg_epis<BN, WN>();
#define DG_LAUNCH(EP)                                                                       \
  dgemm_kernel<T, BM, BN, EP, PK, ABL_NONE, LDW, WN, 0, NS>                                 \
      <<<grid, DG_THREADS + LDW * 64, 0, s>>>(                                              \
      C, (const T*)X, (const T*)W, M, N, K, ldx, S, MB, ss, xm, partial_wt(), aux)
  if (epi == EPI_PARTIAL) DG_LAUNCH(EPI_PARTIAL);
  else if (epi == EPI_OUT) DG_LAUNCH(EPI_OUT);
  else if (epi == EPI_SILU) {
    if constexpr ((E >> EPI_SILU) & 1) DG_LAUNCH(EPI_SILU);
  }
#undef DG_LAUNCH
}

template <typename T>
void dgemm_t(int cfg, int epi, void* C, const void* X, const void* W, int M, int N, int K,
             int64_t ldx, int S, int64_t ss, const DgAux& a, hipStream_t s) {
  switch (cfg) {
    case 0: dgemm_cfg<T, 256, 128, false>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 1: dgemm_cfg<T, 256, 64, false>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 2: dgemm_cfg<T, 128, 128, false>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 3: dgemm_cfg<T, 128, 64, false>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 4: dgemm_cfg<T, 256, 128, true>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 5: dgemm_cfg<T, 128, 128, true>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 6: dgemm_cfg<T, 256, 128, true, 4>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 7: dgemm_cfg<T, 128, 128, true, 4>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 8: dgemm_sl_cfg<T, 256, 128, 4>(epi, C, X, W, M, N, K, ldx, S, ss, s); break;
    case 9: dgemm_sl_cfg<T, 128, 128, 6>(epi, C, X, W, M, N, K, ldx, S, ss, s); break;
    case 10: dgemm_cfg<T, 128, 128, true>(epi, C, X, W, M, N, K, ldx, S, ss, a, s, 1); break;
    case 11: dgemm_cfg<T, 256, 64, true>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 12: dgemm_cfg<T, 256, 80, true, 4, 1>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 13: dgemm_cfg<T, 256, 112, true, 4, 1>(epi, C, X, W, M, N, K, ldx, S, ss, a, s); break;
    case 14: dgemm_cfg<T, 128, 64, true>(epi, C, X, W, M, N, K, ldx, S, ss, a, s, 1); break;
    default: break;                 // the host checks cfg < dgemm_num_cfgs()
  }
}

int dg_cfg_epis(int cfg) {
  switch (cfg) {
    case 8: case 9: return (1 << EPI_PARTIAL) | (1 << EPI_OUT) | (1 << EPI_SILU);
    case 12: return dg_epis<80, 1>();
    case 13: return dg_epis<112, 1>();
    case 1: case 3: case 11: case 14: return dg_epis<64, 2>();
    default: return dg_epis<128, 2>();
  }
}

template <typename T, int BM, int BN, int MOE>
void moe_dgemm_t(int epi, void* C, const void* A, const void* Wp, int max_rows, int N, int K,
                 int64_t lda, int S, int64_t ss, const DgAux& aux, hipStream_t s) {
  // 1-D grid, row blocks fastest: a column tile's blocks (one expert each) are dispatched
  // together, so each XCD's L2 holds the activation rows of the experts it is dealt.
  // BM = 96 (a decode step's ~64 +- 3 sd pairs per expert in ONE block, a third fewer
  // padding rows than 128): 2 x 4 MFMA waves and 4 loader waves (12 A pieces per step).
  // BN = 256 (2 x 4 waves of 64 columns): a block's gathered rows are re-read by half as
  // many column tiles -- at ~64 rows per expert the activation stream is 0.375 of the
  // weight stream instead of 0.75.
  constexpr int WN = (BN == 256 || BM == 96) ? 4 : 2;
  constexpr int LDW = (BM == 96 || (BN == 256 && BM == 128)) ? 4 : 0;
  const int MB = max_rows / BM;
  const dim3 grid((unsigned)(MB * (N / BN) * S));
#define MOE_LAUNCH(EP)                                                                      \
  dgemm_kernel<T, BM, BN, EP, true, ABL_NONE, LDW, WN, MOE>                                 \
      <<<grid, DG_THREADS + LDW * 64, 0, s>>>(C, (const T*)A, (const T*)Wp, max_rows, N, K, \
                                              lda, S, MB, ss, 0, partial_wt(), aux)
  if constexpr (MOE == 1) {
    MOE_LAUNCH(EPI_SILU);
  } else {
    if (epi == EPI_PARTIAL) MOE_LAUNCH(EPI_PARTIAL);
    else MOE_LAUNCH(EPI_OUT);
  }
#undef MOE_LAUNCH
}

}  // namespace

void launch_moe_dgemm(int dtype, int mode, void* C, const void* A, const void* Wp, int max_rows,
                      int N, int K, int64_t lda, int S, int64_t slice_stride, int bm, int bn,
                      const int* sorted_ids, const int* block_expert, const int* meta,
                      int npairs, int topk, hipStream_t s) {
  DgAux aux{};
  aux.sorted_ids = sorted_ids;
  aux.block_expert = block_expert;
  aux.meta = meta;
  aux.npairs = npairs;
  aux.topk = topk;
  aux.wexp = (int64_t)N * K;                     // one expert's packed weight, elements
  const int epi = mode == 1 ? EPI_SILU : S > 1 ? EPI_PARTIAL : EPI_OUT;
#define MOE_BN(TT, BMM, MODE)                                                               \
  if (bn == 256) moe_dgemm_t<TT, BMM, 256, MODE>(epi, C, A, Wp, max_rows, N, K, lda, S, slice_stride, aux, s); \
  else moe_dgemm_t<TT, BMM, 128, MODE>(epi, C, A, Wp, max_rows, N, K, lda, S, slice_stride, aux, s);
#define MOE_BM(TT, MODE)                                                                    \
  if (bm == 64) { MOE_BN(TT, 64, MODE) }                                                    \
  else if (bm == 96) { MOE_BN(TT, 96, MODE) }                                               \
  else { MOE_BN(TT, 128, MODE) }
#define MOE_T(TT)                                                                           \
  if (mode == 1) {                                                                          \
    MOE_BM(TT, 1)                                                                           \
  } else {                                                                                  \
    MOE_BM(TT, 2)                                                                           \
  }
  if (dtype == DT_BF16) { MOE_T(bf16) } else { MOE_T(f16) }
#undef MOE_T
#undef MOE_BM
#undef MOE_BN
}

int dgemm_num_cfgs() { return kNumCfgs; }
void dgemm_cfg_info(int cfg, int* bm, int* bn, int* packed) {
  *bm = kCfg[cfg].bm;
  *bn = kCfg[cfg].bn;
  *packed = kCfg[cfg].pk;
}
int dgemm_cfg_epis(int cfg) { return cfg >= 0 && cfg < kNumCfgs ? dg_cfg_epis(cfg) : 0; }
int dgemm_block_k() { return DG_BK; }
// the split-loader configs (8, 9) have no fan-in or row-scale epilogue
bool dgemm_cfg_has_aux(int cfg) { return cfg != 8 && cfg != 9; }

void launch_dgemm(int dtype, int cfg, int epi, void* C, const void* X, const void* W, int M,
                  int N, int K, int64_t ldx, int S, int64_t slice_stride, const DgAux& aux,
                  hipStream_t s) {
  if (dtype == DT_BF16) dgemm_t<bf16>(cfg, epi, C, X, W, M, N, K, ldx, S, slice_stride, aux, s);
  else dgemm_t<f16>(cfg, epi, C, X, W, M, N, K, ldx, S, slice_stride, aux, s);
}

void launch_dgemm_pack(int dtype, bool silu, void* P, const void* W, int N, int K,
                       hipStream_t s) {
  const int64_t chunks = (int64_t)N * K / 8;
  const dim3 grid((unsigned)((chunks + 255) / 256));
#define PACK(T, E) \
  dgemm_pack_kernel<T, 128, E><<<grid, 256, 0, s>>>((T*)P, (const T*)W, N, K)
  if (dtype == DT_BF16) {
    if (silu) { PACK(bf16, EPI_SILU); }
    else { PACK(bf16, EPI_OUT); }
  } else {
    if (silu) { PACK(f16, EPI_SILU); }
    else { PACK(f16, EPI_OUT); }
  }
#undef PACK
}

// 256 x 128 packed tile with one part removed, fp32 slices (profiling only)
void launch_dgemm_ablate(int mode, float* C, const void* X, const void* W, int M, int N, int K,
                         int64_t ldx, int S, int64_t ss, hipStream_t s) {
  const int MB = (M + 255) / 256;
  const dim3 grid((unsigned)(MB * (N / 128) * S));
#define AB(MODE)                                                                     \
  dgemm_kernel<bf16, 256, 128, EPI_PARTIAL, true, MODE><<<grid, DG_THREADS, 0, s>>>( \
      C, (const bf16*)X, (const bf16*)W, M, N, K, ldx, S, MB, ss, 0, partial_wt(), DgAux{})
  switch (mode) {
    case ABL_NO_MFMA: AB(ABL_NO_MFMA); break;
    case ABL_NO_DMA: AB(ABL_NO_DMA); break;
    case ABL_NO_A: AB(ABL_NO_A); break;
    case ABL_NO_B: AB(ABL_NO_B); break;
    default: AB(ABL_NONE); break;
  }
#undef AB
}

}  // namespace kgc
