// K9r: full-K "ring" decode GEMM for gfx950, M = 32..512 rows (the batch-256 decode step).
//
//   C[M, N] = X[M, K] . W[N, K]^T      bf16 in, fp32 MFMA accumulation
//
// Why a second mid-batch kernel beside K9m (gemm_decode.hip).  K9m fills the chip on the
// narrow projections (o: N = 4096, qkv: 6144) by splitting K, and the fp32 K-slices it
// writes (o at S = 4: 16.8 MB, qkv at S = 5: 31.5 MB, down at S = 8: 33.5 MB per layer)
// cost as much HBM traffic as the weights, plus a read-back in the consumer.  K9r instead
// sizes the OUTPUT tile so that ~256 tiles cover the whole [M, N] output (o at M = 256:
// 64 x 64, qkv: 64 x 96, gate_up + SiLU: 128 x 224) and walks the whole K in one
// workgroup: no partials, the epilogue writes bf16 straight to the consumer.
//
// A workgroup's intake is then (BM + BN) x K x 2 bytes (1 MB for o), which the per-CU
// L1/LDS-DMA path (~64 B/clk) can only sustain with many bytes in flight: every K-step
// (BK = 64) is one ring slot of (BM + BN) x 128 B in LDS, and the ring is as deep as LDS
// allows (NS slots, NS - 1 K-steps in flight: 8 x 16 KB for 64 x 64, 7 x 20 KB for
// 64 x 96), retired with counted `s_waitcnt vmcnt` and ONE raw s_barrier per step.
//   * both operands by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction) into
//     128-B rows with the 16-B chunk XOR swizzle (chunk ^ row % 8) applied on the SOURCE
//     address, conflict-free ds_read_b128 fragment reads (same image as K9m);
//   * weights pre-packed once at load time as [N/G][K/64][G x 64] (G-row groups, swizzle
//     baked in; G = BN makes every K-step of a column tile one contiguous block);
//   * XCD-aware tile order: workgroups b, b+8, b+16, ... share an XCD (round-robin
//     dispatch; speed only, never correctness), so the BM-row blocks of one weight column
//     tile run side by side on one XCD and the weight tile is fetched from HBM once and
//     served from that XCD's L2 to the others; with split-K the K-slice is fixed per XCD;
//   * optional loader waves (LW): the MFMA waves never issue a DMA or wait on vmcnt;
//   * epilogues: OUT (bf16 tile), SILU (merged [gate; up] weight packed with 8-row
//     gate / up interleave inside every 16-row group: lane fr < 8 holds gate, its xor-8
//     partner the matching up column, one DPP-free shuffle per element; any BN % 16 == 0
//     works, e.g. 224 = 112 gate + 112 up columns, 256 tiles for Llama-3-8B's 14336),
//     PARTIAL (fp32 K-slices, write-through, for the long-K down projection where a
//     2-4 way split still pays).
// Reference parity: SURVEY.md §2.5 K9 (decode GEMMs of the vLLM engine image the
// reference deploys, /root/reference/values-01-minimal-example2.yaml:6-7).
#include "common.h"
#include "launch.h"
#include "research.h"
#include <cstdlib>

namespace kgc {

namespace {

constexpr int RG_BK = 64, RG_ROWB = 128;     // K-step, LDS row bytes (BK bf16)
enum { RG_PARTIAL = 0, RG_OUT = 1, RG_SILU = 2 };

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

template <int AUX>
__device__ __forceinline__ void rg_glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_wave_base, 16, 0, AUX);
}

template <int N>
__device__ __forceinline__ void rg_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most min(Y, younger) K-steps of L DMAs each are still in flight
template <int L, int Y>
__device__ __forceinline__ void rg_wait(int younger) {
  if constexpr (Y == 0) {
    rg_vmcnt<0>();
  } else {
    if (younger >= Y) { rg_vmcnt<L * Y>(); return; }
    rg_wait<L, Y - 1>(younger);
  }
}

__device__ __forceinline__ float rg_silu(float g) { return g / (1.f + __expf(-g)); }
__device__ __forceinline__ int rg_swz(int row, int chunk) { return chunk ^ (row & 7); }

// packed row p of a merged [gate; up] weight (I = N / 2 outputs): in every 16-row group,
// rows 0-7 are gate columns 8g..8g+7, rows 8-15 the up columns of the same outputs
__device__ __forceinline__ int64_t rg_silu_row(int64_t p, int I) {
  const int64_t g = p >> 4;
  const int i = (int)(p & 15);
  return i < 8 ? g * 8 + i : I + g * 8 + (i - 8);
}

// CW = WM * WN MFMA waves and LW loader waves.  The weight operand is packed with
// G = BN (ring_pack): every K-step of a column tile is one contiguous BN x 128 B block.
// NSB = 0: one ring of NS slots, each holding a K-step of both operands, every loader
// issuing both.  NSB > 0 (split rings): the activation ring has NS slots and the weight
// ring NSB slots of their own; loader waves [0, LW/2) move activations, [LW/2, LW)
// weights, each group waiting only on its own DMAs -- the weight stream (HBM, long
// latency, small slots) can run many more K-steps ahead than the activation stream (L2,
// large slots) within the same 160 KiB.
template <int BM, int BN, int WM, int WN, int LW, int NS, int WAUX, int EPI, int NSB = 0>
__global__ __launch_bounds__((WM * WN + LW) * 64, 1) void ring_gemm_kernel(
    void* __restrict__ Cv, const bf16* __restrict__ X, const bf16* __restrict__ Wp, int M,
    int N, int K, int64_t ldx, int S, int MB, int64_t slice_stride, int xmap, int wt, int abl) {
  constexpr int CW = WM * WN;
  constexpr bool SPLIT = NSB > 0;
  static_assert(LW >= 1 && (!SPLIT || LW % 2 == 0), "dedicated loader waves");
  constexpr int LWA = SPLIT ? LW / 2 : LW, LWB = SPLIT ? LW / 2 : LW;
  constexpr int D = NS - 1;                       // activation K-steps in flight
  constexpr int DB = SPLIT ? NSB - 1 : D;         // weight K-steps in flight
  constexpr int PA = BM / 8, PB = BN / 8;         // 1-KiB DMA pieces per K-step
  static_assert(PA % LWA == 0, "activation pieces split evenly over the loaders");
  // loader w issues LA activation pieces and LB (+1 for w < RB) weight pieces per step:
  // compile-time counts, so the per-step issue is a straight run of DMAs with no branch
  constexpr int LA = PA / LWA, LB = PB / LWB, RB = PB % LWB;
  constexpr int LMAX = SPLIT ? (LA > LB + (RB ? 1 : 0) ? LA : LB + (RB ? 1 : 0))
                             : LA + LB + (RB ? 1 : 0);
  constexpr int XSLOT = BM * RG_ROWB, WSLOT = BN * RG_ROWB;
  constexpr int SLOT = SPLIT ? XSLOT : (BM + BN) * RG_ROWB;
  constexpr int LDS_BYTES = SPLIT ? NS * XSLOT + NSB * WSLOT : NS * SLOT;
  constexpr int MT = BM / WM / 16, NT = BN / WN / 16;
  static_assert(MT * WM * 16 == BM && NT * WN * 16 == BN, "wave tiling");
  static_assert(NS >= 2 && (!SPLIT || NSB >= 2) && LDS_BYTES <= 163840,
                "LDS rings exceed 160 KiB");
  static_assert(SPLIT ? ((D - 1) * LA <= 63 && (DB - 1) * (LB + (RB ? 1 : 0)) <= 63)
                       : (D - 1) * LMAX <= 63, "vmcnt range");
  // ONE shared array (a second __shared__ object can make hipcc emit vmcnt(0) before the
  // first ds_read of every step)
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  char* const wring = lds + NS * XSLOT;           // SPLIT: the weight ring

  // the wave index as a scalar: role selection is one SALU branch
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool issuer = wave >= CW;
  const bool consumer = wave < CW;
  const int iw = wave - CW;                       // loader index (issuers only)

  // ---- tile coordinates (XCD-aware when the host says the grid divides evenly)
  int z, mb, nb;
  if (xmap) {
    const int r8 = blockIdx.x & 7, q = blockIdx.x >> 3, cpg = 8 / S;
    z = r8 % S;
    mb = q % MB;
    nb = (q / MB) * cpg + r8 / S;
  } else {
    z = blockIdx.x % S;
    const int j = blockIdx.x / S;
    mb = j % MB;
    nb = j / MB;
  }
  const int m0 = mb * BM;
  const int nk_all = K / RG_BK;
  const int kb0 = nk_all * z / S;
  const int nk = nk_all * (z + 1) / S - kb0;
  // the row blocks of one column tile walk K in the same order; column tiles start at
  // different steps (spread the X line fetches)
  const int rot = nk >= 4 ? (nb * 37) % nk : 0;

  // ---- loader state.  Every DMA address is a wave-uniform base (the operand, the
  // column tile, the K-step: SGPRs) plus a per-lane 32-bit byte offset fixed for the whole
  // walk, so a K-step costs a loader one scalar add and one m0 write per DMA.  (Rebuilding
  // each address with 64-bit VALU math, and choosing the piece kind at run time, made the
  // loader's per-step issue ~650 cycles -- measured, it sits between two barriers.)
  const int drow = lane >> 3, dchunk = (lane & 7) ^ drow;
  uint32_t voa[LA], vob[LB + 1];
  const char* const Xb = reinterpret_cast<const char*>(X);
  const int64_t wstep = (int64_t)BN * RG_BK * 2;  // bytes per K-step of one column tile
  const char* const Wb = reinterpret_cast<const char*>(Wp) + (int64_t)nb * nk_all * wstep;
  // SPLIT: loaders [0, LWA) are the activation group (ia), [LWA, LW) the weight group (ib)
  const bool a_loader = issuer && (!SPLIT || iw < LWA);
  const bool b_loader = issuer && (!SPLIT || iw >= LWA);
  const int ia = iw, ib = SPLIT ? iw - LWA : iw;
  const int extra_b = (RB && ib < RB) ? 1 : 0;
  if (issuer) {
#pragma unroll
    for (int t = 0; t < LA; ++t) {
      int r = m0 + (ia * LA + t) * 8 + drow;
      r = r < M ? r : M - 1;                      // padded rows re-read the last row
      voa[t] = (uint32_t)(((int64_t)r * ldx + dchunk * 8) * 2);
    }
#pragma unroll
    for (int t = 0; t < LB + 1; ++t) {
      const int q = t < LB ? ib * LB + t : LWB * LB + ib;  // B piece: tile rows 8q .. 8q+7
      vob[t] = (uint32_t)((q * 8 * RG_BK + lane * 8) * 2);
    }
  }

  auto kstep = [&](int step) {
    int st = step + rot;
    st = st >= nk ? st - nk : st;
    return kb0 + st;
  };
  // weights: WAUX = 2 (nt) streams them past L2 (each weight byte is read by ONE
  // workgroup when BM covers all rows); activations keep the default policy
  auto issue_b = [&](int step, char* base) {
    const char* wa = Wb + (int64_t)kstep(step) * wstep;
#pragma unroll
    for (int t = 0; t < LB; ++t) rg_glds16<WAUX>(wa + vob[t], base + (ib * LB + t) * 1024);
    if (RB && extra_b) rg_glds16<WAUX>(wa + vob[LB], base + (LWB * LB + ib) * 1024);
  };
  auto issue_a = [&](int step, char* base) {
    const char* xa = Xb + (int64_t)kstep(step) * (RG_BK * 2);
#pragma unroll
    for (int t = 0; t < LA; ++t) rg_glds16<0>(xa + voa[t], base + (ia * LA + t) * 1024);
  };
  auto issue = [&](int step) {                    // unified ring: both operands, one slot
    char* base = lds + (step % NS) * SLOT;
    issue_b(step, base + PA * 1024);
    issue_a(step, base);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wm = consumer ? wave / WN : 0, wn = consumer ? wave % WN : 0;
  const int fr = lane & 15, fq = lane >> 4;
  const int a_row0 = wm * (BM / WM) + fr;
  const int b_row0 = wn * (BN / WN) + fr;

  if constexpr (!SPLIT) {
    if (issuer) {
#pragma unroll
      for (int p = 0; p < D; ++p)
        if (p < nk) issue(p);
    }
  } else {
    if (a_loader) {
#pragma unroll
      for (int p = 0; p < D; ++p)
        if (p < nk) issue_a(p, lds + p * XSLOT);
    } else if (b_loader) {
#pragma unroll
      for (int p = 0; p < DB; ++p)
        if (p < nk) issue_b(p, wring + p * WSLOT);
    }
  }
  for (int it = 0; it < nk; ++it) {
    // step `it` must have landed; younger steps may stay in flight
    const int younger = nk - 1 - it;
    if constexpr (!SPLIT) {
      if (issuer) {
        if (RB && extra_b) rg_wait<LA + LB + 1, D - 1>(younger);
        else rg_wait<LA + LB, D - 1>(younger);
      }
    } else {
      if (a_loader) rg_wait<LA, D - 1>(younger);
      else if (b_loader) {
        if (RB && extra_b) rg_wait<LB + 1, DB - 1>(younger);
        else rg_wait<LB, DB - 1>(younger);
      }
    }
    __builtin_amdgcn_s_barrier();
    // every wave is past the reads of step it - 1, whose slots the next issues reuse
    if constexpr (!SPLIT) {
      if (issuer && it + D < nk) issue(it + D);
    } else {
      if (a_loader && it + D < nk) issue_a(it + D, lds + ((it + D) % NS) * XSLOT);
      else if (b_loader && it + DB < nk) issue_b(it + DB, wring + ((it + DB) % NSB) * WSLOT);
    }
    if (!consumer || (abl & 1)) continue;
    const char* sa = SPLIT ? lds + (it % NS) * XSLOT : lds + (it % NS) * SLOT;
    const char* sb = SPLIT ? wring + (it % (SPLIT ? NSB : 1)) * WSLOT : sa + BM * RG_ROWB;
#pragma unroll
    for (int ks = 0; ks < RG_BK / 32; ++ks) {
      const int c = ks * 4 + fq;
      Pack8<bf16> af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int r = a_row0 + i * 16;
        af[i].u = *reinterpret_cast<const u32x4*>(sa + r * RG_ROWB + (rg_swz(r, c) << 4));
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int r = b_row0 + n * 16;
        bfr[n].u = *reinterpret_cast<const u32x4*>(sb + r * RG_ROWB + (rg_swz(r, c) << 4));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[i][n] = mfma16x16x32(af[i].v, bfr[n].v, acc[i][n]);
    }
  }

  // ---- epilogue.  Lane (fq, fr) holds C[4*fq + e][fr] of every 16x16 tile: stored
  // straight from there a wave instruction writes four 32-64 B row pieces, and the
  // per-launch cost of those scattered 2 / 4-byte stores measured 7-20 us (the loop
  // without DMAs or MFMAs, KGC_RING_ABLATE=7: o 9.2 us, gate_up 24 us).  The tile goes
  // through LDS instead (the ring is free now) and every wave, loaders included,
  // writes whole rows with 16-B stores (write-through for the fp32 K-slices).
  constexpr int OCOLS = EPI == RG_SILU ? BN / 2 : BN;          // output columns of the tile
  constexpr int EB = EPI == RG_PARTIAL ? 4 : 2;                  // output element bytes
  constexpr int ROWB = OCOLS * EB + 16;                          // padded staging row
  constexpr int CPR = OCOLS * EB / 16;                           // 16-B chunks per row
  static_assert(OCOLS * EB % 16 == 0, "16-B rows");
  static_assert(BM * ROWB <= LDS_BYTES, "staging tile fits in the ring");
  __builtin_amdgcn_s_barrier();                 // every wave is done reading the ring
  if (consumer) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rt = wm * (BM / WM) + i * 16 + fq * 4 + e;
        char* srow = lds + rt * ROWB;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int ct = wn * (BN / WN) + n * 16 + fr;
          if constexpr (EPI == RG_PARTIAL) {
            *reinterpret_cast<float*>(srow + ct * 4) = acc[i][n][e];
          } else if constexpr (EPI == RG_OUT) {
            *reinterpret_cast<bf16*>(srow + ct * 2) = (bf16)acc[i][n][e];
          } else {
            // the up half of each 16-column group sits in lanes fr + 8 (all lanes shuffle)
            const float g = acc[i][n][e];
            const float u = __shfl_xor(g, 8, 64);
            if (fr < 8)
              *reinterpret_cast<bf16*>(srow + (((ct >> 4) << 3) + fr) * 2) =
                  (bf16)(rg_silu(g) * u);
          }
        }
      }
    }
  }
  __syncthreads();
  constexpr int NTH = (CW + LW) * 64;
  const int ldc = EPI == RG_SILU ? N / 2 : N;
  for (int c = tid; c < BM * CPR; c += NTH) {
    const int r = c / CPR, j = c - (c / CPR) * CPR;
    const int grow = m0 + r;
    if (grow >= M) continue;
    const u32x4 v = *reinterpret_cast<const u32x4*>(lds + r * ROWB + j * 16);
    if constexpr (EPI == RG_PARTIAL) {
      float* gp = reinterpret_cast<float*>(Cv) + z * slice_stride + (int64_t)grow * N +
                  (int64_t)nb * BN + j * 4;
      if (wt) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(gp), "v"(v) : "memory");
      else *reinterpret_cast<u32x4*>(gp) = v;
    } else {
      bf16* gp = reinterpret_cast<bf16*>(Cv) + (int64_t)grow * ldc + (int64_t)nb * OCOLS + j * 8;
      *reinterpret_cast<u32x4*>(gp) = v;
    }
  }
}

// P[grp][kb][r][pos] (16-B chunks) = W[row(grp * G + r)][kb * 64 + (pos ^ r % 8) * 8 ..]
__global__ __launch_bounds__(256) void ring_pack_kernel(bf16* __restrict__ P,
                                                        const bf16* __restrict__ W, int N,
                                                        int K, int G, int silu) {
  const int nk_all = K / RG_BK;
  const int64_t chunk = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * K / 8;
  if (chunk >= total) return;
  const int pos = (int)(chunk & 7);
  const int64_t rowi = chunk >> 3;                 // (grp, kb, r) flattened
  const int r = (int)(rowi % G);
  const int64_t t = rowi / G;
  const int kb = (int)(t % nk_all);
  const int64_t grp = t / nk_all;
  const int64_t p = grp * G + r;
  const int64_t wrow = silu ? rg_silu_row(p, N >> 1) : p;
  const int64_t s = wrow * K + kb * RG_BK + rg_swz(r, pos) * 8;
  reinterpret_cast<u32x4*>(P)[chunk] = *reinterpret_cast<const u32x4*>(W + s);
}

struct RingCfg { int bm, bn, wm, wn, lw, ns, waux, nsb; };
// id -> tile.  One workgroup per CU, ~256 workgroups at the target M.  BM = 256 (all rows
// of a batch-256 step) reads every weight byte from HBM exactly once: measured, row
// blocks of one column tile dispatched side by side on an XCD do NOT share the weight
// lines through L2 (64 x 64 full-K o_proj: 25.5 us = 4 x 33.5 MB at the chip's rate).
// The narrow projections then split K (o: 256 x 64, S = 4; qkv: 256 x 96, S = 4);
// gate_up + SiLU: 256 x 112 (7 gate / up groups of 16: 256 tiles at S = 1) or 256 x 128.
// Dedicated loader waves throughout (the MFMA waves never issue a DMA: 1.3-1.6x faster).
// ids 12-17: split rings (activation ring of `ns` slots, weight ring of `nsb`).
constexpr int kRingCfgs = 18;
constexpr RingCfg kRing[kRingCfgs] = {
    {256, 64, 4, 2, 4, 4, 2, 0},  {256, 64, 4, 2, 8, 4, 2, 0},  {256, 96, 4, 2, 4, 3, 2, 0},
    {256, 96, 4, 2, 8, 3, 2, 0},  {256, 112, 4, 1, 4, 3, 2, 0}, {256, 112, 4, 1, 8, 3, 2, 0},
    {256, 128, 4, 2, 4, 3, 2, 0}, {256, 128, 4, 2, 8, 3, 2, 0}, {128, 128, 2, 2, 4, 5, 0, 0},
    {128, 64, 2, 2, 4, 6, 0, 0},  {128, 96, 2, 2, 4, 5, 0, 0},  {128, 112, 4, 1, 4, 5, 0, 0},
    {256, 64, 4, 2, 8, 3, 2, 8},  {256, 96, 4, 2, 8, 3, 2, 5},  {256, 112, 4, 1, 4, 3, 2, 4},
    {256, 128, 4, 2, 8, 3, 2, 4}, {256, 64, 4, 2, 8, 2, 2, 12}, {128, 128, 2, 2, 8, 3, 2, 6}};

template <int C>
void ring_launch(int epi, void* Cp, const void* X, const void* W, int M, int N, int K,
                 int64_t ldx, int S, int64_t ss, hipStream_t s) {
  constexpr RingCfg c = kRing[C];
  const int MB = (M + c.bm - 1) / c.bm;
  const dim3 grid((unsigned)(MB * (N / c.bn) * S));
  const int nbt = N / c.bn;
  const int xm = (8 % S == 0 && nbt % (8 / S) == 0) ? 1 : 0;
  static const int wt = [] {
    const char* e = getenv("KGC_PARTIAL_WT");
    return e ? atoi(e) : 1;
  }();
  // profiling only: bit 0 drops the MFMAs (KGC_RING_ABLATE=1)
  static const int abl = [] {
    const char* e = getenv("KGC_RING_ABLATE");
    return e ? atoi(e) : 0;
  }();
#define RG_LAUNCH(E)                                                                        \
  ring_gemm_kernel<c.bm, c.bn, c.wm, c.wn, c.lw, c.ns, c.waux, E, c.nsb>                    \
      <<<grid, (c.wm * c.wn + c.lw) * 64, 0, s>>>(Cp, (const bf16*)X, (const bf16*)W, M, N, \
                                                  K, ldx, S, MB, ss, xm, wt, abl)
  if (epi == RG_PARTIAL) RG_LAUNCH(RG_PARTIAL);
  else if (epi == RG_OUT) RG_LAUNCH(RG_OUT);
  else RG_LAUNCH(RG_SILU);
#undef RG_LAUNCH
}

template <int... Is>
void ring_dispatch(int cfg, int epi, void* C, const void* X, const void* W, int M, int N, int K,
                   int64_t ldx, int S, int64_t ss, hipStream_t s,
                   std::integer_sequence<int, Is...>) {
  ((cfg == Is ? (ring_launch<Is>(epi, C, X, W, M, N, K, ldx, S, ss, s), 0) : 0), ...);
}

}  // namespace

int ring_num_cfgs() { return kRingCfgs; }
void ring_cfg_info(int cfg, int* bm, int* bn, int* threads, int* slots) {
  *bm = kRing[cfg].bm;
  *bn = kRing[cfg].bn;
  *threads = (kRing[cfg].wm * kRing[cfg].wn + kRing[cfg].lw) * 64;
  *slots = kRing[cfg].ns * 100 + kRing[cfg].nsb;
}

void launch_ring_gemm(int cfg, int epi, void* C, const void* X, const void* Wp, int M, int N,
                      int K, int64_t ldx, int S, int64_t slice_stride, hipStream_t s) {
  ring_dispatch(cfg, epi, C, X, Wp, M, N, K, ldx, S, slice_stride, s,
                std::make_integer_sequence<int, kRingCfgs>{});
}

void launch_ring_pack(bool silu, void* P, const void* W, int N, int K, int G, hipStream_t s) {
  const int64_t chunks = (int64_t)N * K / 8;
  const dim3 grid((unsigned)((chunks + 255) / 256));
  ring_pack_kernel<<<grid, 256, 0, s>>>((bf16*)P, (const bf16*)W, N, K, G, silu ? 1 : 0);
}

}  // namespace kgc
