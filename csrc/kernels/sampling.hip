// K10 sampler: 1024-thread workgroups over the rows of logits [B, V] (a row's vocabulary
// split over several workgroups at small batch), then a per-row merge.
//   temperature <= 1e-5        -> argmax (first index on ties)
//   otherwise x = logit * (1 / temp) -> optional top-k threshold (4-pass radix select on the
//                                 order-preserving uint32 image of x), optional top-p
//                                 threshold (radix select on softmax mass, over the top-k
//                                 support) -> Gumbel-max over the kept support.
// The Gumbel noise is a counter-based hash of (seed, column), bit-identical to
// ops/reference.uniform_noise, so sampled ids are reproducible per request seed.
//
// Vocab-parallel mode (TP > 1, rows without top-k / top-p): each rank runs the
// (Gumbel-)argmax over its own vocabulary shard with the noise of the GLOBAL column
// (vocab_off + i), and emits one packed (value, index) int64 per row; a MAX all-reduce
// of those 8 bytes per row over the TP group picks the token the unsharded sampler
// would have picked -- instead of all-gathering B x V logits to every rank.
#include "common.h"
#include "launch.h"
#include <algorithm>
#include <cstdlib>

namespace kgc {

constexpr int SMP_NT = 1024;
constexpr int SMP_NBIN = 2048;   // distance-from-max bins of the top-k / top-p pre-pass
constexpr int SMP_DB = 64;       // bins per nat of logit distance

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Gumbel noise.  Row key: both halves of the request seed through lowbias32, once per
// row.  Column gi: ONE lowbias32 round of key ^ gi * golden ratio -> u in (0, 1) ->
// G = -ln2 * log2(-ln2 * log2 u) = -ln(-ln u) on v_log_f32.  (Two hashes and two libm
// logf per logit made the temperature pass VALU-bound: ~70 VALU per logit, 78 us per
// decode step at B = 256 x 128K.)  ops/reference.py uniform_noise / gumbel compute the
// same values in fp32.
__device__ __forceinline__ uint32_t row_key(uint64_t seed) {
  return mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + 0x632BE5ABu));
}
__device__ __forceinline__ float gumbel(uint32_t key, int gi) {
  const uint32_t h = mix32(key ^ ((uint32_t)gi * 0x9E3779B9u));
  // 23 bits: u in [2^-24, 1 - 2^-24], every value exact in fp32.  (24 bits + 0.5 rounded
  // the top value to u = 1.0 -> E = 0 -> G = +inf: that column won its row outright,
  // whatever its logit -- for one row in ~130 at V = 128K.)
  const float u = ((float)(h >> 9) + 0.5f) * (1.0f / 8388608.0f);
  return -0.69314718f * __builtin_amdgcn_logf(-0.69314718f * __builtin_amdgcn_logf(u));
}

__device__ __forceinline__ uint32_t ord_key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_val(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <typename T>
__device__ __forceinline__ float load_logit(const T* row, int i) { return to_f(row[i]); }

// Inclusive prefix sum of one value per thread over a SMP_NT-thread block: wave64
// shuffle scans, then the wave totals (scratch: SMP_NT / 64 floats).
__device__ __forceinline__ float block_scan_incl(float v, float* wtot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  if (lane == 63) wtot[w] = v;
  __syncthreads();
  float off = 0.f;
  for (int j = 0; j < w; ++j) off += wtot[j];
  __syncthreads();
  return v + off;
}

// f(i, logit) over row[lo, hi) by a SMP_NT-thread block.  16-bit rows are read as
// 16-byte vectors (8 logits per load, 4 loads in flight per thread): every pass over
// a 128K-entry row is then ~16 dependent round trips per thread instead of ~125.
template <typename T, typename F>
__device__ __forceinline__ void visit_row(const T* __restrict__ row, int lo, int hi, int tid,
                                          F&& f) {
  if constexpr (sizeof(T) == 2) {
    const int a = min(hi, (lo + 7) & ~7);
    const int e = max(a, hi & ~7);
    if ((reinterpret_cast<uintptr_t>(row) & 15) == 0) {
      for (int i = lo + tid; i < a; i += SMP_NT) f(i, to_f(row[i]));
      // 4 vectors per thread in flight: the loads of a trip are unconditional (clamped
      // to the last full vector) so none waits behind a branch; only f is predicated.
      constexpr int U = 4, VS = 8 * SMP_NT;
      for (int v = a + 8 * tid; v < e; v += U * VS) {
        Pack8<T> p[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          p[u].u = *reinterpret_cast<const u32x4*>(row + min(v + u * VS, e - 8));
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (v + u * VS < e) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f(v + u * VS + j, to_f(p[u].h[j]));
          }
        }
      }
      for (int i = e + tid; i < hi; i += SMP_NT) f(i, to_f(row[i]));
      return;
    }
  }
  for (int i = lo + tid; i < hi; i += SMP_NT) f(i, to_f(row[i]));
}

__device__ __forceinline__ void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

// Grid (B, S): the S blocks of a row split its vocabulary for the (Gumbel-)argmax pass,
// the expensive one (two logs and two hashes per logit).  A row with a top-k / top-p
// threshold has every block compute that threshold over the whole row first (cheap
// vectorised passes, run in parallel), so no single block walks the row alone.
// Each block writes its (value, index) candidate packed into one uint64 (value's
// order-preserving image high, inverted index low: max = larger value, then lower
// index) and sample_merge_kernel reduces the S candidates of a row.
template <typename T>
__global__ __launch_bounds__(SMP_NT) void sample_kernel(
    uint64_t* __restrict__ partial, const T* __restrict__ logits, int64_t row_stride, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const int64_t* __restrict__ seeds, int vocab_off) {
  __shared__ float red_v[SMP_NT / 64];
  __shared__ int red_i[SMP_NT / 64];
  __shared__ float hist_f[256];
  __shared__ float hist_d[SMP_NBIN];
  __shared__ float scan_w[SMP_NT / 64];
  __shared__ uint32_t sel_bin;
  __shared__ float sel_f;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* row = logits + (int64_t)b * row_stride;
  const float temp = temperature[b];
  const bool greedy = temp <= 1e-5f;
  const int k = (greedy || top_k == nullptr) ? 0 : top_k[b];          // null: vocab-parallel
  const float p = (greedy || top_p == nullptr) ? 1.f : top_p[b];
  const bool use_k = k > 0 && k < V;
  const bool use_p = p < 1.f;
  const int S = gridDim.y, y = blockIdx.y;
  const int i_lo = (int)((int64_t)V * y / S);
  const int i_hi = (int)((int64_t)V * (y + 1) / S);

  // ---------- thresholds (kept support = x >= thr)
  // Both selects first bin the row by distance from its max (SMP_DB bins per nat, so
  // a row spreads over hundreds of bins), then resolve the bin holding the k-th value
  // / the p-mass crossing exactly with radix passes restricted to that bin's few
  // elements.  Every "where does the running total cross the target" search is a
  // block-parallel prefix sum: a serial scan by one thread cost ~100 cycles per bin
  // (~300 us per top-p row with the 2048 + 4 x 256 bins).
  // The selects run on the raw logits: x = raw / temp is order-preserving (temp > 0),
  // so "raw >= thr" keeps exactly the tokens "x >= thr * ..." would, and no pass but
  // the final one pays the fp32 division (the masses use raw * (1 / temp)).
  float thr = -INFINITY;
  if (use_k || use_p) {
    float mx = -INFINITY;
    visit_row(row, 0, V, tid, [&](int, float r) { mx = fmaxf(mx, r); });
    mx = block_max<SMP_NT>(mx, red_v);
    const float it = 1.f / temp;                   // x = raw * it for the softmax mass
    auto dbin = [&](float x) -> int {
      const float d = (mx - x) * it * (float)SMP_DB;
      return d < (float)(SMP_NBIN - 1) ? (int)d : SMP_NBIN - 1;   // -inf / NaN -> last
    };
    // distance bins in value order (bin 0 = largest values): first bin whose running
    // total reaches `target` -> sel_bin, the total before it -> sel_f; 2 bins / thread
    auto cross_dist = [&](float target) {
      if (tid == 0) { sel_bin = SMP_NBIN - 1; sel_f = 0.f; }
      const float h0 = hist_d[2 * tid], h1 = hist_d[2 * tid + 1];
      const float incl = block_scan_incl(h0 + h1, scan_w);
      const float excl = incl - h0 - h1;
      if (excl < target && excl + h0 >= target) { sel_bin = 2 * tid; sel_f = excl; }
      else if (excl + h0 < target && incl >= target) { sel_bin = 2 * tid + 1; sel_f = excl + h0; }
      __syncthreads();
    };
    // radix bins visited from 255 down to `lowest`: first one whose running total
    // (starting at `start`) reaches `target` -> sel_bin, the total before it -> sel_f;
    // none -> bin `fallback`, the total over the visited bins
    auto cross_radix = [&](const float* h, float start, float target, int lowest, int fallback) {
      const int pos = tid, bin = 255 - pos;
      const float v = (pos < 256 && bin >= lowest) ? h[bin] : 0.f;
      const float incl = start + block_scan_incl(v, scan_w);
      const float excl = incl - v;
      if (tid == SMP_NT - 1) { sel_bin = fallback; sel_f = incl; }
      __syncthreads();
      if (pos < 256 && bin >= lowest && excl < target && incl >= target) {
        sel_bin = bin;
        sel_f = excl;
      }
      __syncthreads();
    };
    if (use_k) {
      for (int j = tid; j < SMP_NBIN; j += SMP_NT) hist_d[j] = 0.f;
      __syncthreads();
      visit_row(row, 0, V, tid, [&](int, float r) { atomicAdd(&hist_d[dbin(r)], 1.f); });
      __syncthreads();
      cross_dist((float)k);
      const int kbin = (int)sel_bin;
      uint32_t prefix = 0, mask = 0;
      float remaining = (float)k - sel_f;       // counts: exact in fp32 up to 2^24
      for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) hist_f[tid] = 0.f;
        __syncthreads();
        visit_row(row, 0, V, tid, [&](int, float r) {
          const uint32_t kk = ord_key(r);
          if (dbin(r) == kbin && (kk & mask) == prefix) atomicAdd(&hist_f[(kk >> shift) & 255], 1.f);
        });
        __syncthreads();
        cross_radix(hist_f, 0.f, remaining, 0, 0);
        remaining -= sel_f;
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
      }
      thr = key_val(prefix);
    }
    if (use_p) {
      // normaliser and p-mass histogram over the current support (mx is still its max)
      for (int j = tid; j < SMP_NBIN; j += SMP_NT) hist_d[j] = 0.f;
      __syncthreads();
      float z = 0.f;
      visit_row(row, 0, V, tid, [&](int, float r) {
        if (r >= thr) {
          const float e = __expf((r - mx) * it);
          z += e;
          atomicAdd(&hist_d[dbin(r)], e);
        }
      });
      z = block_sum<SMP_NT>(z, red_v);
      const float target = p * z;
      cross_dist(target);
      const int pbin = (int)sel_bin;
      uint32_t prefix = 0, mask = 0;
      float above = sel_f;
      const uint32_t kthr = ord_key(thr);
      for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) hist_f[tid] = 0.f;
        __syncthreads();
        visit_row(row, 0, V, tid, [&](int, float r) {
          const uint32_t kk = ord_key(r);
          if (kk >= kthr && dbin(r) == pbin && (kk & mask) == prefix)
            atomicAdd(&hist_f[(kk >> shift) & 255], __expf((r - mx) * it));
        });
        __syncthreads();
        cross_radix(hist_f, above, target, 1, 0);
        above = sel_f;
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
      }
      thr = fmaxf(thr, key_val(prefix));
    }
  }

  // ---------- (Gumbel-)argmax over the support
  const uint32_t key = row_key((uint64_t)seeds[b]);
  const float inv_t = greedy ? 1.f : 1.f / temp;
  float best = -INFINITY;
  int besti = 0x7fffffff;
  visit_row(row, i_lo, i_hi, tid, [&](int i, float r) {
    const int gi = i + vocab_off;                 // global column (vocab-parallel shard)
    float x = r;
    if (!greedy) {
      if (r < thr) return;
      x = r * inv_t + gumbel(key, gi);
    }
    argmax_merge(best, besti, x, gi);
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(besti, o, 64);
    argmax_merge(best, besti, v2, i2);
  }
  if (lane == 0) { red_v[w] = best; red_i[w] = besti; }
  __syncthreads();
  if (tid == 0) {
    float bv = red_v[0];
    int bi = red_i[0];
    for (int j = 1; j < SMP_NT / 64; ++j) argmax_merge(bv, bi, red_v[j], red_i[j]);
    partial[(int64_t)b * S + y] = ((uint64_t)ord_key(bv) << 32) | (uint32_t)(~(uint32_t)bi);
  }
}

// One thread per row: the largest packed candidate of the row's S blocks.
__global__ __launch_bounds__(256) void sample_merge_kernel(int64_t* __restrict__ out,
                                                           const uint64_t* __restrict__ partial,
                                                           int B, int S) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  uint64_t best = 0;
  for (int y = 0; y < S; ++y) best = max(best, partial[(int64_t)b * S + y]);
  const uint32_t idx = ~(uint32_t)(best & 0xffffffffu);
  out[b] = (best == 0 || idx >= 0x7fffffffu) ? 0 : (int64_t)idx;
}

// ---------------------------------------------------------------------------------------
// Cooperative variant for rows with top-k / top-p: the S workgroups of a row split the
// threshold passes too (each visits V / S logits per pass) and combine their partial
// histograms in a per-row global workspace, with a workgroup barrier per pass (counters
// in the zero-initialised workspace; B * S <= 256, so every workgroup of the grid is
// co-resident and the barriers cannot deadlock; spins are bounded anyway).  The
// single-workgroup kernel above computes every threshold over the whole row in each of
// the S workgroups: ~230 us per top-p row at batch 1.
// Candidates of the crossing distance bin: when a row has at most SMP_CAP of them, each
// workgroup finishes the threshold with the 4 radix passes over that list in its own LDS
// (fixed-point masses: integer sums, so every workgroup of the row lands on the same key)
// instead of 4 global passes over the row with a row barrier each.
constexpr int SMP_CAP = 2048;

// Phase stamps of the cooperative kernel (profiling only, off by default): workgroup
// (0, 0) records wall_clock64() (100 MHz) at each phase boundary when enabled.
__device__ int g_smp_stamp_on;
__device__ uint64_t g_smp_stamps[16];
#define SMP_STAMP(i)                                                                         \
  do {                                                                                       \
    if (g_smp_stamp_on && b == 0 && y == 0 && tid == 0) g_smp_stamps[i] = wall_clock64();   \
  } while (0)

// sticky "a cooperative row barrier gave up" word, read and cleared by the host
__device__ uint32_t g_smp_err;

struct CoopWs {
  uint32_t bar[16];
  uint32_t maxkey;
  uint32_t err;
  float z;
  float pad;
  uint32_t ncand[2];
  uint32_t pad2[2];
  float hist_k[SMP_NBIN];
  float hist_p[SMP_NBIN];
  float hist_r[8][256];
  uint32_t cand_key[2][SMP_CAP];
  float cand_w[2][SMP_CAP];
};

int sample_coop_ws_bytes() { return (int)sizeof(CoopWs); }

template <typename T>
__global__ __launch_bounds__(SMP_NT) void sample_coop_kernel(
    uint64_t* __restrict__ partial, const T* __restrict__ logits, int64_t row_stride, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const int64_t* __restrict__ seeds, CoopWs* __restrict__ wsa) {
  __shared__ float red_v[SMP_NT / 64];
  __shared__ int red_i[SMP_NT / 64];
  __shared__ float hist_f[256];
  __shared__ float hist_d[SMP_NBIN];
  __shared__ float scan_w[SMP_NT / 64];
  __shared__ uint32_t sel_bin;
  __shared__ float sel_f, sel_t;
  __shared__ uint32_t cand_k[SMP_CAP];
  __shared__ uint64_t cand_m[SMP_CAP];
  __shared__ uint64_t hist_u[256];
  __shared__ uint64_t sel_u;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* row = logits + (int64_t)b * row_stride;
  CoopWs* ws = wsa + b;
  const float temp = temperature[b];
  const bool greedy = temp <= 1e-5f;
  const int k = greedy ? 0 : top_k[b];
  const float p = greedy ? 1.f : top_p[b];
  const bool use_k = k > 0 && k < V;
  const bool use_p = p < 1.f;
  const int S = gridDim.y, y = blockIdx.y;
  const int i_lo = (int)((int64_t)V * y / S);
  const int i_hi = (int)((int64_t)V * (y + 1) / S);
  int nbar = 0;
  SMP_STAMP(0);
  // all S workgroups of this row: arrive, wait for the others (bounded).  Everything a
  // workgroup hands to the others goes through agent-scope atomics or write-through
  // stores, and every read of it is an agent-scope (sc1) atomic load, so the barrier needs
  // no release / acquire fence: the __syncthreads() before the arrive drains every wave's
  // stores and atomics (vmcnt(0)), and the counter is an atomic (cdna_hip_programming.md
  // §6 Guideline 16, the write-through form).  Plain loads here only read the logits.
  auto row_barrier = [&]() {
    __syncthreads();
    if (tid == 0) {
      uint32_t* c = &ws->bar[nbar];
      __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long dl = spin_deadline(KGC_COOP_SPIN_MS);
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)S) {
        __builtin_amdgcn_s_sleep(1);
        if (spin_expired(dl)) {
          // a row's workgroups were not co-resident (another kernel held CUs): the
          // thresholds below are wrong -- flag it in the sticky device word the host
          // reads after every step (ops.SamplerHealth) so the step is never served
          atomicOr(&ws->err, 1u);
          atomicOr(&g_smp_err, 1u);
          break;
        }
      }
    }
    __syncthreads();
    ++nbar;
  };
  auto gload = [](const float* p_) { return __hip_atomic_load(p_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };

  float thr = -INFINITY;
  if (use_k || use_p) {
    float mx = -INFINITY;
    visit_row(row, i_lo, i_hi, tid, [&](int, float r) { mx = fmaxf(mx, r); });
    mx = block_max<SMP_NT>(mx, red_v);
    if (tid == 0) atomicMax(&ws->maxkey, ord_key(mx));
    SMP_STAMP(1);
    row_barrier();
    SMP_STAMP(2);
    mx = key_val(__hip_atomic_load(&ws->maxkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const float it = 1.f / temp;
    auto dbin = [&](float x) -> int {
      const float d = (mx - x) * it * (float)SMP_DB;
      return d < (float)(SMP_NBIN - 1) ? (int)d : SMP_NBIN - 1;
    };
    auto cross_dist = [&](float target) {
      if (tid == 0) { sel_bin = SMP_NBIN - 1; sel_f = 0.f; }
      const float h0 = hist_d[2 * tid], h1 = hist_d[2 * tid + 1];
      const float incl = block_scan_incl(h0 + h1, scan_w);
      const float excl = incl - h0 - h1;
      if (excl < target && excl + h0 >= target) { sel_bin = 2 * tid; sel_f = excl; }
      else if (excl + h0 < target && incl >= target) { sel_bin = 2 * tid + 1; sel_f = excl + h0; }
      __syncthreads();
    };
    auto cross_radix = [&](const float* h, float start, float target, int lowest, int fallback) {
      const int pos = tid, bin = 255 - pos;
      const float v = (pos < 256 && bin >= lowest) ? h[bin] : 0.f;
      const float incl = start + block_scan_incl(v, scan_w);
      const float excl = incl - v;
      if (tid == SMP_NT - 1) { sel_bin = fallback; sel_f = incl; }
      __syncthreads();
      if (pos < 256 && bin >= lowest && excl < target && incl >= target) {
        sel_bin = bin;
        sel_f = excl;
      }
      __syncthreads();
    };
    // this workgroup's LDS histogram -> the row's global one (non-zero bins only)
    auto publish = [&](const float* h, float* g, int n) {
      __syncthreads();
      for (int j = tid; j < n; j += SMP_NT)
        if (h[j] != 0.f) atomicAdd(&g[j], h[j]);
    };
    auto fetch = [&](float* h, const float* g, int n) {
      for (int j = tid; j < n; j += SMP_NT) h[j] = gload(&g[j]);
      __syncthreads();
    };
    // append this workgroup's candidates (weight >= 0) to the row's list t; write-through
    // stores, published by the row barrier that follows
    auto collect = [&](int t, auto&& weight) {
      // staged in LDS (cand_k / cand_m are free until local_select), then ONE global
      // atomic per workgroup reserves its range of the row's list.  sel_bin doubles as the
      // LDS counter: every wave has read the previous selection (kbin / pbin) first
      __syncthreads();
      if (tid == 0) sel_bin = 0;
      __syncthreads();
      visit_row(row, i_lo, i_hi, tid, [&](int, float r) {
        const float wt = weight(r);
        if (wt >= 0.f) {
          const uint32_t slot = atomicAdd(&sel_bin, 1u);
          if (slot < (uint32_t)SMP_CAP) {
            cand_k[slot] = ord_key(r);
            cand_m[slot] = __float_as_uint(wt);
          }
        }
      });
      __syncthreads();
      const uint32_t n = sel_bin;
      if (tid == 0)   // an overflowing workgroup pushes the row's count past SMP_CAP
        sel_u = __hip_atomic_fetch_add(&ws->ncand[t], n > (uint32_t)SMP_CAP ? (uint32_t)SMP_CAP + 1 : n,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const uint32_t base = (uint32_t)sel_u;
      for (uint32_t j = tid; j < n && j < (uint32_t)SMP_CAP && base + j < (uint32_t)SMP_CAP; j += SMP_NT) {
        __hip_atomic_store(&ws->cand_key[t][base + j], cand_k[j], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ws->cand_w[t][base + j], __uint_as_float((uint32_t)cand_m[j]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    // the 4 radix passes of a threshold over the n <= SMP_CAP candidates of list t, in LDS:
    // the key of the candidate at which the running mass (keys descending) first reaches
    // `need` (fixed point: mass * scale); bins below `lowest` never cross (fallback bin 0)
    auto local_select = [&](int t, int n, float scale, float need, int lowest) -> uint32_t {
      for (int j = tid; j < n; j += SMP_NT) {
        cand_k[j] = __hip_atomic_load(&ws->cand_key[t][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cand_m[j] = (uint64_t)(gload(&ws->cand_w[t][j]) * scale);
      }
      uint64_t rem = need > 0.f ? (uint64_t)(need * scale) : 0;
      uint32_t prefix = 0, mask = 0;
      for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) hist_u[tid] = 0;
        __syncthreads();
        for (int j = tid; j < n; j += SMP_NT)
          if ((cand_k[j] & mask) == prefix) atomicAdd(&hist_u[(cand_k[j] >> shift) & 255], cand_m[j]);
        __syncthreads();
        if (w == 0) {   // one wave scans the 256 bins, 4 per lane, from bin 255 down
          uint64_t v[4], sum = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int bn = 255 - 4 * lane - i;
            v[i] = bn >= lowest ? hist_u[bn] : 0;
            sum += v[i];
          }
          uint64_t incl = sum;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const uint64_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
          }
          if (lane == 63) { sel_bin = 0; sel_u = incl; }    // no crossing: keep the whole bin
          uint64_t run = incl - sum;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int bn = 255 - 4 * lane - i;
            if (bn >= lowest && run < rem && run + v[i] >= rem) { sel_bin = bn; sel_u = run; }
            run += v[i];
          }
        }
        __syncthreads();
        rem -= sel_u;
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
      }
      return prefix;
    };
    // wave 0: over h[0..n) (n <= 128, ascending distance = descending logit), the first
    // bin whose running total (from `start`) reaches `target` -> sel_bin, the total before
    // it -> sel_f; no crossing: the last bin.  Lane l scans bins 2l, 2l + 1.
    auto wave_cross = [&](const float* h, int n, float start, float target) {
      if (w == 0) {
        const float v0 = 2 * lane < n ? h[2 * lane] : 0.f;
        const float v1 = 2 * lane + 1 < n ? h[2 * lane + 1] : 0.f;
        float incl = v0 + v1;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const float u = __shfl_up(incl, o, 64);
          if (lane >= o) incl += u;
        }
        incl += start;
        const float e0 = incl - v0 - v1, e1 = e0 + v0;
        if (2 * lane == n - 1) { sel_bin = n - 1; sel_f = e0; }
        if (2 * lane + 1 == n - 1) { sel_bin = n - 1; sel_f = e1; }
        if (2 * lane < n && e0 < target && e1 >= target) { sel_bin = 2 * lane; sel_f = e0; }
        else if (2 * lane + 1 < n && e1 < target && incl >= target) { sel_bin = 2 * lane + 1; sel_f = e1; }
      }
      __syncthreads();
    };
    // The crossing distance bin of a threshold, two-level: per-thread register counters over
    // NCB coarse bins (2 nats = 128 distance bins each) -- no LDS atomic per logit -- summed
    // over the row, then LDS-atomic distance bins only for the logits of the crossing
    // coarse bin.  wt(r) = the logit's weight (< 0: not counted); g = the row's global
    // histogram (NCB coarse + 128 fine bins); target_of(row total) = the weight to reach.
    // Returns the distance bin; sel_f = the weight above it, sel_t = the target.
    constexpr int NCB = SMP_NBIN / 128;
    auto dist_cross = [&](auto&& wt, float* g, auto&& target_of) -> int {
      float acc[NCB];
#pragma unroll
      for (int j = 0; j < NCB; ++j) acc[j] = 0.f;
      visit_row(row, i_lo, i_hi, tid, [&](int, float r) {
        const float x = wt(r);
        if (x < 0.f) return;
        const int cb = dbin(r) >> 7;
#pragma unroll
        for (int j = 0; j < NCB; ++j) acc[j] += cb == j ? x : 0.f;
      });
      if (tid < 128) hist_d[tid] = 0.f;
      __syncthreads();
      // reduce-scatter of the NCB = 16 counters over the wave by recursive halving: 8 + 4 +
      // 2 + 1 shuffles (not 16 x 6), then 2 to finish; lanes 4c..4c+3 hold coarse bin c
#pragma unroll
      for (int half = NCB / 2, off = 32; half >= 1; half >>= 1, off >>= 1) {
        const bool hi = (lane & off) != 0;
#pragma unroll
        for (int j = 0; j < half; ++j) {
          const float mine = hi ? acc[half + j] : acc[j];
          const float other = hi ? acc[j] : acc[half + j];
          acc[j] = mine + __shfl_xor(other, off, 64);
        }
      }
      acc[0] += __shfl_xor(acc[0], 2, 64);
      acc[0] += __shfl_xor(acc[0], 1, 64);
      if ((lane & 3) == 0 && acc[0] != 0.f) atomicAdd(&hist_d[lane >> 2], acc[0]);
      publish(hist_d, g, NCB);
      row_barrier();
      fetch(hist_d, g, NCB);
      // the row's total weight, summed in the same order in every workgroup
      float total = 0.f;
      for (int j = 0; j < NCB; ++j) total += hist_d[j];
      const float target = target_of(total);
      if (tid == 0) sel_t = target;
      wave_cross(hist_d, NCB, 0.f, target);
      const int cbin = (int)sel_bin;
      const float above = sel_f;
      __syncthreads();
      if (tid < 128) hist_d[tid] = 0.f;
      __syncthreads();
      visit_row(row, i_lo, i_hi, tid, [&](int, float r) {
        const int d = dbin(r);
        if ((d >> 7) != cbin) return;
        const float x = wt(r);
        if (x >= 0.f) atomicAdd(&hist_d[d & 127], x);
      });
      publish(hist_d, g + NCB, 128);
      row_barrier();
      fetch(hist_d, g + NCB, 128);
      wave_cross(hist_d, 128, above, target);
      return cbin * 128 + (int)sel_bin;
    };
    if (use_k) {
      SMP_STAMP(3);
      const int kbin_ = dist_cross([&](float) { return 1.f; }, ws->hist_k,
                                   [&](float) { return (float)k; });
      SMP_STAMP(4);
      const int kbin = kbin_;
      uint32_t prefix = 0, mask = 0;
      float remaining = (float)k - sel_f;
      collect(0, [&](float r) { return dbin(r) == kbin ? 1.f : -1.f; });
      row_barrier();
      const int nk = (int)__hip_atomic_load(&ws->ncand[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      SMP_STAMP(5);
      if (nk <= SMP_CAP) {
        prefix = local_select(0, nk, 1.f, remaining, 0);
        mask = 0xffffffffu;   // skip the global passes below
      }
      SMP_STAMP(6);
      for (int q = 0, shift = 24; shift >= 0 && mask != 0xffffffffu; ++q, shift -= 8) {
        if (tid < 256) hist_f[tid] = 0.f;
        __syncthreads();
        visit_row(row, i_lo, i_hi, tid, [&](int, float r) {
          const uint32_t kk = ord_key(r);
          if (dbin(r) == kbin && (kk & mask) == prefix) atomicAdd(&hist_f[(kk >> shift) & 255], 1.f);
        });
        publish(hist_f, ws->hist_r[q], 256);
        row_barrier();
        fetch(hist_f, ws->hist_r[q], 256);
        cross_radix(hist_f, 0.f, remaining, 0, 0);
        remaining -= sel_f;
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
      }
      thr = key_val(prefix);
    }
    if (use_p) {
      SMP_STAMP(7);
      // the mass target p * z, z = the row's softmax mass over the top-k support (the
      // coarse histogram's total)
      const int pbin_ = dist_cross([&](float r) { return r >= thr ? __expf((r - mx) * it) : -1.f; },
                                   ws->hist_p, [&](float zt) { return p * zt; });
      const float target = sel_t;
      SMP_STAMP(8);
      const int pbin = pbin_;
      uint32_t prefix = 0, mask = 0;
      float above = sel_f;
      const uint32_t kthr = ord_key(thr);
      collect(1, [&](float r) {
        return (ord_key(r) >= kthr && dbin(r) == pbin) ? __expf((r - mx) * it) : -1.f;
      });
      row_barrier();
      const int np = (int)__hip_atomic_load(&ws->ncand[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      SMP_STAMP(9);
      if (np <= SMP_CAP) {
        // masses <= 1 each, <= 2^11 of them: 2^40 fixed point stays far below 2^64
        prefix = local_select(1, np, 1099511627776.f, target - above, 1);
        mask = 0xffffffffu;
      }
      SMP_STAMP(10);
      for (int q = 4, shift = 24; shift >= 0 && mask != 0xffffffffu; ++q, shift -= 8) {
        if (tid < 256) hist_f[tid] = 0.f;
        __syncthreads();
        visit_row(row, i_lo, i_hi, tid, [&](int, float r) {
          const uint32_t kk = ord_key(r);
          if (kk >= kthr && dbin(r) == pbin && (kk & mask) == prefix)
            atomicAdd(&hist_f[(kk >> shift) & 255], __expf((r - mx) * it));
        });
        publish(hist_f, ws->hist_r[q], 256);
        row_barrier();
        fetch(hist_f, ws->hist_r[q], 256);
        cross_radix(hist_f, above, target, 1, 0);
        above = sel_f;
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
      }
      thr = fmaxf(thr, key_val(prefix));
    }
  }
  SMP_STAMP(11);
  // ---------- (Gumbel-)argmax over this workgroup's slice of the support
  const uint32_t key = row_key((uint64_t)seeds[b]);
  const float inv_t = greedy ? 1.f : 1.f / temp;
  float best = -INFINITY;
  int besti = 0x7fffffff;
  visit_row(row, i_lo, i_hi, tid, [&](int i, float r) {
    float x = r;
    if (!greedy) {
      if (r < thr) return;
      x = r * inv_t + gumbel(key, i);
    }
    argmax_merge(best, besti, x, i);
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(besti, o, 64);
    argmax_merge(best, besti, v2, i2);
  }
  if (lane == 0) { red_v[w] = best; red_i[w] = besti; }
  __syncthreads();
  if (tid == 0) {
    float bv = red_v[0];
    int bi = red_i[0];
    for (int j = 1; j < SMP_NT / 64; ++j) argmax_merge(bv, bi, red_v[j], red_i[j]);
    partial[(int64_t)b * S + y] = ((uint64_t)ord_key(bv) << 32) | (uint32_t)(~(uint32_t)bi);
  }
  // The workspace is persistent and must be all-zero for the next call: the last of the
  // row's workgroups to finish (every read of the workspace is behind it: __syncthreads()
  // drains this workgroup's loads) clears what this call used.  After the argmax pass, so
  // the clearing stays off the row's critical path; the next launch sees the plain stores.
  if (use_k || use_p) {
    __shared__ int last;
    __syncthreads();
    if (tid == 0)
      last = __hip_atomic_fetch_add(&ws->bar[15], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (uint32_t)(S - 1);
    __syncthreads();
    if (last) {
      if (use_k) {
        for (int j = tid; j < SMP_NBIN; j += SMP_NT) ws->hist_k[j] = 0.f;
        for (int j = tid; j < 4 * 256; j += SMP_NT) ws->hist_r[j / 256][j % 256] = 0.f;
      }
      if (use_p) {
        for (int j = tid; j < SMP_NBIN; j += SMP_NT) ws->hist_p[j] = 0.f;
        for (int j = tid; j < 4 * 256; j += SMP_NT) ws->hist_r[4 + j / 256][j % 256] = 0.f;
      }
      if (tid < 16) ws->bar[tid] = 0;
      if (tid == 0) {
        ws->maxkey = 0;
        ws->z = 0.f;
        ws->ncand[0] = 0;
        ws->ncand[1] = 0;
      }
    }
  }
  SMP_STAMP(12);
}

void sample_stamps_enable(bool on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_smp_stamp_on), &v, sizeof(v));
}

void sample_stamps_read(uint64_t* out16) {
  (void)hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_smp_stamps), 16 * sizeof(uint64_t));
}

// Workgroups per row of the cooperative sampler (0: use the single-workgroup-threshold
// kernel).  The whole grid must be co-resident (one 1024-thread workgroup per CU is always
// available), so B * S <= the device's CU count (256 on a whole MI355X, fewer in a
// partitioned mode); with S = 1 a row's barriers wait for nobody.  Measured on MI355X
// (profiles/sample_microbench.jsonl): 16 per row up to B = 16, then CUs / B; at B = 256
// one workgroup per row (top-p 549 -> 268 us against the older kernel).
int sample_coop_splits(int B) {
  static int cus[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 0;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 1;   // unknown: never co-resident enough for more than one row -> older kernel
    cus[dev] = n;
  }
  if (B > cus[dev]) return 0;
  return std::max(1, std::min(16, cus[dev] / B));
}

void launch_sample_coop(int dtype, int64_t* out, uint64_t* partial, void* ws, const void* logits,
                        int64_t row_stride, int B, int V, const float* temperature,
                        const int* top_k, const float* top_p, const int64_t* seeds,
                        hipStream_t s) {
  if (B == 0) return;
  const dim3 grid(B, sample_coop_splits(B));
  CoopWs* w = reinterpret_cast<CoopWs*>(ws);       // persistent, all-zero between calls
  if (dtype == DT_BF16)
    sample_coop_kernel<bf16><<<grid, SMP_NT, 0, s>>>(partial, (const bf16*)logits, row_stride, V,
                                                     temperature, top_k, top_p, seeds, w);
  else if (dtype == DT_F16)
    sample_coop_kernel<f16><<<grid, SMP_NT, 0, s>>>(partial, (const f16*)logits, row_stride, V,
                                                    temperature, top_k, top_p, seeds, w);
  else
    sample_coop_kernel<float><<<grid, SMP_NT, 0, s>>>(partial, (const float*)logits, row_stride,
                                                      V, temperature, top_k, top_p, seeds, w);
  sample_merge_kernel<<<(B + 255) / 256, 256, 0, s>>>(out, partial, B, grid.y);
}

// Vocab-parallel: the row's packed candidate, biased (top bit flipped) so that a SIGNED
// int64 max -- what RCCL / gloo reduce -- orders it like the unsigned packing.
constexpr uint64_t VP_BIAS = 0x8000000000000000ull;

__global__ __launch_bounds__(256) void sample_vp_merge_kernel(int64_t* __restrict__ packed,
                                                              const uint64_t* __restrict__ partial,
                                                              int B, int S) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  uint64_t best = 0;
  for (int y = 0; y < S; ++y) best = max(best, partial[(int64_t)b * S + y]);
  packed[b] = (int64_t)(best ^ VP_BIAS);
}

// after the MAX all-reduce over the TP group: packed candidate -> token id
__global__ __launch_bounds__(256) void sample_vp_unpack_kernel(int64_t* __restrict__ out,
                                                               const int64_t* __restrict__ packed,
                                                               int B) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const uint64_t best = (uint64_t)packed[b] ^ VP_BIAS;
  const uint32_t idx = ~(uint32_t)(best & 0xffffffffu);
  out[b] = (best == 0 || idx >= 0x7fffffffu) ? 0 : (int64_t)idx;
}

int sample_splits(int B) {
  // enough 1024-thread blocks to cover the chip at small batch; 1 block/row at large
  return B >= 512 ? 1 : std::min(32, (512 + B - 1) / B);
}

static void sample_blocks(int dtype, uint64_t* partial, const void* logits, int64_t row_stride,
                          int B, int V, const float* temperature, const int* top_k,
                          const float* top_p, const int64_t* seeds, int vocab_off, dim3 grid,
                          hipStream_t s) {
  if (dtype == DT_BF16)
    sample_kernel<bf16><<<grid, SMP_NT, 0, s>>>(partial, (const bf16*)logits, row_stride, V,
                                                temperature, top_k, top_p, seeds, vocab_off);
  else if (dtype == DT_F16)
    sample_kernel<f16><<<grid, SMP_NT, 0, s>>>(partial, (const f16*)logits, row_stride, V,
                                               temperature, top_k, top_p, seeds, vocab_off);
  else
    sample_kernel<float><<<grid, SMP_NT, 0, s>>>(partial, (const float*)logits, row_stride, V,
                                                 temperature, top_k, top_p, seeds, vocab_off);
}

void launch_sample(int dtype, int64_t* out, uint64_t* partial, const void* logits,
                   int64_t row_stride, int B, int V, const float* temperature, const int* top_k,
                   const float* top_p, const int64_t* seeds, hipStream_t s) {
  if (B == 0) return;
  const dim3 grid(B, sample_splits(B));
  sample_blocks(dtype, partial, logits, row_stride, B, V, temperature, top_k, top_p, seeds, 0,
                grid, s);
  sample_merge_kernel<<<(B + 255) / 256, 256, 0, s>>>(out, partial, B, grid.y);
}

void launch_sample_vp(int dtype, int64_t* packed, uint64_t* partial, const void* logits,
                      int64_t row_stride, int B, int V, const float* temperature,
                      const int64_t* seeds, int vocab_off, hipStream_t s) {
  if (B == 0) return;
  const dim3 grid(B, sample_splits(B));
  sample_blocks(dtype, partial, logits, row_stride, B, V, temperature, nullptr, nullptr, seeds,
                vocab_off, grid, s);
  sample_vp_merge_kernel<<<(B + 255) / 256, 256, 0, s>>>(packed, partial, B, grid.y);
}

void launch_sample_vp_unpack(int64_t* out, const int64_t* packed, int B, hipStream_t s) {
  if (B == 0) return;
  sample_vp_unpack_kernel<<<(B + 255) / 256, 256, 0, s>>>(out, packed, B);
}

}  // namespace kgc

namespace kgc {
void* sample_err_addr() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_smp_err)) != hipSuccess) return nullptr;
  return p;
}
}  // namespace kgc
