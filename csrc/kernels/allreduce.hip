// K12: one-shot / two-shot all-reduce over xGMI peer memory (SURVEY.md §2.5 K12;
// the reference only toggles it: values-01-minimal-example8.yaml:32
// `--disable-custom-all-reduce`).
//
// Every TP rank owns one uncached IPC buffer: [ArSignal][data parity 0][data parity 1]
// [fused parity 0][fused parity 1] (the last two for allreduce_rms_kernel).
// The peers' buffers are mapped into each process (hipIpcOpenMemHandle), so a kernel
// reads the other GPUs' HBM directly over the point-to-point xGMI links -- all 7 links
// of an MI355X in parallel, instead of RCCL's ring that is bound by one link per step.
//
//  one-shot (small messages, latency bound): copy in -> flag barrier -> every rank
//     sums all NR inputs (reads (NR-1) x bytes remote).
//  two-shot (medium): copy in -> barrier -> rank r reduces segment r in place ->
//     barrier -> every rank gathers the NR reduced segments (reads 2 (NR-1)/NR x bytes).
//
// Barriers are per workgroup: block b of every rank touches the same element set, so
// block b only waits for block b of its peers.  The grid is ALWAYS AR_MAX_BLOCKS wide
// (empty blocks still take part in the barrier): the per-block epoch parity protects
// element v across calls only if v maps to the same block in every call (epoch flags, monotonically increasing,
// never reset).  Data regions alternate by epoch parity so a slow peer still reading
// epoch e never sees epoch e+1's copy-in.  The epoch counter lives in device memory, so
// the launch is hipGraph-capturable (kernel arguments are frozen at capture).
// Spins are bounded: a missing peer sets ArSignal::err (checked by the host) instead of
// hanging the GPU.
#include <cstring>
#include <stdexcept>
#include <string>

#include "common.h"
#include "launch.h"

namespace kgc {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 64;    // one-shot / two-shot / one-shot fused grid
constexpr int AR2_BLOCKS = 128;      // row-segmented two-shot fused grid (2 rows per block at
                                     // M = 256; 4 ranks' grids must fit one GPU in the tests)
constexpr int AR_THREADS = 512;
constexpr int AR3_BLOCKS = 256;      // the WIDE plain two-shot grid (large decode messages:
                                     // 4x the loads in flight of the 64-block grid)

struct ArSignal {
  uint32_t counter[AR_MAX_BLOCKS];                     // local: last epoch per block
  uint32_t flag[2][AR_MAX_BLOCKS][AR_MAX_RANKS];       // written by peers
  uint32_t err;
  uint32_t pad[63];
  // the row-segmented two-shot fused kernel's own epochs and flags (its grid differs)
  uint32_t counter2[AR2_BLOCKS];
  uint32_t flag2[2][AR2_BLOCKS][AR_MAX_RANKS];
  // the wide plain two-shot kernel's own epochs and flags (its grid differs again)
  uint32_t counter3[AR3_BLOCKS];
  uint32_t flag3[2][AR3_BLOCKS][AR_MAX_RANKS];
};

size_t allreduce_signal_bytes() { return (sizeof(ArSignal) + 4095) & ~size_t(4095); }

__device__ __forceinline__ void ar_store_flag(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ar_load_flag(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Flag set of one grid geometry (SET): 0 the plain / one-shot fused kernels
// (AR_MAX_BLOCKS), 1 the row-segmented fused kernel (AR2_BLOCKS), 2 the wide plain
// two-shot kernel (AR3_BLOCKS) -- counter[blk] and flag[phase][blk][rank] of each.
template <int SET>
__device__ __forceinline__ uint32_t* ar_counter(ArSignal* s, int blk) {
  if constexpr (SET == 1) return &s->counter2[blk];
  else if constexpr (SET == 2) return &s->counter3[blk];
  else return &s->counter[blk];
}
template <int SET>
__device__ __forceinline__ uint32_t* ar_flag(ArSignal* s, int phase, int blk, int r) {
  if constexpr (SET == 1) return &s->flag2[phase][blk][r];
  else if constexpr (SET == 2) return &s->flag3[phase][blk][r];
  else return &s->flag[phase][blk][r];
}
template <int SET>
constexpr int ar_grid() { return SET == 1 ? AR2_BLOCKS : SET == 2 ? AR3_BLOCKS : AR_MAX_BLOCKS; }

// Publish this block's writes to every peer, then wait for block `blk` of every peer.
// `blk` is the block's index within ITS RANK's grid: blockIdx.x on a real rank, the
// position inside the rank's slice of the grid in world emulation (all ranks' blocks in
// one launch on one device, see launch_allreduce_emu).
template <int NR, int SET = 0>
__device__ __forceinline__ void ar_barrier(const ArPtrs& P, int rank, int blk, int phase,
                                           uint32_t epoch) {
  // every wave drains its own stores first (vmcnt is per wave; do not rely on the
  // barrier's implicit wait), then one lane per peer releases at system scope
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < NR) {
    __threadfence_system();   // release: copy-in / reduced data visible system-wide
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ArSignal* peer = reinterpret_cast<ArSignal*>(P.sig[threadIdx.x]);
    ar_store_flag(ar_flag<SET>(peer, phase, blk, rank), epoch);
    ArSignal* self = reinterpret_cast<ArSignal*>(P.sig[rank]);
    uint32_t* f = ar_flag<SET>(self, phase, blk, threadIdx.x);
    const unsigned long long dl = spin_deadline(KGC_PEER_SPIN_MS);
    // a group that already failed (sticky err) does not wait again: one time-out per
    // dead peer, not one per collective (graph warm-ups run dozens back to back)
    const bool failed = ar_load_flag(&self->err) != 0u;
    while (!failed && (int32_t)(ar_load_flag(f) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (spin_expired(dl)) {        // a peer is gone: fail loudly on the host
        // ... on EVERY rank's host: the word is raised in each peer's signal too, so the
        // driver rank sees a time-out that only a worker rank observed (that worker
        // would otherwise carry on with a stale peer input, silently, unchecked)
        for (int p = 0; p < NR; ++p)
          __hip_atomic_fetch_or(&reinterpret_cast<ArSignal*>(P.sig[p])->err,
                                1u << threadIdx.x, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __threadfence_system();   // acquire
  }
  __syncthreads();
}

__device__ __forceinline__ u32x4 ld_peer(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// this rank's next epoch for block blk (read by thread 0, shared through LDS)
template <int SET>
__device__ __forceinline__ uint32_t ar_epoch(const ArPtrs& P, int rank, int blk) {
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0)
    s_epoch = *ar_counter<SET>(reinterpret_cast<ArSignal*>(P.sig[rank]), blk) + 1;
  __syncthreads();
  return s_epoch;
}

// ---- plain all-reduce body: block `blk` of rank `rank` (ar_grid<SET>() blocks per rank;
// SET 0 the 64-block grid of both forms, SET 2 the wide two-shot grid with its own epochs,
// flags and data regions -- element v -> block (v / AR_THREADS) % grid must be the same in
// every call of a set, so the two grids never share them)
template <typename T, int NR, bool TWO, int SET = 0>
__device__ __forceinline__ void allreduce_body(const ArPtrs& P, int rank, int blk, T* inout,
                                               int64_t nvec, int64_t cap_vec) {
  const uint32_t epoch = ar_epoch<SET>(P, rank, blk);
  const int64_t par_off = (int64_t)(epoch & 1) * cap_vec;
  u32x4* io = reinterpret_cast<u32x4*>(inout);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]) + par_off;
  const int64_t stride = (int64_t)ar_grid<SET>() * AR_THREADS;
  const int64_t first = (int64_t)blk * AR_THREADS + threadIdx.x;

  for (int64_t v = first; v < nvec; v += stride) mine[v] = io[v];
  ar_barrier<NR, SET>(P, rank, blk, 0, epoch);

  auto reduce_at = [&](int64_t v) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    Pack8<T> in[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r)
      in[r].u = ld_peer(reinterpret_cast<const u32x4*>(P.data[r]) + par_off + v);
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += to_f<T>(in[r].h[j]);
    Pack8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.h[j] = from_f<T>(acc[j]);
    return o.u;
  };

  if constexpr (!TWO) {
    for (int64_t v = first; v < nvec; v += stride) io[v] = reduce_at(v);
  } else {
    // Every phase walks the SAME element -> block mapping as the copy-in (element v
    // belongs to block (v / AR_THREADS) % AR_MAX_BLOCKS): block b's barrier then covers
    // exactly the elements block b reads.  (Indexing the segment from its own start
    // would hand block b elements another block copied in, whose peers it never waited
    // for -- a race whenever the segment start is not a multiple of the grid stride.)
    const int64_t seg = nvec / NR;    // host guarantees nvec % NR == 0
    const int64_t lo = (int64_t)rank * seg, hi = lo + seg;
    for (int64_t v = first; v < nvec; v += stride)
      if (v >= lo && v < hi) mine[v] = reduce_at(v);
    ar_barrier<NR, SET>(P, rank, blk, 1, epoch);
    for (int64_t v = first; v < nvec; v += stride) {
      const int r = (int)(v / seg);   // owner of the reduced segment holding v
      io[v] = ld_peer(reinterpret_cast<const u32x4*>(P.data[r]) + par_off + v);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) *ar_counter<SET>(reinterpret_cast<ArSignal*>(P.sig[rank]), blk) = epoch;
}

template <typename T, int NR, bool TWO, int SET = 0>
__global__ __launch_bounds__(AR_THREADS) void allreduce_kernel(ArPtrs P, int rank, T* inout,
                                                               int64_t nvec, int64_t cap_vec) {
  allreduce_body<T, NR, TWO, SET>(P, rank, blockIdx.x, inout, nvec, cap_vec);
}

// World emulation: every rank's blocks in ONE grid on one device, each rank with its own
// signal / data buffers and its own input -- the 8-rank barrier, parity and segment logic
// run exactly as on 8 GPUs.  The grid is block-major (blockIdx = blk * NR + rank): the NR
// blocks that wait for each other are adjacent in dispatch order, so with blocks
// dispatched in order (as observed) the oldest unfinished group is always resident and
// the grid never deadlocks whatever its size -- which eight processes sharing one GPU
// cannot promise (their kernels need not be co-resident at all).  A violation would show
// as the bounded spin's error word, never a hang.
template <typename T, int NR, bool TWO, int SET = 0>
__global__ __launch_bounds__(AR_THREADS) void allreduce_emu_kernel(ArPtrs P, ArWorld W,
                                                                   int64_t nvec, int64_t cap_vec) {
  const int rank = blockIdx.x % NR, blk = blockIdx.x / NR;
  allreduce_body<T, NR, TWO, SET>(P, rank, blk, reinterpret_cast<T*>(W.a[rank]), nvec, cap_vec);
}

// ---- fused one-shot all-reduce + residual add + RMSNorm (row-parallel o / down
// projections at TP > 1):  h = sum_r in_r (rounded to T, as the all-reduce stores it);
// residual += h (rounded);  out = rms_norm(residual) * w  -- the same rounding points
// as xgmi_allreduce followed by fused_add_rms_norm (norm.hip), in one launch and one
// pass over the peers' rows.
// Rows map to blocks (row % AR_MAX_BLOCKS) in the copy-in and in the reduce, so block
// b's barrier covers exactly the rows block b reads.  This kernel has its own IPC data
// regions (P.data points past the plain all-reduce's two), so a peer block still in an
// earlier call of the OTHER kernel -- whose element -> block mapping differs -- never
// reads memory this one overwrites.
constexpr int ARN_MAXV = 4;   // 512 threads x 4 x 8 = 16384 = widest hidden supported

// residual += h (rounded), out = rms_norm(residual) * w for one row whose all-reduced
// values h (already rounded to T) are in hv[]; every rank computes identical bytes
template <typename T>
__device__ __forceinline__ void ar_add_norm_row(Pack8<T>* hv, const Pack8<T>* wv, T* residual,
                                                T* out, int64_t row, int nv, int H, float eps,
                                                float* scratch) {
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < ARN_MAXV; ++i) {
    const int v = threadIdx.x + i * AR_THREADS;
    if (v >= nv) continue;
    const int64_t e = row * nv + v;
    Pack8<T> res;
    res.u = reinterpret_cast<const u32x4*>(residual)[e];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      hv[i].h[j] = from_f<T>(to_f<T>(hv[i].h[j]) + to_f<T>(res.h[j]));   // residual += h
      const float f = to_f<T>(hv[i].h[j]);
      ss += f * f;
    }
    reinterpret_cast<u32x4*>(residual)[e] = hv[i].u;
  }
  ss = block_sum<AR_THREADS>(ss, scratch);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < ARN_MAXV; ++i) {
    const int v = threadIdx.x + i * AR_THREADS;
    if (v >= nv) continue;
    Pack8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o.h[j] = from_f<T>(to_f<T>(hv[i].h[j]) * inv * to_f<T>(wv[i].h[j]));
    reinterpret_cast<u32x4*>(out)[row * nv + v] = o.u;
  }
}

// sum of the NR ranks' copies of 16-B vector e, rounded to T (the all-reduce's output)
template <typename T, int NR>
__device__ __forceinline__ u32x4 ar_sum_vec(const ArPtrs& P, int64_t par_off, int64_t e) {
  Pack8<T> pk[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r)
    pk[r].u = ld_peer(reinterpret_cast<const u32x4*>(P.data[r]) + par_off + e);
  Pack8<T> o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r) acc += to_f<T>(pk[r].h[j]);
    o.h[j] = from_f<T>(acc);
  }
  return o.u;
}

template <typename T, int NR>
__device__ __forceinline__ void allreduce_rms_body(const ArPtrs& P, int rank, int blk,
                                                   const T* __restrict__ in, T* __restrict__ out,
                                                   T* __restrict__ residual,
                                                   const T* __restrict__ w, int M, int H,
                                                   float eps, int64_t cap_vec) {
  __shared__ float scratch[AR_THREADS / 64];
  const uint32_t epoch = ar_epoch<0>(P, rank, blk);
  const int64_t par_off = (int64_t)(epoch & 1) * cap_vec;
  const int nv = H >> 3;                             // 16-byte vectors per row
  const u32x4* src = reinterpret_cast<const u32x4*>(in);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]) + par_off;

  for (int row = blk; row < M; row += AR_MAX_BLOCKS)
    for (int v = threadIdx.x; v < nv; v += AR_THREADS)
      mine[(int64_t)row * nv + v] = src[(int64_t)row * nv + v];
  ar_barrier<NR>(P, rank, blk, 0, epoch);

  Pack8<T> wv[ARN_MAXV];
#pragma unroll
  for (int i = 0; i < ARN_MAXV; ++i) {
    const int v = threadIdx.x + i * AR_THREADS;
    if (v < nv) wv[i].u = reinterpret_cast<const u32x4*>(w)[v];
  }
  for (int row = blk; row < M; row += AR_MAX_BLOCKS) {   // uniform per block
    Pack8<T> h[ARN_MAXV];
#pragma unroll
    for (int i = 0; i < ARN_MAXV; ++i) {
      const int v = threadIdx.x + i * AR_THREADS;
      if (v < nv) h[i].u = ar_sum_vec<T, NR>(P, par_off, (int64_t)row * nv + v);
    }
    ar_add_norm_row<T>(h, wv, residual, out, row, nv, H, eps, scratch);
  }
  __syncthreads();
  if (threadIdx.x == 0) *ar_counter<0>(reinterpret_cast<ArSignal*>(P.sig[rank]), blk) = epoch;
}

template <typename T, int NR>
__global__ __launch_bounds__(AR_THREADS) void allreduce_rms_kernel(
    ArPtrs P, int rank, const T* __restrict__ in, T* __restrict__ out, T* __restrict__ residual,
    const T* __restrict__ w, int M, int H, float eps, int64_t cap_vec) {
  allreduce_rms_body<T, NR>(P, rank, blockIdx.x, in, out, residual, w, M, H, eps, cap_vec);
}

template <typename T, int NR>
__global__ __launch_bounds__(AR_THREADS) void allreduce_rms_emu_kernel(
    ArPtrs P, ArWorld W, const T* __restrict__ w, int M, int H, float eps, int64_t cap_vec) {
  const int rank = blockIdx.x % NR, blk = blockIdx.x / NR;
  allreduce_rms_body<T, NR>(P, rank, blk, reinterpret_cast<const T*>(W.a[rank]),
                            reinterpret_cast<T*>(W.b[rank]), reinterpret_cast<T*>(W.c[rank]), w,
                            M, H, eps, cap_vec);
}

// ---- row-segmented TWO-SHOT fused all-reduce + residual add + RMSNorm (TP = 4 / 8
// decode at real batch sizes: 256 rows x 8192 = 4 MB per call, 16x the one-shot cap).
//   copy-in:  block b writes its rows {row % AR2_BLOCKS == b} into the own IPC buffer;
//   reduce:   row `row` is owned by rank (row + row / AR2_BLOCKS) % NR -- the rows of one
//             block have different owners, so every rank's reduce spreads over as many
//             blocks as it owns rows; block b sums ITS owned rows over all peers (rounded
//             to T: the all-reduce output) in place; barrier;
//   gather:   block b reads each of its rows from the row's owner -- whole rows, so the
//             residual add and the RMSNorm run right there: the reduced rows are read
//             2 (NR-1)/NR x bytes per rank like the plain two-shot, and no second kernel
//             re-reads them for the norm.
// Every phase maps row -> block the same way (row % AR2_BLOCKS), so block b's barriers
// cover exactly the rows block b reads, and its own epoch counters / flags (counter2 /
// flag2) and data regions keep calls of the other kernels out of its way.  Every rank
// computes the same residual / out bytes from the same owner rows.
template <typename T, int NR>
__device__ __forceinline__ void allreduce_rms2_body(const ArPtrs& P, int rank, int blk,
                                                    const T* __restrict__ in,
                                                    T* __restrict__ out,
                                                    T* __restrict__ residual,
                                                    const T* __restrict__ w, int M, int H,
                                                    float eps, int64_t cap_vec) {
  __shared__ float scratch[AR_THREADS / 64];
  const uint32_t epoch = ar_epoch<1>(P, rank, blk);
  const int64_t par_off = (int64_t)(epoch & 1) * cap_vec;
  const int nv = H >> 3;
  const u32x4* src = reinterpret_cast<const u32x4*>(in);
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]) + par_off;

  for (int row = blk; row < M; row += AR2_BLOCKS)
    for (int v = threadIdx.x; v < nv; v += AR_THREADS)
      mine[(int64_t)row * nv + v] = src[(int64_t)row * nv + v];
  ar_barrier<NR, 1>(P, rank, blk, 0, epoch);
  auto owner = [](int row) { return (row + row / AR2_BLOCKS) % NR; };
  for (int row = blk; row < M; row += AR2_BLOCKS) {
    if (owner(row) != rank) continue;
    for (int v = threadIdx.x; v < nv; v += AR_THREADS) {
      const int64_t e = (int64_t)row * nv + v;
      const u32x4 s = ar_sum_vec<T, NR>(P, par_off, e);
      mine[e] = s;
    }
  }
  ar_barrier<NR, 1>(P, rank, blk, 1, epoch);
  Pack8<T> wv[ARN_MAXV];
#pragma unroll
  for (int i = 0; i < ARN_MAXV; ++i) {
    const int v = threadIdx.x + i * AR_THREADS;
    if (v < nv) wv[i].u = reinterpret_cast<const u32x4*>(w)[v];
  }
  for (int row = blk; row < M; row += AR2_BLOCKS) {
    const u32x4* own = reinterpret_cast<const u32x4*>(P.data[owner(row)]) + par_off;
    Pack8<T> h[ARN_MAXV];
#pragma unroll
    for (int i = 0; i < ARN_MAXV; ++i) {
      const int v = threadIdx.x + i * AR_THREADS;
      if (v < nv) h[i].u = ld_peer(own + (int64_t)row * nv + v);
    }
    ar_add_norm_row<T>(h, wv, residual, out, row, nv, H, eps, scratch);
  }
  __syncthreads();
  if (threadIdx.x == 0) *ar_counter<1>(reinterpret_cast<ArSignal*>(P.sig[rank]), blk) = epoch;
}

template <typename T, int NR>
__global__ __launch_bounds__(AR_THREADS) void allreduce_rms2_kernel(
    ArPtrs P, int rank, const T* __restrict__ in, T* __restrict__ out, T* __restrict__ residual,
    const T* __restrict__ w, int M, int H, float eps, int64_t cap_vec) {
  allreduce_rms2_body<T, NR>(P, rank, blockIdx.x, in, out, residual, w, M, H, eps, cap_vec);
}

template <typename T, int NR>
__global__ __launch_bounds__(AR_THREADS) void allreduce_rms2_emu_kernel(
    ArPtrs P, ArWorld W, const T* __restrict__ w, int M, int H, float eps, int64_t cap_vec) {
  const int rank = blockIdx.x % NR, blk = blockIdx.x / NR;
  allreduce_rms2_body<T, NR>(P, rank, blk, reinterpret_cast<const T*>(W.a[rank]),
                             reinterpret_cast<T*>(W.b[rank]), reinterpret_cast<T*>(W.c[rank]), w,
                             M, H, eps, cap_vec);
}

#define KGC_AR_RANKS(NR_, CALL) \
  switch (NR_) {                \
    case 2: CALL(2); break;     \
    case 4: CALL(4); break;     \
    case 8: CALL(8); break;     \
    default: break;             \
  }

template <typename T>
static void arn_by_ranks(int nranks, const ArPtrs& P, int rank, const void* in, void* out,
                         void* residual, const void* w, int M, int H, float eps, int64_t cap_vec,
                         bool two, hipStream_t s) {
#define KGC_ARN(NR_)                                                                             \
  if (two)                                                                                       \
    allreduce_rms2_kernel<T, NR_><<<AR2_BLOCKS, AR_THREADS, 0, s>>>(                             \
        P, rank, (const T*)in, (T*)out, (T*)residual, (const T*)w, M, H, eps, cap_vec);          \
  else                                                                                           \
    allreduce_rms_kernel<T, NR_><<<AR_MAX_BLOCKS, AR_THREADS, 0, s>>>(                           \
        P, rank, (const T*)in, (T*)out, (T*)residual, (const T*)w, M, H, eps, cap_vec)
  KGC_AR_RANKS(nranks, KGC_ARN)
#undef KGC_ARN
}

int allreduce_rms_max_hidden() { return AR_THREADS * ARN_MAXV * 8; }

void launch_allreduce_rms(int dtype, const ArPtrs& P, int nranks, int rank, const void* in,
                          void* out, void* residual, const void* w, int M, int H, float eps,
                          int64_t cap_vec, bool two_shot, hipStream_t s) {
  if (dtype == DT_BF16)
    arn_by_ranks<bf16>(nranks, P, rank, in, out, residual, w, M, H, eps, cap_vec, two_shot, s);
  else
    arn_by_ranks<f16>(nranks, P, rank, in, out, residual, w, M, H, eps, cap_vec, two_shot, s);
}

template <typename T>
static void ar_by_ranks(int nranks, const ArPtrs& P, int rank, void* inout, int64_t nvec,
                        int64_t cap_vec, bool two, bool wide, hipStream_t s) {
#define KGC_AR(NR_)                                                                          \
  if (two && wide)                                                                           \
    allreduce_kernel<T, NR_, true, 2><<<AR3_BLOCKS, AR_THREADS, 0, s>>>(P, rank, (T*)inout,  \
                                                                        nvec, cap_vec);      \
  else if (two)                                                                              \
    allreduce_kernel<T, NR_, true><<<AR_MAX_BLOCKS, AR_THREADS, 0, s>>>(P, rank, (T*)inout,  \
                                                                        nvec, cap_vec);      \
  else                                                                                       \
    allreduce_kernel<T, NR_, false><<<AR_MAX_BLOCKS, AR_THREADS, 0, s>>>(P, rank, (T*)inout, \
                                                                         nvec, cap_vec)
  KGC_AR_RANKS(nranks, KGC_AR)
#undef KGC_AR
}

int allreduce_max_blocks() { return AR_MAX_BLOCKS; }
int peer_spin_ms() { return KGC_PEER_SPIN_MS; }
int coop_spin_ms() { return KGC_COOP_SPIN_MS; }

void launch_allreduce(int dtype, const ArPtrs& P, int nranks, int rank, void* inout,
                      int64_t nvec, int64_t cap_vec, bool two_shot, bool wide, hipStream_t s) {
  if (dtype == DT_BF16)
    ar_by_ranks<bf16>(nranks, P, rank, inout, nvec, cap_vec, two_shot, wide, s);
  else
    ar_by_ranks<f16>(nranks, P, rank, inout, nvec, cap_vec, two_shot, wide, s);
}

// ---- world emulation launches (tests): kind 0 plain one-shot, 1 plain two-shot,
// 2 fused one-shot, 3 fused two-shot (row-segmented).  W.a = inout / in, W.b = out,
// W.c = residual of each rank; P.data = each rank's data region for the kernel kind.
template <typename T>
static void ar_emu_t(int kind, const ArPtrs& P, const ArWorld& W, int nranks, int64_t nvec,
                     const void* w, int M, int H, float eps, int64_t cap_vec, hipStream_t s) {
  const int g1 = nranks * AR_MAX_BLOCKS, g2 = nranks * AR2_BLOCKS, g3 = nranks * AR3_BLOCKS;
#define KGC_EMU(NR_)                                                                           \
  switch (kind) {                                                                              \
    case 0: allreduce_emu_kernel<T, NR_, false><<<g1, AR_THREADS, 0, s>>>(P, W, nvec, cap_vec); \
      break;                                                                                   \
    case 1: allreduce_emu_kernel<T, NR_, true><<<g1, AR_THREADS, 0, s>>>(P, W, nvec, cap_vec);  \
      break;                                                                                   \
    case 2: allreduce_rms_emu_kernel<T, NR_><<<g1, AR_THREADS, 0, s>>>(P, W, (const T*)w, M, H, \
                                                                       eps, cap_vec);          \
      break;                                                                                   \
    case 4: allreduce_emu_kernel<T, NR_, true, 2><<<g3, AR_THREADS, 0, s>>>(P, W, nvec, cap_vec); \
      break;                                                                                   \
    default: allreduce_rms2_emu_kernel<T, NR_><<<g2, AR_THREADS, 0, s>>>(P, W, (const T*)w, M,  \
                                                                         H, eps, cap_vec);     \
      break;                                                                                   \
  }
  KGC_AR_RANKS(nranks, KGC_EMU)
#undef KGC_EMU
}

void launch_allreduce_emu(int dtype, int kind, const ArPtrs& P, const ArWorld& W, int nranks,
                          int64_t nvec, const void* w, int M, int H, float eps, int64_t cap_vec,
                          hipStream_t s) {
  if (dtype == DT_BF16) ar_emu_t<bf16>(kind, P, W, nranks, nvec, w, M, H, eps, cap_vec, s);
  else ar_emu_t<f16>(kind, P, W, nranks, nvec, w, M, H, eps, cap_vec, s);
}

// ---- phantom TP rank (KGC_TP_PHANTOM, parallel/custom_allreduce.py PhantomAllReduce):
// one process runs rank `rank`'s shard of a TP = NR model on one GPU; the NR - 1 peers are
// local buffers that never run a kernel.  Their arrival flags in this rank's signal are
// raised to `value` (far ahead of any epoch: the barrier's wrap-safe (flag - epoch) test
// then passes for 2^30 calls per block), so the real kernels run their full sequence --
// copy-in, barriers, peer reads, the fused add + norm -- inside the captured graphs.
// Vector stores from one workgroup; a step's kernels are ordered behind it by the stream.
__global__ __launch_bounds__(256) void ar_raise_peer_flags_kernel(ArSignal* s, int rank,
                                                                  int nranks, uint32_t value) {
  for (int i = threadIdx.x; i < 2 * AR_MAX_BLOCKS * AR_MAX_RANKS; i += blockDim.x) {
    const int r = i % AR_MAX_RANKS;
    if (r != rank && r < nranks) (&s->flag[0][0][0])[i] = value;
  }
  for (int i = threadIdx.x; i < 2 * AR2_BLOCKS * AR_MAX_RANKS; i += blockDim.x) {
    const int r = i % AR_MAX_RANKS;
    if (r != rank && r < nranks) (&s->flag2[0][0][0])[i] = value;
  }
  for (int i = threadIdx.x; i < 2 * AR3_BLOCKS * AR_MAX_RANKS; i += blockDim.x) {
    const int r = i % AR_MAX_RANKS;
    if (r != rank && r < nranks) (&s->flag3[0][0][0])[i] = value;
  }
}

void ar_raise_peer_flags(void* sig, int rank, int nranks, uint32_t value, hipStream_t s) {
  ar_raise_peer_flags_kernel<<<1, 256, 0, s>>>(reinterpret_cast<ArSignal*>(sig), rank, nranks,
                                               value);
}

// ---- IPC buffer management (host) ----------------------------------------------
static void ar_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

int64_t wall_clock_rate_khz() {
  int dev = 0, khz = 0;
  ar_check(hipGetDevice(&dev), "hipGetDevice");
  ar_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev),
           "hipDeviceGetAttribute(WallClockRate)");
  return khz;
}

void* ar_alloc(int64_t bytes) {
  void* p = nullptr;
  // uncached: flags and peer-written data must never sit stale in a local L2
  ar_check(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags");
  ar_check(hipMemset(p, 0, bytes), "hipMemset");
  ar_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return p;
}

void ar_free(void* p) { ar_check(hipFree(p), "hipFree"); }

void ar_get_handle(void* p, uint8_t* out64) {
  hipIpcMemHandle_t h;
  ar_check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
  static_assert(sizeof(h) <= 64, "IPC handle larger than 64 bytes");
  memset(out64, 0, 64);
  memcpy(out64, &h, sizeof(h));
}

void* ar_open_handle(const uint8_t* in64) {
  hipIpcMemHandle_t h;
  memcpy(&h, in64, sizeof(h));
  void* p = nullptr;
  ar_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return p;
}

void ar_close_handle(void* p) { ar_check(hipIpcCloseMemHandle(p), "hipIpcCloseMemHandle"); }

// stream-ordered copy of the sticky error word (read on the host once the step is done)
void ar_err_copy_async(void* sig, uint32_t* host_dst, hipStream_t s) {
  ar_check(hipMemcpyAsync(host_dst, &reinterpret_cast<ArSignal*>(sig)->err, 4,
                          hipMemcpyDeviceToHost, s),
           "xgmi allreduce: error word copy");
}

uint32_t ar_read_err(void* sig) {
  uint32_t e = 0;
  ar_check(hipMemcpy(&e, &reinterpret_cast<ArSignal*>(sig)->err, 4, hipMemcpyDeviceToHost),
           "hipMemcpy");
  return e;
}

}  // namespace kgc
