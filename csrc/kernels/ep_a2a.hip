// C7 expert-parallel dispatch / combine over xGMI peer memory, graph-capturable.
//
// The reference's EP all-to-all is an NCCL all_to_allv with host-side counts (BASELINE
// config 4).  Host-known split sizes cannot be replayed from a hipGraph, so here every
// rank exposes an IPC buffer and the routing stays on the device:
//
//   dispatch (source r):  per (token, slot) pair, owner d = expert / E_local; the
//       pair's position among r's pairs for d comes from a wave-ballot prefix scan
//       (deterministic order).  Its activation row, (local expert, pair index) and r's
//       count for d are written straight into d's receive region [r] (one-sided puts
//       over xGMI); the last workgroup to finish raises flag0[r] on every peer.
//   receive (owner d):    wait for flag0 of every source, copy the valid rows into a
//       local [NR * C, H] tensor and emit per-row expert ids (-1 = empty slot) for the
//       grouped expert MLP (K14, ops.fused_moe).
//   return (owner d):     put each result row back into its source's return region at
//       the pair's index; the last workgroup raises flag1[d] on every peer.
//   combine (source r):   wait for flag1 of every owner; out[t] = sum_j w[t, j] * ret[t*k + j].
//
// Traffic is proportional to the actual routing (no padding on the wire).  Regions are
// double-buffered by call parity and the epoch lives in device memory (bumped by a
// 1-thread kernel after the combine), so the whole block replays from a graph.  Spins
// are bounded: a missing peer sets EpSignal::err, which the host checks.
#include "common.h"
#include "launch.h"

namespace kgc {

constexpr int EP_MAX_RANKS = 8;
constexpr int EP_THREADS = 512;
constexpr int EP_WAVES = EP_THREADS / 64;
// dispatch / receive / return: one wave per row (pair / slot), 512 rows in flight.  One
// workgroup per row walked the 4,096 receive slots 64 deep, a dependent route / count load
// per step (~20 us per phase at Mixtral's EP = 8 decode shapes).  The grid stays at 64
// workgroups: each one that publishes pays a system-scope fence and a serialised atomic
// on the uncached signal (128 workgroups measured slower for dispatch / return)
constexpr int EP_BLOCKS = 64;
// the combine publishes nothing and runs a workgroup per token
constexpr int EP_COMBINE_BLOCKS = 128;
constexpr int EP_MAX_PAIRS = 4096;   // T * k of one call (decode buckets)

struct EpSignal {
  uint32_t counter;                     // epoch of the last completed call
  uint32_t done[2];                     // workgroups finished (dispatch, return)
  uint32_t flag[2][EP_MAX_RANKS];       // written by peers: [0] rows arrived, [1] results back
  uint32_t err;
  uint32_t pad[1024 - 4 - 2 * EP_MAX_RANKS];
};

size_t ep_signal_bytes() { return (sizeof(EpSignal) + 4095) & ~size_t(4095); }

__device__ __forceinline__ void ep_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ep_load(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t ep_epoch(const EpPtrs& P, int rank) {
  return reinterpret_cast<EpSignal*>(P.sig[rank])->counter + 1;
}

// byte offsets of one rank's regions for call parity `par` (see ep_region_bytes)
struct EpLayout {
  int64_t x, meta, cnt, ret;
  __host__ __device__ EpLayout(int nr, int C, int H, int esz, int par) {
    const int64_t xb = (int64_t)nr * C * H * esz, mb = (int64_t)nr * C * 8, cb = 256,
                  rb = (int64_t)C * H * esz;
    int64_t o = 0;
    x = o + par * xb;
    o += 2 * xb;
    meta = o + par * mb;
    o += 2 * mb;
    cnt = o + par * cb;
    o += 2 * cb;
    ret = o + par * rb;
  }
};

int64_t ep_region_bytes(int nr, int C, int H, int esz) {
  const int64_t xb = (int64_t)nr * C * H * esz, mb = (int64_t)nr * C * 8, cb = 256,
                rb = (int64_t)C * H * esz;
  return 2 * (xb + mb + cb + rb);
}

// every wave has finished its stores -> one release at system scope -> count the
// workgroup; the last one to arrive publishes `flag[phase][rank] = epoch` to every peer
template <int NR>
__device__ void ep_grid_publish(const EpPtrs& P, int rank, int phase, uint32_t epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) {
    __threadfence_system();
    EpSignal* self = reinterpret_cast<EpSignal*>(P.sig[rank]);
    last = atomicAdd(&self->done[phase], 1u) == gridDim.x - 1;
    if (last) {
      self->done[phase] = 0;
      __threadfence_system();
    }
  }
  __syncthreads();
  if (last && threadIdx.x < NR) {
    EpSignal* peer = reinterpret_cast<EpSignal*>(P.sig[threadIdx.x]);
    ep_store(&peer->flag[phase][rank], epoch);
  }
}

// one thread per peer waits for flag[phase][peer] >= epoch (bounded)
template <int NR>
__device__ void ep_wait_all(const EpPtrs& P, int rank, int phase, uint32_t epoch) {
  if (threadIdx.x < NR) {
    EpSignal* self = reinterpret_cast<EpSignal*>(P.sig[rank]);
    uint32_t* f = &self->flag[phase][threadIdx.x];
    const unsigned long long dl = spin_deadline(KGC_PEER_SPIN_MS);
    const bool failed = ep_load(&self->err) != 0u;   // sticky: fail fast after the first
    while (!failed && (int32_t)(ep_load(f) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (spin_expired(dl)) {      // raised on every rank, as the all-reduce does
        for (int p = 0; p < NR; ++p)
          __hip_atomic_fetch_or(&reinterpret_cast<EpSignal*>(P.sig[p])->err,
                                1u << threadIdx.x, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __threadfence_system();
  }
  __syncthreads();
}

// Destination and rank-local position of every pair, in pair order per destination:
// per wave, a ballot per destination and a popcount below the lane; wave totals then
// an exclusive scan over the waves.  Every workgroup computes the same table.
template <int NR>
__device__ void ep_positions(const int* topk_ids, int npairs, int E_local, int* s_dest,
                             int* s_pos, int* s_cnt) {
  __shared__ int wtot[EP_THREADS / 64][NR];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int base[NR];
#pragma unroll
  for (int d = 0; d < NR; ++d) base[d] = 0;
  for (int p0 = 0; p0 < npairs; p0 += EP_THREADS) {
    const int p = p0 + threadIdx.x;
    // (an out-of-range expert id is clamped to a valid owner, never an OOB index)
    const int d = p < npairs ? min(max(topk_ids[p] / E_local, 0), NR - 1) : -1;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int mypos = 0;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const uint64_t m = __ballot(d == q);
      if (d == q) mypos = __popcll(m & below);
      if (lane == 0) wtot[w][q] = __popcll(m);
    }
    __syncthreads();
    if (p < npairs) {
      int off = base[d];
      for (int v = 0; v < w; ++v) off += wtot[v][d];
      s_dest[p] = d;
      s_pos[p] = off + mypos;
    }
#pragma unroll
    for (int q = 0; q < NR; ++q)
      for (int v = 0; v < EP_THREADS / 64; ++v) base[q] += wtot[v][q];
    __syncthreads();
  }
  if (threadIdx.x < NR) s_cnt[threadIdx.x] = base[threadIdx.x];
  __syncthreads();
}

template <typename T, int NR>
__global__ __launch_bounds__(EP_THREADS) void ep_dispatch_kernel(
    EpPtrs P, int rank, const T* __restrict__ x, const int* __restrict__ topk_ids, int npairs,
    int k, int H, int E_local, int C) {
  __shared__ int s_dest[EP_MAX_PAIRS], s_pos[EP_MAX_PAIRS], s_cnt[NR];
  const uint32_t epoch = ep_epoch(P, rank);
  const int par = epoch & 1;
  const EpLayout L(NR, C, H, sizeof(T), par);
  ep_positions<NR>(topk_ids, npairs, E_local, s_dest, s_pos, s_cnt);
  const int nv = H >> 3;
  const int lane = threadIdx.x & 63;
  for (int p = blockIdx.x * EP_WAVES + (threadIdx.x >> 6); p < npairs; p += gridDim.x * EP_WAVES) {
    const int d = s_dest[p], pos = s_pos[p];
    char* base = reinterpret_cast<char*>(P.data[d]);
    const int64_t slot = (int64_t)rank * C + pos;               // d's region for source `rank`
    const u32x4* src = reinterpret_cast<const u32x4*>(x + (int64_t)(p / k) * H);
    u32x4* dst = reinterpret_cast<u32x4*>(base + L.x) + slot * nv;
    for (int v = lane; v < nv; v += 64) dst[v] = src[v];
    if (lane == 0) {
      int* meta = reinterpret_cast<int*>(base + L.meta) + 2 * slot;
      meta[0] = topk_ids[p] - d * E_local;                     // owner-local expert
      meta[1] = p;                                             // pair index at the source
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < NR) {                   // r's row count for each owner
    char* base = reinterpret_cast<char*>(P.data[threadIdx.x]);
    reinterpret_cast<int*>(base + L.cnt)[rank] = s_cnt[threadIdx.x];
  }
  ep_grid_publish<NR>(P, rank, 0, epoch);
}

// owner: wait for every source, then copy the valid rows into x_local [NR * C, H] and
// write ids (global expert id, or -1) and the (source, pair) of every slot
template <typename T, int NR>
__global__ __launch_bounds__(EP_THREADS) void ep_receive_kernel(
    EpPtrs P, int rank, T* __restrict__ x_local, int* __restrict__ ids, int* __restrict__ route,
    int H, int E_local, int C) {
  const uint32_t epoch = ep_epoch(P, rank);
  const EpLayout L(NR, C, H, sizeof(T), epoch & 1);
  ep_wait_all<NR>(P, rank, 0, epoch);
  const char* base = reinterpret_cast<const char*>(P.data[rank]);
  const int* cnt = reinterpret_cast<const int*>(base + L.cnt);
  const int* meta = reinterpret_cast<const int*>(base + L.meta);
  __shared__ int s_cnt[NR];
  if (threadIdx.x < NR) s_cnt[threadIdx.x] = cnt[threadIdx.x];
  __syncthreads();
  const int nv = H >> 3;
  const int lane = threadIdx.x & 63;
  for (int slot = blockIdx.x * EP_WAVES + (threadIdx.x >> 6); slot < NR * C;
       slot += gridDim.x * EP_WAVES) {
    const int s = slot / C, i = slot % C;
    const bool valid = i < s_cnt[s];
    if (lane == 0) {
      ids[slot] = valid ? meta[2 * slot] + rank * E_local : -1;
      route[slot] = valid ? meta[2 * slot + 1] : -1;
    }
    if (!valid) continue;
    const u32x4* src = reinterpret_cast<const u32x4*>(base + L.x) + (int64_t)slot * nv;
    u32x4* dst = reinterpret_cast<u32x4*>(x_local) + (int64_t)slot * nv;
    for (int v = lane; v < nv; v += 64) dst[v] = src[v];
  }
}

// owner: each valid result row back to its source's return region at its pair index.
// y is the grouped MLP's output in T ([NR * C, H], S = 0) or its down projection's fp32
// split-K slices ([S, >= NR * C, H], summed here and rounded once): the slices never go
// through a separate combine pass, and empty slots are never read.
template <typename T, int NR>
__global__ __launch_bounds__(EP_THREADS) void ep_return_kernel(
    EpPtrs P, int rank, const void* __restrict__ y, int S, int64_t slice_stride,
    const int* __restrict__ route, int H, int C) {
  const uint32_t epoch = ep_epoch(P, rank);
  const EpLayout L(NR, C, H, sizeof(T), epoch & 1);
  const int nv = H >> 3;
  const int lane = threadIdx.x & 63;
  for (int slot = blockIdx.x * EP_WAVES + (threadIdx.x >> 6); slot < NR * C;
       slot += gridDim.x * EP_WAVES) {
    const int p = route[slot];
    if (p < 0) continue;
    const int s = slot / C;
    u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(P.data[s]) + L.ret) +
                 (int64_t)p * nv;
    if (S == 0) {
      const u32x4* src = reinterpret_cast<const u32x4*>(y) + (int64_t)slot * nv;
      for (int v = lane; v < nv; v += 64) dst[v] = src[v];
    } else {
      const float* rowp = reinterpret_cast<const float*>(y) + (int64_t)slot * H;
      for (int v = lane; v < nv; v += 64) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int z = 0; z < S; ++z) {
          const float* src = rowp + z * slice_stride + v * 8;
          const f32x4 a = *reinterpret_cast<const f32x4*>(src);
          const f32x4 b = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc[q] += a[q];
            acc[4 + q] += b[q];
          }
        }
        Pack8<T> o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o.h[q] = from_f<T>(acc[q]);
        dst[v] = o.u;
      }
    }
  }
  ep_grid_publish<NR>(P, rank, 1, epoch);
}

// source: out[t] = sum_j w[t, j] * ret[t * k + j]  (fp32 sum, rounded once)
template <typename T, int NR>
__global__ __launch_bounds__(EP_THREADS) void ep_combine_kernel(
    EpPtrs P, int rank, T* __restrict__ out, const float* __restrict__ topk_w, int ntok, int k,
    int H, int C) {
  const uint32_t epoch = ep_epoch(P, rank);
  const EpLayout L(NR, C, H, sizeof(T), epoch & 1);
  ep_wait_all<NR>(P, rank, 1, epoch);
  const T* ret = reinterpret_cast<const T*>(reinterpret_cast<const char*>(P.data[rank]) + L.ret);
  const int nv = H >> 3;
  // a workgroup per token (the whole row in one pass at H = 4096): ntok is only T here, so
  // a wave per token would leave most of the grid idle
  for (int t = blockIdx.x; t < ntok; t += gridDim.x)
    for (int v = threadIdx.x; v < nv; v += EP_THREADS) {
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
      for (int j = 0; j < k; ++j) {
        const float wj = topk_w[t * k + j];
        Pack8<T> r;
        r.u = reinterpret_cast<const u32x4*>(ret + (int64_t)(t * k + j) * H)[v];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += wj * to_f<T>(r.h[e]);
      }
      Pack8<T> o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.h[e] = from_f<T>(acc[e]);
      reinterpret_cast<u32x4*>(out + (int64_t)t * H)[v] = o.u;
    }
}

// A phantom EP rank (KGC_TP_PHANTOM with --moe-parallel ep: rank `rank` of an EP group
// whose peers do not exist): every peer's arrival flag in this rank's signal, both phases,
// raised far ahead of any epoch (vector stores), so dispatch / receive / return / combine
// run their full sequence in the decode graphs without waiting; the peers' regions hold
// zero counts, so the owner's grouped MLP sees this rank's own rows only.
__global__ void ep_raise_peer_flags_kernel(EpSignal* s, int rank, int nranks, uint32_t value) {
  const int i = threadIdx.x;
  if (i < 2 * EP_MAX_RANKS) {
    const int r = i % EP_MAX_RANKS;
    if (r != rank && r < nranks) ep_store(&(&s->flag[0][0])[i], value);
  }
}

void ep_raise_peer_flags(void* sig, int rank, int nranks, uint32_t value, hipStream_t s) {
  ep_raise_peer_flags_kernel<<<1, 64, 0, s>>>(reinterpret_cast<EpSignal*>(sig), rank, nranks,
                                              value);
}

// after the combine (stream order: every kernel of the call has read the epoch)
__global__ void ep_bump_kernel(EpPtrs P, int rank) {
  EpSignal* self = reinterpret_cast<EpSignal*>(P.sig[rank]);
  self->counter = self->counter + 1;
}

#define KGC_EP_RANKS(NR_, CALL) \
  switch (NR_) {                \
    case 2: CALL(2); break;     \
    case 4: CALL(4); break;     \
    case 8: CALL(8); break;     \
    default: break;             \
  }

template <typename T>
static void ep_dispatch_t(const EpPtrs& P, int nr, int rank, const void* x, const int* ids,
                          int npairs, int k, int H, int E_local, int C, hipStream_t s) {
#define KGC_EPD(NR)                                                                         \
  ep_dispatch_kernel<T, NR><<<EP_BLOCKS, EP_THREADS, 0, s>>>(P, rank, (const T*)x, ids,     \
                                                              npairs, k, H, E_local, C)
  KGC_EP_RANKS(nr, KGC_EPD)
#undef KGC_EPD
}

void launch_ep_dispatch(int dtype, const EpPtrs& P, int nr, int rank, const void* x,
                        const int* topk_ids, int npairs, int k, int H, int E_local, int C,
                        hipStream_t s) {
  if (dtype == DT_BF16) ep_dispatch_t<bf16>(P, nr, rank, x, topk_ids, npairs, k, H, E_local, C, s);
  else ep_dispatch_t<f16>(P, nr, rank, x, topk_ids, npairs, k, H, E_local, C, s);
}

template <typename T>
static void ep_receive_t(const EpPtrs& P, int nr, int rank, void* x_local, int* ids, int* route,
                         int H, int E_local, int C, hipStream_t s) {
#define KGC_EPR(NR)                                                                          \
  ep_receive_kernel<T, NR><<<EP_BLOCKS, EP_THREADS, 0, s>>>(P, rank, (T*)x_local, ids, route, \
                                                             H, E_local, C)
  KGC_EP_RANKS(nr, KGC_EPR)
#undef KGC_EPR
}

void launch_ep_receive(int dtype, const EpPtrs& P, int nr, int rank, void* x_local, int* ids,
                       int* route, int H, int E_local, int C, hipStream_t s) {
  if (dtype == DT_BF16) ep_receive_t<bf16>(P, nr, rank, x_local, ids, route, H, E_local, C, s);
  else ep_receive_t<f16>(P, nr, rank, x_local, ids, route, H, E_local, C, s);
}

template <typename T>
static void ep_return_t(const EpPtrs& P, int nr, int rank, const void* y, int S,
                        int64_t slice_stride, const int* route, int H, int C, hipStream_t s) {
#define KGC_EPT(NR)                                                                          \
  ep_return_kernel<T, NR><<<EP_BLOCKS, EP_THREADS, 0, s>>>(P, rank, y, S, slice_stride, route, \
                                                           H, C)
  KGC_EP_RANKS(nr, KGC_EPT)
#undef KGC_EPT
}

void launch_ep_return(int dtype, const EpPtrs& P, int nr, int rank, const void* y, int S,
                      int64_t slice_stride, const int* route, int H, int C, hipStream_t s) {
  if (dtype == DT_BF16) ep_return_t<bf16>(P, nr, rank, y, S, slice_stride, route, H, C, s);
  else ep_return_t<f16>(P, nr, rank, y, S, slice_stride, route, H, C, s);
}

template <typename T>
static void ep_combine_t(const EpPtrs& P, int nr, int rank, void* out, const float* topk_w,
                         int ntok, int k, int H, int C, hipStream_t s) {
#define KGC_EPC(NR)                                                                          \
  ep_combine_kernel<T, NR><<<EP_COMBINE_BLOCKS, EP_THREADS, 0, s>>>(P, rank, (T*)out, topk_w, ntok, k, \
                                                             H, C)
  KGC_EP_RANKS(nr, KGC_EPC)
#undef KGC_EPC
  ep_bump_kernel<<<1, 1, 0, s>>>(P, rank);
}

void launch_ep_combine(int dtype, const EpPtrs& P, int nr, int rank, void* out,
                       const float* topk_w, int ntok, int k, int H, int C, hipStream_t s) {
  if (dtype == DT_BF16) ep_combine_t<bf16>(P, nr, rank, out, topk_w, ntok, k, H, C, s);
  else ep_combine_t<f16>(P, nr, rank, out, topk_w, ntok, k, H, C, s);
}

int ep_max_pairs() { return EP_MAX_PAIRS; }

void ep_err_copy_async(void* sig, uint32_t* host_dst, hipStream_t s) {
  (void)hipMemcpyAsync(host_dst, &reinterpret_cast<EpSignal*>(sig)->err, 4, hipMemcpyDeviceToHost, s);
}

uint32_t ep_read_err(void* sig) {
  uint32_t e = 0;
  (void)hipMemcpy(&e, &reinterpret_cast<EpSignal*>(sig)->err, 4, hipMemcpyDeviceToHost);
  return e;
}

}  // namespace kgc
