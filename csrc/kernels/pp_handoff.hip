// C5 pipeline-stage handoff over xGMI peer memory, graph-capturable.
//
// Stage s (TP rank t) hands its [B, H] hidden and residual rows to stage s+1 (TP rank t)
// at the end of every decode step.  RCCL send/recv would do the job eagerly; here the
// handoff is a pair of kernels so that each stage's whole decode step -- receive, its
// layers, send -- is ONE hipGraph replay:
//
//   send (stage s):   wait until the receiver has consumed step i - R (credit), write
//                     the rows into ring slot i % R of the receiver's IPC buffer, and
//                     raise the receiver's `avail` to i + 1 (last workgroup, system scope).
//   recv (stage s+1): wait for `avail` >= i + 1, copy the slot into the local static
//                     input tensors, and raise the sender's `credit` to i + 1.
//
// i is each side's own step counter in device memory, advanced by the last workgroup
// of the kernel once every workgroup has read it.  Spins are bounded (sticky `err`).
#include "common.h"
#include "launch.h"

namespace kgc {

constexpr int PP_THREADS = 512;
constexpr int PP_BLOCKS = 64;

struct PpSignal {
  uint32_t count;       // own: steps sent (sender side) / received (receiver side)
  uint32_t done;        // own: workgroups finished in the current kernel
  uint32_t avail;       // receiver side, written by the sender: steps available
  uint32_t credit;      // sender side, written by the receiver: steps consumed
  uint32_t err;
  uint32_t pad[1024 - 5];
};

size_t pp_signal_bytes() { return (sizeof(PpSignal) + 4095) & ~size_t(4095); }

__device__ __forceinline__ uint32_t pp_load(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void pp_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// thread 0 of every workgroup waits for *f >= target (bounded; failure -> err)
__device__ void pp_wait(PpSignal* own, uint32_t* f, uint32_t target) {
  if (threadIdx.x == 0) {
    const unsigned long long dl = spin_deadline(KGC_PEER_SPIN_MS);
    const bool failed = pp_load(&own->err) != 0u;    // sticky: fail fast after the first
    while (!failed && (int32_t)(pp_load(f) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (spin_expired(dl)) {
        atomicOr(&own->err, 1u);
        break;
      }
    }
    __threadfence_system();
  }
  __syncthreads();
}

// all stores of this workgroup drained; the last workgroup raises *remote = value and
// advances the own step counter
__device__ void pp_finish(PpSignal* own, uint32_t* remote, uint32_t value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    if (atomicAdd(&own->done, 1u) == gridDim.x - 1) {
      own->done = 0;
      __threadfence_system();
      pp_store(remote, value);
      own->count = value;
    }
  }
}

__global__ __launch_bounds__(PP_THREADS) void pp_send_kernel(
    void* peer_data, void* peer_sig, void* own_sig, const u32x4* __restrict__ h,
    const u32x4* __restrict__ r, int64_t nvec, int64_t slot_vec, int R) {
  PpSignal* own = reinterpret_cast<PpSignal*>(own_sig);
  PpSignal* peer = reinterpret_cast<PpSignal*>(peer_sig);
  const uint32_t i = own->count;
  pp_wait(own, &own->credit, i + 1 - R);                 // slot i % R is free again
  u32x4* dst = reinterpret_cast<u32x4*>(peer_data) + (int64_t)(i % R) * 2 * slot_vec;
  for (int64_t v = (int64_t)blockIdx.x * PP_THREADS + threadIdx.x; v < nvec;
       v += (int64_t)gridDim.x * PP_THREADS) {
    dst[v] = h[v];
    dst[slot_vec + v] = r[v];
  }
  pp_finish(own, &peer->avail, i + 1);
}

__global__ __launch_bounds__(PP_THREADS) void pp_recv_kernel(
    void* own_data, void* own_sig, void* peer_sig, u32x4* __restrict__ h, u32x4* __restrict__ r,
    int64_t nvec, int64_t slot_vec, int R) {
  PpSignal* own = reinterpret_cast<PpSignal*>(own_sig);
  PpSignal* peer = reinterpret_cast<PpSignal*>(peer_sig);
  const uint32_t i = own->count;
  pp_wait(own, &own->avail, i + 1);
  const u32x4* src = reinterpret_cast<const u32x4*>(own_data) + (int64_t)(i % R) * 2 * slot_vec;
  for (int64_t v = (int64_t)blockIdx.x * PP_THREADS + threadIdx.x; v < nvec;
       v += (int64_t)gridDim.x * PP_THREADS) {
    h[v] = src[v];
    r[v] = src[slot_vec + v];
  }
  pp_finish(own, &peer->credit, i + 1);
}

void launch_pp_send(void* peer_data, void* peer_sig, void* own_sig, const void* h, const void* r,
                    int64_t bytes, int64_t slot_bytes, int R, hipStream_t s) {
  pp_send_kernel<<<PP_BLOCKS, PP_THREADS, 0, s>>>(peer_data, peer_sig, own_sig,
                                                  (const u32x4*)h, (const u32x4*)r, bytes / 16,
                                                  slot_bytes / 16, R);
}

void launch_pp_recv(void* own_data, void* own_sig, void* peer_sig, void* h, void* r,
                    int64_t bytes, int64_t slot_bytes, int R, hipStream_t s) {
  pp_recv_kernel<<<PP_BLOCKS, PP_THREADS, 0, s>>>(own_data, own_sig, peer_sig, (u32x4*)h,
                                                  (u32x4*)r, bytes / 16, slot_bytes / 16, R);
}

uint32_t pp_read_err(void* sig) {
  uint32_t e = 0;
  (void)hipMemcpy(&e, &reinterpret_cast<PpSignal*>(sig)->err, 4, hipMemcpyDeviceToHost);
  return e;
}

}  // namespace kgc
