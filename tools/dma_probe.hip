// Per-CU intake probe for gfx950: how fast can one 512-thread workgroup per CU pull bytes
// into LDS by LDS-DMA (global_load_lds_dwordx4) or into VGPRs (global_load_dwordx4), as a
// function of bytes in flight, from HBM (every workgroup its own region) or from L2 (all
// workgroups of an XCD re-reading one shared region)?  Used to size the K9m decode GEMM's
// operand rings (csrc/kernels/gemm_decode.hip).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/dma_probe tools/dma_probe.hip
//   build/dma_probe            -> one JSON line per (path, source, slot KB, depth)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// SLOT_KB per step; D steps in flight; each of the 8 waves issues SLOT_KB / 8 DMAs per step.
// shared = 1: every workgroup reads the same `region` bytes (L2-resident after first touch)
// SEG > 0: the decode-GEMM weight pattern instead of a contiguous stream: a step reads
// SEG bytes from each of SLOT / SEG rows 8 KB apart (W [N, K] bf16 at K = 4096), walking K
// once (a 128-row x 8-KB tile per workgroup, one of 8 copies per launch: beyond the MALL)
template <int SLOT_KB, int D, bool VGPR, int SEG = 0>
__global__ __launch_bounds__(512, 1) void probe(const char* __restrict__ src, int64_t region,
                                                int steps, int shared, float* sink) {
  constexpr int PER_WAVE = SLOT_KB / 8;            // 1-KiB instructions per wave per step
  constexpr int SLOT = SLOT_KB * 1024;
  __shared__ __attribute__((aligned(16))) char lds[VGPR ? 16 : (D + 1) * SLOT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* base = src + (shared ? 0 : (int64_t)blockIdx.x * region);
  if constexpr (SEG > 0) base = src + ((int64_t)(steps & 7) * gridDim.x + blockIdx.x) * (SLOT / SEG) * 8192;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[D][PER_WAVE > 0 ? PER_WAVE : 1];
  auto issue = [&](int step, int u) {
    const int64_t off = ((int64_t)step * SLOT) % region;
#pragma unroll
    for (int t = 0; t < PER_WAVE; ++t) {
      const char* g = base + off + (wave * PER_WAVE + t) * 1024 + lane * 16;
      if constexpr (SEG > 0) {
        constexpr int LPR = SEG / 16;                 // lanes per row segment
        const int row = ((wave * PER_WAVE + t) * 64 + lane) / LPR;
        const int64_t kofs = ((int64_t)step * SEG) % 8192;
        g = base + (int64_t)row * 8192 + kofs + (lane % LPR) * 16;
      }
      if constexpr (VGPR) {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r[u][t]) : "v"(g) : "memory");
      } else {
        char* l = lds + (step % (D + 1)) * SLOT + (wave * PER_WAVE + t) * 1024;
        __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)l, 16, 0, 0);
      }
    }
  };
#pragma unroll
  for (int u = 0; u < D; ++u) issue(u, u);
  const int nsteps = SEG > 0 ? 8192 / SEG : steps;
  for (int s0 = 0; s0 < nsteps; s0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int s = s0 + u;
      wait_vm<(D - 1) * PER_WAVE>();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (VGPR) {
#pragma unroll
        for (int t = 0; t < PER_WAVE; ++t) acc += r[u][t];
      } else {
        __builtin_amdgcn_s_barrier();
      }
      if (SEG == 0 || s + D < nsteps) issue(s + D, u);
    }
  }
  wait_vm<0>();
  if (acc.x == 0x12345678u) sink[threadIdx.x] = (float)acc.y;   // keep the loads live
}

template <int SLOT_KB, int D, bool VGPR, int SEG = 0>
void run(const char* src, float* sink, int shared, int nblk) {
  const int64_t region = shared ? (int64_t)2 << 20 : (int64_t)8 << 20;   // 2 MB shared / 8 MB own
  const int steps = (int)((8LL << 20) / (SLOT_KB * 1024));                // 8 MB per workgroup
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep)
    probe<SLOT_KB, D, VGPR, SEG><<<nblk, 512>>>(src, region, steps + rep, shared, sink);
  CK(hipEventRecord(e0));
  const int iters = SEG > 0 ? 64 : 5;
  for (int rep = 0; rep < iters; ++rep)
    probe<SLOT_KB, D, VGPR, SEG><<<nblk, 512>>>(src, region, steps + rep, shared, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double s = ms / 1e3 / iters;
  const double bytes = SEG > 0 ? (double)(SLOT_KB * 1024 / SEG) * 8192 : (double)steps * SLOT_KB * 1024;
  std::printf("{\"seg\": %d, \"path\": \"%s\", \"source\": \"%s\", \"slot_kb\": %d, \"depth\": %d, "
              "\"inflight_kb\": %d, \"us\": %.1f, \"GBps_per_cu\": %.1f, \"TBps_chip\": %.2f}\n",
              SEG, VGPR ? "vgpr" : "lds_dma", shared ? "L2" : "HBM", SLOT_KB, D, SLOT_KB * D,
              s * 1e6, bytes / s / 1e9, bytes * nblk / s / 1e12);
  std::fflush(stdout);
}

int main() {
  int nblk = 256;
  char* src;
  float* sink;
  CK(hipMalloc(&src, (size_t)nblk * (8 << 20) + (16 << 20)));
  CK(hipMemset(src, 1, (size_t)nblk * (8 << 20) + (16 << 20)));
  CK(hipMalloc(&sink, 4096));
  // SEG runs touch 8 copies x nblk x (16 KB / SEG) rows x 8 KB <= 1 GB: within the 2 GB buffer
  // contiguous HBM stream vs the weight-tile pattern (128 / 256 / 512 B per row per step)
  run<16, 2, false>(src, sink, 0, nblk);
  run<16, 2, false, 128>(src, sink, 0, nblk);
  run<16, 4, false, 128>(src, sink, 0, nblk);
  run<16, 2, false, 256>(src, sink, 0, nblk);
  run<16, 2, false, 512>(src, sink, 0, nblk);
  run<16, 4, false, 512>(src, sink, 0, nblk);
  run<16, 2, true, 128>(src, sink, 0, nblk);
  CK(hipFree(src));
  CK(hipFree(sink));
  return 0;
}
