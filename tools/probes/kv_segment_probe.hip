// Does the K-cache access shape of the K1w decode kernel cost HBM rate?  Each wave streams
// 8 KB chunks (32 token rows x 256 B) from random chunk addresses, two chunks in flight,
// 8 wave-instructions of 16 B per lane per chunk, in one of two shapes:
//   A (the K1w K read): an instruction covers 16 token rows x one 64-B segment each
//     (lane: row key(m) = 8*(m>>2) + (m&3) (+4), 16 B at qd*16 + s2*64 of the row)
//   B (a [D/32][tokens][32] K layout): an instruction covers 4 runs of 4 rows x 64 B
//     = 4 contiguous 256-B segments
// Same bytes, same chunk order; prints TB/s per shape.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <random>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ __launch_bounds__(64, 2) void probe(const char* __restrict__ buf,
                                               const int* __restrict__ chunk_of, int per_wave,
                                               u32x4* __restrict__ sink) {
  const int lane = threadIdx.x, m = lane & 15, qd = lane >> 4;
  const int w = blockIdx.x;
  auto off = [&](int h, int s2) -> int {
    const int key = 8 * (m >> 2) + (m & 3) + 4 * h;
    if (SHAPE == 0) return key * 256 + s2 * 64 + qd * 16;
    return s2 * 2048 + key * 64 + qd * 16;
  };
  u32x4 acc = {0, 0, 0, 0};
  u32x4 a[8], b[8];
  auto issue = [&](u32x4* f, int c) {
    const char* base = buf + (int64_t)chunk_of[(int64_t)w * per_wave + c] * 8192;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      f[i] = *reinterpret_cast<const u32x4*>(base + off(i >> 2, i & 3));
  };
  issue(a, 0);
  issue(b, 1 < per_wave ? 1 : 0);
  for (int c = 0; c < per_wave; c += 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= a[i];
    issue(a, min(c + 2, per_wave - 1));
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= b[i];
    issue(b, min(c + 3, per_wave - 1));
  }
  sink[w * 64 + lane] = acc;
}

// DEPTH chunks in flight per wave (shape A), named buffers
template <int DEPTH>
__global__ __launch_bounds__(64, 2) void probe_depth(const char* __restrict__ buf,
                                                     const int* __restrict__ chunk_of,
                                                     int per_wave, u32x4* __restrict__ sink) {
  const int lane = threadIdx.x, m = lane & 15, qd = lane >> 4;
  const int w = blockIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 f[DEPTH][8];
  auto issue = [&](int d, int c) {
    const char* base = buf + (int64_t)chunk_of[(int64_t)w * per_wave + c] * 8192;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int key = 8 * (m >> 2) + (m & 3) + 4 * (i >> 2);
      f[d][i] = *reinterpret_cast<const u32x4*>(base + key * 256 + (i & 3) * 64 + qd * 16);
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) issue(d, min(d, per_wave - 1));
  for (int c = 0; c < per_wave; c += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc ^= f[d][i];
      issue(d, min(c + DEPTH + d, per_wave - 1));
    }
  }
  sink[w * 64 + lane] = acc;
}

// contiguous runs of RUN 8-KB sub-chunks (a KV block of 32 * RUN tokens per head): the
// wave's chunk c reads sub-chunk c % RUN of run chunk_of[c / RUN]
template <int RUN>
__global__ __launch_bounds__(64, 2) void probe_run(const char* __restrict__ buf,
                                                   const int* __restrict__ chunk_of, int per_wave,
                                                   u32x4* __restrict__ sink) {
  const int lane = threadIdx.x, m = lane & 15, qd = lane >> 4;
  const int w = blockIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 a[8], b[8];
  auto issue = [&](u32x4* f, int c) {
    const char* base =
        buf + ((int64_t)chunk_of[(int64_t)w * (per_wave / RUN) + c / RUN] * RUN + c % RUN) * 8192;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int key = 8 * (m >> 2) + (m & 3) + 4 * (i >> 2);
      f[i] = *reinterpret_cast<const u32x4*>(base + key * 256 + (i & 3) * 64 + qd * 16);
    }
  };
  issue(a, 0);
  issue(b, 1);
  for (int c = 0; c < per_wave; c += 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= a[i];
    issue(a, min(c + 2, per_wave - 1));
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= b[i];
    issue(b, min(c + 3, per_wave - 1));
  }
  sink[w * 64 + lane] = acc;
}

int main() {
  const int waves = 2048, per_wave = 20;
  const int64_t nchunks = (int64_t)1536 << 20 >> 13;       // 1.5 GB of 8 KB chunks
  char* buf;
  hipMalloc(&buf, nchunks * 8192);
  hipMemset(buf, 1, nchunks * 8192);
  std::vector<int> perm(nchunks);
  for (int64_t i = 0; i < nchunks; ++i) perm[i] = (int)i;
  std::mt19937 rng(1);
  std::shuffle(perm.begin(), perm.end(), rng);
  const int64_t need = (int64_t)waves * per_wave;
  std::vector<int> sets;                                     // several disjoint chunk sets
  const int nsets = (int)(nchunks / need);
  int* d_chunks;
  hipMalloc(&d_chunks, nsets * need * sizeof(int));
  hipMemcpy(d_chunks, perm.data(), nsets * need * sizeof(int), hipMemcpyHostToDevice);
  u32x4* sink;
  hipMalloc(&sink, 2 * waves * 64 * sizeof(u32x4));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int shape = 0; shape < 2; ++shape) {
    for (int rep = 0; rep < 3; ++rep) {
      float best = 1e9;
      for (int it = 0; it < 20; ++it) {
        const int* ch = d_chunks + (int64_t)(it % nsets) * need;
        hipEventRecord(e0);
        if (shape == 0) probe<0><<<waves, 64>>>(buf, ch, per_wave, sink);
        else probe<1><<<waves, 64>>>(buf, ch, per_wave, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (it >= 2) best = std::min(best, ms);
      }
      const double bytes = (double)need * 8192;
      printf("{\"shape\": \"%s\", \"rep\": %d, \"us\": %.2f, \"TBps\": %.3f}\n",
             shape == 0 ? "A 16 rows x 64 B" : "B 4 x 256 B", rep, best * 1e3,
             bytes / (best * 1e-3) / 1e12);
    }
  }
  // in-flight depth (shape A) and waves per SIMD: the grid is 2048 waves (one round at
  // 2 per SIMD) or 4096 (per_wave halved: same bytes)
  for (int depth = 2; depth <= 4; ++depth) {
    for (int wmul = 1; wmul <= 2; ++wmul) {
      const int nw = waves * wmul, pw = per_wave / wmul;
      float best = 1e9;
      for (int it = 0; it < 20; ++it) {
        const int* ch = d_chunks + (int64_t)(it % nsets) * need;
        hipEventRecord(e0);
        if (depth == 2) probe_depth<2><<<nw, 64>>>(buf, ch, pw, sink);
        else if (depth == 3) probe_depth<3><<<nw, 64>>>(buf, ch, pw, sink);
        else probe_depth<4><<<nw, 64>>>(buf, ch, pw, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (it >= 2) best = std::min(best, ms);
      }
      const double bytes = (double)nw * pw * 8192;
      printf("{\"shape\": \"A depth %d, %d waves\", \"us\": %.2f, \"TBps\": %.3f}\n", depth, nw,
             best * 1e3, bytes / (best * 1e-3) / 1e12);
    }
  }
  // KV block size: runs of 1 / 2 / 4 sub-chunks (32 / 64 / 128 tokens per block and head),
  // random run placement (run indices < nchunks / RUN)
  for (int run = 1; run <= 4; run *= 2) {
    std::vector<int> rp(nchunks / run);
    for (size_t i = 0; i < rp.size(); ++i) rp[i] = (int)i;
    std::shuffle(rp.begin(), rp.end(), rng);
    int* d_runs;
    hipMalloc(&d_runs, rp.size() * sizeof(int));
    hipMemcpy(d_runs, rp.data(), rp.size() * sizeof(int), hipMemcpyHostToDevice);
    const int64_t per_set = (int64_t)waves * per_wave / run;
    const int sets = (int)(rp.size() / per_set);
    float best = 1e9;
    for (int it = 0; it < 20; ++it) {
      const int* ch = d_runs + (int64_t)(it % sets) * per_set;
      hipEventRecord(e0);
      // the kernel reads chunk_of[w * (per_wave / RUN) + c / RUN]: per_set entries per set
      if (run == 1) probe_run<1><<<waves, 64>>>(buf, ch, per_wave, sink);
      else if (run == 2) probe_run<2><<<waves, 64>>>(buf, ch, per_wave, sink);
      else probe_run<4><<<waves, 64>>>(buf, ch, per_wave, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (it >= 2) best = std::min(best, ms);
    }
    const double bytes = (double)waves * per_wave * 8192;
    printf("{\"shape\": \"A, %d-token KV blocks (runs of %d x 8 KB)\", \"us\": %.2f, \"TBps\": %.3f}\n",
           32 * run, run, best * 1e3, bytes / (best * 1e-3) / 1e12);
    hipFree(d_runs);
  }
  return 0;
}
