// K10 sampler: one 1024-thread workgroup per row of logits [B, V].
//   temperature <= 1e-5        -> argmax (first index on ties)
//   otherwise x = logit / temp -> optional top-k threshold (4-pass radix select on the
//                                 order-preserving uint32 image of x), optional top-p
//                                 threshold (radix select on softmax mass, over the top-k
//                                 support) -> Gumbel-max over the kept support.
// The Gumbel noise is a counter-based hash of (seed, column), bit-identical to
// ops/reference.uniform_noise, so sampled ids are reproducible per request seed.
#include "common.h"
#include "launch.h"

namespace kgc {

constexpr int SMP_NT = 1024;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
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

__device__ __forceinline__ void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

template <typename T>
__global__ __launch_bounds__(SMP_NT) void sample_kernel(
    int64_t* __restrict__ out, const T* __restrict__ logits, int64_t row_stride, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const int64_t* __restrict__ seeds) {
  __shared__ float red_v[SMP_NT / 64];
  __shared__ int red_i[SMP_NT / 64];
  __shared__ float hist_f[256];
  __shared__ uint32_t hist_u[256];
  __shared__ uint32_t sel_bin;
  __shared__ float sel_f;
  __shared__ uint32_t sel_u;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* row = logits + (int64_t)b * row_stride;
  const float temp = temperature[b];
  const bool greedy = temp <= 1e-5f;
  const int k = greedy ? 0 : top_k[b];
  const float p = greedy ? 1.f : top_p[b];
  const bool use_k = k > 0 && k < V;
  const bool use_p = p < 1.f;

  auto xval = [&](int i) -> float { return greedy ? load_logit(row, i) : load_logit(row, i) / temp; };

  // ---------- thresholds (kept support = x >= thr)
  float thr = -INFINITY;
  if (use_k || use_p) {
    if (use_k) {
      uint32_t prefix = 0, mask = 0;
      int remaining = k;
      for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) hist_u[tid] = 0;
        __syncthreads();
        for (int i = tid; i < V; i += SMP_NT) {
          const uint32_t kk = ord_key(xval(i));
          if ((kk & mask) == prefix) atomicAdd(&hist_u[(kk >> shift) & 255], 1u);
        }
        __syncthreads();
        if (tid == 0) {
          int acc = 0, bin = 0;
          for (bin = 255; bin >= 0; --bin) {
            if (acc + (int)hist_u[bin] >= remaining) break;
            acc += hist_u[bin];
          }
          sel_bin = (uint32_t)max(bin, 0);
          sel_u = (uint32_t)acc;
        }
        __syncthreads();
        remaining -= (int)sel_u;
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
      }
      thr = key_val(prefix);
    }
    if (use_p) {
      // max and normaliser over the current support
      float mx = -INFINITY;
      for (int i = tid; i < V; i += SMP_NT) {
        const float x = xval(i);
        if (x >= thr) mx = fmaxf(mx, x);
      }
      mx = block_max<SMP_NT>(mx, red_v);
      float z = 0.f;
      for (int i = tid; i < V; i += SMP_NT) {
        const float x = xval(i);
        if (x >= thr) z += __expf(x - mx);
      }
      z = block_sum<SMP_NT>(z, red_v);
      const float target = p * z;
      uint32_t prefix = 0, mask = 0;
      float above = 0.f;
      const uint32_t kthr = ord_key(thr);
      for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) hist_f[tid] = 0.f;
        __syncthreads();
        for (int i = tid; i < V; i += SMP_NT) {
          const float x = xval(i);
          const uint32_t kk = ord_key(x);
          if (kk >= kthr && (kk & mask) == prefix)
            atomicAdd(&hist_f[(kk >> shift) & 255], __expf(x - mx));
        }
        __syncthreads();
        if (tid == 0) {
          float acc = above;
          int bin;
          for (bin = 255; bin > 0; --bin) {
            if (acc + hist_f[bin] >= target) break;
            acc += hist_f[bin];
          }
          sel_bin = (uint32_t)bin;
          sel_f = acc;
        }
        __syncthreads();
        above = sel_f;
        prefix |= sel_bin << shift;
        mask |= 255u << shift;
      }
      thr = fmaxf(thr, key_val(prefix));
    }
  }

  // ---------- (Gumbel-)argmax over the support
  const uint64_t seed = (uint64_t)seeds[b];
  const uint32_t key = mix32((uint32_t)seed);
  const uint32_t hi = (uint32_t)(seed >> 32);
  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int i = tid; i < V; i += SMP_NT) {
    float x = xval(i);
    if (!greedy) {
      if (x < thr) continue;
      const uint32_t h = mix32(mix32(key ^ (uint32_t)(i * 0x9E3779B9u)) + hi);
      const float u = ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
      x += -logf(-logf(u));
    }
    argmax_merge(best, besti, x, i);
  }
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
    out[b] = bi == 0x7fffffff ? 0 : bi;
  }
}

void launch_sample(int dtype, int64_t* out, const void* logits, int64_t row_stride, int B,
                   int V, const float* temperature, const int* top_k, const float* top_p,
                   const int64_t* seeds, hipStream_t s) {
  if (B == 0) return;
  if (dtype == DT_BF16)
    sample_kernel<bf16><<<B, SMP_NT, 0, s>>>(out, (const bf16*)logits, row_stride, V,
                                             temperature, top_k, top_p, seeds);
  else if (dtype == DT_F16)
    sample_kernel<f16><<<B, SMP_NT, 0, s>>>(out, (const f16*)logits, row_stride, V,
                                            temperature, top_k, top_p, seeds);
  else
    sample_kernel<float><<<B, SMP_NT, 0, s>>>(out, (const float*)logits, row_stride, V,
                                              temperature, top_k, top_p, seeds);
}

}  // namespace kgc
