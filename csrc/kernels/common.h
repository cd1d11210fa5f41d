// Shared device helpers for the gfx950 (CDNA4) kernels.
// wave64 everywhere: lane = threadIdx.x & 63; reductions use 64-lane shuffles.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kgc {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int WAVE = 64;

// dtype traits: the 16-bit storage type, its 8-wide MFMA operand vector and the MFMA.
template <typename T> struct Vec8;
template <> struct Vec8<bf16> { typedef bf16x8 type; };
template <> struct Vec8<f16> { typedef f16x8 type; };

__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x32(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <typename T> __device__ __forceinline__ float to_f(T x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x) { return (T)x; }

// 16-byte vector of 8 halves, reinterpretable as raw words.
template <typename T>
union Pack8 {
  u32x4 u;
  typename Vec8<T>::type v;
  T h[8];
};

template <typename T>
union Pack4 {
  u32x2 u;
  T h[4];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64); scratch holds NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (NT == 64) return v;
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (NT == 64) return v;
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, scratch[i]);
  __syncthreads();
  return t;
}

__device__ __forceinline__ float fast_exp(float x) { return __expf(x); }

}  // namespace kgc
