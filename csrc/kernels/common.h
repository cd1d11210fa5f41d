// Shared device helpers for the gfx950 (CDNA4) kernels.
// wave64 everywhere: lane = threadIdx.x & 63; reductions use 64-lane shuffles.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

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

// NeoX RoPE of the pair (a at dim i, b at dim i + d/2), with the two products and their
// fused add spelled out so every kernel that rotates (rope_cache.hip, the decode
// prologue, the prefill kernel's q load) rounds identically, whatever -ffp-contract does
__device__ __forceinline__ void neox_rot(float a, float b, float c, float s, float& oa,
                                         float& ob) {
  oa = __builtin_fmaf(a, c, -(b * s));
  ob = __builtin_fmaf(b, c, a * s);
  // the fp32 results exist as such: otherwise the f16 callers' fptrunc(fma) may become a
  // v_fma_mix (one rounding instead of fp32-then-f16) for SOME elements, chosen by the
  // scheduler per instantiation -- 1-ulp differences between kernels that must agree
  asm("" : "+v"(oa), "+v"(ob));
}

// ---- fp8 (OCP e4m3, gfx950) KV cache ---------------------------------------------
// Values are stored as fp8(x / scale) with the per-tensor scale folded into the
// attention math by the kernels (K: softmax scale, V: output), so dequantisation is
// the exact e4m3 -> bf16/f16 widening (every e4m3 value is representable in both).
constexpr float FP8_MAX = 448.f;

__device__ __forceinline__ uint32_t fp8x4(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -FP8_MAX), FP8_MAX);
  b = fminf(fmaxf(b, -FP8_MAX), FP8_MAX);
  c = fminf(fmaxf(c, -FP8_MAX), FP8_MAX);
  d = fminf(fmaxf(d, -FP8_MAX), FP8_MAX);
  const int lo = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, lo, true);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

// bytes [2*HI, 2*HI+1] of w -> 2 T packed in 32 bits
template <typename T, bool HI> __device__ __forceinline__ uint32_t fp8x2_widen(uint32_t w) {
  if constexpr (std::is_same_v<T, bf16>) {
    union { bf16x2_t v; uint32_t u; } r;
    r.v = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.0f, HI);
    return r.u;
  } else {
    union { f16x2_t v; uint32_t u; } r;
    r.v = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(w, 1.0f, HI);
    return r.u;
  }
}

// 8 fp8 bytes -> 8 T (one MFMA operand fragment)
template <typename T>
__device__ __forceinline__ u32x4 fp8x8_widen(u32x2 raw) {
  return u32x4{fp8x2_widen<T, false>(raw.x), fp8x2_widen<T, true>(raw.x),
               fp8x2_widen<T, false>(raw.y), fp8x2_widen<T, true>(raw.y)};
}

// Load one 8-element fragment from a cache row: 16 B of T, or 8 B of fp8 widened.
template <typename T, bool KV8>
__device__ __forceinline__ u32x4 ld_frag8(const void* base, int64_t elem) {
  if constexpr (KV8)
    return fp8x8_widen<T>(*reinterpret_cast<const u32x2*>(
        reinterpret_cast<const uint8_t*>(base) + elem));
  else
    return *reinterpret_cast<const u32x4*>(reinterpret_cast<const T*>(base) + elem);
}


// ---- debug build (KGC_HIP_DEBUG=1 python csrc/build.py -> _kgc_ops_debug.so): device-side
// bounds checks of the indices the attention / KV-write kernels take from the host
// (block tables, slot mapping, context lengths).  A failed check prints once, sets the
// translation unit's sticky error word (read by kgc.debug_errors(), which raises on the
// host) and CLAMPS the index to a valid value -- never a trap, never an out-of-bounds
// access.  In release builds the checks compile to nothing.
#ifdef KGC_DEBUG
static __device__ unsigned int kgc_dbg_err;
#define KGC_DEBUG_TU(name)                                                   \
  uint32_t dbg_err_##name() {                                                \
    unsigned int v = 0, z = 0;                                               \
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(kgc_dbg_err), sizeof(v));       \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(kgc_dbg_err), &z, sizeof(z));         \
    return v;                                                                \
  }
#define KGC_DCHECK_RANGE(v, lo, hi, what)                                                     \
  do {                                                                                        \
    if ((long long)(v) < (long long)(lo) || (long long)(v) >= (long long)(hi)) {              \
      if (atomicOr(&kgc_dbg_err, 1u) == 0u)                                                   \
        printf("kgc debug check: %s = %lld not in [%lld, %lld) at %s:%d (wg %d,%d,%d t %d)\n", \
               what, (long long)(v), (long long)(lo), (long long)(hi), __FILE__, __LINE__,   \
               (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)threadIdx.x);         \
      (v) = (lo);                                                                             \
    }                                                                                         \
  } while (0)
#else
#define KGC_DEBUG_TU(name) \
  uint32_t dbg_err_##name() { return 0; }
#define KGC_DCHECK_RANGE(v, lo, hi, what) \
  do {                                    \
  } while (0)
#endif

// block-table entry i of a sequence's row (debug: column and block id range-checked)
__device__ __forceinline__ int kgc_bt(const int* bt, int i, int bt_stride, int num_blocks) {
  KGC_DCHECK_RANGE(i, 0, bt_stride, "block-table column");
  int v = bt[i];
  KGC_DCHECK_RANGE(v, 0, num_blocks, "block id");
  (void)bt_stride;
  (void)num_blocks;
  return v;
}

// ---- bounded spin-waits -------------------------------------------------------------
// Every cross-workgroup / cross-GPU flag wait (xGMI all-reduce barriers, PP hand-off,
// EP all-to-all, the cooperative sampler's row barriers) gives up after a WALL-CLOCK
// bound, not an iteration count: the time a spin iteration takes depends on the flag's
// memory scope and on what the other waves do, so an iteration bound is not a duration.
// The clock is the constant-rate steady counter (s_memrealtime, 100 MHz on gfx950 =
// hipDeviceAttributeWallClockRate; tests/test_allreduce_gpu.py checks the rate and the
// measured time-out).  On expiry the kernel sets its sticky error word; the host raises
// (engine/health.py) -- a peer that is gone fails the step in seconds, never hangs it.
#ifndef KGC_PEER_SPIN_MS
#define KGC_PEER_SPIN_MS 10000   // xGMI AR / PP / EP: peers can lag by a host hiccup
#endif
#ifndef KGC_COOP_SPIN_MS
#define KGC_COOP_SPIN_MS 2000    // same-kernel workgroups (sampler): microseconds when healthy
#endif
constexpr unsigned long long kWallClockHz = 100000000ull;

__device__ __forceinline__ unsigned long long spin_deadline(unsigned ms) {
  return (unsigned long long)wall_clock64() + (unsigned long long)ms * (kWallClockHz / 1000ull);
}
__device__ __forceinline__ bool spin_expired(unsigned long long deadline) {
  return (unsigned long long)wall_clock64() > deadline;
}

}  // namespace kgc
