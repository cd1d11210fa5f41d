// K4 RMSNorm / fused residual-add + RMSNorm, K8 LayerNorm (OPT), K6 helper.
// One workgroup per row; each thread owns up to MAXV 16-byte vectors of the row
// held in registers between the reduction and the scale pass (single HBM read).
#include "common.h"
#include "launch.h"

namespace kgc {

constexpr int NORM_NT = 256;
constexpr int NORM_MAXV = 4;  // 256 thr * 4 vec * 8 elems = 8192 = Llama-3-70B hidden

template <typename T, bool ADD>
__global__ __launch_bounds__(NORM_NT) void rms_norm_kernel(
    T* __restrict__ out, const T* __restrict__ x, T* __restrict__ residual,
    const T* __restrict__ w, int H, int64_t x_stride, float eps) {
  __shared__ float scratch[NORM_NT / 64];
  const int row = blockIdx.x;
  const int nv = H >> 3;
  const T* xr = x + row * x_stride;
  T* rr = ADD ? residual + (int64_t)row * H : nullptr;
  Pack8<T> v[NORM_MAXV], wv[NORM_MAXV];
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {   // weight loads issued before the reduction
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) wv[i].u = *reinterpret_cast<const u32x4*>(w + idx * 8);
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) {
      v[i].u = *reinterpret_cast<const u32x4*>(xr + idx * 8);
      if (ADD) {
        Pack8<T> r;
        r.u = *reinterpret_cast<const u32x4*>(rr + idx * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i].h[j] = from_f<T>(to_f(v[i].h[j]) + to_f(r.h[j]));
        *reinterpret_cast<u32x4*>(rr + idx * 8) = v[i].u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = to_f(v[i].h[j]);
        ss += f * f;
      }
    }
  }
  ss = block_sum<NORM_NT>(ss, scratch);
  const float inv = rsqrtf(ss / (float)H + eps);
  T* orow = out + (int64_t)row * H;
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) {
      Pack8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.h[j] = from_f<T>(to_f(v[i].h[j]) * inv * to_f(wv[i].h[j]));
      *reinterpret_cast<u32x4*>(orow + idx * 8) = o.u;
    }
  }
}

// Split-K reduction fused into the residual add + RMSNorm that consumes a row-parallel
// projection (o_proj -> post-attention norm, down_proj -> next layer's input norm):
//   h = sum_z Cs[z, row, :] (rounded to T, as the unfused reduce stores it)
//   residual += h;  out = rms_norm(residual) * w
// The [M, H] projection output is never written and one launch per projection goes.
template <typename T, int SK>
__global__ __launch_bounds__(NORM_NT) void splitk_add_rms_norm_kernel(
    T* __restrict__ out, const float* __restrict__ Cs, T* __restrict__ residual,
    const T* __restrict__ w, int H, int S_, int64_t slice_stride, float eps) {
  // SK > 0: the slice count is a compile-time constant, so every slice load of a thread
  // is issued before the first add (one memory round trip instead of S)
  const int S = SK > 0 ? SK : S_;
  __shared__ float scratch[NORM_NT / 64];
  const int row = blockIdx.x;
  const int nv = H >> 3;
  const float* cr = Cs + (int64_t)row * H;
  T* rr = residual + (int64_t)row * H;
  Pack8<T> v[NORM_MAXV], wv[NORM_MAXV];
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) wv[i].u = *reinterpret_cast<const u32x4*>(w + idx * 8);
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) {
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
#pragma unroll
      for (int z = 0; z < (SK > 0 ? SK : 1); ++z) {
        const float* src = cr + z * slice_stride + idx * 8;
        a += *reinterpret_cast<const f32x4*>(src);
        b += *reinterpret_cast<const f32x4*>(src + 4);
      }
      for (int z = SK > 0 ? SK : 1; z < S; ++z) {
        const float* src = cr + z * slice_stride + idx * 8;
        a += *reinterpret_cast<const f32x4*>(src);
        b += *reinterpret_cast<const f32x4*>(src + 4);
      }
      Pack8<T> r;
      r.u = *reinterpret_cast<const u32x4*>(rr + idx * 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[i].h[q] = from_f<T>(to_f(from_f<T>(a[q])) + to_f(r.h[q]));
        v[i].h[4 + q] = from_f<T>(to_f(from_f<T>(b[q])) + to_f(r.h[4 + q]));
      }
      *reinterpret_cast<u32x4*>(rr + idx * 8) = v[i].u;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = to_f(v[i].h[j]);
        ss += f * f;
      }
    }
  }
  ss = block_sum<NORM_NT>(ss, scratch);
  const float inv = rsqrtf(ss / (float)H + eps);
  T* orow = out + (int64_t)row * H;
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) {
      Pack8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.h[j] = from_f<T>(to_f(v[i].h[j]) * inv * to_f(wv[i].h[j]));
      *reinterpret_cast<u32x4*>(orow + idx * 8) = o.u;
    }
  }
}

// The same for H = NVT * 2048 and a compile-time slice count: no per-vector guards, so
// every slice, residual and weight load of a thread is issued before the first add (the
// guarded loop above issued vector i + 1's loads only after vector i's adds: at H = 4096
// two dependent round trips per row)
template <typename T, int SK, int NVT, int NT>
__global__ __launch_bounds__(NT) void splitk_add_rms_norm_nv_kernel(
    T* __restrict__ out, const float* __restrict__ Cs, T* __restrict__ residual,
    const T* __restrict__ w, int H, int64_t slice_stride, float eps) {
  __shared__ float scratch[NT / 64];
  const int row = blockIdx.x;
  const float* cr = Cs + (int64_t)row * H;
  T* rr = residual + (int64_t)row * H;
  f32x4 a[NVT][SK], b[NVT][SK];
  Pack8<T> r[NVT], wv[NVT];
#pragma unroll
  for (int i = 0; i < NVT; ++i) {
    const int idx = threadIdx.x + i * NT;
#pragma unroll
    for (int z = 0; z < SK; ++z) {
      const float* src = cr + z * slice_stride + idx * 8;
      a[i][z] = *reinterpret_cast<const f32x4*>(src);
      b[i][z] = *reinterpret_cast<const f32x4*>(src + 4);
    }
    r[i].u = *reinterpret_cast<const u32x4*>(rr + idx * 8);
    wv[i].u = *reinterpret_cast<const u32x4*>(w + idx * 8);
  }
  float ss = 0.f;
  Pack8<T> v[NVT];
#pragma unroll
  for (int i = 0; i < NVT; ++i) {
    f32x4 sa = a[i][0], sb = b[i][0];
#pragma unroll
    for (int z = 1; z < SK; ++z) {
      sa += a[i][z];
      sb += b[i][z];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[i].h[q] = from_f<T>(to_f(from_f<T>(sa[q])) + to_f(r[i].h[q]));
      v[i].h[4 + q] = from_f<T>(to_f(from_f<T>(sb[q])) + to_f(r[i].h[4 + q]));
    }
    *reinterpret_cast<u32x4*>(rr + (threadIdx.x + i * NT) * 8) = v[i].u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = to_f(v[i].h[j]);
      ss += f * f;
    }
  }
  ss = block_sum<NT>(ss, scratch);
  const float inv = rsqrtf(ss / (float)H + eps);
  T* orow = out + (int64_t)row * H;
#pragma unroll
  for (int i = 0; i < NVT; ++i) {
    Pack8<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.h[j] = from_f<T>(to_f(v[i].h[j]) * inv * to_f(wv[i].h[j]));
    *reinterpret_cast<u32x4*>(orow + (threadIdx.x + i * NT) * 8) = o.u;
  }
}

template <typename T>
__global__ __launch_bounds__(NORM_NT) void layer_norm_kernel(
    T* __restrict__ out, const T* __restrict__ x, const T* __restrict__ w,
    const T* __restrict__ b, int H, float eps) {
  __shared__ float scratch[NORM_NT / 64];
  const int row = blockIdx.x;
  const int nv = H >> 3;
  const T* xr = x + (int64_t)row * H;
  Pack8<T> v[NORM_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) {
      v[i].u = *reinterpret_cast<const u32x4*>(xr + idx * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += to_f(v[i].h[j]);
    }
  }
  const float mean = block_sum<NORM_NT>(s, scratch) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = to_f(v[i].h[j]) - mean;
        ss += d * d;
      }
    }
  }
  const float inv = rsqrtf(block_sum<NORM_NT>(ss, scratch) / (float)H + eps);
  T* orow = out + (int64_t)row * H;
#pragma unroll
  for (int i = 0; i < NORM_MAXV; ++i) {
    const int idx = threadIdx.x + i * NORM_NT;
    if (idx < nv) {
      Pack8<T> wv, bv, o;
      wv.u = *reinterpret_cast<const u32x4*>(w + idx * 8);
      bv.u = *reinterpret_cast<const u32x4*>(b + idx * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o.h[j] = from_f<T>((to_f(v[i].h[j]) - mean) * inv * to_f(wv.h[j]) + to_f(bv.h[j]));
      *reinterpret_cast<u32x4*>(orow + idx * 8) = o.u;
    }
  }
}

template <typename T>
static void rms_dispatch(void* out, const void* x, void* res, const void* w, int rows, int H,
                         int64_t xs, float eps, hipStream_t s) {
  if (rows == 0) return;
  if (res)
    rms_norm_kernel<T, true><<<rows, NORM_NT, 0, s>>>((T*)out, (const T*)x, (T*)res,
                                                      (const T*)w, H, xs, eps);
  else
    rms_norm_kernel<T, false><<<rows, NORM_NT, 0, s>>>((T*)out, (const T*)x, nullptr,
                                                       (const T*)w, H, xs, eps);
}

void launch_rms_norm(int dtype, void* out, const void* x, void* residual, const void* w,
                     int rows, int H, int64_t x_stride, float eps, hipStream_t s) {
  if (dtype == DT_BF16) rms_dispatch<bf16>(out, x, residual, w, rows, H, x_stride, eps, s);
  else rms_dispatch<f16>(out, x, residual, w, rows, H, x_stride, eps, s);
}

// NT threads per row, NVT 8-element vectors per thread (H = NT * NVT * 8): 512 threads at
// H = 4096 keep every slice load of a thread in flight at S = 8 (at 256 threads x 2
// vectors the S = 8 variant ran 7.5 us against 5.6 at S = 4)
template <typename T, int NVT, int NT>
static bool splitk_add_rms_nv(T* out, const float* Cs, T* residual, const T* w, int rows, int H,
                              int S, int64_t ss, float eps, hipStream_t s) {
#define SKV(K)                                                                                  \
  splitk_add_rms_norm_nv_kernel<T, K, NVT, NT><<<rows, NT, 0, s>>>(out, Cs, residual, w, H, ss, \
                                                                  eps)
  switch (S) {
    case 2: SKV(2); return true;
    case 3: SKV(3); return true;
    case 4: SKV(4); return true;
    case 5: SKV(5); return true;
    case 6: SKV(6); return true;
    case 8: SKV(8); return true;
    default: return false;
  }
#undef SKV
}

template <typename T>
static void splitk_add_rms_dispatch(T* out, const float* Cs, T* residual, const T* w, int rows,
                                    int H, int S, int64_t ss, float eps, hipStream_t s) {
  if (H == 2048 && splitk_add_rms_nv<T, 1, 256>(out, Cs, residual, w, rows, H, S, ss, eps, s)) return;
  if (H == 4096 && splitk_add_rms_nv<T, 1, 512>(out, Cs, residual, w, rows, H, S, ss, eps, s)) return;
  if (H == 8192 && splitk_add_rms_nv<T, 2, 512>(out, Cs, residual, w, rows, H, S, ss, eps, s)) return;
#define SKN(K) splitk_add_rms_norm_kernel<T, K><<<rows, NORM_NT, 0, s>>>(out, Cs, residual, w, \
                                                                         H, S, ss, eps)
  switch (S) {
    case 2: SKN(2); break;
    case 3: SKN(3); break;
    case 4: SKN(4); break;
    case 5: SKN(5); break;
    case 6: SKN(6); break;
    case 8: SKN(8); break;
    default: SKN(0); break;
  }
#undef SKN
}

void launch_splitk_add_rms_norm(int dtype, void* out, const float* Cs, void* residual,
                                const void* w, int rows, int H, int S, int64_t slice_stride,
                                float eps, hipStream_t s) {
  if (rows == 0) return;
  if (dtype == DT_BF16)
    splitk_add_rms_dispatch<bf16>((bf16*)out, Cs, (bf16*)residual, (const bf16*)w, rows, H, S,
                                  slice_stride, eps, s);
  else
    splitk_add_rms_dispatch<f16>((f16*)out, Cs, (f16*)residual, (const f16*)w, rows, H, S,
                                 slice_stride, eps, s);
}

void launch_layer_norm(int dtype, void* out, const void* x, const void* w, const void* b,
                       int rows, int H, float eps, hipStream_t s) {
  if (rows == 0) return;
  if (dtype == DT_BF16)
    layer_norm_kernel<bf16><<<rows, NORM_NT, 0, s>>>((bf16*)out, (const bf16*)x,
                                                     (const bf16*)w, (const bf16*)b, H, eps);
  else
    layer_norm_kernel<f16><<<rows, NORM_NT, 0, s>>>((f16*)out, (const f16*)x, (const f16*)w,
                                                    (const f16*)b, H, eps);
}

}  // namespace kgc
