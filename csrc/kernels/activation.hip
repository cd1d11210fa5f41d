// K7 SiLU-and-mul: out[t, i] = silu(x[t, i]) * x[t, I + i] over the fused gate_up
// projection output.  16-byte vector loads/stores (8 halves per lane), one vector
// per thread on a 2-D grid (memory-bound; no index division).
#include "common.h"
#include "launch.h"

namespace kgc {

// grid (ceil(I/8/256), rows): one 16-byte vector per thread, no index division
template <typename T>
__global__ __launch_bounds__(256) void silu_mul_kernel(T* __restrict__ out,
                                                       const T* __restrict__ x, int I) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c * 8 >= I) return;
  const int64_t r = blockIdx.y;
  const T* xr = x + r * 2 * I;
  Pack8<T> g, u, o;
  g.u = *reinterpret_cast<const u32x4*>(xr + c * 8);
  u.u = *reinterpret_cast<const u32x4*>(xr + I + c * 8);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gf = to_f(g.h[j]);
    o.h[j] = from_f<T>(gf / (1.f + __expf(-gf)) * to_f(u.h[j]));
  }
  *reinterpret_cast<u32x4*>(out + r * I + c * 8) = o.u;
}

void launch_silu_mul(int dtype, void* out, const void* x, int64_t rows, int I, hipStream_t s) {
  for (int64_t r0 = 0; r0 < rows; r0 += 65535) {   // gridDim.y <= 65535
    const int64_t n = std::min<int64_t>(rows - r0, 65535);
    const dim3 grid(((I >> 3) + 255) / 256, (unsigned)n);
    if (dtype == DT_BF16)
      silu_mul_kernel<bf16><<<grid, 256, 0, s>>>((bf16*)out + r0 * I, (const bf16*)x + r0 * 2 * I, I);
    else
      silu_mul_kernel<f16><<<grid, 256, 0, s>>>((f16*)out + r0 * I, (const f16*)x + r0 * 2 * I, I);
  }
}

}  // namespace kgc
