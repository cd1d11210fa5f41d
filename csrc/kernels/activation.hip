// K7 SiLU-and-mul: out[t, i] = silu(x[t, i]) * x[t, I + i] over the fused gate_up
// projection output.  16-byte vector loads/stores (8 halves per lane), grid capped
// at 256 CUs x 8 blocks with a grid-stride loop (memory-bound).
#include "common.h"
#include "launch.h"

namespace kgc {

template <typename T>
__global__ __launch_bounds__(256) void silu_mul_kernel(T* __restrict__ out,
                                                       const T* __restrict__ x, int64_t rows,
                                                       int I) {
  const int nv = I >> 3;
  const int64_t total = rows * nv;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / nv;
    const int c = (int)(i - r * nv);
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
}

void launch_silu_mul(int dtype, void* out, const void* x, int64_t rows, int I, hipStream_t s) {
  if (rows == 0) return;
  const int64_t total = rows * (I >> 3);
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 2048);
  if (dtype == DT_BF16)
    silu_mul_kernel<bf16><<<grid, 256, 0, s>>>((bf16*)out, (const bf16*)x, rows, I);
  else
    silu_mul_kernel<f16><<<grid, 256, 0, s>>>((f16*)out, (const f16*)x, rows, I);
}

}  // namespace kgc
