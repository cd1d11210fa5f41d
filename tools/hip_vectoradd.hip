// gfx950 smoke test for a GPU pod: c = a + b over 1M floats, checked on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void vadd(const float* a, const float* b, float* c, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = a[i] + b[i];
}

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::printf("FAILED: %s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const int n = 1 << 20;
  int devs = 0;
  CHECK(hipGetDeviceCount(&devs));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  std::printf("devices: %d, device 0: %s (%s), %d CUs\n", devs, p.name, p.gcnArchName,
              p.multiProcessorCount);
  std::vector<float> a(n), b(n), c(n);
  for (int i = 0; i < n; ++i) { a[i] = i; b[i] = 2.f * i; }
  float *da, *db, *dc;
  CHECK(hipMalloc(&da, n * 4)); CHECK(hipMalloc(&db, n * 4)); CHECK(hipMalloc(&dc, n * 4));
  CHECK(hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice));
  vadd<<<(n + 255) / 256, 256>>>(da, db, dc, n);
  CHECK(hipGetLastError());
  CHECK(hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; ++i)
    if (c[i] != 3.f * i) { std::printf("FAILED at %d\n", i); return 1; }
  std::printf("Test PASSED\n");
  CHECK(hipFree(da)); CHECK(hipFree(db)); CHECK(hipFree(dc));
  return 0;
}
