// microbench4.hip — HBM ceilings at 1 GiB (beyond the 256 MiB MALL): read, write, copy,
// and the mixed 2-stream-read + 1-stream-write shape of the round kernels.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void rd(const uint4* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t c = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) { uint4 v = a[i]; c ^= v.x ^ v.w; }
  if (c == 0x12345678u) out[0] = c;
}
__global__ __launch_bounds__(256) void wr(uint4* __restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) a[i] = make_uint4(i, 0, 0, 0);
}
__global__ __launch_bounds__(256) void cp(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) b[i] = a[i];
}
__global__ __launch_bounds__(256) void mix(const uint4* __restrict__ a, const uint4* __restrict__ b, uint4* __restrict__ c, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint4 x = a[i], y = b[i];
    c[i] = make_uint4(x.x | y.x, x.y | y.y, x.z | y.z, x.w | y.w);
  }
}
int main() {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const uint64_t B = 1ull << 30, n = B / 16;
  uint4 *a, *b, *c; uint32_t* out;
  CK(hipMalloc(&a, B)); CK(hipMalloc(&b, B)); CK(hipMalloc(&c, B)); CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 1, B)); CK(hipMemset(b, 2, B)); CK(hipMemset(c, 3, B));
  float ms;
  auto T = [&](auto&& f, const char* name, double bytes) {
    for (uint32_t grid : {2048u, 8192u}) {
      f(grid); CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) f(grid); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"test\":\"%s\",\"grid\":%u,\"us\":%.1f,\"GBps\":%.0f}\n", name, grid, ms * 200, bytes / (ms * 1e-3 / 5) / 1e9);
    }
    return 0;
  };
  T([&](uint32_t g) { rd<<<g, 256>>>(a, n, out); }, "read_1GiB", (double)B);
  T([&](uint32_t g) { wr<<<g, 256>>>(a, n); }, "write_1GiB", (double)B);
  T([&](uint32_t g) { cp<<<g, 256>>>(a, b, n); }, "copy_1GiB(rd+wr bytes)", 2.0 * B);
  T([&](uint32_t g) { mix<<<g, 256>>>(a, b, c, n); }, "2rd1wr_1GiB(all bytes)", 3.0 * B);
  return 0;
}
