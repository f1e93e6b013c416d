// microbench.hip — access-pattern ceilings on MI355X that bound the round kernels.
// Not product code: measures streaming copy, random 8-byte gather, random
// 8-byte atomicOr and random 8-byte store rates at table sizes below and above
// the 256 MiB Infinity Cache.  Output: one JSON line per measurement.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) b[i] = a[i];
}

__global__ void gather_kernel(const uint64_t* __restrict__ t, uint64_t* __restrict__ out, uint64_t n, uint32_t mask, uint32_t reps, uint32_t salt) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint64_t acc = 0;
    for (uint32_t r = 0; r < reps; ++r) acc |= t[hash32((uint32_t)i * reps + r + salt) & mask];
    out[i] = acc;
  }
}

__global__ void atomic_kernel(uint64_t* t, uint64_t n, uint32_t mask, uint32_t reps, uint32_t salt) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    for (uint32_t r = 0; r < reps; ++r)
      atomicOr((unsigned long long*)&t[hash32((uint32_t)i * reps + r + salt) & mask], 1ull << ((i + r) & 63));
}

__global__ void store_kernel(uint64_t* t, uint64_t n, uint32_t mask, uint32_t reps, uint32_t salt) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    for (uint32_t r = 0; r < reps; ++r) t[hash32((uint32_t)i * reps + r + salt) & mask] = i;
}

__global__ void lds_or_kernel(uint64_t* out, uint32_t iters) {
  __shared__ unsigned long long tile[16384];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) tile[i] = 0;
  __syncthreads();
  uint32_t x = blockIdx.x * 1024 + threadIdx.x;
  for (uint32_t it = 0; it < iters; ++it) {
    x = hash32(x + it);
    atomicOr(&tile[x & 16383], 1ull << (x >> 26));
  }
  __syncthreads();
  unsigned long long acc = 0;
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) acc ^= tile[i];
  if (acc == 0x123456789ull) out[0] = acc;
}

int main() {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const uint64_t maxbytes = 1ull << 31;
  uint64_t *buf, *buf2;
  CK(hipMalloc(&buf, maxbytes)); CK(hipMalloc(&buf2, maxbytes));
  CK(hipMemset(buf, 0x11, maxbytes)); CK(hipMemset(buf2, 0, maxbytes));
  float ms;
  // streaming copy
  for (uint64_t bytes : {128ull << 20, 1ull << 30}) {
    uint64_t n = bytes / 16;
    for (int w = 0; w < 2; ++w) copy_kernel<<<8192, 256>>>((uint4*)buf, (uint4*)buf2, n);
    CK(hipEventRecord(a));
    for (int r = 0; r < 10; ++r) copy_kernel<<<8192, 256>>>((uint4*)buf, (uint4*)buf2, n);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"test\":\"copy\",\"bytes\":%llu,\"GBps\":%.1f}\n", (unsigned long long)bytes, 2.0 * bytes * 10 / (ms * 1e-3) / 1e9);
  }
  const uint64_t nthreads = 1ull << 24;  // 16M lanes, 2 ops each
  for (uint64_t tbytes : {8ull << 20, 64ull << 20, 128ull << 20, 1ull << 30, 2ull << 30}) {
    uint32_t mask = (uint32_t)(tbytes / 8 - 1);
    for (int kind = 0; kind < 3; ++kind) {
      for (int w = 0; w < 2; ++w) {
        if (kind == 0) gather_kernel<<<16384, 256>>>(buf, buf2 + (1ull << 27) * 0, nthreads, mask, 2, w);
        if (kind == 1) atomic_kernel<<<16384, 256>>>(buf, nthreads, mask, 2, w);
        if (kind == 2) store_kernel<<<16384, 256>>>(buf, nthreads, mask, 2, w);
      }
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      const int reps = 5;
      for (int r = 0; r < reps; ++r) {
        if (kind == 0) gather_kernel<<<16384, 256>>>(buf, buf2, nthreads, mask, 2, 100 + r);
        if (kind == 1) atomic_kernel<<<16384, 256>>>(buf, nthreads, mask, 2, 100 + r);
        if (kind == 2) store_kernel<<<16384, 256>>>(buf, nthreads, mask, 2, 100 + r);
      }
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      double ops = 2.0 * nthreads * reps;
      const char* nm = kind == 0 ? "gather8" : kind == 1 ? "atomicOr8" : "store8";
      printf("{\"test\":\"%s\",\"table_bytes\":%llu,\"Gops\":%.2f,\"us_per_16M_lanes\":%.1f}\n", nm,
             (unsigned long long)tbytes, ops / (ms * 1e-3) / 1e9, ms * 1e3 / reps);
    }
  }
  // LDS 64-bit OR atomics (128 KiB tile per block)
  {
    const uint32_t iters = 1024, blocks = 1024, threads = 1024;
    lds_or_kernel<<<blocks, threads>>>(buf2, iters);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    lds_or_kernel<<<blocks, threads>>>(buf2, iters);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"test\":\"lds_or64\",\"Gops\":%.1f}\n", (double)iters * blocks * threads / (ms * 1e-3) / 1e9);
  }
  return 0;
}
