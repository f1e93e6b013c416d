// microbench3.hip — floors for the frontier (sparse-round) kernels on MI355X.
// Not product code.  One JSON line per measurement:
//   philox   : one Philox4x32-10 + k=2 peer draws per node over 2^24 nodes (compute floor of a round)
//   stream   : read 128 MiB as u64 / u128 lanes with a data-dependent branch (D-scan floor)
//   atomic   : random 8-byte atomicOr over a 128 MiB table, with and without a used return value
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../gossip-protocol_amd/csrc/philox.h"

using namespace gossip;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ __launch_bounds__(1024) void philox_kernel(uint64_t N, uint32_t t, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t n = blockIdx.x * 1024ull + threadIdx.x; n < N; n += gridDim.x * 1024ull) {
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)n, t, 0u, 0u}, 0x5EED0003u, 0u);
    acc ^= peer_from_word(r.x, N - 1, (uint32_t)n) + peer_from_word(r.y, N - 1, (uint32_t)n);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(1024) void philox_lds_kernel(uint64_t N, uint32_t t, const uint32_t* summ, uint32_t* out) {
  __shared__ uint4 s4[8192];
  const uint32_t* s = (const uint32_t*)s4;
  for (uint32_t i = threadIdx.x; i < 8192; i += 1024) s4[i] = ((const uint4*)summ)[i];
  __syncthreads();
  uint32_t acc = 0;
  for (uint64_t n = blockIdx.x * 1024ull + threadIdx.x; n < N; n += gridDim.x * 1024ull) {
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)n, t, 0u, 0u}, 0x5EED0003u, 0u);
    const uint32_t p0 = peer_from_word(r.x, N - 1, (uint32_t)n), p1 = peer_from_word(r.y, N - 1, (uint32_t)n);
    acc += (s[p0 >> 9] >> ((p0 >> 4) & 31)) & 1;
    acc += (s[p1 >> 9] >> ((p1 >> 4) & 31)) & 1;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void stream64_kernel(const uint64_t* __restrict__ D, uint64_t n, uint32_t* out) {
  uint32_t c = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) c += D[i] != 0;
  if (c == 0x12345678u) out[0] = c;
}

__global__ __launch_bounds__(256) void stream128_kernel(const uint4* __restrict__ D, uint64_t n, uint32_t* out) {
  uint32_t c = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint4 v = D[i];
    c += (v.x | v.y | v.z | v.w) != 0;
  }
  if (c == 0x12345678u) out[0] = c;
}

__global__ __launch_bounds__(256) void atomic_kernel(uint64_t* t, uint64_t n, uint32_t mask, uint32_t salt, uint32_t* out,
                                                     int ret) {
  uint64_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    uint64_t* a = &t[hash32((uint32_t)i + salt) & mask];
    const unsigned long long v = 1ull << (i & 63);
    if (ret) acc += atomicOr((unsigned long long*)a, v);
    else atomicOr((unsigned long long*)a, v);
  }
  if (ret && acc == 0x123456789ull) out[0] = 1;
}

int main() {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint64_t N = 1ull << 24;
  uint64_t* buf;
  uint32_t *out, *summ;
  CK(hipMalloc(&buf, N * 8 * 2));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&summ, 131072));
  CK(hipMemset(buf, 0, N * 16));
  CK(hipMemset(summ, 0x11, 131072));
  float ms;
  auto time = [&](auto&& launch, int reps) -> float {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
  };
  for (uint32_t grid : {256u, 512u, 1024u, 2048u}) {
    float us = time([&] { philox_kernel<<<grid, 1024>>>(N, 7, out); }, 20);
    printf("{\"test\":\"philox\",\"nodes\":%llu,\"grid\":%u,\"us\":%.1f}\n", (unsigned long long)N, grid, us);
  }
  for (uint32_t grid : {256u, 512u}) {
    float us = time([&] { philox_lds_kernel<<<grid, 1024>>>(N, 7, summ, out); }, 20);
    printf("{\"test\":\"philox_lds\",\"nodes\":%llu,\"grid\":%u,\"us\":%.1f}\n", (unsigned long long)N, grid, us);
  }
  for (uint32_t grid : {1024u, 2048u, 4096u}) {
    float us = time([&] { stream64_kernel<<<grid, 256>>>(buf, N, out); }, 20);
    printf("{\"test\":\"stream64\",\"bytes\":%llu,\"grid\":%u,\"us\":%.1f,\"GBps\":%.0f}\n",
           (unsigned long long)(N * 8), grid, us, N * 8 / us / 1e3);
    us = time([&] { stream128_kernel<<<grid, 256>>>((const uint4*)buf, N / 2, out); }, 20);
    printf("{\"test\":\"stream128\",\"bytes\":%llu,\"grid\":%u,\"us\":%.1f,\"GBps\":%.0f}\n",
           (unsigned long long)(N * 8), grid, us, N * 8 / us / 1e3);
  }
  const uint64_t nat = 1ull << 22;
  for (int ret : {0, 1}) {
    float us = time([&] { atomic_kernel<<<2048, 256>>>(buf, nat, (uint32_t)(N - 1), 99, out, ret); }, 10);
    printf("{\"test\":\"atomicOr8\",\"ret\":%d,\"ops\":%llu,\"table_bytes\":%llu,\"us\":%.1f,\"Gops\":%.1f}\n", ret,
           (unsigned long long)nat, (unsigned long long)(N * 8), us, nat / us / 1e3);
  }
  return 0;
}
