// microbench2.hip — piece-size and atomic-scope ceilings for the binned round.
//  frag_write P: each lane-group writes P-byte pieces at scattered piece slots
//  frag_read  P: same pattern, reads
//  wg_atomic:    64-bit atomicOr at workgroup scope into a block-private region
//                of R bytes (is it performed in L2?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// pieces of P bytes (P/8 u64 lanes per piece); piece slot chosen by hash -> scattered
template <int P>
__global__ void frag_write(uint64_t* buf, uint64_t npieces, uint32_t salt) {
  constexpr int L = P / 8;
  const uint64_t gl = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t piece = gl / L, sub = gl % L;
  if (piece >= npieces) return;
  const uint64_t slot = hash32((uint32_t)piece ^ salt) % npieces;
  buf[slot * L + sub] = gl;
}
template <int P>
__global__ void frag_read(const uint64_t* buf, uint64_t* out, uint64_t npieces, uint32_t salt) {
  constexpr int L = P / 8;
  const uint64_t gl = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t piece = gl / L, sub = gl % L;
  if (piece >= npieces) return;
  const uint64_t slot = hash32((uint32_t)piece ^ salt) % npieces;
  uint64_t v = buf[slot * L + sub];
  if (v == 0x1234567ull) out[0] = v;
}

template <int SCOPE>
__global__ void region_atomic(uint64_t* buf, uint32_t region_words, uint32_t iters) {
  uint64_t* r = buf + (uint64_t)blockIdx.x * region_words;
  uint32_t x = blockIdx.x * 1024 + threadIdx.x;
  for (uint32_t i = 0; i < iters; ++i) {
    x = hash32(x + i);
    __hip_atomic_fetch_or(&r[x % region_words], 1ull << (x >> 26), __ATOMIC_RELAXED, SCOPE);
  }
}

int main() {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const uint64_t bytes = 512ull << 20;
  uint64_t *buf, *out;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, bytes));
  float ms;
#define RUNP(P) { uint64_t np = bytes / P; uint64_t lanes = np * (P / 8); uint32_t grid = (uint32_t)((lanes + 255) / 256); \
    frag_write<P><<<grid, 256>>>(buf, np, 1); CK(hipDeviceSynchronize()); \
    CK(hipEventRecord(a)); for (int r = 0; r < 5; ++r) frag_write<P><<<grid, 256>>>(buf, np, r); CK(hipEventRecord(b)); \
    CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b)); \
    printf("{\"test\":\"frag_write\",\"piece\":%d,\"GBps\":%.1f}\n", P, 5.0 * bytes / (ms * 1e-3) / 1e9); \
    frag_read<P><<<grid, 256>>>(buf, out, np, 1); CK(hipDeviceSynchronize()); \
    CK(hipEventRecord(a)); for (int r = 0; r < 5; ++r) frag_read<P><<<grid, 256>>>(buf, out, np, r); CK(hipEventRecord(b)); \
    CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b)); \
    printf("{\"test\":\"frag_read\",\"piece\":%d,\"GBps\":%.1f}\n", P, 5.0 * bytes / (ms * 1e-3) / 1e9); }
  RUNP(8) RUNP(16) RUNP(32) RUNP(64) RUNP(128) RUNP(256) RUNP(512)
  for (uint32_t rb : {65536u, 131072u}) {
    const uint32_t words = rb / 8, blocks = 1024, iters = 256;
    for (int sc = 0; sc < 2; ++sc) {
      if (sc == 0) region_atomic<__HIP_MEMORY_SCOPE_WORKGROUP><<<blocks, 1024>>>(buf, words, iters);
      else region_atomic<__HIP_MEMORY_SCOPE_AGENT><<<blocks, 1024>>>(buf, words, iters);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      if (sc == 0) region_atomic<__HIP_MEMORY_SCOPE_WORKGROUP><<<blocks, 1024>>>(buf, words, iters);
      else region_atomic<__HIP_MEMORY_SCOPE_AGENT><<<blocks, 1024>>>(buf, words, iters);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"test\":\"region_atomicOr\",\"scope\":\"%s\",\"region_bytes\":%u,\"Gops\":%.1f}\n", sc ? "agent" : "workgroup", rb,
             (double)blocks * 1024 * iters / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
