// microbench7.hip — random 64-B row gathers (K = 16 u32 versions: the ANTIENTROPY dense round's
// peer and in-edge rows) and random 8-B word gathers from a 4 GiB table, by allocation type:
// hipMalloc (coarse-grained, cached in L2 by 128-B lines) against hipExtMallocWithFlags fine-grained
// and uncached.  Question: does an uncached table fetch only the 64 B a row needs?  Not product code.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// 4 lanes per row (16 B each), U rows in flight per lane group; rows written contiguously to out
template <int U>
__global__ __launch_bounds__(256) void gather_rows(const uint4* __restrict__ T, uint4* __restrict__ out, uint32_t rmask,
                                                   uint64_t nrows) {
  const uint32_t q = threadIdx.x & 3;
  const uint64_t g0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 2, ng = ((uint64_t)gridDim.x * 256) >> 2;
  for (uint64_t r0 = g0; r0 < nrows; r0 += ng * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t r = r0 + (uint64_t)u * ng;
      const uint32_t src = mix((uint32_t)r * 2654435761u) & rmask;
      v[u] = r < nrows ? T[(uint64_t)src * 4 + q] : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t r = r0 + (uint64_t)u * ng;
      if (r < nrows) out[r * 4 + q] = v[u];
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void gather_words(const uint64_t* __restrict__ T, uint64_t* __restrict__ sink,
                                                    uint32_t wmask, uint64_t n) {
  uint64_t acc = 0;
  const uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, ni = (uint64_t)gridDim.x * 256;
  for (uint64_t b = i0; b < n; b += ni * U) {
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * ni;
      v[u] = i < n ? T[mix((uint32_t)i * 40503u + 7u) & wmask] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if (acc == 0x12345ull) sink[0] = acc;
}

__global__ __launch_bounds__(256) void stream_copy(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) b[i] = a[i];
}

int main() {
  const uint64_t bytes = 4ull << 30;  // 2^26 rows of 64 B
  const uint64_t nrows = bytes / 64;
  uint4* out;
  uint64_t* sink;
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* kinds[] = {"hipMalloc", "finegrained", "uncached"};
  const unsigned flags[] = {0u, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
  for (int k = 0; k < 3; ++k) {
    void* T = nullptr;
    if (k == 0) CK(hipMalloc(&T, bytes));
    else CK(hipExtMallocWithFlags(&T, bytes, flags[k]));
    CK(hipMemset(T, 1, bytes));
    CK(hipDeviceSynchronize());
    auto run = [&](const char* name, double units, auto launch) -> int {
      launch();
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("{\"alloc\": \"%s\", \"case\": \"%s\", \"ms\": %.3f, \"G_units_per_s\": %.2f}\n", kinds[k], name, best,
             units / (best * 1e6));
      fflush(stdout);
      return 0;
    };
    if (run("gather_rows64_U4", (double)nrows, [&] { gather_rows<4><<<4096, 256>>>((const uint4*)T, out, (uint32_t)(nrows - 1), nrows); }))
      return 1;
    if (run("gather_rows64_U8", (double)nrows, [&] { gather_rows<8><<<4096, 256>>>((const uint4*)T, out, (uint32_t)(nrows - 1), nrows); }))
      return 1;
    if (run("gather_words8_U8", (double)nrows, [&] { gather_words<8><<<4096, 256>>>((const uint64_t*)T, sink, (uint32_t)(bytes / 8 - 1), nrows); }))
      return 1;
    if (run("gather_words8_16MiB_U8", (double)nrows, [&] { gather_words<8><<<4096, 256>>>((const uint64_t*)T, sink, (1u << 21) - 1, nrows); }))
      return 1;
    if (run("stream_copy_4GiB_GBps", (double)bytes * 2 / 1e3, [&] { stream_copy<<<4096, 256>>>((const uint4*)T, out, bytes / 16); }))
      return 1;
    CK(hipFree(T));
  }
  return 0;
}
