// microbench6.hip — random 8-B gathers from a window of S that one XCD's blocks share (held in
// that XCD's L2), against the whole 1 GiB table: can a serve pass read its replies from L2 instead
// of an LDS tile image?  Models the 2^27-node serve (2^28 gathers into a 2^27-word S, replies
// written contiguously).  Not product code.
//   Block b runs on XCD b % 8 (round-robin dispatch); XCD x walks windows x * nwin + w, w = 0..nwin-1,
//   in order; its 32 blocks split each window's gathers.  Index = hash(i) within the window.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// STORE: 0 none (xor into a sink), 1 plain contiguous stores, 2 non-temporal contiguous stores
template <int U, int STORE>
__global__ __launch_bounds__(1024) void gather_win(const uint64_t* __restrict__ S, uint64_t* __restrict__ out,
                                                   uint32_t win_log, uint32_t nwin, uint32_t per_block,
                                                   uint64_t* sink) {
  const uint32_t x = blockIdx.x & 7u, j = blockIdx.x >> 3, nb = gridDim.x >> 3;
  const uint32_t wmask = (1u << win_log) - 1u;
  uint64_t acc = 0;
  for (uint32_t w = 0; w < nwin; ++w) {
    const uint64_t win = (uint64_t)(x * nwin + w);
    const uint64_t base = win << win_log;
    uint64_t* o = out + (win * nb + j) * per_block;
    for (uint32_t i0 = 0; i0 < per_block; i0 += 1024u * U) {
      uint64_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = min(i0 + u * 1024u + threadIdx.x, per_block - 1);
        v[u] = S[base + (mix(i * 2654435761u + (uint32_t)win * 40503u + j) & wmask)];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t i = i0 + u * 1024u + threadIdx.x;
        if (i >= per_block) break;
        if (STORE == 1) o[i] = v[u];
        else if (STORE == 2) __builtin_nontemporal_store(v[u], &o[i]);
        else acc ^= v[u];
      }
    }
  }
  if (STORE == 0 && acc == 0x1234567ull) sink[0] = acc;
}

// streams of the same shape as the serve's non-gather traffic: read 2^28 u16, write 2^28 u64
__global__ __launch_bounds__(1024) void streams(const uint16_t* __restrict__ ids, uint64_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = blockIdx.x * 1024ull + threadIdx.x; i < n; i += gridDim.x * 1024ull)
    __builtin_nontemporal_store((uint64_t)ids[i] * 3u, &out[i]);
}

int main() {
  const uint32_t NLOG = 27;  // S words
  const uint64_t NS = 1ull << NLOG, NG = 1ull << 28;  // gathers
  uint64_t *S, *out, *sink;
  uint16_t* ids;
  CK(hipMalloc(&S, NS * 8)); CK(hipMalloc(&out, NG * 8)); CK(hipMalloc(&sink, 64)); CK(hipMalloc(&ids, NG * 2));
  CK(hipMemset(S, 1, NS * 8)); CK(hipMemset(ids, 1, NG * 2));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const uint32_t grid = 256;
  auto run = [&](const char* name, auto launch) -> int {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
    }
    printf("{\"case\": \"%s\", \"ms\": %.3f, \"G_per_s\": %.1f}\n", name, best, NG / (best * 1e6));
    fflush(stdout);
    return 0;
  };
  char nm[128];
  for (uint32_t wl : {14u, 16u, 17u, 18u, 19u, 27u - 3u}) {  // window words: 128 KB .. 4 MB, and 1/8 of S
    const uint32_t nwin = (uint32_t)(NS >> wl) / 8;
    const uint32_t per_block = (uint32_t)(NG / ((uint64_t)nwin * grid));
    snprintf(nm, sizeof nm, "win_%uKB_nostore", (8u << wl) >> 10);
    run(nm, [&] { gather_win<8, 0><<<grid, 1024>>>(S, out, wl, nwin, per_block, sink); });
    snprintf(nm, sizeof nm, "win_%uKB_store", (8u << wl) >> 10);
    run(nm, [&] { gather_win<8, 1><<<grid, 1024>>>(S, out, wl, nwin, per_block, sink); });
    snprintf(nm, sizeof nm, "win_%uKB_ntstore", (8u << wl) >> 10);
    run(nm, [&] { gather_win<8, 2><<<grid, 1024>>>(S, out, wl, nwin, per_block, sink); });
  }
  run("win_18_U4_ntstore", [&] { gather_win<4, 2><<<grid, 1024>>>(S, out, 18, 64, (uint32_t)(NG / (64ull * 8 * grid)), sink); });
  run("win_18_U16_ntstore", [&] { gather_win<16, 2><<<grid, 1024>>>(S, out, 18, 64, (uint32_t)(NG / (64ull * 8 * grid)), sink); });
  run("streams_u16_to_u64", [&] { streams<<<grid * 4, 1024>>>(ids, out, NG); });
  return 0;
}
