// microbench5.hip — scattered piece writes/reads at 1 GiB: does a write piece that starts or ends
// inside a 64-B chunk (shared with a piece written at another time) cost HBM bandwidth?
// Models bin_serve's response runs (random lengths, random order).  Not product code.
//   order[i] = destination word of thread i; the words of one piece are consecutive in order[],
//   pieces are shuffled.  Variants differ only in piece lengths / alignment.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void scat_wr(const uint32_t* __restrict__ order, uint64_t* __restrict__ buf, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint32_t w = order[i];
    if (w != 0xFFFFFFFFu) buf[w] = i;
  }
}
__global__ __launch_bounds__(256) void scat_rd(const uint32_t* __restrict__ order, const uint64_t* __restrict__ buf, uint64_t n,
                                               uint64_t* out) {
  uint64_t c = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint32_t w = order[i];
    if (w != 0xFFFFFFFFu) c ^= buf[w];
  }
  if (c == 0x123456789ull) out[0] = c;
}

int main() {
  const uint64_t NW = 1ull << 27;  // 1 GiB of u64 words
  uint64_t* buf; uint32_t* order; uint64_t* out;
  CK(hipMalloc(&buf, NW * 8)); CK(hipMalloc(&order, NW * 4)); CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 0, NW * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::mt19937_64 rng(12345);
  std::vector<uint32_t> h(NW);
  struct Piece { uint32_t start, len; };
  // kind: 0 sequential; 1 random len [1,31] unaligned; 2 same lens, each piece padded to 8 words (64-B chunks);
  //       3 len 16 aligned 128 B; 4 len 16 at +8 B; 5 random len [1,15]; 6 len 8 aligned 64 B;
  //       7 random len [1,31], pieces placed in 64-B aligned slots, only len words written (partial chunk at the end)
  const char* names[] = {"sequential", "rand1-31_unaligned", "rand1-31_padded64", "16w_aligned128", "16w_off8B",
                         "rand1-15_unaligned", "8w_aligned64", "rand1-31_aligned_start_partial_end"};
  for (int kind = 0; kind < 8; ++kind) {
    std::vector<Piece> ps;
    uint64_t pos = 0, useful = 0;
    if (kind == 4) pos = 1;
    while (true) {
      uint32_t len;
      if (kind == 0) len = 64;
      else if (kind == 1 || kind == 2 || kind == 7) len = 1 + rng() % 31;
      else if (kind == 3 || kind == 4) len = 16;
      else if (kind == 5) len = 1 + rng() % 15;
      else len = 8;
      const uint32_t span = (kind == 2 || kind == 7) ? (len + 7) & ~7u : len;
      if (pos + span > NW) break;
      ps.push_back({(uint32_t)pos, kind == 2 ? span : len});
      useful += len;
      pos += span;
    }
    if (kind != 0) std::shuffle(ps.begin(), ps.end(), rng);
    uint64_t i = 0;
    for (auto& p : ps)
      for (uint32_t j = 0; j < p.len; ++j) h[i++] = p.start + j;
    const uint64_t n = i;
    for (; i < NW; ++i) h[i] = 0xFFFFFFFFu;
    CK(hipMemcpy(order, h.data(), NW * 4, hipMemcpyHostToDevice));
    for (int rw = 0; rw < 2; ++rw) {
      auto run = [&]() { if (rw == 0) scat_wr<<<8192, 256>>>(order, buf, n); else scat_rd<<<8192, 256>>>(order, buf, n, out); };
      run(); CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 5; ++r) run();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / 5;
      printf("{\"test\":\"%s\",\"op\":\"%s\",\"pieces\":%zu,\"words\":%lu,\"useful_words\":%lu,\"us\":%.1f,"
             "\"data_GBps\":%.0f,\"useful_GBps\":%.0f}\n",
             names[kind], rw ? "read" : "write", ps.size(), (unsigned long)n, (unsigned long)useful, us,
             n * 8.0 / us / 1e3, useful * 8.0 / us / 1e3);
      fflush(stdout);
    }
  }
  return 0;
}
