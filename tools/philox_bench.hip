// philox_bench.hip — throughput of Philox4x32-10 formulations on gfx950 (which
// multiply instruction the ten rounds use).  Every variant must give the same
// words; each kernel draws one call per counter n in [0, N) and folds the words
// into one u32 per thread (no dead code), timed with hipEvents.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/philox_bench.hip -o exp/philox_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

struct u4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// V0: one 32x32->64 product per multiply (v_mad_u64_u32), the library's form
__device__ __forceinline__ void mul_v0(uint32_t a, uint32_t m, uint32_t& hi, uint32_t& lo) {
  const uint64_t p = (uint64_t)m * a;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}
// V1: separate high and low halves (v_mul_hi_u32 + v_mul_lo_u32)
__device__ __forceinline__ void mul_v1(uint32_t a, uint32_t m, uint32_t& hi, uint32_t& lo) {
  hi = __umulhi(a, m);
  lo = a * m;
}
// V2: 24-bit multiplies only (v_mul_u32_u24 / v_mul_hi_u32_u24): a = ah:al (8:24), m = mh:ml (8:24)
__device__ __forceinline__ void mul_v2(uint32_t a, uint32_t m, uint32_t& hi, uint32_t& lo) {
  const uint32_t al = a & 0xFFFFFFu, ah = a >> 24, ml = m & 0xFFFFFFu, mh = m >> 24;
  // al*ml: 48 bits; the masks let the compiler pick v_mul_u32_u24 / v_mul_hi_u32_u24
  uint32_t p0l, p0h;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p0l) : "v"(al), "v"(ml));
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(p0h) : "v"(al), "v"(ml));
  const uint64_t p0 = (uint64_t)p0h << 32 | p0l;
  // cross terms, each < 2^32: (al*mh + ah*ml) << 24, sum < 2^33
  const uint64_t c = (uint64_t)(al * mh) + (uint64_t)(ah * ml);
  const uint32_t hh = ah * mh;  // << 48
  const uint64_t p = p0 + (c << 24) + ((uint64_t)hh << 48);
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

template <int V>
__device__ __forceinline__ u4 philox(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0, lo0, hi1, lo1;
    if (V == 0) { mul_v0(c.x, 0xD2511F53u, hi0, lo0); mul_v0(c.z, 0xCD9E8D57u, hi1, lo1); }
    if (V == 1) { mul_v1(c.x, 0xD2511F53u, hi0, lo0); mul_v1(c.z, 0xCD9E8D57u, hi1, lo1); }
    if (V == 2) { mul_v2(c.x, 0xD2511F53u, hi0, lo0); mul_v2(c.z, 0xCD9E8D57u, hi1, lo1); }
    c = u4{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

template <int V>
__global__ __launch_bounds__(256) void draw_kernel(uint32_t N, uint32_t t, uint32_t k0, uint32_t k1, uint32_t* out) {
  uint32_t acc = 0;
  for (uint32_t n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
    const u4 r = philox<V>(u4{n, t, 0u, 0u}, k0, k1);
    acc ^= r.x + 3 * r.y + 5 * r.z + 7 * r.w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int V>
float run(uint32_t N, uint32_t grid, uint32_t* out, uint64_t* sum) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  draw_kernel<V><<<grid, 256>>>(N, 1, 0x1234u, 0x9876u, out);  // warm-up
  hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) draw_kernel<V><<<grid, 256>>>(N, 1, 0x1234u, 0x9876u, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  static uint32_t h[1 << 20];
  hipMemcpy(h, out, grid * 256 * 4, hipMemcpyDeviceToHost);
  uint64_t s = 0;
  for (uint32_t i = 0; i < grid * 256; ++i) s = s * 31 + h[i];
  *sum = s;
  return ms / reps;
}

int main() {
  const uint32_t N = 1u << 27, grid = 4096;
  uint32_t* out;
  if (hipMalloc(&out, grid * 256 * 4) != hipSuccess) return 1;
  uint64_t s0, s1, s2;
  const float t0 = run<0>(N, grid, out, &s0);
  const float t1 = run<1>(N, grid, out, &s1);
  const float t2 = run<2>(N, grid, out, &s2);
  printf("2^27 Philox4x32-10 calls: mad_u64 %.1f us, mul_hi+mul_lo %.1f us, u24 %.1f us; same words: %s %s\n",
         t0 * 1e3, t1 * 1e3, t2 * 1e3, s0 == s1 ? "yes" : "NO", s0 == s2 ? "yes" : "NO");
  hipFree(out);
  return s0 == s1 && s0 == s2 ? 0 : 2;
}
