// philox.h — Philox4x32-10 counter-based generator, host + device.
//
// Peer selection in the reference is the harness-given Topology[node.ID()]
// (main.go:72).  The random modes replace it with counter-based draws so that
// every GPU (and the CPU restatement) derives the same peers from
// (seed, node, round) with no stored state.  Constants and round structure are
// Random123's, identical to /opt/rocm/include/rocrand/rocrand_philox4x32_10.h
// :62-65 (constants) and :270-302 (ten rounds + key bump).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gossip {

struct u32x4 {
  uint32_t x, y, z, w;
};

// a ^ b ^ c: one v_bitop3_b32 (truth table 0x96) on gfx950, which has no v_xor3
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // one 32x32->64 product each (v_mad_u64_u32 on gfx950) gives both halves
    const uint64_t m0 = (uint64_t)0xD2511F53u * c.x, m1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(m0 >> 32), lo0 = (uint32_t)m0;
    const uint32_t hi1 = (uint32_t)(m1 >> 32), lo1 = (uint32_t)m1;
    c = u32x4{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__host__ __device__ __forceinline__ uint32_t lane_of(const u32x4& x, uint32_t q) {
  return q == 0 ? x.x : q == 1 ? x.y : q == 2 ? x.z : x.w;
}

// Uniform over [0, N) \ {n} by integer arithmetic only.
// N < 2^32, so N-1 fits 32 bits and the scaling is one high-half product.
__host__ __device__ __forceinline__ uint32_t peer_from_word(uint32_t x, uint64_t nm1, uint32_t n) {
  const uint32_t p = (uint32_t)(((uint64_t)x * (uint32_t)nm1) >> 32);
  return p + (p >= n ? 1u : 0u);
}

// Rumor origins: stream tag 2.
__host__ __device__ __forceinline__ uint32_t origin_of(uint32_t r, uint64_t N, uint32_t k0, uint32_t k1) {
  const u32x4 x = philox4x32_10(u32x4{r, 0u, 2u, 0u}, k0, k1);
  return (uint32_t)(((uint64_t)x.x * N) >> 32);
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

constexpr uint64_t kGold64 = 0x9E3779B97F4A7C15ull;

}  // namespace gossip
