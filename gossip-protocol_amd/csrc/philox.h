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

// Fault model (the reference's lossy SyncRPC,
// main.go:77-87): the edge n -> p_j(n) of round t is lost in both directions
// when a partition separates its ends (nodes split into `parts` contiguous
// blocks) or when its loss draw, stream tag 4, falls below `loss` (P = loss/2^32).
// Stall mode (main.go:77-87, the expired 2 s context): a node
// whose initiated exchanges were lost in D rounds in a row initiates none until
// reset.  stall = the per-node streaks of all N nodes (random modes), or null.
struct Faults {
  uint32_t loss;   // 0: no loss
  uint32_t parts;  // 0 or 1: no partition
  uint64_t N;
  const uint8_t* stall = nullptr;
  uint32_t D = 0;
  __host__ __device__ bool any() const { return loss != 0 || parts > 1 || stall != nullptr; }
};

__host__ __device__ __forceinline__ uint32_t part_of(uint32_t n, const Faults& f) {
  return (uint32_t)(((uint64_t)n * f.parts) / f.N);
}

// Nodes reachable from n: [lo, hi) = n's partition block (q = part_of(n): the
// nodes m with q*N <= m*P < (q+1)*N), or everything.  Computed once per node,
// so the per-edge test is a range check.
struct Reach {
  uint32_t lo, hi;
};
// A stalled initiator reaches nobody: every edge it would start is lost.
__host__ __device__ __forceinline__ Reach reach_of(uint32_t n, const Faults& f) {
  if (f.stall && f.stall[n] >= f.D) return Reach{0xFFFFFFFFu, 0u};
  if (f.parts <= 1) return Reach{0u, 0xFFFFFFFFu};
  const uint64_t q = part_of(n, f);
  return Reach{(uint32_t)((q * f.N + f.parts - 1) / f.parts), (uint32_t)(((q + 1) * f.N + f.parts - 1) / f.parts)};
}

// the loss draws of edges 4q .. 4q+3 of node n in round t; FLOOD walks draw one per message:
// value slot x in the tag word's upper half (x = 0: the random modes' draw), DESIGN.md §2.9
__host__ __device__ __forceinline__ u32x4 loss_draws(uint32_t n, uint32_t t, uint32_t q, uint32_t k0, uint32_t k1,
                                                     uint32_t x = 0) {
  return philox4x32_10(u32x4{n, t, 4u | (x << 16), q}, k0, k1);
}

// edge n -> p lost?  rc = reach_of(n), lossw = lane j & 3 of loss_draws(n, t, j >> 2)
__host__ __device__ __forceinline__ bool edge_lost(const Faults& f, const Reach& rc, uint32_t p, uint32_t lossw) {
  return p < rc.lo || p >= rc.hi || lossw < f.loss;
}

// Rumor origins: stream tag 2.
// ANTIENTROPY churn word of node n in round t: with fanout k <= 3 the last
// word of the node's first peer draw x0 = Philox({n, t, 0, 0}) (peers use words 0 .. k-1), so
// one cipher per node serves both; else Philox({n, t, 1, 0}).x (x0 unused)
__host__ __device__ __forceinline__ uint32_t ae_churn_word(const u32x4& x0, uint32_t n, uint32_t t, uint32_t k,
                                                           uint32_t k0, uint32_t k1) {
  return k <= 3 ? x0.w : philox4x32_10(u32x4{n, t, 1u, 0u}, k0, k1).x;
}
// the first peer draw, computed only where ae_churn_word reads it
__host__ __device__ __forceinline__ u32x4 ae_first_draw(uint32_t n, uint32_t t, uint32_t k, uint32_t k0, uint32_t k1) {
  return k <= 3 ? philox4x32_10(u32x4{n, t, 0u, 0u}, k0, k1) : u32x4{0u, 0u, 0u, 0u};
}

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
