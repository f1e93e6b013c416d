// antientropy.h — version-vector anti-entropy kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gossip {

struct AeArgs {
  const uint32_t* V;     // S_t rows  [N][K]
  uint32_t* Vn;          // S_{t+1} rows (seeded with a copy of V)
  const uint8_t* alive;  // alive flags before round t's churn
  uint8_t* alive_n;      // after
  const uint32_t* target;  // global max vector (constant between injections)
  uint64_t* partial;
  uint64_t N;
  uint32_t K, L, k, t;
  uint32_t key0, key1, fail, rec;
  uint32_t flags;
};

uint32_t ae_lanes(uint32_t K);
hipError_t launch_ae_init(uint32_t* V, uint32_t* target, uint64_t N, uint32_t K, uint32_t k0, uint32_t k1,
                          hipStream_t st);
hipError_t launch_ae_inject(uint32_t* V, uint32_t* target, uint64_t node, uint32_t K, uint32_t c, hipStream_t st);
hipError_t launch_ae_round(const AeArgs& a, hipStream_t st);
hipError_t launch_ae_stats(const AeArgs& a, const uint32_t* V, const uint8_t* alive, hipStream_t st);

}  // namespace gossip
