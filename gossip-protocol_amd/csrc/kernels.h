// kernels.h — HIP round kernels for gfx950 (declarations + launch helpers).
//
// Device layout: rumor words are structure-of-arrays,
// word w of local node i at S[w * Nl + i]; the gathered image of all shards is
// [G][W][Nl], which for W == 1 is simply the global node order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox.h"

namespace gossip {

struct RoundArgs {
  const uint64_t* S;      // own shard S_t            [W][Nl]
  const uint64_t* G;      // gathered exchange image  [G][W][Nl] (S_t, or F_t for FLOOD)
  uint64_t* Snext;        // own shard S_{t+1}        [W][Nl]
  uint64_t* partial;      // stats partial vector (device, zeroed per round)
  uint64_t N, Nl, lo, nown;
  uint32_t W, R, k, t;
  uint32_t key0, key1;
  uint32_t flags;
  uint32_t mode;
  Faults fa;              // random modes: lost edges (philox.h)
  // FLOOD only
  const uint64_t* Sprev;  // own shard S_{t-1}
  uint64_t* skip;         // own shard sender-skip masks
  const uint32_t *orow, *ocol, *irow, *icol;
};

// FLOOD with faults: one walk per (value x, node u) of one shard
// (G == 1), index x * N + u, down u's row in the topology message's order.
constexpr uint32_t kWalkNone = 0xFFFFFFFFu;  // snd: no first sender (a client's value); cur: no walk
struct FloodWalks {
  uint32_t* cur;  // next position in u's row
  uint8_t* att;   // lost attempts on that position
  uint32_t* snd;  // first sender of x at u
  uint32_t D;     // lost attempts that expire a neighbour's context (0: never)
};

hipError_t launch_round_random(const RoundArgs& a, hipStream_t st);
hipError_t launch_round_flood_walks(const RoundArgs& a, const FloodWalks& fw, hipStream_t st);
// Stall streaks after round t (random modes), all N nodes; fa.stall is the array.
hipError_t launch_stall_update(uint8_t* stall, uint64_t N, uint32_t k, uint32_t t, uint32_t key0, uint32_t key1,
                               const Faults& fa, hipStream_t st);
hipError_t launch_round_flood(const RoundArgs& a, hipStream_t st);
hipError_t launch_stats(const RoundArgs& a, hipStream_t st);
hipError_t launch_frontier(const uint64_t* S, const uint64_t* Sprev, uint64_t* F, uint64_t n, hipStream_t st);
// fw (FLOOD with faults, or null): a value new at its node starts its walk next round
hipError_t launch_inject(uint64_t* S, uint64_t Nl, uint64_t lo, uint64_t hi, uint64_t N, uint32_t R, uint32_t key0,
                         uint32_t key1, int64_t node, uint32_t rumor, hipStream_t st, const FloodWalks* fw = nullptr);
hipError_t launch_hash(const uint64_t* S, uint64_t Nl, uint64_t nown, uint32_t W, uint64_t N, uint64_t lo,
                       uint64_t* out, hipStream_t st);
hipError_t launch_philox(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out, uint32_t n, hipStream_t st);
// Small values a sharded round hands to a device-side collective (counts, partials):
// out[i] = in64[i] or in32[i] (widened) for i < n, then out[slot] = value when slot >= 0.
hipError_t launch_publish(const uint64_t* in64, const uint32_t* in32, uint64_t* out, uint32_t n, int32_t slot,
                          uint64_t value, hipStream_t st);

}  // namespace gossip
