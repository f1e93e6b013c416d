// round.h — end-of-round hand-off of the running totals to the host.
//
// The host enqueues rounds ahead of the stats it has read.
// After every round a one-block kernel copies the totals into a host-mapped
// ring slot and then writes the slot's sequence word, which the host polls:
// no event or copy-engine transfer sits between rounds.  (Doing it in the last
// block of the round's final kernel needs a device-scope release per block,
// which costs more than the launch on gfx950.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gossip {

struct RoundSync {
  uint64_t* ring;  // host-mapped slot: [plen] totals, then [plen] = seq
  uint32_t plen;
  uint32_t seq;
};

// One block: copies partial (plen u64) to rs.ring, then writes rs.ring[plen] =
// rs.seq.  Enqueued after the round's last kernel (its stats atomics are then
// complete and visible).
hipError_t launch_round_snapshot(const uint64_t* partial, const RoundSync& rs, hipStream_t st);

}  // namespace gossip
