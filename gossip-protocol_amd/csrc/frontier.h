// frontier.h — sparse rounds of the random modes (W == 1, one shard).
//
// When almost every node is in one class — all-zero early in a run, all-full
// late in it — an edge between two majority nodes moves nothing, so a round
// only has to find the edges that touch a "rare" node.  Two occupancy bitmaps
// (nonzero, full) are kept exact by every round; a coarse summary of the rare
// set sits in LDS so that the peer test of an edge almost never leaves the CU.
// Deltas are OR-ed into D (zero between rounds) and committed in place.
// DESIGN.md §3.3 has the rules and the byte accounting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox.h"
#include "round.h"

namespace gossip {

#ifndef GOSSIP_SUMM_LOG
#define GOSSIP_SUMM_LOG 20
#endif
constexpr uint32_t kSummBits = 1u << GOSSIP_SUMM_LOG;  // LDS summary: at most 2^20 bits (128 KiB)

struct FrontierBufs {
  uint64_t* nzb;      // [ceil(N/64)] bit n: S[n] != 0
  uint64_t* fullb;    // [ceil(N/64)] bit n: S[n] == full mask
  uint32_t* summ;     // [summ_words] bit b: some rare node in [b*g, (b+1)*g)
  uint64_t* D;        // [N] pending push deltas (atomic OR), zero outside a sparse round
  uint64_t* P;        // [N] pending pull deltas (plain store by the node's own lane), zero outside
  uint8_t* dirtyD;    // [ceil(N/64)] group g has a push delta (not kept in all_d rounds)
  uint8_t* dirtyP;    // [ceil(N/64)] group g has a pull delta
  uint32_t glog;      // g = 1 << glog nodes per summary bit
  uint32_t summ_words;
  uint64_t id0;       // global id of node 0 of these arrays (a shard's first node; 0 on one GPU): the hash uses global ids
};

uint32_t frontier_glog(uint64_t N);
size_t frontier_bytes(uint64_t N);
void frontier_carve(uint64_t N, void* base, FrontierBufs* f);

// Coarse summary (f.summ, 1 bit per 2^f.glog nodes) of the rare set of an
// N-node bitmap pair: maj 0 -> f.nzb, maj 1 -> not f.fullb.  No early exit.
hipError_t launch_frontier_summary(const FrontierBufs& f, uint64_t N, uint32_t maj, hipStream_t st);

// The commit half of a sparse round on its own: S |= D | P for the dirty (or,
// all_d, every) groups, D/P/flags cleared, bitmaps and running totals updated.
hipError_t launch_frontier_commit(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                  bool all_d, uint32_t flags, hipStream_t st);

// Absolute stats of S into partial (zeroed by the caller) + both bitmaps.
hipError_t launch_frontier_rebuild(const FrontierBufs& f, const uint64_t* S, uint64_t N, uint64_t* partial,
                                   uint32_t R, uint32_t flags, hipStream_t st);

// Client broadcast that keeps the running totals (partial) and both bitmaps
// exact: node >= 0 sets one bit, node < 0 injects every rumor at its origin.
hipError_t launch_frontier_inject(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                  uint32_t key0, uint32_t key1, int64_t node, uint32_t rumor, uint32_t flags,
                                  hipStream_t st);

// One sparse round, in place on S.  maj = 0: rare = nonzero nodes; maj = 1:
// rare = nodes not yet full (either choice is exact; it only moves time).
// partial holds the totals of S_t on entry and those of S_{t+1} on exit; the
// last commit block hands them to the host through rs.  With no rare node the
// round is a no-op (every kernel returns at once).
// all_d: the scan does not flag push-dirty groups and the commit reads D of
// every group instead — cheaper once pushes touch most groups (a random byte
// store per push costs about as much as the push atomic itself).  Exact either way.
hipError_t launch_frontier_round(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                 uint32_t k, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode, uint32_t maj,
                                 bool all_d, const Faults& fa, uint32_t flags, const RoundSync& rs,
                                 hipStream_t st);

}  // namespace gossip
