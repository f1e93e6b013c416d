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
constexpr uint32_t kSummBits = 1u << GOSSIP_SUMM_LOG;  // LDS summary: at most 2^20 bits (128 KiB; 2^19 / 2^18 slower, §3.7)

struct FrontierBufs {
  uint64_t* nzb;      // [ceil(N/64)] bit n: S[n] != 0
  uint64_t* fullb;    // [ceil(N/64)] bit n: S[n] == full mask
  uint32_t* summ;     // [summ_words] bit b: some rare node in [b*g, (b+1)*g)
  // [N] pending deltas, zero outside a sparse round: pushes and (round 4) the node's own pull
  // deltas alike, atomic ORs (one array: the commit reads and clears one word per node, not two)
  uint64_t* D;
  uint8_t* dirtyD;    // [ceil(N/64)] group g has a delta (not kept in all_d rounds)
  uint32_t glog;      // g = 1 << glog nodes per summary bit
  uint32_t summ_words;
  // Mid-level summary (one shard, 2^25 < N <= 2^30: the exact bitmaps no longer fit an XCD's
  // L2): bit b = some rare node in [b*g2, (b+1)*g2), g2 = 1 << g2log (8 up to 2^27 nodes), at
  // most 2 MiB so it stays L2-resident; a peer that hits the LDS summary is tested here before
  // its exact bitmap word is fetched from the MALL / HBM.  Null: not kept.
  uint32_t* summ2;
  uint32_t g2log, summ2_words;
  // one-shard rounds decide on the device, from the exact rare count of S_t: summ2 is built and
  // used when 1 - (1 - r)^g >= mid_frac (the LDS summary is that saturated)
  float mid_frac;
  // round 5: the scan's edges with a possibly rare end go through a per-wave LDS queue and are
  // resolved 128 at a time (one chain of round trips per 128 edges, not per wave batch); 0: the
  // per-batch resolution (param scan_queue)
  uint32_t scan_q;
  // round 6, binned sparse scan (frontier.hip K1a / K1b): set per round by the engine when the
  // round takes it (null: the LDS-summary scan).  brec: [bregions][k * 4096] u32 records,
  // btab: [bregions][btiles + 1] u16 run starts (+ btabT); all carved from the dense round's record slab.
  uint32_t* brec;
  uint16_t* btab;
  uint16_t* btabT;   // [btiles + 1][bregions]: btab transposed (K1b reads a tile's column contiguously)
  uint32_t btiles, bregions;
  uint64_t id0;      // global id of node 0 of these arrays (a shard's first node; 0 on one GPU): the hash uses global ids
};

uint32_t frontier_glog(uint64_t N);
// mid-level summary of N nodes: log2 of its group size, its u32 words (0: none below 2^25 or past 2^30 nodes)
uint32_t frontier_g2log(uint64_t N);
uint32_t frontier_summ2_words(uint64_t N);
size_t frontier_bytes(uint64_t N);
// the binned sparse scan's geometry: tiles of 2^19 peers, regions of 4096 senders; ok for
// k <= 4 and N <= 2^29; bytes of its record array and of its run-start table
bool bs_path_ok(uint64_t N, uint32_t k);
uint32_t bs_tiles(uint64_t N);
uint32_t bs_regions(uint64_t N);
size_t bs_rec_bytes(uint64_t N, uint32_t k);
size_t bs_tab_bytes(uint64_t N);
void frontier_carve(uint64_t N, void* base, FrontierBufs* f);

// Coarse summary (f.summ, 1 bit per 2^f.glog nodes) of the rare set of an
// N-node bitmap pair: maj 0 -> f.nzb, maj 1 -> not f.fullb, and the mid-level
// summary f.summ2 when f has one.  No early exit.
hipError_t launch_frontier_summary(const FrontierBufs& f, uint64_t N, uint32_t maj, hipStream_t st);

// how a sparse round's push deltas reach its commit (launch_frontier_round)
constexpr uint32_t kSparseFlags = 0, kSparseAllD = 1, kSparseDirect = 2;

// The commit half of a sparse round on its own: S |= D | P for the dirty (or,
// kSparseAllD, every) groups, D/P/flags cleared, bitmaps and running totals updated.
hipError_t launch_frontier_commit(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                  uint32_t dmode, uint32_t flags, hipStream_t st);

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
// dmode (how the push deltas reach the commit; exact in every mode):
//   kSparseFlags  the scan flags the push-dirty groups, the commit visits those;
//   kSparseAllD   the scan flags none and the commit reads D of every group —
//                 cheaper once pushes touch most groups (a random byte store per
//                 push costs about as much as the push atomic itself);
//   kSparseDirect (maj = 0 only) pushes into a majority (empty) peer are OR-ed
//                 straight into S: no kernel of the round reads a majority node's
//                 S_t (its value is known to be 0), so the round stays synchronous.
//                 A majority node's own pull is OR-ed into its S word the same way.
//                 Pushes into rare peers still go to D (flagged).  The commit then
//                 visits every group once, reads D / P only where flagged and
//                 recomputes the totals absolutely (S is read once; D is neither
//                 read nor cleared outside the flagged groups).
hipError_t launch_frontier_round(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                 uint32_t k, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode, uint32_t maj,
                                 uint32_t dmode, const Faults& fa, uint32_t flags, const RoundSync& rs,
                                 hipStream_t st);

}  // namespace gossip
