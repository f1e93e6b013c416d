// sharded.h — sparse rounds of the random modes across G shards (W == 1).
//
// One engine per GPU owns nodes [lo, lo + nown).  A sparse round (one class of
// nodes rare, as in frontier.h) moves only what touches the rare set:
//   1. each shard lists its own rare nodes {id, S_t} in id order   (sx_compact)
//   2. the driver all-gathers the lists                              (RCCL)
//   3. every shard builds the same global rare index from them: a bitmap over
//      all N nodes, per-word rank counts (exact membership and value lookup)
//      and the LDS summary of frontier.h                               (sx_index)
//   4. every shard scans its own nodes with their global Philox peers: pulls
//      land in P, pushes to its own nodes in D, pushes to other shards become
//      messages {node at the owner, delta} grouped by owner            (sx_scan)
//   5. the driver all-to-alls the messages                             (RCCL)
//   6. received pushes are OR-ed into D                                (sx_apply)
//   7. the frontier commit updates S, bitmaps and the shard's totals.
// Peers depend only on the global node id, the round and the seed, so the
// result equals the one-GPU round bit for bit.  DESIGN.md §5.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "frontier.h"
#include "philox.h"

namespace gossip {

struct SxItem {  // 16-byte exchange item
  uint64_t node;
  uint64_t value;
};

struct SxGeom {
  uint64_t N, Nl, lo, nown;  // global nodes, nodes per shard, first owned node, owned nodes
  uint32_t G, rank, k, R;
};

struct SxBufs {
  uint32_t* wcount;    // [nwl + 1] rare nodes per local bitmap word
  uint32_t* wpos;      // [nwl + 1] their exclusive prefix; [nwl] = list length
  SxItem* rare_send;   // [Nl] own rare nodes, id order (then padding up to the driver's stride)
  uint64_t* grb;       // [nwg] global rare bitmap
  uint32_t* gcnt;      // [nwg + 1] popcounts of grb words
  uint32_t* gpre;      // [nwg + 1] rare nodes before each word
  FrontierBufs gsum;   // summary view of grb (nzb = grb, maj 0)
  uint64_t* cbase;     // [G + 1] list position of shard g's first rare node
  SxItem* msg;         // [cap] push messages as the scan emits them: node = owner << 40 | node at owner
  SxItem* msg_out;     // [cap] grouped by owner, node = node at owner
  uint32_t* msg_cnt;   // [G + 2] per-owner counts, [G] = total, [G + 1] spare (G <= 1024)
  uint32_t* msg_fill;  // [G] grouping cursors
  uint64_t cap;        // k * nown: every owned node sends at most k pushes
  void* tmp;           // device-scan scratch
  size_t tmp_bytes;
};

size_t sx_bytes(const SxGeom& g);
void sx_carve(const SxGeom& g, void* base, SxBufs* b);

// 1. own rare nodes (maj 0: nonzero, maj 1: not full) -> b.rare_send; count at b.wpos[nwl]
hipError_t sx_compact(const SxGeom& g, const SxBufs& b, const FrontierBufs& lf, const uint64_t* S, uint32_t maj,
                      hipStream_t st);
// 3. global index from the gathered lists: recv[q * stride + i], i < counts of shard q
//    (b.cbase must hold the prefix of the counts)
//    rare = total rare nodes; small totals skip the O(N) per-word ranks and summary pass
//    mid: also the mid-level summary of the global bitmap (past 2^25 nodes, saturated rounds)
hipError_t sx_index(const SxGeom& g, const SxBufs& b, const SxItem* recv, uint64_t stride, uint64_t rare,
                    hipStream_t st, bool mid = false);
// 4. scan of the owned nodes; messages grouped by owner into b.msg_out, counts in b.msg_cnt
hipError_t sx_scan(const SxGeom& g, const SxBufs& b, const FrontierBufs& lf, const uint64_t* S, const SxItem* recv,
                   uint64_t stride, uint64_t rare, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode,
                   uint32_t maj, bool all_d, const Faults& fa, hipStream_t st, bool mid = false);
// 6. received pushes into D (and the push-dirty flags unless all_d)
hipError_t sx_apply(const FrontierBufs& lf, const SxItem* in, uint64_t n, bool all_d, hipStream_t st);

// Class-coded state exchange for dense rounds on the state image: a shard
// sends its two occupancy bitmaps (empty / full), the mixed nodes before each bitmap word,
// and the words of its mixed nodes only.  A shard's slot: [nz: nwl words][full: nwl words]
// [prefix: nwl uint32, padded to whole words], nwl = ceil(Nl / 64).
inline uint64_t cc_slot_words(uint64_t Nl) {
  const uint64_t nwl = (Nl + 63) / 64;
  return 2 * nwl + (nwl + 1) / 2;
}
// The own mixed words in id order -> out; the prefix at b.wpos, their count at b.wpos[nwl]
hipError_t cc_compact(const SxGeom& g, const SxBufs& b, const FrontierBufs& lf, const uint64_t* S, uint64_t* out,
                      hipStream_t st);
// slots = every shard's slot ([G][cc_slot_words]), vals = shard q's mixed words at q * stride:
// writes the other shards' slices of image
hipError_t cc_expand(const SxGeom& g, const uint64_t* slots, const uint64_t* vals, uint64_t stride,
                     uint64_t* image, uint32_t R, hipStream_t st);

}  // namespace gossip
