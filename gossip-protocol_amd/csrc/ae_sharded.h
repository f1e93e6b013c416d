// ae_sharded.h — anti-entropy rounds with rows sharded over G engines (DESIGN.md §5.3,
// SURVEY.md §8(e) "Design B": request / reply buckets over all-to-all, max-merge on the owner).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gossip {

struct AexArgs {
  const uint32_t* V;        // own rows S_t [Nl][K] (node lo + i)
  uint32_t* Vn;             // own rows S_{t+1}
  // The all-gathered image, one word pair per 64 nodes (global ids; a shard's slot is its
  // Nl / 64 pairs, 64-aligned): [w][0] alive bits after round t's churn, [w][1] stale bits of
  // S_t (row != target).  The owner computes both for its nodes (churn at gossip_exchange_buffers,
  // stale bits of S_{t+1} in the stats pass), so one 16-B load answers both for any peer.
  uint64_t* img;
  bool write_stale;         // the stats pass writes the own stale words (not for gossip_state_hash)
  const uint32_t* target;   // global max vector [K]
  uint64_t* partial;        // [0] full [1] alive [2] messages [3] hash [4..4+K) per component
  uint64_t* cnt;            // [G + 1] items per owner (the last: own-own exchanges)
  uint32_t* bcnt;           // [blocks][G + 1] per-block counts (aex_block_table_words)
  uint64_t* boff;           // [blocks][G + 1] per-block offsets
  uint32_t* req;            // request items, grouped by owner: {p, n, row[K]} padded to rw words
  uint32_t* loc;            // own-own exchanges {n_local, p_local}
  uint64_t* dirty;          // [ceil(Nl / 64)] own rows of Vn raised above S_t this round (serve / merge);
                            // null: not tracked (a round with many items: the next one copies every row)
  uint8_t* verdict;         // [nown] per own node, from the count pass: bit j = exchange j listed (k <= 8)
  uint64_t N, Nl, lo, nown;
  uint32_t G, rank, K, L, k, t, key0, key1, fail, rec, flags, rw, pw;
};

// entries of the per-block tables (bcnt, boff) for nown own nodes and G shards
size_t aex_block_table_words(uint64_t nown, uint32_t G);

// Vn = S_t before round t: patch = Vn holds S_{t-1} and dirty marks the rows round t-1 raised
// (the only rows where S_t differs): those rows are copied from V; else a full copy.  Both
// leave dirty cleared for round t.
hipError_t launch_aex_seed_next(AexArgs a, uint64_t* dirty, bool patch, hipStream_t st);
// churn of round t of the own nodes, in place in the own slot's alive words (round t - 1 -> t)
hipError_t launch_aex_churn(const AexArgs& a, hipStream_t st);
// the own nodes' exchanges of round t (after the all-gather): messages counted, those with a
// stale end listed (count pass, scan, fill pass)
hipError_t launch_aex_requests(const AexArgs& a, hipStream_t st);
// requests received (m items): max-merge into Vn, responses V_t[p] in the received order
hipError_t launch_aex_serve(const AexArgs& a, const uint32_t* in, uint64_t m, uint32_t* resp, hipStream_t st);
// the responses to the own requests (in request order), the own-own exchanges, then the
// stats of S_{t+1} and its own stale bits: a full pass, or (inc, with a.dirty tracked and the
// own stale words of S_t in the image) over the raised rows only, partial[3] = the hash delta
hipError_t launch_aex_finish(const AexArgs& a, const uint32_t* resp, uint64_t nreq, uint64_t nloc, bool inc,
                             hipStream_t st);
// own stale bits of V against target (after set_target)
hipError_t launch_aex_stale(const AexArgs& a, const uint32_t* V, hipStream_t st);
// initial versions of the own rows (Philox tag 3 with global node ids)
hipError_t launch_aex_init(uint32_t* V, uint64_t lo, uint64_t nown, uint32_t K, uint32_t k0, uint32_t k1,
                           hipStream_t st);
// every own node alive (the own slot's alive words; nodes >= N not)
hipError_t launch_aex_fill_alive(const AexArgs& a, hipStream_t st);
// max over the own rows into out[K] (zeroed here)
hipError_t launch_aex_local_max(const uint32_t* V, uint64_t nown, uint32_t K, uint32_t* out, hipStream_t st);

}  // namespace gossip
