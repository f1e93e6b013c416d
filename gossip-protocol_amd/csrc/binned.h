// binned.h — propagation-blocked round pipeline (W == 1, one shard).
//
// Every random access of a round is moved into LDS: edges are binned by
// destination tile in a sender-tile pass, pull requests are served from an LDS
// copy of the peer tile, and pushes plus pull responses are OR-ed into an LDS
// copy of the receiving tile.  Global traffic is streaming or short runs.
// DESIGN.md §3.2 has the data layout and the byte accounting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox.h"
#include "round.h"

namespace gossip {

constexpr uint32_t kTileD = 16384;   // destination tile (nodes): one 128 KiB LDS image of u64 words
constexpr uint32_t kTileDLog = 14;
constexpr uint32_t kRecPerRegion = 16384;  // records staged per sender tile (LDS, 4 B each)
constexpr uint32_t kMaxSenders = 8192;     // senders per sender tile (their values staged once, 8 B each)
constexpr uint32_t kMaxTilesD = 4096;     // tiles with sender values staged in LDS (N <= 2^26); past it, up to
                                          // kSbMaxTiles (2^27 nodes), emit re-reads them from S

// Sharded dense rounds (sb_*): the pull pass stages no sender values, so its
// tile counters cover the whole image (N <= kSbMaxTiles * kTileD = 2^27).
constexpr uint32_t kSbMaxTiles = 8192;
// one-shard rounds take the big regions (make_bin_geom(big)) past this many destination tiles
// (2^24 nodes): the big emit costs more per sender, the walks gain more from longer runs
constexpr uint32_t kBigFromTiles = 1024;

// One emit pass of a sharded dense round: senders [snd0, snd0 + nsnd) (global
// ids), edges whose peer lies in [dst0, dst0 + dstn), directions in dmask
// (bit 0 push, bit 1 pull); wvals = 0: the records carry no sender value
// (the pull pass).
// Indices [lo, lo + n) with [skip0, skip1) spliced out: at(i) = lo + i, moved
// past the hole.  A launch over part of the regions or tiles.
struct IdxRange {
  uint32_t lo, n, skip0, skip1;
  __host__ __device__ uint32_t at(uint32_t i) const {
    const uint32_t x = lo + i;
    return x >= skip0 ? x + (skip1 - skip0) : x;
  }
  static IdxRange all(uint32_t n) { return IdxRange{0u, n, 0u, 0u}; }
};

struct EmitRange {
  uint64_t snd0, nsnd, dst0, dstn;
  uint32_t dmask, wvals;
  IdxRange rs;  // sender regions of this launch
};

struct BinGeom {
  uint64_t N;
  uint32_t k;
  uint32_t ts, ts_log;   // sender tile size (power of two <= kMaxSenders, ts * k <= kRecPerRegion)
  uint32_t rp;           // records per sender region = ts * k
  uint32_t nt_s, nt_d;   // sender tiles, destination tiles
  uint32_t apply_grid;   // host only: persistent apply blocks (0 = one per tile; gossip_set_param)
  uint32_t serve_grid;   // host only: persistent serve blocks of one-shard rounds (0 = one per tile)
  uint32_t push_waves;   // push-pull apply: waves [0, push_waves) walk the pushes, the rest the responses
  uint32_t aos;          // push records also packed {value, id} (BinBufs::prec; one shard, big regions)
  uint32_t split;        // one shard: record ids as two u16 arrays (BinBufs::dst / src) instead of ids
};

// big: regions of up to 2 * kMaxSenders senders and 2 * kRecPerRegion records (one shard
// past kMaxTilesD tiles: the emit's 16-bit packed tile counters, binned.hip V = 4)
BinGeom make_bin_geom(uint64_t N, uint32_t k, bool big = false);
bool bin_path_ok(uint64_t N, uint32_t k, uint32_t W, uint32_t G);

struct BinBufs {
  uint32_t* ids;    // [nt_s][rp]   p_local | n_local << 14 | flags (null with split)
  uint16_t* dst;    // split: [nt_s][rp] p_local | no-push << 14 | no-pull << 15 (serve, the push walk)
  uint16_t* src;    // split: [nt_s][rp] n_local | no-pull << 15 (the reply walk)
  uint64_t* vals;   // [nt_s][rp]   S_t[sender] (null with aos)
  uint32_t* prec;   // aos: [nt_s][rp][3] {S_t[sender] lo, hi, id}: a push in one 12-B piece
  uint64_t* resp;   // [nt_s][rp]   pull response S_t[p] & ~S_t[n]
  uint16_t* off;    // [nt_s][nt_d + 1] run starts inside each sender region
  uint16_t* offT;   // [nt_d + 1][nt_s]
  uint64_t* nzb;    // occupancy bitmaps of S_{t+1} written by K3 (frontier.h), or null
  uint64_t* fullb;
  // one shard: the persistent serve's / apply's tile queues, 8 counters each (one per XCD), zeroed
  // by the round's transpose kernel (binned.hip TileQueue); null: the static tile order
  uint32_t* dyn;
};

size_t bin_bytes(const BinGeom& g);
// [rows][cols] u16 table -> [cols][rows] (64 x 64 LDS tiles)
void bin_transpose_u16(const uint16_t* in, uint16_t* out, uint32_t rows, uint32_t cols, hipStream_t st);
void bin_carve(const BinGeom& g, void* base, BinBufs* b);

// One dense round, in place on S.  The totals in partial are cleared and
// recomputed (layout as stats_kernel's plus [4+R] = nonzero nodes); a
// one-block kernel hands them to the host through rs.  filt (needs exact
// nzb/fullb): bit 0 drops pulls from empty peers, bit 1 pushes into full
// peers — exact, it only removes edges that move nothing.  parts (placement trials): bit 0 emit +
// transpose, bit 1 serve, bit 2 apply; a round is all three.
constexpr uint32_t kBinAll = 7u;
hipError_t launch_binned_round(const BinGeom& g, const BinBufs& b, uint64_t* S, uint64_t* partial, uint32_t R,
                               uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode, uint32_t filt,
                               const Faults& fa, uint32_t flags, const RoundSync& rs, hipStream_t st,
                               uint32_t parts = kBinAll);

// Dense round of a sharded engine (G > 1) after the state all-gather
// (DESIGN.md §5): push pass P = every sender of the image, records for the
// own nodes' tiles; pull pass Q = the own senders, records for every tile of
// the image, served from LDS images of the gathered state; apply over the
// own tiles writes S_{t+1} of the own slice, its occupancy bitmaps and the
// own nodes' totals (global ids in the hash).
struct SbGeom {
  BinGeom p, q;
  uint64_t lo, nown;
};
struct SbBufs {
  BinBufs p, q;
};
bool sb_path_ok(uint64_t N, uint32_t k, uint64_t nown);
SbGeom make_sb_geom(uint64_t N, uint32_t k, uint64_t lo, uint64_t nown);
size_t sb_bytes(const SbGeom& g);
void sb_carve(const SbGeom& g, void* base, SbBufs* b);
// image: the gathered S_t (global ids); Snext: the own slice of S_{t+1};
// nzb/fullb: bitmaps over the own nodes; partial must be zero on entry.
// launch_sb_round = launch_sb_pre (reads only the own slice of the image: the
// pull pass, the push pass over the own senders, serving the own tiles — it may
// run while the all-gather fills the other slices) + launch_sb_post (the rest).
hipError_t launch_sb_pre(const SbGeom& g, const SbBufs& b, const uint64_t* image, uint32_t R, uint32_t t,
                         uint32_t key0, uint32_t key1, uint32_t mode, const Faults& fa, hipStream_t st);
hipError_t launch_sb_post(const SbGeom& g, const SbBufs& b, const uint64_t* image, uint64_t* Snext,
                          uint64_t* partial, uint32_t R, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode,
                          const Faults& fa, uint32_t flags, uint64_t* nzb, uint64_t* fullb, hipStream_t st);
hipError_t launch_sb_round(const SbGeom& g, const SbBufs& b, const uint64_t* image, uint64_t* Snext,
                           uint64_t* partial, uint32_t R, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode,
                           const Faults& fa, uint32_t flags, uint64_t* nzb, uint64_t* fullb, hipStream_t st);

// Exchange dense rounds of a sharded engine: no state image.
// Each shard emits one item per live edge of its own senders, grouped by the
// owner of the peer ({p at its owner | direction flags, S_t[n]}); the items go
// to their owners (all-to-all); each owner bins what it received by its own
// destination tile, answers the pulls from LDS images of S_t and returns the
// replies in the received order (all-to-all back); then every shard ORs the
// pushes it received and the replies to its own pulls into LDS images of its
// tiles.  Per-shard work is O(nodes per shard) at any G.
constexpr uint32_t kXdNoPush = 1u << 30;  // wire item id: p at the owner [0, 30) | these two flags
constexpr uint32_t kXdNoPull = 1u << 31;
// received items binned per LDS region (<= 16384; at <= 8192 their values are staged in LDS
// too: G = 8 probe 17.44 ms against 17.62 ms with 16384, profiles/r02_xd)
constexpr uint32_t kXdBinRegion = 8192;
struct XdGeom {
  uint64_t N, Nl, lo, nown;
  uint32_t G, rank, k;
  BinGeom s;  // own senders: ts, ts_log, rp (region records), nt_s regions; nt_d own tiles; N = nown
  BinGeom r;  // received items: rp = kXdBinRegion, nt_s regions of this round (xd_bin_regions), nt_d own tiles
};
struct XdBufs {
  uint32_t *rcnt, *roff;      // [s.nt_s][G] items per (sender region, owner) and their send positions
  uint32_t* rlofs;            // [s.nt_s][G + 1] each region's owner runs in its own order (prefix)
  uint32_t* ocnt;             // [G] items per owner
  uint32_t* sid;              // send items, owner-major [cap_s]
  uint64_t* sval;
  uint16_t* snl;              // the sender of each send item (index in its region), kept here
  uint64_t* rep_in;           // replies to the send items, in send order [cap_s]
  uint32_t* rid;              // received items [cap_r]
  uint64_t* rval;
  BinBufs rb;                 // received items binned by own tile (regions of kXdBinRegion)
  uint64_t* rep_out;          // replies to the received items, in received order [cap_r]
};
bool xd_path_ok(uint64_t N, uint32_t k, uint64_t Nl, uint32_t G);
XdGeom make_xd_geom(uint64_t N, uint32_t k, uint64_t Nl, uint64_t lo, uint64_t nown, uint32_t G, uint32_t rank);
uint64_t xd_send_cap(const XdGeom& g);
size_t xd_send_bytes(const XdGeom& g);  // rcnt .. rep_in
void xd_carve_send(const XdGeom& g, void* base, XdBufs* b);
size_t xd_recv_bytes(const XdGeom& g, uint64_t cap_r);  // rid .. rep_out
void xd_carve_recv(const XdGeom& g, uint64_t cap_r, void* base, XdBufs* b);
// Edge filter of an exchange round (filt = 0: none): cls = every shard's occupancy bitmaps
// of S_t, [nz: nwl u64][full: nwl u64] per shard (gossip_xd_classes, all-gathered).
struct XdFilter {
  const uint64_t* cls;
  uint32_t nwl, filt;  // filt bit 0: drop pull-only edges into empty peers, bit 1: push-only into full
  uint8_t* keep;       // [nown] the count pass's verdict per sender (bit j: edge j kept; k <= 8), read by emit
};
// own senders' items: counts per (region, owner), send positions, then the items
hipError_t launch_xd_requests(const XdGeom& g, const XdBufs& b, const uint64_t* S, uint32_t R, uint32_t t,
                              uint32_t key0, uint32_t key1, uint32_t mode, const Faults& fa, const XdFilter& xf,
                              hipStream_t st);
// n_in received items: bin by own tile, serve the pulls from S_t, replies in received order (b.rep_out)
hipError_t launch_xd_serve(XdGeom g, const XdBufs& b, const uint64_t* S, uint64_t n_in, uint32_t R,
                           hipStream_t st);
// S_{t+1} = S_t | pushes received | replies to the own pulls, stats of the own nodes (global ids in the hash)
hipError_t launch_xd_apply(XdGeom g, const XdBufs& b, const uint64_t* S, uint64_t* Snext, uint64_t n_in,
                           uint64_t* partial, uint32_t R, uint32_t mode, uint32_t flags, uint64_t* nzb,
                           uint64_t* fullb, hipStream_t st);

}  // namespace gossip
