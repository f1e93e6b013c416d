// binned.hip — propagation-blocked push / pull / push-pull round for gfx950.
//
// Reference hot path: (*NodeState).Gossip, main.go:65-89 — each informed node
// sends its value to its peers (:72-81).  A synchronous round over N nodes is
// N*k random 8-byte reads (pull) and N*k random 8-byte OR-updates (push) —
// ~55 G/s and ~27 G/s on MI355X (profiles/r01_v0/microbench.jsonl) — so the
// round is restructured so that every random access lands in LDS:
//
//   K1 bin_emit   (one block per sender tile of ts nodes)
//        reads S_t[sender] (streaming), draws Philox peers, counting-sorts the
//        edge records {p_local | n_local<<14, S_t[n]} by destination tile in
//        LDS and writes them out as one contiguous region per sender tile.
//   K1b transpose the per-region run offsets so a destination tile finds its
//        runs with two contiguous row reads.
//   K2 bin_serve  (one block per destination tile, pull modes)
//        LDS image of S_t[tile]; for every record aimed at the tile writes the
//        pull response S_t[p] next to the record (nonzero ones only, flagged).
//   K3 bin_apply  (one block per destination tile)
//        LDS image acc = S_t[tile]; ORs in the pushes aimed at the tile and the
//        responses owed to the tile's own senders (ds_or_b64), writes
//        S_{t+1}[tile] and folds the convergence stats (ballot + 64x64 bit
//        transpose popcounts).
//
// OR is commutative and idempotent and every read is of S_t, so the record
// order inside a run (decided by LDS atomics) never changes a result bit.
#include <type_traits>

#include "binned.h"
#include "philox.h"
#include "round.h"
#include "wave.h"

namespace gossip {

namespace {

constexpr int kEmitThreads = 1024;
constexpr uint32_t kEmitGrid = 256;  // one persistent emit block per CU (128 / 64 slower: DESIGN.md §3.7)
constexpr int kTileThreads = 1024;
constexpr uint32_t kServeGrid = 256;  // persistent serve: one block per CU (the tile image takes 128 KiB of LDS)
constexpr uint32_t kApplyGrid = 256;  // persistent apply, likewise
constexpr int kUnrollSeq = 8;  // records in flight per lane in the sequential response walker
// push-pull apply: waves [0, push_waves) walk the pushes, the rest the responses
// (BinGeom::push_waves, this default up to 2^25 nodes)
constexpr uint32_t kPushWaves = 8;
// past 2^25 nodes the pushes come in short runs (~4 records at 2^27) and their walk
// sets the pace: 12 of the 16 waves (2^27 apply 2930 -> 2710 us, 10: 2745;
// profiles/r03_var27); 10 at 2^24 was slower (549 vs 542 us, round 2)
constexpr uint32_t kPushWavesBig = 12;
// push-pull apply: the block's waves split between the push walk (fragmented runs)
// and the response walk (sequential regions), which then run side by side
constexpr bool kApplySplit = true;
// Record buffers are written once and read once (or twice) per round: emit's record
// stores carry the non-temporal hint, so the streamed records do not displace the
// state image from the caches (bench: serve -28 us, apply -10 us per dense round).
// The same hint on the other record accesses was slower or equal.
template <typename T>
__device__ __forceinline__ void rec_st(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}
// A packed push {value lo, hi, id} moves as one 12-B access (global_load/store_dwordx3)
typedef uint32_t u32x3v __attribute__((ext_vector_type(3)));
__device__ __forceinline__ void prec_st(uint32_t* p, uint32_t a, uint32_t b, uint32_t c) {
  u32x3v v = {a, b, c};
  __builtin_memcpy(p, &v, 12);
}
__device__ __forceinline__ void prec_ld(const uint32_t* p, uint32_t& a, uint32_t& b, uint32_t& c) {
  u32x3v v;
  __builtin_memcpy(&v, p, 12);
  a = v.x;
  b = v.y;
  c = v.z;
}

// record id word: p_local [0,14) | n_local [14,28) | flags.  K1 rewrites every
// id each round, so a flag never outlives its round.
constexpr uint32_t kIdVZ = 1u << 28;  // no push on this record (sender empty, or the peer already full)
constexpr uint32_t kIdVF = 1u << 29;  // no pull (sender full, or the peer empty)
constexpr uint32_t kIdNMask = (1u << 14) - 1u;

// Split record ids (BinGeom::split, one shard): the id word becomes two u16 arrays, so serve
// and the push walk read 2 B (dst) instead of 4 and the reply walk 2 B (src): 12 B per node
// less per dense round.  dst = p_local | no-push << 14 | no-pull << 15; src = n_local |
// no-pull << 15.  The readers rebuild the u32 id fields they use.
constexpr uint16_t kDstVZ = 1u << 14, kDstVF = 1u << 15, kSrcVF = 1u << 15;
__device__ __forceinline__ uint16_t dst_of(uint32_t id) {
  return (uint16_t)((id & (kTileD - 1)) | ((id & kIdVZ) ? kDstVZ : 0u) | ((id & kIdVF) ? kDstVF : 0u));
}
__device__ __forceinline__ uint16_t src_of(uint32_t id) {
  return (uint16_t)(((id >> kTileDLog) & kIdNMask) | ((id & kIdVF) ? kSrcVF : 0u));
}
__device__ __forceinline__ uint32_t id_of_dst(uint32_t d) {
  return (d & (kTileD - 1)) | ((d & kDstVZ) ? kIdVZ : 0u) | ((d & kDstVF) ? kIdVF : 0u);
}
__device__ __forceinline__ uint32_t id_of_src(uint32_t s) {
  return ((s & kIdNMask) << kTileDLog) | ((s & kSrcVF) ? kIdVF : 0u);
}
__device__ __forceinline__ uint32_t id_of_pair(uint32_t d, uint32_t s) { return id_of_dst(d) | id_of_src(s); }

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  // blocks are dealt round-robin over the 8 XCDs: give each XCD a contiguous
  // range of tiles so neighbouring runs share its L2 (speed only)
  if (n & 7u) return b;
  return (b & 7u) * (n >> 3) + (b >> 3);
}

// Dynamic tile order of the persistent serve / apply (BinBufs::dyn, one shard, nv a multiple of 8):
// a block on XCD x (blockIdx.x % 8, as xcd_remap assumes) takes the next tile of x's contiguous
// range (xcd_remap's order) from x's counter, then steals from the other XCDs' ranges once x's is
// dry, so the kernel ends when the last tile does, not when the slowest block's static share does.
// Every tile is taken exactly once whichever XCD runs a block (speed only).
struct TileQueue {
  uint32_t* c;  // 8 counters, zeroed by the round's transpose kernel
  uint32_t nv;
  __device__ uint32_t claim() const {  // (one thread) the next tile, or nv
    const uint32_t per = nv >> 3, x0 = blockIdx.x & 7u;
    for (uint32_t h = 0; h < 8; ++h) {
      const uint32_t x = (x0 + h) & 7u;
      if (__atomic_load_n(&c[x], __ATOMIC_RELAXED) >= per) continue;  // dry: no atomic
      const uint32_t i = atomicAdd(&c[x], 1u);
      if (i < per) return x * per + i;
    }
    return nv;
  }
};

// Which directions an edge n -> p carries (bit 0 push, bit 1 pull; 0: no
// record).  From the sender alone: a push needs S_t[n] != 0, a pull is
// pointless once n holds every rumor.  filt bit 0 also drops pull-only edges
// whose peer is empty, bit 1 push-only edges whose peer is full (the peer's
// class from the occupancy bitmaps): exact, such an edge moves no bit.
__device__ __forceinline__ uint32_t sender_dirs(uint32_t mode, uint64_t v, uint64_t fm) {
  const uint32_t push = (mode == 1 || mode == 3) && v != 0;
  const uint32_t pull = (mode == 2 || mode == 3) && v != fm;
  return push | (pull << 1);
}

__device__ __forceinline__ uint32_t peer_filter(uint32_t d, uint32_t p, uint32_t filt, const uint64_t* nzb,
                                                const uint64_t* fullb) {
  // only one-way edges are probed: a two-way record stays anyway
  if ((filt & 1u) && d == 2u && !((nzb[p >> 6] >> (p & 63u)) & 1ull)) d = 0u;
  if ((filt & 2u) && d == 1u && ((fullb[p >> 6] >> (p & 63u)) & 1ull)) d = 0u;
  return d;
}

// record flags: kIdVZ = no push on this record, kIdVF = no pull
__device__ __forceinline__ uint32_t dir_flags(uint32_t d) { return ((d & 1u) ? 0u : kIdVZ) | ((d & 2u) ? 0u : kIdVF); }

// Region counting sort, middle step: cur[0, nt) holds the records per
// destination tile; writes each run's start to off_row[0, nt] (u16, the total
// last), turns cur into the fill pointers and returns the total.  Every thread
// of the (kEmitThreads) block calls it; it ends with a barrier.
__device__ __forceinline__ uint32_t region_offsets(uint32_t* cur, uint32_t nt, uint16_t* off_row, uint32_t* wsum,
                                                   uint32_t* wpre) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t per = (nt + kEmitThreads - 1) / kEmitThreads;
  const uint32_t lo = min(tid * per, nt), hi = min(lo + per, nt);
  uint32_t mine = 0;
  for (uint32_t d = lo; d < hi; ++d) mine += cur[d];
  uint32_t inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  if (tid == 0) {
    uint32_t a = 0;
    for (int w = 0; w < kEmitThreads / 64; ++w) {
      wpre[w] = a;
      a += wsum[w];
    }
    wpre[kEmitThreads / 64] = a;
  }
  __syncthreads();
  uint32_t run = wpre[wave] + inc - mine;
  for (uint32_t d = lo; d < hi; ++d) {
    const uint32_t c = cur[d];
    cur[d] = run;
    off_row[d] = (uint16_t)run;
    run += c;
  }
  const uint32_t total = wpre[kEmitThreads / 64];
  if (tid == 0) off_row[nt] = (uint16_t)total;
  __syncthreads();
  return total;
}

// region_offsets over 16-bit counters packed two per word (tile d in half d & 1 of
// cur[d >> 1]; regions of <= 32768 records, so no half overflows)
__device__ __forceinline__ uint32_t region_offsets_packed(uint32_t* cur, uint32_t nt, uint16_t* off_row,
                                                          uint32_t* wsum, uint32_t* wpre) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t nw = (nt + 1) >> 1;  // this thread: whole words [lo, hi)
  const uint32_t per = (nw + kEmitThreads - 1) / kEmitThreads;
  const uint32_t lo = min(tid * per, nw), hi = min(lo + per, nw);
  uint32_t mine = 0;
  for (uint32_t w = lo; w < hi; ++w) mine += (cur[w] & 0xFFFFu) + (cur[w] >> 16);
  uint32_t inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  if (tid == 0) {
    uint32_t a = 0;
    for (int w = 0; w < kEmitThreads / 64; ++w) {
      wpre[w] = a;
      a += wsum[w];
    }
    wpre[kEmitThreads / 64] = a;
  }
  __syncthreads();
  uint32_t run = wpre[wave] + inc - mine;
  for (uint32_t w = lo; w < hi; ++w) {
    const uint32_t c0 = cur[w] & 0xFFFFu, c1 = cur[w] >> 16;
    const uint32_t r0 = run, r1 = run + c0;
    cur[w] = r0 | (r1 << 16);
    off_row[2 * w] = (uint16_t)r0;
    if (2 * w + 1 < nt) off_row[2 * w + 1] = (uint16_t)r1;
    run = r1 + c1;
  }
  const uint32_t total = wpre[kEmitThreads / 64];
  if (tid == 0) off_row[nt] = (uint16_t)total;
  __syncthreads();
  return total;
}

// KREG > 0: the k (<= KREG) peers of each sender stay in registers between passes.
// FAULTS: edge loss / partitions active; off, none of that code exists.
// V = 0: one shard.  V = 1, 2: one pass of a sharded dense round (EmitRange):
// senders [snd0, snd0 + nsnd) of the gathered image S (global ids), only edges
// whose peer lies in [dst0, dst0 + dstn), only the directions in dmask, tiles
// counted from dst0.  V = 2 (pull pass) stores no sender values, so its tile
// counters can cover kSbMaxTiles tiles of the whole image.  V = 3: one shard
// past 4096 tiles (N > 2^26): the sender values are not staged in LDS (the
// tile counters take that room) but re-read from S — the region's slice, which
// this block has just streamed, so the reads hit L2.  V = 4: as V = 3 with regions
// twice as large (up to 16384 senders, 32768 records; 16-bit tile counters packed in
// pairs make the room), so the runs stay twice as long at N > 2^26; no next-region
// prefetch (its registers).  V = 6, 7: the big regions of V = 4 for the sharded passes of
// V = 1 (push, values written beside the u32 ids) and V = 2 (pull, no values); V = 8, 9: the
// same with V = 5's peers kept between the passes (no faults, k <= 2).
template <int KREG, bool FAULTS, int V>
__global__ __launch_bounds__(kEmitThreads) void bin_emit_kernel(BinGeom g, const uint64_t* __restrict__ S, BinBufs b,
                                                                  uint32_t R, uint32_t t, uint32_t key0,
                                                                  uint32_t key1, uint32_t mode, uint32_t filt,
                                                                  Faults fa, EmitRange er) {
  constexpr bool SHARD = V == 1 || V == 2 || V >= 6;
  constexpr bool STAGE = V == 0 || V == 1;  // sender values staged in LDS
  constexpr bool BIG = V >= 4;               // packed 16-bit tile counters, double regions
  // V = 5: BIG without faults, k <= 2 (the launch checks): the count pass keeps each sender's
  // peers and edge directions in the LDS staging room ({p0, p1, dirs} in a u64: p < 2^27), so
  // the placement pass draws no Philox again (one cipher per sender instead of two)
  constexpr bool PKC = V == 5 || V == 8 || V == 9;
  constexpr bool NOVALS = V == 7 || V == 9;  // the sharded pull pass writes no sender values
  constexpr uint32_t kMaxT = V >= 2 ? kSbMaxTiles : kMaxTilesD;
  constexpr uint32_t kMaxS = BIG ? 2 * kMaxSenders : kMaxSenders;
  __shared__ uint32_t cur[BIG ? kMaxT / 2 : kMaxT];
  __shared__ __align__(16) uint32_t st_ids[BIG ? 2 * kRecPerRegion : kRecPerRegion];  // p_local | n_local << 14, by tile (BIG: then the u64 sender values)
  __shared__ uint64_t sval[STAGE ? kMaxS : 1];  // S_t of each sender, once (not once per record)
  __shared__ uint32_t wsum[kEmitThreads / 64];
  __shared__ uint32_t wpre[kEmitThreads / 64 + 1];

  const uint32_t tid = threadIdx.x;
  const uint64_t nm1 = g.N - 1, fm = full_mask1(R);
  constexpr uint32_t kQ = kMaxS / kEmitThreads;  // senders per thread upper bound
  const uint64_t snd0 = SHARD ? er.snd0 : 0ull, nsnd = SHARD ? er.nsnd : g.N;
  const uint32_t dmask = SHARD ? er.dmask : 3u;
  // destination tile of peer p, false when p lies outside the pass's range
  auto tile_of = [&](uint32_t p, uint32_t* tl, uint32_t* pl) -> bool {
    const uint32_t rel = SHARD ? p - (uint32_t)er.dst0 : p;
    *tl = rel >> kTileDLog;
    *pl = rel & (kTileD - 1);
    return !SHARD || rel < (uint32_t)er.dstn;
  };

  // persistent over sender regions s = blockIdx.x, +gridDim.x, ...: the next
  // region's sender values are loaded while this one is sorted and written
  auto load_values = [&](uint32_t s, uint64_t* v) {
    const uint64_t base = (uint64_t)s << g.ts_log;
    const uint32_t nsend = (uint32_t)min<uint64_t>(g.ts, nsnd - base);
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
      // clamp, never branch around a load: a guarded load is waited on alone
      const uint64_t x = S[snd0 + base + min(i, nsend - 1)];
      v[q] = i < nsend ? x : 0ull;
    }
  };
  uint64_t v[kQ], vn[kQ];
  // regions r = blockIdx.x, +gridDim.x, ... of the launch; V != 0 launches may
  // cover a subrange of the regions (er.rs: the part of a dense sharded round
  // that overlaps the all-gather, or the rest)
  const uint32_t nr = SHARD ? er.rs.n : g.nt_s;
  auto region = [&](uint32_t r) -> uint32_t { return SHARD ? er.rs.at(r) : r; };
  auto count_tile = [&](uint32_t tl) {
    if constexpr (BIG) atomicAdd(&cur[tl >> 1], 1u << ((tl & 1u) << 4));
    else atomicAdd(&cur[tl], 1u);
  };
  auto place_tile = [&](uint32_t tl) -> uint32_t {
    if constexpr (BIG) {
      const uint32_t sh = (tl & 1u) << 4;
      return (atomicAdd(&cur[tl >> 1], 1u << sh) >> sh) & 0xFFFFu;
    } else {
      return atomicAdd(&cur[tl], 1u);
    }
  };
  if (!BIG && blockIdx.x < nr) load_values(region(blockIdx.x), v);
  // one shard, big regions, b.dyn: regions from one queue (b.dyn[16], zeroed by the round's transpose
  // for the next round), so the launch ends with its last region, not its slowest block's share
  const bool dynq = BIG && !SHARD && b.dyn != nullptr;
  __shared__ uint32_t s_claim;
  for (uint32_t r = blockIdx.x;;) {
  __syncthreads();  // the previous region's write-out has read cur/st_ids/sval (and s_claim is read)
  if (dynq) {
    if (tid == 0) s_claim = atomicAdd(&b.dyn[16], 1u);
    __syncthreads();
    r = s_claim;
  }
  if (r >= nr) break;
  const uint32_t s = region(r);
  const uint64_t base = (uint64_t)s << g.ts_log;
  const uint32_t nsend = (uint32_t)min<uint64_t>(g.ts, nsnd - base);

  for (uint32_t d = tid; d < (BIG ? (g.nt_d + 1) >> 1 : g.nt_d); d += kEmitThreads) cur[d] = 0;
  if (BIG) load_values(s, v);
#pragma unroll
  for (uint32_t q = 0; q < kQ; ++q) {
    const uint32_t i = tid + q * kEmitThreads;
    if (STAGE && i < g.ts) sval[i] = v[q];
  }
  if (!BIG && r + gridDim.x < nr) load_values(region(r + gridDim.x), vn);
  __syncthreads();
  // pass A: per-destination-tile counts of the records (edges that carry something)
  uint32_t pr[KREG > 0 ? kQ * KREG : 1];
  uint32_t ed[KREG > 0 ? kQ : 1];  // 2 bits per edge j: directions (sender_dirs, then peer_filter)
  if (KREG > 0) {
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
      ed[q] = 0;
#pragma unroll
      for (int j = 0; j < KREG; ++j) pr[q * KREG + j] = 0;
      const uint32_t d = i < nsend ? sender_dirs(mode, v[q], fm) & dmask : 0u;
      if (!d) continue;
      const uint32_t n = (uint32_t)(snd0 + base + i);
      const u32x4 x = philox4x32_10(u32x4{n, t, 0u, 0u}, key0, key1);
      const u32x4 lw = FAULTS && fa.loss ? loss_draws(n, t, 0u, key0, key1) : u32x4{0, 0, 0, 0};
      const Reach rc = FAULTS ? reach_of(n, fa) : Reach{0u, 0xFFFFFFFFu};  // n's partition block
#pragma unroll
      for (int j = 0; j < KREG; ++j) {
        pr[q * KREG + j] = peer_from_word(lane_of(x, j), nm1, n);
        const bool lost = FAULTS && edge_lost(fa, rc, pr[q * KREG + j], lane_of(lw, j));
        uint32_t tl, pl;
        const bool in = tile_of(pr[q * KREG + j], &tl, &pl);
        if ((uint32_t)j < g.k && !lost && in) ed[q] |= d << (2 * j);
      }
    }
    if (filt) {  // every probe issued before any is used (32-bit words: half the registers)
      const uint32_t* nz32 = (const uint32_t*)b.nzb;
      const uint32_t* full32 = (const uint32_t*)b.fullb;
      uint32_t wz[KREG > 0 ? kQ * KREG : 1];
#pragma unroll
      for (uint32_t q = 0; q < kQ; ++q)
#pragma unroll
        for (int j = 0; j < KREG; ++j) {
          const uint32_t p = pr[q * KREG + j];
          // only edges that carry nothing else are probed: a two-way record stays anyway
          wz[q * KREG + j] = ((filt & 1u) && ((ed[q] >> (2 * j)) & 3u) == 2u) ? nz32[p >> 5] : ~0u;
        }
#pragma unroll
      for (uint32_t q = 0; q < kQ; ++q)
#pragma unroll
        for (int j = 0; j < KREG; ++j)
          if (!((wz[q * KREG + j] >> (pr[q * KREG + j] & 31u)) & 1u)) ed[q] &= ~(2u << (2 * j));
#pragma unroll
      for (uint32_t q = 0; q < kQ; ++q)
#pragma unroll
        for (int j = 0; j < KREG; ++j) {
          const uint32_t p = pr[q * KREG + j];
          wz[q * KREG + j] = ((filt & 2u) && ((ed[q] >> (2 * j)) & 3u) == 1u) ? full32[p >> 5] : 0u;
        }
#pragma unroll
      for (uint32_t q = 0; q < kQ; ++q)
#pragma unroll
        for (int j = 0; j < KREG; ++j)
          if ((wz[q * KREG + j] >> (pr[q * KREG + j] & 31u)) & 1u) ed[q] &= ~(1u << (2 * j));
    }
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q)
#pragma unroll
      for (int j = 0; j < KREG; ++j)
        if ((ed[q] >> (2 * j)) & 3u) {
          uint32_t tl, pl;
          tile_of(pr[q * KREG + j], &tl, &pl);
          count_tile(tl);
        }
  } else if (PKC) {
    uint64_t* pkl = (uint64_t*)st_ids;  // kMaxS u64 = the staging room, free until placement
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
      uint64_t pk = 0;
      const uint32_t d = i < nsend ? sender_dirs(mode, v[q], fm) & dmask : 0u;
      if (d) {
        const uint32_t n = (uint32_t)(snd0 + base + i);
        const u32x4 x = philox4x32_10(u32x4{n, t, 0u, 0u}, key0, key1);
#pragma unroll
        for (uint32_t j = 0; j < 2; ++j) {
          if (j >= g.k) break;
          const uint32_t p = peer_from_word(lane_of(x, j), nm1, n);
          uint32_t tl, pl;
          const bool in = tile_of(p, &tl, &pl);  // (one shard: always inside)
          const uint32_t dd = in ? peer_filter(d, p, filt, b.nzb, b.fullb) : 0u;
          if (!dd) continue;
          count_tile(tl);
          pk |= ((uint64_t)p << (27 * j)) | ((uint64_t)dd << (54 + 2 * j));
        }
      }
      pkl[i] = pk;
    }
  } else {
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
      if (i >= nsend) break;
      const uint32_t d = sender_dirs(mode, v[q], fm) & dmask;
      if (!d) continue;
      const uint32_t n = (uint32_t)(snd0 + base + i);
      u32x4 x{0, 0, 0, 0}, lw{0, 0, 0, 0};
      const Reach rc = FAULTS ? reach_of(n, fa) : Reach{0u, 0xFFFFFFFFu};  // n's partition block (§2.8)
      for (uint32_t j = 0; j < g.k; ++j) {
        if ((j & 3u) == 0) {
          x = philox4x32_10(u32x4{n, t, 0u, j >> 2}, key0, key1);
          if (FAULTS && fa.loss) lw = loss_draws(n, t, j >> 2, key0, key1);
        }
        const uint32_t p = peer_from_word(lane_of(x, j & 3u), nm1, n);
        if (FAULTS && edge_lost(fa, rc, p, lane_of(lw, j & 3u))) continue;
        uint32_t tl, pl;
        if (!tile_of(p, &tl, &pl)) continue;
        if (peer_filter(d, p, filt, b.nzb, b.fullb)) count_tile(tl);
      }
    }
  }
  __syncthreads();

  uint16_t* off_row = b.off + (size_t)s * (g.nt_d + 1);
  const uint32_t total = BIG ? region_offsets_packed(cur, g.nt_d, off_row, wsum, wpre)
                             : region_offsets(cur, g.nt_d, off_row, wsum, wpre);

  // pass B: each record to its slot (k <= KREG: the peers and directions from
  // registers; else the same draws and probes again)
  if (KREG > 0) {
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
#pragma unroll
      for (int j = 0; j < KREG; ++j) {
        const uint32_t d = (ed[q] >> (2 * j)) & 3u;
        if (!d) continue;
        uint32_t tl, pl;
        tile_of(pr[q * KREG + j], &tl, &pl);
        const uint32_t pos = place_tile(tl);
        st_ids[pos] = pl | (i << kTileDLog) | dir_flags(d);
      }
    }
  } else if (PKC) {
    uint64_t mine[kQ];
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) mine[q] = ((const uint64_t*)st_ids)[tid + q * kEmitThreads];
    __syncthreads();  // every sender's peers are read before any record takes the room
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
#pragma unroll
      for (uint32_t j = 0; j < 2; ++j) {
        const uint32_t dd = (uint32_t)(mine[q] >> (54 + 2 * j)) & 3u;
        if (!dd) continue;
        const uint32_t p = (uint32_t)(mine[q] >> (27 * j)) & ((1u << 27) - 1u);
        uint32_t tl, pl;
        tile_of(p, &tl, &pl);
        const uint32_t pos = place_tile(tl);
        st_ids[pos] = pl | (i << kTileDLog) | dir_flags(dd);
      }
    }
  } else {
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
      if (i >= nsend) break;
      const uint32_t d0 = sender_dirs(mode, v[q], fm) & dmask;
      if (!d0) continue;
      const uint32_t n = (uint32_t)(snd0 + base + i);
      u32x4 x{0, 0, 0, 0}, lw{0, 0, 0, 0};
      const Reach rc = FAULTS ? reach_of(n, fa) : Reach{0u, 0xFFFFFFFFu};  // n's partition block (§2.8)
      for (uint32_t j = 0; j < g.k; ++j) {
        if ((j & 3u) == 0) {
          x = philox4x32_10(u32x4{n, t, 0u, j >> 2}, key0, key1);
          if (FAULTS && fa.loss) lw = loss_draws(n, t, j >> 2, key0, key1);
        }
        const uint32_t p = peer_from_word(lane_of(x, j & 3u), nm1, n);
        if (FAULTS && edge_lost(fa, rc, p, lane_of(lw, j & 3u))) continue;
        uint32_t tl, pl;
        if (!tile_of(p, &tl, &pl)) continue;
        const uint32_t d = peer_filter(d0, p, filt, b.nzb, b.fullb);
        if (!d) continue;
        const uint32_t pos = place_tile(tl);
        st_ids[pos] = pl | (i << kTileDLog) | dir_flags(d);
      }
    }
  }
  __syncthreads();

  uint32_t* gids = b.ids + (size_t)s * g.rp;
  uint64_t* gvals = b.vals + (size_t)s * g.rp;
  uint16_t* gdst = b.dst + (size_t)s * g.rp;
  uint16_t* gsrc = b.src + (size_t)s * g.rp;
  // the one-shard emits (BinGeom::split); V = 1, 2, 6, 7: sharded passes (u32 ids)
  constexpr bool split = !SHARD;
  if constexpr (BIG) {
    // ids out first, then the region's sender values take the staging room and each
    // push is written packed {value, id} (BinGeom::aos), its value read from LDS: the
    // values are the ones in v[] (no second read of S), and no record gathers its
    // sender's word from L2 / MALL (a 64-B fetch per 8-B value at 2^27 nodes: emit 158 B
    // of fetch per node, profiles/r03_a/pmc_dense_2p27.json).  The ids are read back from
    // the region just written (plain stores: L2-resident; a register copy of 32 ids per
    // lane spilled 39 VGPRs).
    for (uint32_t e = tid; e < total; e += kEmitThreads) {
      const uint32_t id = st_ids[e];
      if (split) {
        gdst[e] = dst_of(id);
        gsrc[e] = src_of(id);
      } else {
        gids[e] = id;
      }
    }
    if constexpr (!NOVALS) {
      __syncthreads();  // every staged id is out
      uint64_t* sv = (uint64_t*)st_ids;  // 2 * kRecPerRegion u32 = kMaxS u64
      // (V = 5 keeps v[] live through the count pass rather than rereading S here: 5.86 vs
      // 5.98 ms per 2^27 dense round, profiles/r04_e/summary.txt)
#pragma unroll
      for (uint32_t q = 0; q < kQ; ++q) sv[tid + q * kEmitThreads] = v[q];
      __syncthreads();
      if constexpr (SHARD) {  // V = 6, 8: every value slot beside its u32 id (no holes)
#pragma unroll 4
        for (uint32_t e = tid; e < total; e += kEmitThreads)
          rec_st(&gvals[e], sv[(gids[e] >> kTileDLog) & kIdNMask]);
      } else {
        uint32_t* gprec = b.prec + (size_t)s * g.rp * 3;
#pragma unroll 4
        for (uint32_t e = tid; e < total; e += kEmitThreads) {
          const uint32_t id = split ? id_of_pair(gdst[e], gsrc[e]) : gids[e];
          const uint64_t x = sv[(id >> kTileDLog) & kIdNMask];  // (one-shard big regions always pack: g.aos)
          prec_st(&gprec[3 * e], (uint32_t)x, (uint32_t)(x >> 32), id);
        }
      }
    }
  } else
  for (uint32_t e = tid; e < total; e += kEmitThreads) {
    const uint32_t id = st_ids[e];
    // every value slot is stored (also where the flags say no push), so the
    // region is written without holes (a partly written 64-B chunk costs HBM
    // a read-modify-write: profiles/r01_experiments/microbench5_scattered_pieces.jsonl)
    if (split) {
      rec_st(&gdst[e], dst_of(id));
      rec_st(&gsrc[e], src_of(id));
    } else {
      rec_st(&gids[e], id);
    }
    if (STAGE) {
      rec_st(&gvals[e], sval[(id >> kTileDLog) & kIdNMask]);
    }
    if (V >= 3) rec_st(&gvals[e], S[base + ((id >> kTileDLog) & kIdNMask)]);
  }
  if constexpr (!BIG) {
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) v[q] = vn[q];
  }
  if (!dynq) r += gridDim.x;
  }
}

// Run offsets [rows][cols] -> [cols][rows] in 64x64 tiles: a (64, 4) block, 16 loads in flight per
// thread before any store (the 32x32 version with 4 per thread was latency-bound: 149 us for
// the 134 MB table at 2^27 nodes, 1.8 TB/s), u32 LDS slots so the transposed reads are
// conflict-free.
constexpr uint32_t kTrT = 64, kTrRows = 4;
__global__ __launch_bounds__(kTrT * kTrRows) void transpose_u16_kernel(const uint16_t* __restrict__ in,
                                                                       uint16_t* __restrict__ out, uint32_t rows,
                                                                       uint32_t cols, uint64_t* __restrict__ partial,
                                                                       uint32_t plen, uint32_t* __restrict__ dyn) {
  // the dense round's stats are absolute: clear the totals before K3 adds to them; and the
  // serve / apply tile queues (16 counters)
  if (blockIdx.x == 0 && blockIdx.y == 0) {
    for (uint32_t i = threadIdx.y * kTrT + threadIdx.x; i < plen; i += kTrT * kTrRows) partial[i] = 0;
    if (dyn && threadIdx.y == 0 && threadIdx.x < 17) dyn[threadIdx.x] = 0;  // (dyn[16]: the next emit's)
  }
  __shared__ uint32_t tile[kTrT][kTrT + 1];
  constexpr uint32_t kPer = kTrT / kTrRows;
  const uint32_t c0 = blockIdx.x * kTrT, r0 = blockIdx.y * kTrT, tx = threadIdx.x, ty = threadIdx.y;
  uint16_t v[kPer];
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint32_t r = r0 + ty + i * kTrRows, c = c0 + tx;
    v[i] = (r < rows && c < cols) ? in[(size_t)r * cols + c] : (uint16_t)0;
  }
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) tile[ty + i * kTrRows][tx] = v[i];
  __syncthreads();
#pragma unroll
  for (uint32_t i = 0; i < kPer; ++i) {
    const uint32_t c = c0 + ty + i * kTrRows, r = r0 + tx;
    if (r < rows && c < cols) out[(size_t)c * rows + r] = (uint16_t)tile[tx][ty + i * kTrRows];
  }
}

// launch of transpose_u16_kernel over a [rows][cols] table
void launch_transpose_u16(const uint16_t* in, uint16_t* out, uint32_t rows, uint32_t cols, uint64_t* partial,
                          uint32_t plen, hipStream_t st, uint32_t* dyn = nullptr) {
  const dim3 tg((cols + kTrT - 1) / kTrT, (rows + kTrT - 1) / kTrT);
  transpose_u16_kernel<<<tg, dim3(kTrT, kTrRows), 0, st>>>(in, out, rows, cols, partial, plen, dyn);
}


// Writes the finished tile (LDS) to S_{t+1} and folds the round stats
// (definitions as in stats_kernel): fully-informed count by ballot, per-rumor
// counts as column popcounts of each wave's 64x64 bit matrix, optional hash.
// hid0: global id of node 0 (sharded rounds hash global ids)
__device__ __forceinline__ void tile_epilogue(const unsigned long long* acc, uint64_t node0, uint64_t N, uint64_t hid0,
                                              uint64_t* __restrict__ Snext, uint64_t* __restrict__ partial,
                                              uint32_t R, uint32_t flags, uint32_t* cnt, uint64_t* red_hash,
                                              uint32_t* red_full, uint32_t* red_nz, uint64_t* __restrict__ nzb,
                                              uint64_t* __restrict__ fullb, uint64_t* btot) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t fm = full_mask1(R);
  const bool do_hash = (flags & 1u) != 0;
  uint64_t hash = 0;
  uint32_t full = 0, nzc = 0, c_lane = 0;
  // Per-rumor counts: the lane's 16 words are summed bit-sliced (a carry-save
  // adder tree: planes of weight 1, 2, 4, 8, 16 per rumor bit), then each
  // plane's 64x64 matrix is transposed once per wave — five transposes for
  // 1024 nodes instead of sixteen.
  constexpr uint32_t kQ = kTileD / kTileThreads;
  static_assert(kQ == 16, "tile_epilogue: the adder tree sums 16 words per lane");
  uint64_t plane[5];
  {
    uint64_t ones = 0, twos = 0, fours = 0, eights = 0, sixteens = 0;
    auto csa = [](uint64_t& h, uint64_t& l, uint64_t a, uint64_t b, uint64_t c) {
      const uint64_t u = a ^ b;
      h = (a & b) | (u & c);
      l = u ^ c;
    };
    uint64_t xs[2], twosA, twosB, foursA, foursB, eightsA, eightsB;
    uint64_t hash_key = (hid0 + node0 + tid) * kGold64;
    auto word = [&](uint32_t q) -> uint64_t {
      const uint32_t i = q * kTileThreads + tid;
      const uint64_t n = node0 + i;
      const bool valid = n < N;
      const uint64_t x = valid ? (uint64_t)acc[i] : 0ull;
      if (valid) Snext[n] = x;
      if (do_hash && x) hash += mix64(x + hash_key);
      hash_key += (uint64_t)kTileThreads * kGold64;
      const uint64_t fw = __ballot(valid && x == fm);
      const uint64_t nz = __ballot(x != 0);
      full += (uint32_t)__popcll(fw);
      nzc += (uint32_t)__popcll(nz);
      // a wave holds 64 consecutive nodes: one word of each occupancy bitmap
      if (nzb && lane == 0 && (n - lane) < N) {
        nzb[n >> 6] = nz;
        fullb[n >> 6] = fw;
      }
      return x;
    };
#pragma unroll
    for (uint32_t h8 = 0; h8 < 2; ++h8) {
#pragma unroll
      for (uint32_t h4 = 0; h4 < 2; ++h4) {
        xs[0] = word(h8 * 8 + h4 * 4 + 0);
        xs[1] = word(h8 * 8 + h4 * 4 + 1);
        csa(twosA, ones, ones, xs[0], xs[1]);
        xs[0] = word(h8 * 8 + h4 * 4 + 2);
        xs[1] = word(h8 * 8 + h4 * 4 + 3);
        csa(twosB, ones, ones, xs[0], xs[1]);
        if (h4 == 0) csa(foursA, twos, twos, twosA, twosB);
        else csa(foursB, twos, twos, twosA, twosB);
      }
      if (h8 == 0) csa(eightsA, fours, fours, foursA, foursB);
      else csa(eightsB, fours, fours, foursA, foursB);
    }
    csa(sixteens, eights, eights, eightsA, eightsB);
    plane[0] = ones;
    plane[1] = twos;
    plane[2] = fours;
    plane[3] = eights;
    plane[4] = sixteens;
  }
#pragma unroll
  for (uint32_t p = 0; p < 5; ++p) {
    if (__ballot(plane[p] != 0) == 0) continue;
    if (__ballot(plane[p] != fm) == 0) {  // every lane has every rumor at this weight
      c_lane += 64u << p;
      continue;
    }
    c_lane += (uint32_t)__popcll(transpose64(plane[p], lane)) << p;
  }
  if (lane < R && c_lane) atomicAdd(&cnt[lane], c_lane);  // bits >= R are never set
  hash = wave_sum64(hash);
  if (lane == 0) {
    red_hash[wave] = hash;
    red_full[wave] = full;
    red_nz[wave] = nzc;
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t h = 0, f = 0, z = 0;
    for (int w = 0; w < kTileThreads / 64; ++w) {
      h += red_hash[w];
      f += red_full[w];
      z += red_nz[w];
    }
    if (btot) {  // a persistent block: its tiles' totals stay in LDS until block_totals_flush
      btot[0] += f;
      btot[1] += h;
      btot[2] += z;
    } else {
      if (f) atomicAdd((unsigned long long*)&partial[0], (unsigned long long)f);
      if (h) atomicAdd((unsigned long long*)&partial[3], (unsigned long long)h);
      if (z) atomicAdd((unsigned long long*)&partial[4 + R], (unsigned long long)z);  // nonzero nodes
    }
  }
  if (!btot && tid < R && cnt[tid]) atomicAdd((unsigned long long*)&partial[4 + tid], (unsigned long long)cnt[tid]);
}

// A persistent apply block's totals (tile_epilogue with btot), once, after its last tile: ~67
// same-address atomics per block instead of per tile (8192 tiles at 2^27).  All-dense rounds
// 510 -> 502 us at 2^24, equal at 2^27 (profiles/r05_bt/).
__device__ __forceinline__ void block_totals_flush(uint64_t* __restrict__ partial, uint32_t R, const uint32_t* cnt,
                                                   const uint64_t* btot) {
  const uint32_t tid = threadIdx.x;
  __syncthreads();
  if (tid == 0) {
    if (btot[0]) atomicAdd((unsigned long long*)&partial[0], (unsigned long long)btot[0]);
    if (btot[1]) atomicAdd((unsigned long long*)&partial[3], (unsigned long long)btot[1]);
    if (btot[2]) atomicAdd((unsigned long long*)&partial[4 + R], (unsigned long long)btot[2]);
  }
  if (tid < R && cnt[tid]) atomicAdd((unsigned long long*)&partial[4 + tid], (unsigned long long)cnt[tid]);
}

// Orders this wave's LDS accesses (a wave's LDS operations complete in order;
// the fences keep the compiler from moving them across).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Visits every record of the runs (s, T) for s in [0, nt_s): a wave takes 64 * RPL
// consecutive runs at a time (RPL consecutive runs per lane) and scans their lengths; the
// concatenated records are then walked in windows of 64*U, lane-strided (so
// each load instruction reads consecutive records of a run).  The owner of a
// record comes from a per-wave LDS bitmap of run starts in the window and a
// list of the window's runs: rank = (run starts at or before it) - 1, one
// popcount and one LDS read per record, no search.  load(rec) receives the
// global record index s * rp + pos, or -1 past the end.
// LDS per wave: wmask[U] u64, wlist[64 * RPL] i32.  The walk is shared by the waves
// [w0, w0 + nwaves) of the block (nwaves = 0: every wave).
// Software-pipelined: load(rec) issues a window's loads into a Buf and proc(buf) consumes the
// previous window's, so one window's memory latency overlaps the other's LDS work (a wave's
// loads retire in order: proc waits only for the older window).
template <int U, typename Buf, int RPL = 1, typename LD, typename PR>
__device__ __forceinline__ void for_each_run_record_pipe(const BinGeom& g, const uint16_t* rowb, const uint16_t* rowe,
                                                         uint64_t* wmask_all, int32_t* wlist_all, LD&& load,
                                                         PR&& proc, uint32_t w0 = 0, uint32_t nwaves = 0) {
  // RPL runs per lane (consecutive): a wave takes 64 * RPL runs at a time
  constexpr uint32_t kWin = 64 * U, kRuns = 64 * RPL;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (nwaves == 0) nwaves = blockDim.x >> 6;
  uint64_t* wm = wmask_all + wave * U;
  int32_t* wl = wlist_all + wave * kRuns;
  const uint64_t below = (1ull << lane) - 1ull, upto = (2ull << lane) - 1ull;
  const uint32_t step = nwaves * kRuns;
  uint32_t nbe[RPL], nen[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) nbe[r] = nen[r] = 0;
  if ((wave - w0) * kRuns < g.nt_s) {
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const uint32_t sc = min((wave - w0) * kRuns + lane * RPL + r, g.nt_s - 1);
      nbe[r] = rowb[sc];
      nen[r] = rowe[sc];
    }
  }
  Buf pend;
  bool have = false;
  for (uint32_t s0 = (wave - w0) * kRuns; s0 < g.nt_s; s0 += step) {
    uint32_t len[RPL], exc[RPL];
    int32_t basep[RPL];
    uint32_t lsum = 0;
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const uint32_t s = s0 + lane * RPL + r;
      const uint32_t be = s < g.nt_s ? nbe[r] : 0u, en = s < g.nt_s ? nen[r] : 0u;
      len[r] = en - be;
      exc[r] = lsum;  // (the lane's own part: the wave's prefix is added below)
      basep[r] = (int32_t)(s * g.rp + be);
      lsum += len[r];
    }
    if (s0 + step < g.nt_s) {
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const uint32_t sc = min(s0 + step + lane * RPL + r, g.nt_s - 1);
        nbe[r] = rowb[sc];
        nen[r] = rowe[sc];
      }
    }
    uint32_t inc = lsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    const uint32_t total = __shfl(inc, 63, 64);
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      exc[r] += inc - lsum;
      basep[r] -= (int32_t)exc[r];
    }
    for (uint32_t f0 = 0; f0 < total; f0 += kWin) {
      if (lane < (uint32_t)U) wm[lane] = 0;
      wave_sync();
      bool in[RPL];
      uint32_t before = 0;
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        in[r] = len[r] != 0 && exc[r] < f0 + kWin && exc[r] + len[r] > f0;
        before += (uint32_t)__popcll(__ballot(in[r]) & below);
      }
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        if (in[r]) {
          const uint32_t pos = exc[r] > f0 ? exc[r] - f0 : 0u;
          atomicOr((unsigned long long*)&wm[pos >> 6], 1ull << (pos & 63u));
          wl[before] = basep[r];
          ++before;
        }
      }
      wave_sync();
      int32_t rec[U];
      uint32_t pre = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t w = wm[u];
        const uint32_t rank = pre + (uint32_t)__popcll(w & upto) - 1u;
        pre += (uint32_t)__popcll(w);
        const uint32_t f = f0 + u * 64 + lane;
        rec[u] = f < total ? wl[rank & (kRuns - 1u)] + (int32_t)f : -1;
      }
      wave_sync();  // the next window rewrites wm/wl
      Buf nb = load(rec);
      if (have) proc(pend);
      pend = nb;
      have = true;
    }
  }
  if (have) proc(pend);
}

template <int U>
struct PushBuf {
  int32_t rec[U];
  uint32_t id[U];
  uint64_t v[U];
};
template <int U>
struct IdBuf {
  int32_t rec[U];
  uint32_t id[U];
};
constexpr int kUnrollPipe = 4;  // records per lane and window in the pipelined walks (8: 2^27 dense round 5737 vs 5686 us)
// Serve's walk: windows of 8 records per lane over groups of 128 runs (2 per lane): more loads in
// flight per wave than 4 over 64 (its buffers are ids only).  2^27 dense round 5601-5613 -> 5558-5576
// us, 2^24 equal; 8 over 256 runs, 16 over 128, and apply's push walk over 128 runs or with 6 / 8 records per lane: slower
// (profiles/r04_ak/).
constexpr int kServeU = 8, kServeRPL = 2, kPushRPL = 1;

// The pushes aimed at tile X (its runs in every sender region) ORed into acc,
// by the waves [0, nwaves) (0: all).  VZ: the record id's no-push flag.
// LAYOUT 0: u32 ids + values (sharded passes), 1: split u16 ids + values, 2: split + packed pushes
template <uint32_t VZ, int LAYOUT>
__device__ __forceinline__ void push_walk(const BinGeom& g, const BinBufs& b, uint32_t X, unsigned long long* acc,
                                          uint64_t* wmask, int32_t* wlist, uint32_t nwaves) {
  const uint32_t* __restrict__ gids = b.ids;
  const uint64_t* __restrict__ gvals = b.vals;
  const uint32_t* __restrict__ gprec = b.prec;
  constexpr bool aos = LAYOUT == 2, SPLIT = LAYOUT >= 1;
  const uint16_t* rowb = b.offT + (size_t)X * g.nt_s;
  constexpr int U = kUnrollPipe;
  for_each_run_record_pipe<U, PushBuf<U>, kPushRPL>(g, rowb, rowb + g.nt_s, wmask, wlist, [&](const int32_t* rec) {
    PushBuf<U> bf;
#pragma unroll
    for (int u = 0; u < U; ++u) bf.rec[u] = rec[u];
    if constexpr (aos) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t* r = &gprec[3ull * (uint32_t)(rec[u] >= 0 ? rec[u] : 0)];
        uint32_t lo, hi;
        prec_ld(r, lo, hi, bf.id[u]);
        bf.v[u] = (uint64_t)lo | ((uint64_t)hi << 32);
      }
    } else {
      if constexpr (SPLIT) {
#pragma unroll
        for (int u = 0; u < U; ++u) bf.id[u] = (uint32_t)*(&b.dst[rec[u] >= 0 ? rec[u] : 0]);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) bf.id[u] = *(&gids[rec[u] >= 0 ? rec[u] : 0]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) bf.v[u] = *(&gvals[rec[u] >= 0 ? rec[u] : 0]);
    }
    return bf;
  }, [&](const PushBuf<U>& bf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t id = SPLIT && !aos ? id_of_dst(bf.id[u]) : bf.id[u];
      const uint64_t v = bf.rec[u] < 0 || (id & VZ) ? 0ull : bf.v[u];
      const uint32_t p = id & (kTileD - 1);
      // no read-before-OR: the LDS read's latency stalled the wave (0.7 % of the 2^27 dense round,
      // profiles/r04_ag)
      if (v) atomicOr(&acc[p], (unsigned long long)v);
    }
  }, 0u, nwaves);
}

// Tile image in registers (the next tile's loads fly during the current walk).
constexpr uint32_t kTileQ = kTileD / kTileThreads / 2;  // uint4 per thread
// Slots [Q0, Q0 + Q) of this thread's part of the tile (x[i] = slot Q0 + i).
template <uint32_t Q0 = 0, uint32_t Q = kTileQ>
__device__ __forceinline__ void tile_regs_load(uint4 (&x)[Q], const uint64_t* __restrict__ S, uint64_t node0,
                                               uint64_t N) {
  const uint32_t tid = threadIdx.x;
  if (node0 + kTileD <= N && ((uintptr_t)(S + node0) & 15u) == 0) {
    const uint4* src = (const uint4*)(S + node0);
#pragma unroll
    for (uint32_t q = 0; q < Q; ++q) x[q] = src[(Q0 + q) * kTileThreads + tid];
  } else {
#pragma unroll
    for (uint32_t q = 0; q < Q; ++q) {
      const uint64_t n = node0 + 2ull * ((Q0 + q) * kTileThreads + tid);
      const uint64_t a = n < N ? S[n] : 0ull, b = n + 1 < N ? S[n + 1] : 0ull;
      x[q] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
  }
}

// K2 — one block per destination tile T (pull modes): LDS image of S_t[T];
// every record aimed at T from a sender that is not yet fully informed gets
// its pull response S_t[p] written next to it when nonzero (every one, in dense rounds).
// VF: the record id's no-pull flag (kIdVF; exchange rounds' binned items: kXbVF).
template <uint32_t VF, bool SPLIT = false>
__global__ __launch_bounds__(kTileThreads) void bin_serve_kernel(BinGeom g, const uint64_t* __restrict__ S, BinBufs b,
                                                                  uint32_t R, IdxRange tr) {
  __shared__ unsigned long long img[kTileD];
  __shared__ uint64_t wmask[(kTileThreads / 64) * kServeU];
  __shared__ int32_t wlist[(kTileThreads / 64) * 64 * kServeRPL];
  // persistent: virtual block v = blockIdx.x, +gridDim.x, ... serves tile
  // tr.at(xcd_remap(v, tr.n)) (the XCD of v is that of blockIdx.x, as with one
  // block per tile); the next tile's image loads into registers during a walk
  const uint32_t nv = tr.n;
  // b.dyn: tiles from the per-XCD queues (TileQueue; the whole range only), claimed one ahead
  const bool dyn = b.dyn && tr.lo == 0 && tr.skip0 == tr.skip1 && nv >= 8 && (nv & 7u) == 0;
  const TileQueue tq{b.dyn, nv};
  __shared__ uint32_t s_claim;
  auto tile_of = [&](uint32_t v) { return tr.at(dyn ? v : xcd_remap(v, nv)); };
  uint4 x[kTileQ];
  uint32_t v0 = blockIdx.x;
  if (dyn) {
    if (threadIdx.x == 0) s_claim = tq.claim();
    __syncthreads();
    v0 = s_claim;
  }
  if (v0 < nv) tile_regs_load(x, S, (uint64_t)tile_of(v0) << kTileDLog, g.N);
  for (uint32_t v = v0, vn; v < nv; v = vn) {
  const uint32_t T = tile_of(v);
  __syncthreads();  // the previous walk is done with img (and every thread has read s_claim)
#pragma unroll
  for (uint32_t q = 0; q < kTileQ; ++q) ((uint4*)img)[q * kTileThreads + threadIdx.x] = x[q];
  if (dyn && threadIdx.x == 0) s_claim = tq.claim();
  __syncthreads();
  vn = dyn ? s_claim : v + gridDim.x;
  if (vn < nv) tile_regs_load(x, S, (uint64_t)tile_of(vn) << kTileDLog, g.N);
  const uint32_t* gids = b.ids;
  uint64_t* __restrict__ gresp = b.resp;
  const uint16_t* rowb = b.offT + (size_t)T * g.nt_s;
  constexpr int U = kServeU;
  auto proc = [&](const IdBuf<U>& bf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t id = SPLIT ? id_of_dst(bf.id[u]) : bf.id[u];
      if (bf.rec[u] < 0 || (id & VF)) continue;
      gresp[bf.rec[u]] = (uint64_t)img[id & (kTileD - 1)];
    }
  };
  for_each_run_record_pipe<U, IdBuf<U>, kServeRPL>(g, rowb, rowb + g.nt_s, wmask, wlist, [&](const int32_t* rec) {
    IdBuf<U> bf;
#pragma unroll
    for (int u = 0; u < U; ++u) bf.rec[u] = rec[u];
    if constexpr (SPLIT) {
#pragma unroll
      for (int u = 0; u < U; ++u) bf.id[u] = (uint32_t)*(&b.dst[rec[u] >= 0 ? rec[u] : 0]);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) bf.id[u] = *(&gids[rec[u] >= 0 ? rec[u] : 0]);
    }
    return bf;
  }, proc);
  }
}


uint32_t serve_grid(uint32_t tiles, uint32_t cap = kServeGrid) { return cap == 0 || tiles < cap ? tiles : cap; }

// K3 — one block per tile X: acc = S_t[X]; OR in the pushes aimed at X (its
// runs) and the pull responses owed to X's own senders (their regions, read
// sequentially); write S_{t+1}[X] and fold the stats.  One shard: g = gq, b =
// bq.  Sharded dense round: g/b the push pass (every sender, tiles of the own
// nodes), gq/bq the pull pass (own senders, tiles of the whole image); S and
// Snext are the own slices (Nn nodes, global ids from hid0).
template <int LAYOUT>
__global__ __launch_bounds__(kTileThreads) void bin_apply_kernel(BinGeom g, BinBufs b, BinGeom gq, BinBufs bq,
                                                                  const uint64_t* S, uint64_t* Snext,  // may alias
                                                                  uint64_t Nn, uint64_t hid0,
                                                                  uint64_t* __restrict__ partial, uint32_t R,
                                                                  uint32_t mode, uint32_t flags) {
  __shared__ unsigned long long acc[kTileD];
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red_hash[kTileThreads / 64];
  __shared__ uint32_t red_full[kTileThreads / 64];
  __shared__ uint32_t red_nz[kTileThreads / 64];
  __shared__ uint64_t wmask[(kTileThreads / 64) * kUnrollPipe];
  __shared__ int32_t wlist[(kTileThreads / 64) * 64 * kPushRPL];
  const uint32_t tid = threadIdx.x;
  // persistent (grid apply_grid(nt_d)): virtual block v = blockIdx.x,
  // +gridDim.x, ... applies tile xcd_remap(v, nt_d) (same XCD as blockIdx.x);
  // the next tile's S_t loads into registers during the current tile's work.  In
  // place stays safe: only this block reads or writes S[X] of its tiles.
  const uint32_t nv = g.nt_d;
  // b.dyn (one shard): tiles from the per-XCD queues (TileQueue), else the static order
  const bool dyn = b.dyn && nv >= 8 && (nv & 7u) == 0;
  const TileQueue tq{b.dyn ? b.dyn + 8 : nullptr, nv};
  __shared__ uint32_t s_claim;
  __shared__ uint64_t btot[3];  // the block's totals over its tiles (cnt too: not reset per tile)
  if (tid < 64) cnt[tid] = 0;
  if (tid < 3) btot[tid] = 0;
  for (uint32_t v = blockIdx.x;;) {
  __syncthreads();  // the previous epilogue is done with acc, cnt and s_claim
  if (dyn) {
    if (tid == 0) s_claim = tq.claim();
    __syncthreads();
    v = s_claim;
  }
  if (v >= nv) break;
  const uint32_t X = dyn ? v : xcd_remap(v, nv);
  const uint64_t node0 = (uint64_t)X << kTileDLog;
  {
    uint4 xr[kTileQ];
    tile_regs_load(xr, S, node0, Nn);
#pragma unroll
    for (uint32_t q = 0; q < kTileQ; ++q) ((uint4*)acc)[q * kTileThreads + tid] = xr[q];
  }
  __syncthreads();
  const uint32_t wave = tid >> 6;
  const bool split = kApplySplit && mode == 3;
  const uint32_t pw = g.push_waves;
  const bool do_push = (mode == 1 || mode == 3) && (!split || wave < pw);
  const bool do_pull = (mode == 2 || mode == 3) && (!split || wave >= pw);
  // split: waves [0, pw) walk the pushes, the others the responses
  const uint32_t qt0 = split ? pw * 64 : 0u, qnt = split ? kTileThreads - pw * 64 : kTileThreads;
  constexpr bool SPLIT = LAYOUT >= 1;
  if (do_push) push_walk<kIdVZ, LAYOUT>(g, b, X, acc, wmask, wlist, split ? pw : 0u);  // pushes aimed at this tile
  if (do_pull) {  // responses owed to this tile's own senders
    const uint32_t* __restrict__ qids = bq.ids;
    const uint64_t* __restrict__ gresp = bq.resp;
    const uint32_t per = kTileD >> gq.ts_log;
    const uint32_t s0 = X * per, s1 = min(s0 + per, gq.nt_s);
    for (uint32_t s = s0; s < s1; ++s) {
      const uint32_t total = bq.off[(size_t)s * (gq.nt_d + 1) + gq.nt_d];
      const size_t reg = (size_t)s * gq.rp;
      const uint32_t nb = (s - s0) << gq.ts_log;
      const uint32_t qtid = tid - qt0;
      for (uint32_t p0 = 0; p0 < total; p0 += qnt * kUnrollSeq) {
        uint64_t r[kUnrollSeq];
        uint32_t id[kUnrollSeq];
        // id and response loads are independent: both fly together
#pragma unroll
        for (int u = 0; u < kUnrollSeq; ++u) {
          const uint32_t pos = min(p0 + u * qnt + qtid, total - 1);
          if constexpr (SPLIT) id[u] = id_of_src(*(&bq.src[reg + pos]));
          else id[u] = *(&qids[reg + pos]);
          r[u] = *(&gresp[reg + pos]);
        }
#pragma unroll
        for (int u = 0; u < kUnrollSeq; ++u) {
          // a full sender's slot was never written this round (K2 skips it)
          if (p0 + u * qnt + qtid >= total || (id[u] & kIdVF)) continue;
          const uint32_t node = nb + ((id[u] >> kTileDLog) & kIdNMask);
          if (r[u]) atomicOr(&acc[node], (unsigned long long)r[u]);
        }
      }
    }
  }
  __syncthreads();
  tile_epilogue(acc, node0, Nn, hid0, Snext, partial, R, flags, cnt, red_hash, red_full, red_nz, b.nzb, b.fullb,
                btot);
  if (!dyn) v += gridDim.x;
  }
  block_totals_flush(partial, R, cnt, btot);
}

// Apply grid: one persistent block per CU (BinGeom::apply_grid = 0: one block per tile).
uint32_t apply_grid(const BinGeom& g) {
  const uint32_t cap = g.apply_grid;
  return cap == 0 || g.nt_d < cap ? g.nt_d : cap;
}

}  // namespace

// [rows][cols] u16 table -> [cols][rows] (the binned sparse scan's run table, frontier.hip)
void bin_transpose_u16(const uint16_t* in, uint16_t* out, uint32_t rows, uint32_t cols, hipStream_t st) {
  launch_transpose_u16(in, out, rows, cols, nullptr, 0u, st);
}

BinGeom make_bin_geom(uint64_t N, uint32_t k, bool big) {
  BinGeom g{};
  g.N = N;
  g.k = k;
  uint32_t ts = big ? 2 * kMaxSenders : kMaxSenders, lg = big ? 14 : 13;
  while (ts * k > (big ? 2 * kRecPerRegion : kRecPerRegion)) {
    ts >>= 1;
    --lg;
  }
  g.ts = ts;
  g.ts_log = lg;
  g.rp = ts * k;
  g.nt_s = (uint32_t)((N + ts - 1) / ts);
  g.nt_d = (uint32_t)((N + kTileD - 1) / kTileD);
  g.apply_grid = kApplyGrid;
  g.serve_grid = kServeGrid;
  g.push_waves = N > (1ull << 25) ? kPushWavesBig : kPushWaves;
  // big regions (past kMaxTilesD tiles) make runs of ~4 records, and the apply pass's push
  // walk is bound by the number of distinct lines it fetches: a push packed as one 12-B
  // piece beside the 4-B id (for serve and the reply walk) touches fewer than the two
  // arrays' 16-B + 32-B pieces of a run
  g.aos = big ? 1u : 0u;  // (packed pushes at 2^24: 570 vs 520 us per dense round)
  g.split = 1u;  // (sharded geometries clear it: their passes keep u32 ids)
  return g;
}

bool bin_path_ok(uint64_t N, uint32_t k, uint32_t W, uint32_t G) {
  if (W != 1 || G != 1 || k == 0 || k > 64 || N < 2) return false;
  const BinGeom g = make_bin_geom(N, k);
  // past 4096 tiles the emit re-reads sender values from S (V = 3); record indices are int32
  return g.nt_d <= kSbMaxTiles && (uint64_t)g.nt_s * g.rp < (1ull << 31);
}

size_t bin_bytes(const BinGeom& g) {
  const size_t recs = (size_t)g.nt_s * g.rp;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  return (g.split ? 2 * al(recs * 2) : al(recs * 4)) + (g.aos ? al(recs * 12) : al(recs * 8)) + al(recs * 8) +
         2 * al((size_t)g.nt_s * (g.nt_d + 1) * 2) + 256 +
         256;  // the tile queues (dyn)
}

void bin_carve(const BinGeom& g, void* base, BinBufs* b) {
  const size_t recs = (size_t)g.nt_s * g.rp;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  char* p = (char*)base;
  b->ids = nullptr;
  b->dst = b->src = nullptr;
  if (g.split) {
    b->dst = (uint16_t*)p;
    p += al(recs * 2);
    b->src = (uint16_t*)p;
    p += al(recs * 2);
  } else {
    b->ids = (uint32_t*)p;
    p += al(recs * 4);
  }
  b->vals = g.aos ? nullptr : (uint64_t*)p;
  b->prec = g.aos ? (uint32_t*)p : nullptr;
  p += g.aos ? al(recs * 12) : al(recs * 8);
  b->resp = (uint64_t*)p;
  p += al(recs * 8);
  b->off = (uint16_t*)p;
  p += al((size_t)g.nt_s * (g.nt_d + 1) * 2);
  b->offT = (uint16_t*)p;
  p += al((size_t)g.nt_s * (g.nt_d + 1) * 2);
  p += 256;
  b->dyn = (uint32_t*)p;  // 16 u32 (sharded passes clear it: their order stays static)

}

namespace {
// K1 + the run-offset transpose of a one-shard dense round
void launch_bin_emit(const BinGeom& g, const BinBufs& b, uint64_t* S, uint64_t* partial, uint32_t R, uint32_t t,
                     uint32_t key0, uint32_t key1, uint32_t mode, uint32_t filt, const Faults& fa,
                     const RoundSync& rs, hipStream_t st) {
  const uint32_t eg = g.nt_s < kEmitGrid ? g.nt_s : kEmitGrid;  // persistent: one block per CU
#define GOSSIP_EMIT(KR, F, VV) \
  bin_emit_kernel<KR, F, VV><<<eg, kEmitThreads, 0, st>>>(g, S, b, R, t, key0, key1, mode, filt, fa, EmitRange{})
#define GOSSIP_EMIT_V(VV)                                                 \
  if (g.k <= 2) {                                                        \
    if (fa.any()) GOSSIP_EMIT(2, true, VV); else GOSSIP_EMIT(2, false, VV); \
  } else {                                                                \
    if (fa.any()) GOSSIP_EMIT(0, true, VV); else GOSSIP_EMIT(0, false, VV); \
  }
  if (g.ts > kMaxSenders || g.rp > kRecPerRegion) {  // make_bin_geom(big): V = 4, 5
    // 16 senders per lane keep no room for their peers in registers (KREG = 2 spills 78
    // VGPRs): V = 5 keeps them in LDS between the passes, V = 4 draws them again
    if (fa.any()) GOSSIP_EMIT(0, true, 4);
    else if (g.k <= 2) GOSSIP_EMIT(0, false, 5);
    else GOSSIP_EMIT(0, false, 4);
  } else if (g.nt_d <= kMaxTilesD) {
    GOSSIP_EMIT_V(0)
  } else {
    GOSSIP_EMIT_V(3)
  }
#undef GOSSIP_EMIT_V
#undef GOSSIP_EMIT
  launch_transpose_u16(b.off, b.offT, g.nt_s, g.nt_d + 1, partial, rs.plen, st, b.dyn);
}
}  // namespace

hipError_t launch_binned_round(const BinGeom& g, const BinBufs& b, uint64_t* S, uint64_t* partial, uint32_t R,
                               uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode, uint32_t filt,
                               const Faults& fa, uint32_t flags, const RoundSync& rs, hipStream_t st,
                               uint32_t parts) {
  if (!b.nzb || !b.fullb) filt = 0;  // the bitmaps exist only with the frontier buffers
  if (parts & 1u) launch_bin_emit(g, b, S, partial, R, t, key0, key1, mode, filt, fa, rs, st);
  const bool pull = mode == 2 || mode == 3;
  if ((parts & 2u) && pull && g.split)
    bin_serve_kernel<kIdVF, true><<<serve_grid(g.nt_d, g.serve_grid), kTileThreads, 0, st>>>(g, S, b, R,
                                                                                          IdxRange::all(g.nt_d));
  else if ((parts & 2u) && pull)
    bin_serve_kernel<kIdVF, false><<<serve_grid(g.nt_d, g.serve_grid), kTileThreads, 0, st>>>(g, S, b, R,
                                                                                           IdxRange::all(g.nt_d));
  // in place: K3 of tile X reads and writes only S[X] (push values and pull
  // responses come from the record buffers), and K1/K2 have finished reading S_t
  if (!(parts & 4u)) return hipGetLastError();
  if (g.aos)
    bin_apply_kernel<2><<<apply_grid(g), kTileThreads, 0, st>>>(g, b, g, b, S, S, g.N, 0, partial, R, mode, flags);
  else if (g.split)
    bin_apply_kernel<1><<<apply_grid(g), kTileThreads, 0, st>>>(g, b, g, b, S, S, g.N, 0, partial, R, mode, flags);
  else
    bin_apply_kernel<0><<<apply_grid(g), kTileThreads, 0, st>>>(g, b, g, b, S, S, g.N, 0, partial, R, mode, flags);
  return hipGetLastError();  // the engine enqueues the round's snapshot (round.h) after its timing event
}

// --- sharded dense rounds ------------------------------------------------

bool sb_path_ok(uint64_t N, uint32_t k, uint64_t nown) {
  if (k == 0 || k > 64 || N < 2 || nown == 0) return false;
  const SbGeom g = make_sb_geom(N, k, 0, nown);
  return g.q.nt_d <= kSbMaxTiles && g.p.nt_d <= kMaxTilesD && (uint64_t)g.p.nt_s * g.p.rp < (1ull << 31);
}

SbGeom make_sb_geom(uint64_t N, uint32_t k, uint64_t lo, uint64_t nown) {
  SbGeom g{};
  g.lo = lo;
  g.nown = nown;
  // region sizes as on one shard (make_bin_geom), big past 4096 image tiles: at 2^27 nodes runs
  // of ~2 records become ~4 (dense round per rank 4.93 -> 4.14 ms at 2 x 2^26, 2.87 -> 2.56 ms at
  // 4 x 2^25); with 2^26 or 2^25 image nodes the big emit costs more than that saves (4 x 2^24:
  // 1.18 -> 1.23 ms; profiles/r04_ad).  Peers are drawn over the global id space.
  g.p = g.q = make_bin_geom(N, k, (N + kTileD - 1) / kTileD > kMaxTilesD);
  g.p.split = g.q.split = 0u;
  g.p.aos = g.q.aos = 0u;  // (the sharded passes keep u32 ids + values)
  g.p.nt_s = (uint32_t)((N + g.p.ts - 1) / g.p.ts);      // every sender
  g.p.nt_d = (uint32_t)((nown + kTileD - 1) / kTileD);   // own tiles
  g.q.nt_s = (uint32_t)((nown + g.q.ts - 1) / g.q.ts);   // own senders
  g.q.nt_d = (uint32_t)((N + kTileD - 1) / kTileD);      // every tile of the image
  return g;
}

size_t sb_bytes(const SbGeom& g) { return bin_bytes(g.p) + bin_bytes(g.q); }

void sb_carve(const SbGeom& g, void* base, SbBufs* b) {
  bin_carve(g.p, base, &b->p);
  bin_carve(g.q, (char*)base + bin_bytes(g.p), &b->q);
  b->p.nzb = b->p.fullb = b->q.nzb = b->q.fullb = nullptr;
  b->p.dyn = b->q.dyn = nullptr;
}

namespace {
// the P regions and image tiles that lie inside the own slice: they need no
// remote data, so they run while the all-gather is in flight
IdxRange own_regions(const SbGeom& g) {
  const uint64_t a = (g.lo + g.p.ts - 1) / g.p.ts, b = (g.lo + g.nown) / g.p.ts;
  return b > a ? IdxRange{(uint32_t)a, (uint32_t)(b - a), 0u, 0u} : IdxRange{0u, 0u, 0u, 0u};
}
IdxRange own_tiles(const SbGeom& g) {
  const uint64_t a = (g.lo + kTileD - 1) / kTileD, b = (g.lo + g.nown) / kTileD;
  return b > a ? IdxRange{(uint32_t)a, (uint32_t)(b - a), 0u, 0u} : IdxRange{0u, 0u, 0u, 0u};
}
// every index of [0, n) outside x
IdxRange rest_of(uint32_t n, const IdxRange& x) { return IdxRange{0u, n - x.n, x.lo, x.lo + x.n}; }

void sb_emit(const BinGeom& gg, const BinBufs& bb, const uint64_t* image, uint32_t R, uint32_t t, uint32_t key0,
             uint32_t key1, uint32_t mode, const Faults& fa, const EmitRange& er, bool vals, hipStream_t st) {
  if (er.rs.n == 0) return;
  const uint32_t eg = er.rs.n < kEmitGrid ? er.rs.n : kEmitGrid;
#define GOSSIP_EMIT(KR, F, VV) \
  bin_emit_kernel<KR, F, VV><<<eg, kEmitThreads, 0, st>>>(gg, image, bb, R, t, key0, key1, mode, 0u, fa, er)
#define GOSSIP_EMIT_V(VV)                                                 \
  if (gg.k <= 2) {                                                        \
    if (fa.any()) GOSSIP_EMIT(2, true, VV); else GOSSIP_EMIT(2, false, VV); \
  } else {                                                                \
    if (fa.any()) GOSSIP_EMIT(0, true, VV); else GOSSIP_EMIT(0, false, VV); \
  }
  if (gg.ts > kMaxSenders || gg.rp > kRecPerRegion) {  // big regions (make_sb_geom): V = 6-9
    if (fa.any()) {
      if (vals) GOSSIP_EMIT(0, true, 6); else GOSSIP_EMIT(0, true, 7);
    } else if (gg.k <= 2) {
      if (vals) GOSSIP_EMIT(0, false, 8); else GOSSIP_EMIT(0, false, 9);
    } else {
      if (vals) GOSSIP_EMIT(0, false, 6); else GOSSIP_EMIT(0, false, 7);
    }
  } else if (vals) {
    GOSSIP_EMIT_V(1)
  } else {
    GOSSIP_EMIT_V(2)
  }
#undef GOSSIP_EMIT_V
#undef GOSSIP_EMIT
}

void sb_transpose(const BinGeom& gg, const BinBufs& bb, uint64_t* partial, hipStream_t st) {
  launch_transpose_u16(bb.off, bb.offT, gg.nt_s, gg.nt_d + 1, partial, 0u, st);
}

EmitRange push_range(const SbGeom& g, const IdxRange& rs) { return EmitRange{0, g.p.N, g.lo, g.nown, 1u, 1u, rs}; }
EmitRange pull_range(const SbGeom& g) {
  return EmitRange{g.lo, g.nown, 0, g.q.N, 2u, 0u, IdxRange::all(g.q.nt_s)};
}
}  // namespace

hipError_t launch_sb_pre(const SbGeom& g, const SbBufs& b, const uint64_t* image, uint32_t R, uint32_t t,
                         uint32_t key0, uint32_t key1, uint32_t mode, const Faults& fa, hipStream_t st) {
  const bool push = mode == 1 || mode == 3, pull = mode == 2 || mode == 3;
  if (pull) {
    sb_emit(g.q, b.q, image, R, t, key0, key1, mode, fa, pull_range(g), false, st);
    sb_transpose(g.q, b.q, nullptr, st);
    const IdxRange ot = own_tiles(g);
    if (ot.n) bin_serve_kernel<kIdVF><<<serve_grid(ot.n), kTileThreads, 0, st>>>(g.q, image, b.q, R, ot);
  }
  if (push) sb_emit(g.p, b.p, image, R, t, key0, key1, mode, fa, push_range(g, own_regions(g)), true, st);
  return hipGetLastError();
}

hipError_t launch_sb_post(const SbGeom& g, const SbBufs& b, const uint64_t* image, uint64_t* Snext,
                          uint64_t* partial, uint32_t R, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode,
                          const Faults& fa, uint32_t flags, uint64_t* nzb, uint64_t* fullb, hipStream_t st) {
  const bool push = mode == 1 || mode == 3, pull = mode == 2 || mode == 3;
  if (push) {
    sb_emit(g.p, b.p, image, R, t, key0, key1, mode, fa, push_range(g, rest_of(g.p.nt_s, own_regions(g))), true,
            st);
    sb_transpose(g.p, b.p, nullptr, st);
  }
  if (pull) {
    const IdxRange rt = rest_of(g.q.nt_d, own_tiles(g));
    if (rt.n) bin_serve_kernel<kIdVF><<<serve_grid(rt.n), kTileThreads, 0, st>>>(g.q, image, b.q, R, rt);
  }
  BinBufs bp = b.p;
  bp.nzb = nzb;
  bp.fullb = fullb;
  bin_apply_kernel<0><<<apply_grid(g.p), kTileThreads, 0, st>>>(g.p, bp, g.q, b.q, image + g.lo, Snext, g.nown, g.lo, partial,
                                                      R, mode, flags);
  return hipGetLastError();
}

hipError_t launch_sb_round(const SbGeom& g, const SbBufs& b, const uint64_t* image, uint64_t* Snext,
                           uint64_t* partial, uint32_t R, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode,
                           const Faults& fa, uint32_t flags, uint64_t* nzb, uint64_t* fullb, hipStream_t st) {
  const hipError_t e = launch_sb_pre(g, b, image, R, t, key0, key1, mode, fa, st);
  if (e != hipSuccess) return e;
  return launch_sb_post(g, b, image, Snext, partial, R, t, key0, key1, mode, fa, flags, nzb, fullb, st);
}


// --- exchange dense rounds (binned.h: XdGeom) ---------------

namespace {

constexpr uint32_t kXdMaxG = 256;
// sender regions of the exchange rounds: at most this many items (xd_emit stages them in
// LDS, 6 B each), and the count / emit grid.  8192 items and 512 blocks (two emit blocks per
// CU) measured the same at G = 8 (9.81 vs 9.81-9.87 ms per rank, profiles/r02_xd/region)
constexpr uint32_t kXdSendRegion = 16384;  // (8192: no gain at G = 8)
static_assert(kXdSendRegion <= kRecPerRegion, "xd sender regions: at most kRecPerRegion items");
// binned received item: p_local [0, 14) | slot in its region [14, 28) | no push | no pull
constexpr uint32_t kXbVZ = 1u << 28;
constexpr uint32_t kXbVF = 1u << 29;
constexpr uint32_t kXbSlotMask = kXdBinRegion - 1u;
constexpr uint32_t kXdPref = 2048;
constexpr int kUnrollXd = 4;  // replies in flight per lane in apply (each finds its owner run first)  // apply's LDS copy of its regions' (G + 1)-entry prefix rows

__device__ __forceinline__ uint32_t xd_owner(uint32_t p, uint32_t Nl32, uint32_t G) {
  const uint32_t o = p / Nl32;
  return o < G ? o : G - 1u;
}

// The exchange-round edge filter: xf.cls holds every shard's occupancy
// bitmaps of S_t ([nz: nwl words][full: nwl words] per shard, all-gathered); a one-way
// edge is dropped when it moves nothing — a pull-only edge (empty sender) whose peer is
// empty (filt bit 0), a push-only edge (full sender) whose peer is full (bit 1).  Returns
// the directions kept (sender_dirs' bits), 0 = no item.
__device__ __forceinline__ uint32_t xd_filter(const XdFilter& xf, uint32_t d, uint32_t o, uint32_t pl) {
  const uint64_t* slot = xf.cls + (size_t)o * 2 * xf.nwl;
  if ((xf.filt & 1u) && d == 2u && !((slot[pl >> 6] >> (pl & 63u)) & 1ull)) return 0u;
  if ((xf.filt & 2u) && d == 1u && ((slot[xf.nwl + (pl >> 6)] >> (pl & 63u)) & 1ull)) return 0u;
  return d;
}

// the live edges n -> p of sender n in round t (draws as bin_emit's; a lost edge
// carries nothing in either direction)
template <bool FAULTS, typename F>
__device__ __forceinline__ void xd_edges(uint32_t k, uint32_t n, uint64_t nm1, uint32_t t, uint32_t key0,
                                         uint32_t key1, const Faults& fa, F&& fn) {
  u32x4 x{0, 0, 0, 0}, lw{0, 0, 0, 0};
  const Reach rc = FAULTS ? reach_of(n, fa) : Reach{0u, 0xFFFFFFFFu};
  for (uint32_t j = 0; j < k; ++j) {
    if ((j & 3u) == 0) {
      x = philox4x32_10(u32x4{n, t, 0u, j >> 2}, key0, key1);
      if (FAULTS && fa.loss) lw = loss_draws(n, t, j >> 2, key0, key1);
    }
    const uint32_t p = peer_from_word(lane_of(x, j & 3u), nm1, n);
    if (FAULTS && edge_lost(fa, rc, p, lane_of(lw, j & 3u))) continue;
    fn(p, j);
  }
}

// items per (sender region, owner of the peer).  (Reading the senders' classes from the
// occupancy bitmaps instead of S_t made count + emit slower: S_t streamed here is still
// in the MALL when emit reads it, profiles/r02_xd/variants3.)
template <bool FAULTS>
__global__ __launch_bounds__(kEmitThreads) void xd_count_kernel(XdGeom g, const uint64_t* __restrict__ S,
                                                                 uint32_t* __restrict__ rcnt, uint32_t R, uint32_t t,
                                                                 uint32_t key0, uint32_t key1, uint32_t mode,
                                                                 Faults fa, XdFilter xf) {
  __shared__ uint32_t cnt[kXdMaxG];
  const uint32_t tid = threadIdx.x, Nl32 = (uint32_t)g.Nl;
  const uint64_t fm = full_mask1(R), nm1 = g.N - 1;
  for (uint32_t s = blockIdx.x; s < g.s.nt_s; s += gridDim.x) {
    __syncthreads();
    for (uint32_t o = tid; o < g.G; o += kEmitThreads) cnt[o] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)s << g.s.ts_log;
    const uint32_t nsend = (uint32_t)min<uint64_t>(g.s.ts, g.nown - base);
    // (one LDS atomic per edge: aggregating a wave's lanes per owner with ballots measured
    // 2.6x slower, profiles/r02_xd/variants3)
    for (uint32_t i = tid; i < nsend; i += kEmitThreads) {
      const uint32_t d = sender_dirs(mode, S[base + i], fm);
      uint32_t keep = 0;  // filtered rounds: edge j survives the class probe (emit reads it, no second probe)
      if (d)
        xd_edges<FAULTS>(g.k, (uint32_t)(g.lo + base + i), nm1, t, key0, key1, fa, [&](uint32_t p, uint32_t j) {
          const uint32_t o = xd_owner(p, Nl32, g.G);
          if (xf.filt && !xd_filter(xf, d, o, p - o * Nl32)) return;
          keep |= 1u << j;
          atomicAdd(&cnt[o], 1u);
        });
      if (xf.filt) xf.keep[base + i] = (uint8_t)keep;
    }
    __syncthreads();
    for (uint32_t o = tid; o < g.G; o += kEmitThreads) rcnt[(size_t)s * g.G + o] = cnt[o];
  }
}

// send positions: owner-major, then sender region; ocnt = items per owner.  One
// block per owner o: the items of owners < o (its base) and o's column scan.
__global__ __launch_bounds__(1024) void xd_scan_kernel(const uint32_t* __restrict__ rcnt, uint32_t* __restrict__ roff,
                                                        uint32_t* __restrict__ ocnt, uint32_t nrs, uint32_t G) {
  __shared__ uint32_t scratch[1024 / 64 + 1];
  const uint32_t o = blockIdx.x;
  const uint32_t per = (nrs + 1023) / 1024;
  const uint32_t lo = min(threadIdx.x * per, nrs), hi = min(lo + per, nrs);
  uint32_t before = 0, mine = 0;
  for (uint32_t s = lo; s < hi; ++s) {
    const uint32_t* row = rcnt + (size_t)s * G;
    for (uint32_t q = 0; q < o; ++q) before += row[q];
    mine += row[o];
  }
  uint32_t base, total;
  (void)block_exscan<1024>(before, scratch, &base);
  uint32_t run = base + block_exscan<1024>(mine, scratch, &total);
  for (uint32_t s = lo; s < hi; ++s) {
    const uint32_t c = rcnt[(size_t)s * G + o];
    roff[(size_t)s * G + o] = run;
    run += c;
  }
  if (threadIdx.x == 0) ocnt[o] = total;
}

// the items of sender region s, counting-sorted by owner in LDS and written to
// their send positions; rlofs[s] = the region's owner runs (G + 1 prefix)
template <bool FAULTS>
__global__ __launch_bounds__(kEmitThreads) void xd_emit_kernel(XdGeom g, const uint64_t* __restrict__ S, XdBufs b,
                                                                uint32_t* __restrict__ rlofs, uint32_t R, uint32_t t,
                                                                uint32_t key0, uint32_t key1, uint32_t mode,
                                                                Faults fa, XdFilter xf) {
  __shared__ uint32_t cur[kXdMaxG];
  __shared__ uint32_t lofs[kXdMaxG + 1];
  __shared__ uint32_t st_id[kXdSendRegion];
  __shared__ uint16_t st_nl[kXdSendRegion];
  const uint32_t tid = threadIdx.x, Nl32 = (uint32_t)g.Nl, G = g.G;
  const uint64_t fm = full_mask1(R), nm1 = g.N - 1;
  for (uint32_t s = blockIdx.x; s < g.s.nt_s; s += gridDim.x) {
    __syncthreads();  // the previous region's write-out is done with the LDS
    if (tid == 0) {
      uint32_t a = 0;
      for (uint32_t o = 0; o < G; ++o) {
        lofs[o] = a;
        cur[o] = a;
        a += b.rcnt[(size_t)s * G + o];
      }
      lofs[G] = a;
    }
    __syncthreads();
    for (uint32_t o = tid; o <= G; o += kEmitThreads) rlofs[(size_t)s * (G + 1) + o] = lofs[o];
    const uint64_t base = (uint64_t)s << g.s.ts_log;
    const uint32_t nsend = (uint32_t)min<uint64_t>(g.s.ts, g.nown - base);
    for (uint32_t i = tid; i < nsend; i += kEmitThreads) {
      const uint32_t d = sender_dirs(mode, S[base + i], fm);
      if (!d) continue;
      const uint32_t keep = xf.filt ? xf.keep[base + i] : ~0u;
      xd_edges<FAULTS>(g.k, (uint32_t)(g.lo + base + i), nm1, t, key0, key1, fa, [&](uint32_t p, uint32_t j) {
        if (!((keep >> j) & 1u)) return;  // dropped by the count pass's class probe
        const uint32_t o = xd_owner(p, Nl32, G), pl = p - o * Nl32;
        const uint32_t de = d;
        const uint32_t pos = atomicAdd(&cur[o], 1u);
        st_id[pos] = pl | ((de & 1u) ? 0u : kXdNoPush) | ((de & 2u) ? 0u : kXdNoPull);
        st_nl[pos] = (uint16_t)i;
      });
    }
    __syncthreads();
    const uint32_t total = lofs[G];
    for (uint32_t e = tid; e < total; e += kEmitThreads) {
      uint32_t lo = 0, hi = G;  // the owner: the last o with lofs[o] <= e
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (lofs[mid] <= e) lo = mid;
        else hi = mid;
      }
      const size_t dst = (size_t)b.roff[(size_t)s * G + lo] + (e - lofs[lo]);
      const uint32_t id = st_id[e], nl = st_nl[e];
      rec_st(&b.sid[dst], id);
      rec_st(&b.snl[dst], (uint16_t)nl);
      rec_st(&b.sval[dst], (uint64_t)((id & kXdNoPush) ? 0ull : S[base + nl]));  // the region's slice: L2 hits
    }
  }
}

// received items binned by own destination tile (one region of kXdBinRegion
// items per pass of the block); the binned id keeps the item's slot
__global__ __launch_bounds__(kEmitThreads) void xd_bin_kernel(XdGeom g, XdBufs b, uint64_t n_in) {
  // regions of <= 8192 items also stage the values in LDS (all global accesses in order)
  constexpr bool kStageV = kXdBinRegion <= 8192;
  __shared__ uint32_t cur[kSbMaxTiles];
  __shared__ uint32_t st[kXdBinRegion];
  __shared__ uint64_t sv[kStageV ? kXdBinRegion : 1];
  __shared__ uint32_t wsum[kEmitThreads / 64];
  __shared__ uint32_t wpre[kEmitThreads / 64 + 1];
  constexpr uint32_t kQ = kXdBinRegion / kEmitThreads;
  const uint32_t tid = threadIdx.x, nt = g.r.nt_d;
  for (uint32_t r = blockIdx.x; r < g.r.nt_s; r += gridDim.x) {
    __syncthreads();
    for (uint32_t d = tid; d < nt; d += kEmitThreads) cur[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)r * kXdBinRegion;
    const uint32_t nitems = (uint32_t)min<uint64_t>(kXdBinRegion, n_in - base);
    uint32_t id[kQ];
    uint64_t iv[kStageV ? kQ : 1];
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
      id[q] = i < nitems ? b.rid[base + i] : 0u;
      if constexpr (kStageV) iv[q] = b.rval[base + min(i, nitems - 1)];
      if (i < nitems) atomicAdd(&cur[min((id[q] & (kXdNoPush - 1u)) >> kTileDLog, nt - 1u)], 1u);
    }
    __syncthreads();
    const uint32_t total = region_offsets(cur, nt, b.rb.off + (size_t)r * (nt + 1), wsum, wpre);
    uint32_t* gids = b.rb.ids + (size_t)r * g.r.rp;
    uint64_t* gvals = b.rb.vals + (size_t)r * g.r.rp;
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t i = tid + q * kEmitThreads;
      if (i >= nitems) continue;
      const uint32_t p = id[q] & (kXdNoPush - 1u);
      const uint32_t pos = atomicAdd(&cur[min(p >> kTileDLog, nt - 1u)], 1u);  // (p < nown: emit's items)
      st[pos] = (p & (kTileD - 1)) | (i << kTileDLog) | ((id[q] & kXdNoPush) ? kXbVZ : 0u) |
                ((id[q] & kXdNoPull) ? kXbVF : 0u);
      if constexpr (kStageV) sv[pos] = (id[q] & kXdNoPush) ? 0ull : iv[q];
    }
    __syncthreads();
    for (uint32_t e = tid; e < total; e += kEmitThreads) {
      const uint32_t x = st[e];
      rec_st(&gids[e], x);
      if constexpr (kStageV) {
        rec_st(&gvals[e], (uint64_t)sv[e]);
        continue;
      }
      // the region's values were streamed in with the ids' lines: L2 hits (all of a
      // thread's gathers in flight at once measured slower: 239 -> 323 us)
      rec_st(&gvals[e], (uint64_t)((x & kXbVZ) ? 0ull : b.rval[base + ((x >> kTileDLog) & kXbSlotMask)]));
    }
  }
}

// the responses (binned order) back to the received order, one region per pass
__global__ __launch_bounds__(kEmitThreads) void xd_unperm_kernel(XdGeom g, XdBufs b, uint64_t n_in) {
  __shared__ uint64_t buf[kXdBinRegion];
  const uint32_t tid = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < g.r.nt_s; r += gridDim.x) {
    __syncthreads();
    const uint64_t base = (uint64_t)r * kXdBinRegion;
    const uint32_t nitems = (uint32_t)min<uint64_t>(kXdBinRegion, n_in - base);
    const uint32_t* gids = b.rb.ids + (size_t)r * g.r.rp;
    const uint64_t* gresp = b.rb.resp + (size_t)r * g.r.rp;
    constexpr uint32_t kQ = kXdBinRegion / kEmitThreads;
    uint32_t x[kQ];
    uint64_t rv[kQ];
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q) {
      const uint32_t e = min(tid + q * kEmitThreads, nitems - 1);  // (nitems >= 1)
      x[q] = gids[e];
      rv[q] = gresp[e];
    }
#pragma unroll
    for (uint32_t q = 0; q < kQ; ++q)
      if (tid + q * kEmitThreads < nitems)
        buf[(x[q] >> kTileDLog) & kXbSlotMask] = (x[q] & kXbVF) ? 0ull : rv[q];  // serve wrote only the pulls
    __syncthreads();
    for (uint32_t i = tid; i < nitems; i += kEmitThreads) b.rep_out[base + i] = buf[i];
  }
}

// S_{t+1}[X] = S_t[X] | pushes received for X | replies to the pulls of X's own senders
__global__ __launch_bounds__(kTileThreads) void xd_apply_kernel(XdGeom g, XdBufs b, const uint32_t* __restrict__ rlofs,
                                                                 const uint64_t* S, uint64_t* Snext,
                                                                 uint64_t* __restrict__ partial, uint32_t R,
                                                                 uint32_t mode, uint32_t flags, uint64_t* nzb,
                                                                 uint64_t* fullb) {
  __shared__ unsigned long long acc[kTileD];
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red_hash[kTileThreads / 64];
  __shared__ uint32_t red_full[kTileThreads / 64];
  __shared__ uint32_t red_nz[kTileThreads / 64];
  __shared__ uint64_t wmask[(kTileThreads / 64) * kUnrollPipe];
  __shared__ int32_t wlist[(kTileThreads / 64) * 64 * kPushRPL];
  __shared__ uint32_t pl[kXdPref];  // the tile's sender regions: owner-run prefix rows (G + 1 each)
  __shared__ uint32_t po[kXdPref];  // and the runs' send positions (G each, stride G + 1)
  const uint32_t tid = threadIdx.x, G = g.G;
  const uint32_t nv = g.r.nt_d;
  const uint32_t per = kTileD >> g.s.ts_log;
  const uint32_t wave = tid >> 6, nwav = kTileThreads / 64;
  const bool split = kApplySplit && mode == 3;
  const bool do_push = (mode == 1 || mode == 3) && (!split || wave < nwav / 2);
  const bool do_pull = (mode == 2 || mode == 3) && (!split || wave >= nwav / 2);
  const uint32_t qt0 = split ? kTileThreads / 2 : 0u, qnt = split ? kTileThreads / 2 : kTileThreads;
  __shared__ uint64_t btot[3];  // the block's totals over its tiles (cnt too: not reset per tile)
  if (tid < 64) cnt[tid] = 0;
  if (tid < 3) btot[tid] = 0;
  for (uint32_t v = blockIdx.x; v < nv; v += gridDim.x) {
    const uint32_t X = xcd_remap(v, nv);
    const uint64_t node0 = (uint64_t)X << kTileDLog;
    const uint32_t s0 = X * per, s1 = min(s0 + per, g.s.nt_s);
    __syncthreads();  // the previous epilogue is done with acc, cnt and the prefix rows
    {
      uint4 xr[kTileQ];
      tile_regs_load(xr, S, node0, g.nown);
#pragma unroll
      for (uint32_t q = 0; q < kTileQ; ++q) ((uint4*)acc)[q * kTileThreads + tid] = xr[q];
    }
    for (uint32_t i = tid; i < (s1 - s0) * (G + 1); i += kTileThreads) {
      const uint32_t s = s0 + i / (G + 1), o = i % (G + 1);
      pl[i] = rlofs[(size_t)s * (G + 1) + o];
      po[i] = o < G ? b.roff[(size_t)s * G + o] : 0u;
    }
    __syncthreads();
    if (do_push) push_walk<kXbVZ, 0>(g.r, b.rb, X, acc, wmask, wlist, split ? nwav / 2 : 0u);
    if (do_pull) {  // replies, in send order: region s's items are G runs (one per owner)
      const uint32_t qtid = tid - qt0;
      for (uint32_t s = s0; s < s1; ++s) {
        const uint32_t* rl = pl + (s - s0) * (G + 1);
        const uint32_t* ro = po + (s - s0) * (G + 1);
        const uint32_t total = rl[G];
        const uint32_t nb = (s - s0) << g.s.ts_log;
        for (uint32_t f0 = 0; f0 < total; f0 += qnt * kUnrollXd) {
          uint64_t rv[kUnrollXd];
          uint32_t nl[kUnrollXd];
#pragma unroll
          for (int u = 0; u < kUnrollXd; ++u) {
            const uint32_t f = min(f0 + u * qnt + qtid, total - 1);
            uint32_t lo = 0, hi = G;  // f's owner run
            while (hi - lo > 1) {
              const uint32_t mid = (lo + hi) >> 1;
              if (rl[mid] <= f) lo = mid;
              else hi = mid;
            }
            const size_t pos = (size_t)ro[lo] + (f - rl[lo]);
            rv[u] = *(&b.rep_in[pos]);
            nl[u] = b.snl[pos];
          }
#pragma unroll
          for (int u = 0; u < kUnrollXd; ++u) {
            if (f0 + u * qnt + qtid >= total) continue;
            const uint32_t node = nb + nl[u];
            if (rv[u]) atomicOr(&acc[node], (unsigned long long)rv[u]);
          }
        }
      }
    }
    __syncthreads();
    tile_epilogue(acc, node0, g.nown, g.lo, Snext, partial, R, flags, cnt, red_hash, red_full, red_nz, nzb, fullb,
                  btot);
  }
  block_totals_flush(partial, R, cnt, btot);
}

}  // namespace

bool xd_path_ok(uint64_t N, uint32_t k, uint64_t Nl, uint32_t G) {
  if (G < 2 || G > kXdMaxG || k == 0 || k > 64 || N < 2 || Nl >= (1ull << 30) || N > 0xFFFFFFFFull) return false;
  const BinGeom s = make_bin_geom(Nl, k);
  const uint32_t per = kTileD >> s.ts_log;
  // apply's prefix rows; tiles of one shard; send positions and record indices fit u32 / int32
  return (uint64_t)per * (G + 1) <= kXdPref && (Nl + kTileD - 1) / kTileD <= kSbMaxTiles &&
         (uint64_t)k * Nl < (1ull << 31);
}

XdGeom make_xd_geom(uint64_t N, uint32_t k, uint64_t Nl, uint64_t lo, uint64_t nown, uint32_t G, uint32_t rank) {
  XdGeom g{};
  g.N = N;
  g.Nl = Nl;
  g.lo = lo;
  g.nown = nown;
  g.G = G;
  g.rank = rank;
  g.k = k;
  g.s = make_bin_geom(nown ? nown : 1, k);
  g.s.split = 0u;  // exchange items keep u32 ids (p_local | slot << 14 | flags)
  g.s.aos = 0u;
  while (g.s.ts > 64 && g.s.ts * k > kXdSendRegion) {
    g.s.ts >>= 1;
    --g.s.ts_log;
  }
  g.s.rp = g.s.ts * k;
  g.s.nt_s = (uint32_t)(((nown ? nown : 1) + g.s.ts - 1) / g.s.ts);
  g.r = g.s;
  g.r.N = nown;
  g.r.ts = kXdBinRegion;
  g.r.ts_log = 31 - __builtin_clz(kXdBinRegion);
  g.r.rp = kXdBinRegion;
  g.r.nt_s = 0;  // set per round from the received count
  return g;
}

uint64_t xd_send_cap(const XdGeom& g) { return (uint64_t)g.k * g.nown; }

namespace {
size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

size_t xd_send_bytes(const XdGeom& g) {
  const size_t cap = xd_send_cap(g) + 1, tab = (size_t)g.s.nt_s * g.G;
  return 2 * al256(tab * 4) + al256((tab + g.s.nt_s) * 4) + al256(g.G * 4) + al256(cap * 4) + al256(cap * 8) +
         al256(cap * 2) + al256(cap * 8);
}

void xd_carve_send(const XdGeom& g, void* base, XdBufs* b) {
  const size_t cap = xd_send_cap(g) + 1, tab = (size_t)g.s.nt_s * g.G;
  char* p = (char*)base;
  auto take = [&](size_t bytes) {
    char* r = p;
    p += al256(bytes);
    return r;
  };
  b->rcnt = (uint32_t*)take(tab * 4);
  b->roff = (uint32_t*)take(tab * 4);
  b->rlofs = (uint32_t*)take((tab + g.s.nt_s) * 4);
  b->ocnt = (uint32_t*)take(g.G * 4);
  b->sid = (uint32_t*)take(cap * 4);
  b->sval = (uint64_t*)take(cap * 8);
  b->snl = (uint16_t*)take(cap * 2);
  b->rep_in = (uint64_t*)take(cap * 8);
}

namespace {
uint32_t xd_regions(uint64_t cap_r) { return (uint32_t)((cap_r + kXdBinRegion - 1) / kXdBinRegion); }
}  // namespace

size_t xd_recv_bytes(const XdGeom& g, uint64_t cap_r) {
  const uint32_t nr = xd_regions(cap_r) ? xd_regions(cap_r) : 1;
  const size_t recs = (size_t)nr * kXdBinRegion, offs = (size_t)nr * (g.r.nt_d + 1);
  return al256(recs * 4) + al256(recs * 8) + al256(recs * 4) + 3 * al256(recs * 8) + 2 * al256(offs * 2);
}

void xd_carve_recv(const XdGeom& g, uint64_t cap_r, void* base, XdBufs* b) {
  const uint32_t nr = xd_regions(cap_r) ? xd_regions(cap_r) : 1;
  const size_t recs = (size_t)nr * kXdBinRegion, offs = (size_t)nr * (g.r.nt_d + 1);
  char* p = (char*)base;
  auto take = [&](size_t bytes) {
    char* r = p;
    p += al256(bytes);
    return r;
  };
  b->rid = (uint32_t*)take(recs * 4);
  b->rval = (uint64_t*)take(recs * 8);
  b->rb.ids = (uint32_t*)take(recs * 4);
  b->rb.vals = (uint64_t*)take(recs * 8);
  b->rb.resp = (uint64_t*)take(recs * 8);
  b->rep_out = (uint64_t*)take(recs * 8);
  b->rb.off = (uint16_t*)take(offs * 2);
  b->rb.offT = (uint16_t*)take(offs * 2);
  b->rb.nzb = b->rb.fullb = nullptr;
  b->rb.dyn = nullptr;
}

hipError_t launch_xd_requests(const XdGeom& g, const XdBufs& b, const uint64_t* S, uint32_t R, uint32_t t,
                              uint32_t key0, uint32_t key1, uint32_t mode, const Faults& fa, const XdFilter& xf,
                              hipStream_t st) {
  if (g.nown == 0) return hipMemsetAsync(b.ocnt, 0, g.G * 4, st);
  const uint32_t eg = g.s.nt_s < kEmitGrid ? g.s.nt_s : kEmitGrid;
  // (count: 1024 blocks instead of one per CU took the same time, profiles/r02_xd/variants3)
  if (fa.any()) xd_count_kernel<true><<<eg, kEmitThreads, 0, st>>>(g, S, b.rcnt, R, t, key0, key1, mode, fa, xf);
  else xd_count_kernel<false><<<eg, kEmitThreads, 0, st>>>(g, S, b.rcnt, R, t, key0, key1, mode, fa, xf);
  xd_scan_kernel<<<g.G, 1024, 0, st>>>(b.rcnt, b.roff, b.ocnt, g.s.nt_s, g.G);
  if (fa.any()) xd_emit_kernel<true><<<eg, kEmitThreads, 0, st>>>(g, S, b, b.rlofs, R, t, key0, key1, mode, fa, xf);
  else xd_emit_kernel<false><<<eg, kEmitThreads, 0, st>>>(g, S, b, b.rlofs, R, t, key0, key1, mode, fa, xf);
  return hipGetLastError();
}

hipError_t launch_xd_serve(XdGeom g, const XdBufs& b, const uint64_t* S, uint64_t n_in, uint32_t R,
                           hipStream_t st) {
  g.r.nt_s = xd_regions(n_in);
  if (g.r.nt_s == 0) return hipSuccess;
  const uint32_t eg = g.r.nt_s < kEmitGrid ? g.r.nt_s : kEmitGrid;
  xd_bin_kernel<<<eg, kEmitThreads, 0, st>>>(g, b, n_in);
  launch_transpose_u16(b.rb.off, b.rb.offT, g.r.nt_s, g.r.nt_d + 1, nullptr, 0u, st);
  bin_serve_kernel<kXbVF><<<serve_grid(g.r.nt_d), kTileThreads, 0, st>>>(g.r, S, b.rb, R, IdxRange::all(g.r.nt_d));
  // replies back to the received order in LDS (writing them there from serve, scattered,
  // measured 4x slower: profiles/r02_xd)
  xd_unperm_kernel<<<eg, kEmitThreads, 0, st>>>(g, b, n_in);
  return hipGetLastError();
}

hipError_t launch_xd_apply(XdGeom g, const XdBufs& b, const uint64_t* S, uint64_t* Snext, uint64_t n_in,
                           uint64_t* partial, uint32_t R, uint32_t mode, uint32_t flags, uint64_t* nzb,
                           uint64_t* fullb, hipStream_t st) {
  if (g.nown == 0) return hipSuccess;
  g.r.nt_s = xd_regions(n_in);
  const uint32_t grid = g.r.nt_d < kApplyGrid ? g.r.nt_d : kApplyGrid;
  xd_apply_kernel<<<grid, kTileThreads, 0, st>>>(g, b, b.rlofs, S, Snext, partial, R, mode, flags, nzb, fullb);
  return hipGetLastError();
}

}  // namespace gossip
