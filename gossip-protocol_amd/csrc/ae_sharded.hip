// ae_sharded.hip — anti-entropy (configs[4]) with the rows sharded by node id over G
// engines: SURVEY.md §8(e) "Design B" — all-to-all of request buckets (the pushed
// row) and reply buckets (the pulled row), max-merge on the owner; the global max
// vector by an all-reduce MAX (ncclMax) of the shards' maxima.
//
// Reference: (*NodeState).Gossip, main.go:65-89 — here each exchange of the round
// model is one SyncRPC-shaped request/reply between the two ends'
// owners.  Every shard receives every shard's alive bits (its churn: ae_churn_word, a
// per-node Philox draw) and stale bits (row != target) each round, one 16-B word pair per 64 nodes:
// an exchange between two rows equal to the target moves nothing, so only exchanges with
// a stale end travel.
#include "ae_sharded.h"

#include <algorithm>
#include <type_traits>

#include "philox.h"
#include "wave.h"

namespace gossip {

namespace {

constexpr int kAxBlock = 256;
constexpr uint32_t kAxStatsGrid = 1024;  // stats blocks (256 / 8192: slower)
constexpr uint32_t kAxMaxG = 1024;

// {alive, stale} word pair of the 64 nodes around global node n (one 16-B load)
__device__ __forceinline__ uint4 pair_of(const uint64_t* img, uint64_t n) { return ((const uint4*)img)[n >> 6]; }
__device__ __forceinline__ bool alive_in(const uint4& w, uint64_t n) {
  return (((n & 63) < 32 ? w.x >> (n & 31) : w.y >> (n & 31)) & 1u) != 0;
}
__device__ __forceinline__ bool stale_in(const uint4& w, uint64_t n) {
  return (((n & 63) < 32 ? w.z >> (n & 31) : w.w >> (n & 31)) & 1u) != 0;
}

// the own nodes' churn of round t: alive words of the own slot, round t - 1 -> t, in place
__global__ __launch_bounds__(kAxBlock) void aex_churn_kernel(AexArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t chunks = (a.nown + 63) / 64, w0 = a.lo / 64;
  for (uint64_t ch = (uint64_t)blockIdx.x * (kAxBlock / 64) + (threadIdx.x >> 6); ch < chunks;
       ch += (uint64_t)gridDim.x * (kAxBlock / 64)) {
    const uint64_t w = w0 + ch, n = w * 64 + lane;
    bool al = false;
    if (ch * 64 + lane < a.nown) {
      const bool was = (a.img[2 * w] >> lane) & 1ull;
      const u32x4 x0 = ae_first_draw((uint32_t)n, a.t, a.k, a.key0, a.key1);
      const uint32_t x = ae_churn_word(x0, (uint32_t)n, a.t, a.k, a.key0, a.key1);
      al = was ? !(x < a.fail) : (x < a.rec);
    }
    const uint64_t b = __ballot(al);
    if (lane == 0) a.img[2 * w] = b;
  }
}

// Node range of block b (contiguous, so the fill pass reproduces the count pass's
// per-block counts exactly).
__device__ __forceinline__ void block_range(const AexArgs& a, uint64_t* i0, uint64_t* i1) {
  const uint64_t per = (a.nown + gridDim.x - 1) / gridDim.x;
  *i0 = min<uint64_t>((uint64_t)blockIdx.x * per, a.nown);
  *i1 = min<uint64_t>(*i0 + per, a.nown);
}

// FILL = false: per-block item counts per owner (+ own-own exchanges in slot G) into
// bcnt[b][G + 1] and the messages into partial[2].  FILL = true: the same walk, items
// written at boff[b][q] + LDS cursor (request items {p, n, row[K]}, own-own pairs).
template <bool FILL>
__global__ __launch_bounds__(kAxBlock) void aex_list_kernel(AexArgs a, uint32_t* bcnt, const uint64_t* boff) {
  constexpr uint32_t kStage = kAxBlock * 8;  // items one pass of the block lists at most (k <= 8)
  __shared__ uint32_t c[kAxMaxG + 1];
  __shared__ uint64_t red[kAxBlock / 64];
  __shared__ uint32_t st_at[FILL ? kStage : 1], st_i[FILL ? kStage : 1], st_p[FILL ? kStage : 1];
  __shared__ uint32_t st_n;
  for (uint32_t q = threadIdx.x; q <= a.G; q += kAxBlock) c[q] = 0;
  if (threadIdx.x == 0) st_n = 0;
  __syncthreads();
  uint64_t i0, i1;
  block_range(a, &i0, &i1);
  const uint64_t nm1 = a.N - 1;
  uint64_t msgs = 0;
  // k <= 8: the count pass leaves each node's listed exchanges in a verdict byte, and the fill
  // pass redraws only the peers of nodes that list one (late rounds: a few thousand); the
  // request items it lists are staged in LDS and their rows copied by L lanes per item
  // (coalesced 4K-byte rows: a lane per item reading its own row was 1.4 ms of a G = 8 round)
  const bool verdicts = a.k <= 8;
  for (uint64_t b0 = i0; b0 < i1; b0 += kAxBlock) {  // block-uniform trip count (the staging barriers)
    const uint64_t i = b0 + threadIdx.x;
    const uint64_t n = a.lo + i;
    uint32_t vb = 0;
    bool sn = false, go = i < i1;
    if (go && FILL && verdicts) {
      vb = a.verdict[i];
      go = vb != 0;
    } else if (go) {
      const uint4 wn = pair_of(a.img, n);
      if (!alive_in(wn, n)) {
        if (!FILL && verdicts) a.verdict[i] = 0;
        go = false;
      }
      sn = go && stale_in(wn, n);
    }
    if (go) {
      u32x4 x{0, 0, 0, 0};
      uint32_t listed = 0;
      for (uint32_t j = 0; j < a.k; ++j) {
        if ((j & 3u) == 0) x = philox4x32_10(u32x4{(uint32_t)n, a.t, 0u, j >> 2}, a.key0, a.key1);
        const uint32_t p = peer_from_word(lane_of(x, j & 3u), nm1, (uint32_t)n);
        if (FILL && verdicts) {
          if (!((vb >> j) & 1u)) continue;
        } else {
          const uint4 wp = pair_of(a.img, p);
          if (!alive_in(wp, p)) continue;
          ++msgs;
          if (!sn && !stale_in(wp, p)) continue;  // two target rows: nothing moves
          listed |= 1u << j;
        }
        const uint32_t q = (uint32_t)(p / a.Nl);
        const uint32_t slot = q == a.rank ? a.G : q;
        const uint32_t pos = atomicAdd(&c[slot], 1u);
        if (!FILL) continue;
        const uint64_t at = boff[(uint64_t)blockIdx.x * (a.G + 1) + slot] + pos;
        if (slot == a.G) {
          a.loc[2 * at] = (uint32_t)i;
          a.loc[2 * at + 1] = (uint32_t)(p - a.lo);
        } else if (verdicts) {
          const uint32_t e = atomicAdd(&st_n, 1u);
          st_at[e] = (uint32_t)at;
          st_i[e] = (uint32_t)i;
          st_p[e] = p;
        } else {
          uint32_t* it = a.req + at * a.rw;
          it[0] = p;
          it[1] = (uint32_t)n;
          const uint32_t* row = a.V + i * a.K;
          for (uint32_t cc = 0; cc < a.K; ++cc) it[2 + cc] = row[cc];
        }
      }
      if (!FILL && verdicts) a.verdict[i] = (uint8_t)listed;
    }
    if (FILL && verdicts) {
      __syncthreads();
      const uint32_t m = st_n, L = a.L, per = kAxBlock / L, cc = threadIdx.x % L;
      for (uint32_t e = threadIdx.x / L; e < m; e += per) {
        uint32_t* it = a.req + (uint64_t)st_at[e] * a.rw;
        const uint32_t il = st_i[e];
        if (cc < a.K) it[2 + cc] = a.V[(uint64_t)il * a.K + cc];
        if (cc == 0) {
          it[0] = st_p[e];
          it[1] = (uint32_t)(a.lo + il);
        }
      }
      __syncthreads();  // every copy has read st_n and the stage
      if (threadIdx.x == 0) st_n = 0;
      __syncthreads();  // the next pass stages after the reset
    }
  }
  __syncthreads();
  if (!FILL) {
    for (uint32_t q = threadIdx.x; q <= a.G; q += kAxBlock) bcnt[(uint64_t)blockIdx.x * (a.G + 1) + q] = c[q];
    msgs = wave_sum64(msgs);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = msgs;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t s = 0;
      for (int w = 0; w < kAxBlock / 64; ++w) s += red[w];
      if (s) atomicAdd((unsigned long long*)&a.partial[2], (unsigned long long)s);
    }
  }
}

// One block per slot q (owners 0..G-1, then G = own-own): exclusive scan of the
// per-block counts; requests are laid out by owner (cnt[q] items from base[q]),
// the own-own list from 0.
__global__ __launch_bounds__(kAxBlock) void aex_scan_kernel(AexArgs a, const uint32_t* bcnt, uint64_t* boff,
                                                            uint32_t nblocks) {
  const uint32_t q = blockIdx.x;
  __shared__ uint64_t tot[kAxBlock / 64];
  __shared__ uint64_t qbase;
  if (threadIdx.x == 0) {
    uint64_t b = 0;  // owner q's requests start after those of owners < q
    if (q < a.G)
      for (uint32_t r = 0; r < q; ++r) b += a.cnt[r];
    qbase = b;
  }
  __syncthreads();
  // serial over chunks of the block list, a wave scan each (nblocks is a few thousand at most)
  uint64_t run = qbase;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t b0 = 0; b0 < nblocks; b0 += kAxBlock) {
    const uint32_t b = b0 + threadIdx.x;
    const uint64_t v = b < nblocks ? bcnt[(uint64_t)b * (a.G + 1) + q] : 0;
    uint64_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) tot[wave] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (int w = 0; w < kAxBlock / 64; ++w) {
      before += w < (int)wave ? tot[w] : 0;
      all += tot[w];
    }
    if (b < nblocks) boff[(uint64_t)b * (a.G + 1) + q] = run + before + inc - v;
    run += all;
    __syncthreads();
  }
}

// per-owner totals from the per-block counts (cnt[q], q <= G)
__global__ __launch_bounds__(kAxBlock) void aex_total_kernel(AexArgs a, const uint32_t* bcnt, uint32_t nblocks) {
  const uint32_t q = blockIdx.x;
  uint64_t s = 0;
  for (uint32_t b = threadIdx.x; b < nblocks; b += kAxBlock) s += bcnt[(uint64_t)b * (a.G + 1) + q];
  __shared__ uint64_t red[kAxBlock / 64];
  s = wave_sum64(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kAxBlock / 64; ++w) t += red[w];
    a.cnt[q] = t;
  }
}

// requests received: lanes = components of one item; max-merge the pushed row into
// Vn[p] (only where it is larger than S_t: Vn >= S_t throughout), answer S_t[p]
// Marks own row i of Vn raised above S_t (the next round's patch copies it, launch_aex_seed_next).
// (dirty = null: not tracked this round — many rows change, the next round copies them all)
__device__ __forceinline__ void mark_dirty(const AexArgs& a, uint64_t i) {
  if (a.dirty) atomicOr((unsigned long long*)&a.dirty[i >> 6], 1ull << (i & 63));
}

__global__ __launch_bounds__(kAxBlock) void aex_serve_kernel(AexArgs a, const uint32_t* __restrict__ in, uint64_t m,
                                                             uint32_t* __restrict__ resp) {
  const uint32_t per = kAxBlock / a.L, c = threadIdx.x % a.L;
  for (uint64_t it = (uint64_t)blockIdx.x * per + threadIdx.x / a.L; it < m; it += (uint64_t)gridDim.x * per) {
    if (c >= a.K) continue;
    const uint64_t pl = in[it * a.rw] - a.lo;
    const uint32_t vp = a.V[pl * a.K + c];
    resp[it * a.pw + c] = vp;
    const uint32_t rv = in[it * a.rw + 2 + c];
    if (rv > vp) {
      atomicMax(&a.Vn[pl * a.K + c], rv);
      mark_dirty(a, pl);
    }
  }
}

// the replies to the own requests (request order) and the own-own exchanges
__global__ __launch_bounds__(kAxBlock) void aex_merge_kernel(AexArgs a, const uint32_t* __restrict__ resp,
                                                             uint64_t nreq, uint64_t nloc) {
  const uint32_t per = kAxBlock / a.L, c = threadIdx.x % a.L;
  for (uint64_t it = (uint64_t)blockIdx.x * per + threadIdx.x / a.L; it < nreq + nloc;
       it += (uint64_t)gridDim.x * per) {
    if (c >= a.K) continue;
    if (it < nreq) {
      const uint64_t nl = a.req[it * a.rw + 1] - a.lo;
      const uint32_t rv = resp[it * a.pw + c];
      if (rv > a.V[nl * a.K + c]) {
        atomicMax(&a.Vn[nl * a.K + c], rv);
        mark_dirty(a, nl);
      }
    } else {
      const uint64_t e = it - nreq;
      const uint64_t nl = a.loc[2 * e], pl = a.loc[2 * e + 1];
      const uint32_t vn = a.V[nl * a.K + c], vp = a.V[pl * a.K + c];
      if (vp > vn) {
        atomicMax(&a.Vn[nl * a.K + c], vp);
        mark_dirty(a, nl);
      }
      if (vn > vp) {
        atomicMax(&a.Vn[pl * a.K + c], vn);
        mark_dirty(a, pl);
      }
    }
  }
}

// Stats of the own rows R (S_{t+1}) with the alive bits after the churn: full, alive,
// per-component counts, hash (global ids, every node as on one shard), and the own stale
// words (STATS = false: the stale words only).  One wave per 64 own nodes (lo is 64-aligned:
// the chunk is one word of the global bitmaps); lane (sub, c) holds component c of nodes
// sub*L .. sub*L+L-1, one per sub-step, so every row load is a coalesced 4K-byte row and a
// group's "differs" bits OR-reduce across its L lanes (antientropy.hip ae_stats_kernel).
template <uint32_t L, bool STATS>
__global__ __launch_bounds__(kAxBlock) void aex_stats_kernel(AexArgs a, const uint32_t* __restrict__ R) {
  using BT = typename std::conditional<(L > 32), uint64_t, uint32_t>::type;
  constexpr uint32_t per = 64 / L;
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red[3][kAxBlock / 64];
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, sub = lane / L, c = lane % L;
  const uint32_t tgt = c < a.K ? a.target[c] : 0u;
  const uint64_t chunks = (a.nown + 63) / 64;
  uint64_t hash = 0, full = 0, nal = 0;
  uint32_t c_lane = 0;
  for (uint64_t ch = (uint64_t)blockIdx.x * (kAxBlock / 64) + (threadIdx.x >> 6); ch < chunks;
       ch += (uint64_t)gridDim.x * (kAxBlock / 64)) {
    uint32_t v[L];
#pragma unroll
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t il = ch * 64 + sub * L + i;
      v[i] = (il < a.nown && c < a.K) ? R[il * a.K + c] : 0u;
    }
    const uint64_t aw = a.img[2 * (a.lo / 64 + ch)];  // (nodes past nown: not alive, no row)
    BT bad = 0;
    uint64_t hb = ((uint64_t)c * a.N + a.lo + ch * 64 + sub * L) * kGold64;  // stepped by kGold64 per node
#pragma unroll
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t il = ch * 64 + sub * L + i;
      const bool valid = il < a.nown && c < a.K;
      const bool al = (aw >> (sub * L + i)) & 1ull;
      if (STATS && (a.flags & 1u)) hash += valid && v[i] ? mix64((uint64_t)v[i] + hb) : 0ull;
      hb += kGold64;
      if (STATS) c_lane += (valid && al && v[i] == tgt) ? 1u : 0u;
      bad |= (BT)(valid && v[i] != tgt) << i;
    }
#pragma unroll
    for (uint32_t off = 1; off < L; off <<= 1) bad |= (BT)__shfl_xor(bad, (int)off, 64);
    uint64_t stale = 0;
    if (per <= L) {
#pragma unroll
      for (uint32_t g = 0; g < per; ++g) stale |= (uint64_t)__shfl(bad, (int)(g * L), 64) << (g * L);
    } else {
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) stale |= __ballot(c == 0 && ((bad >> i) & 1u)) << i;
    }
    if (lane == 0 && a.write_stale) a.img[2 * (a.lo / 64 + ch) + 1] = stale;
    if (STATS) {
      full += (uint64_t)__popcll(aw & ~stale);
      nal += (uint64_t)__popcll(aw);
    }
  }
  if (!STATS) return;
  if (c < a.K && c_lane) atomicAdd(&cnt[c], c_lane);
  if (lane != 0) full = nal = 0;  // wave-uniform: counted once per wave
  hash = wave_sum64(hash);
  full = wave_sum64(full);
  nal = wave_sum64(nal);
  if (lane == 0) {
    red[0][threadIdx.x >> 6] = hash;
    red[1][threadIdx.x >> 6] = full;
    red[2][threadIdx.x >> 6] = nal;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    uint64_t sum = 0;
    for (int w = 0; w < kAxBlock / 64; ++w) sum += red[threadIdx.x][w];
    const uint32_t slot = threadIdx.x == 0 ? 3u : threadIdx.x == 1 ? 0u : 1u;
    if (sum) atomicAdd((unsigned long long*)&a.partial[slot], (unsigned long long)sum);
  }
  if (threadIdx.x < a.K && cnt[threadIdx.x])
    atomicAdd((unsigned long long*)&a.partial[4 + threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

// Incremental stats of a round that tracked its raised rows: only dirty rows can
// differ between S_t (V) and S_{t+1} (Vn), so their stale bits are recomputed and their hash terms
// swapped (partial[3] gets the delta); full / alive from the bitmaps; per-component counts = the
// alive non-stale nodes plus the matching components of the alive stale rows (few in such rounds).
// One wave per own chunk, lanes as in aex_stats_kernel.
template <uint32_t L>
__global__ __launch_bounds__(kAxBlock) void aex_stats_inc_kernel(AexArgs a) {
  using BT = typename std::conditional<(L > 32), uint64_t, uint32_t>::type;
  constexpr uint32_t per = 64 / L;
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red[4][kAxBlock / 64];
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, sub = lane / L, c = lane % L;
  const uint32_t tgt = c < a.K ? a.target[c] : 0u;
  const uint64_t chunks = (a.nown + 63) / 64;
  uint64_t dhash = 0, full = 0, nal = 0, fullw = 0;
  uint32_t c_lane = 0;
  for (uint64_t ch = (uint64_t)blockIdx.x * (kAxBlock / 64) + (threadIdx.x >> 6); ch < chunks;
       ch += (uint64_t)gridDim.x * (kAxBlock / 64)) {
    uint64_t* pw = a.img + 2 * (a.lo / 64 + ch);
    const uint64_t aw = pw[0], dw = a.dirty[ch];
    uint64_t sw = pw[1];
    if (dw) {  // the raised rows: stale bits of S_{t+1}, hash terms old -> new
      BT bad = 0;
      uint64_t hb = ((uint64_t)c * a.N + a.lo + ch * 64 + sub * L) * kGold64;
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) {
        const uint32_t b = sub * L + i;
        if (((dw >> b) & 1ull) && c < a.K) {
          const uint64_t il = ch * 64 + b;
          const uint32_t vn = a.Vn[il * a.K + c], vo = a.V[il * a.K + c];
          if (a.flags & 1u) dhash += (vn ? mix64((uint64_t)vn + hb) : 0ull) - (vo ? mix64((uint64_t)vo + hb) : 0ull);
          bad |= (BT)(vn != tgt) << i;
        }
        hb += kGold64;
      }
#pragma unroll
      for (uint32_t off = 1; off < L; off <<= 1) bad |= (BT)__shfl_xor(bad, (int)off, 64);
      uint64_t st = 0;
      if (per <= L) {
#pragma unroll
        for (uint32_t g = 0; g < per; ++g) st |= (uint64_t)__shfl(bad, (int)(g * L), 64) << (g * L);
      } else {
#pragma unroll
        for (uint32_t i = 0; i < L; ++i) st |= __ballot(c == 0 && ((bad >> i) & 1u)) << i;
      }
      sw = (sw & ~dw) | (st & dw);
      if (lane == 0) pw[1] = sw;
    }
    const uint64_t as = aw & sw;
    fullw += (uint64_t)__popcll(aw & ~sw);
    if (as) {  // alive stale rows: their components that match the target
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) {
        const uint32_t b = sub * L + i;
        if (((as >> b) & 1ull) && c < a.K) c_lane += a.Vn[(ch * 64 + b) * a.K + c] == tgt ? 1u : 0u;
      }
    }
    nal += (uint64_t)__popcll(aw);
  }
  full = fullw;
  if (c < a.K && c_lane) atomicAdd(&cnt[c], c_lane);
  if (lane != 0) full = nal = fullw = 0;  // wave-uniform: counted once per wave
  dhash = wave_sum64(dhash);
  full = wave_sum64(full);
  nal = wave_sum64(nal);
  if (lane == 0) {
    red[0][threadIdx.x >> 6] = dhash;
    red[1][threadIdx.x >> 6] = full;
    red[2][threadIdx.x >> 6] = nal;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    uint64_t sum = 0;
    for (int w = 0; w < kAxBlock / 64; ++w) sum += red[threadIdx.x][w];
    const uint32_t slot = threadIdx.x == 0 ? 3u : threadIdx.x == 1 ? 0u : 1u;
    if (sum) atomicAdd((unsigned long long*)&a.partial[slot], (unsigned long long)sum);
  }
  __syncthreads();
  // every alive non-stale node matches the target in every component
  if (threadIdx.x < a.K) {
    uint64_t f = 0;
    for (int w = 0; w < kAxBlock / 64; ++w) f += red[1][w];
    const uint64_t add = f + cnt[threadIdx.x];
    if (add) atomicAdd((unsigned long long*)&a.partial[4 + threadIdx.x], (unsigned long long)add);
  }
}

// Vn rows the previous round raised (dirty) := V rows, dirty cleared: one wave per 64 rows,
// lanes as in the stats pass (coalesced rows); clean words cost one load.
template <uint32_t L>
__global__ __launch_bounds__(kAxBlock) void aex_patch_kernel(AexArgs a) {
  constexpr uint32_t per = 64 / L;
  const uint32_t lane = threadIdx.x & 63, sub = lane / L, c = lane % L;
  const uint64_t chunks = (a.nown + 63) / 64;
  for (uint64_t ch = (uint64_t)blockIdx.x * (kAxBlock / 64) + (threadIdx.x >> 6); ch < chunks;
       ch += (uint64_t)gridDim.x * (kAxBlock / 64)) {
    const uint64_t dw = a.dirty[ch];
    if (!dw) continue;
#pragma unroll
    for (uint32_t i = 0; i < L; ++i) {
      const uint32_t b = sub * L + i;
      const uint64_t il = ch * 64 + b;
      if (((dw >> b) & 1ull) && c < a.K) a.Vn[il * a.K + c] = a.V[il * a.K + c];
    }
    if (lane == 0) a.dirty[ch] = 0;
  }
  (void)per;
}

__global__ __launch_bounds__(kAxBlock) void aex_init_kernel(uint32_t* V, uint64_t lo, uint64_t nown, uint32_t K,
                                                            uint32_t k0, uint32_t k1) {
  const uint32_t c4 = (K + 3) / 4;
  for (uint64_t x = (uint64_t)blockIdx.x * kAxBlock + threadIdx.x; x < nown * c4; x += (uint64_t)gridDim.x * kAxBlock) {
    const uint64_t i = x / c4;
    const uint32_t q = (uint32_t)(x % c4);
    const u32x4 r = philox4x32_10(u32x4{(uint32_t)(lo + i), q, 3u, 0u}, k0, k1);
    for (uint32_t s = 0; s < 4 && 4 * q + s < K; ++s) V[i * K + 4 * q + s] = lane_of(r, s) & 0xFFFFu;
  }
}

__global__ __launch_bounds__(kAxBlock) void aex_fill_alive_kernel(AexArgs a) {
  const uint64_t chunks = (a.nown + 63) / 64, w0 = a.lo / 64;
  for (uint64_t ch = (uint64_t)blockIdx.x * kAxBlock + threadIdx.x; ch < chunks; ch += (uint64_t)gridDim.x * kAxBlock) {
    const uint64_t left = a.nown - ch * 64;
    a.img[2 * (w0 + ch)] = left >= 64 ? ~0ull : (1ull << left) - 1ull;
  }
}

__global__ __launch_bounds__(kAxBlock) void aex_max_kernel(const uint32_t* V, uint64_t nown, uint32_t K, uint32_t* out) {
  __shared__ uint32_t m[64];
  if (threadIdx.x < 64) m[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t x = (uint64_t)blockIdx.x * kAxBlock + threadIdx.x; x < nown * K; x += (uint64_t)gridDim.x * kAxBlock)
    atomicMax(&m[x % K], V[x]);
  __syncthreads();
  if (threadIdx.x < K && m[threadIdx.x]) atomicMax(&out[threadIdx.x], m[threadIdx.x]);
}

uint32_t ax_grid(uint64_t units, uint32_t per_block, uint32_t cap) {
  const uint64_t b = (units + per_block - 1) / per_block;
  return (uint32_t)(b == 0 ? 1 : (b < cap ? b : cap));
}

uint32_t list_blocks(uint64_t nown) { return ax_grid(nown, 4 * kAxBlock, 2048); }

}  // namespace

size_t aex_block_table_words(uint64_t nown, uint32_t G) { return (size_t)list_blocks(nown) * (G + 1); }

hipError_t launch_aex_churn(const AexArgs& a, hipStream_t st) {
  if (a.nown == 0) return hipSuccess;
  aex_churn_kernel<<<ax_grid((a.nown + 63) / 64, kAxBlock / 64, 8192), kAxBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_aex_requests(const AexArgs& a, hipStream_t st) {
  if (a.G > kAxMaxG) return hipErrorInvalidValue;
  const uint32_t nb = list_blocks(a.nown);
  uint32_t* bcnt = a.bcnt;
  uint64_t* boff = a.boff;
  aex_list_kernel<false><<<nb, kAxBlock, 0, st>>>(a, bcnt, nullptr);
  aex_total_kernel<<<a.G + 1, kAxBlock, 0, st>>>(a, bcnt, nb);
  aex_scan_kernel<<<a.G + 1, kAxBlock, 0, st>>>(a, bcnt, boff, nb);
  aex_list_kernel<true><<<nb, kAxBlock, 0, st>>>(a, bcnt, boff);
  return hipGetLastError();
}

hipError_t launch_aex_serve(const AexArgs& a, const uint32_t* in, uint64_t m, uint32_t* resp, hipStream_t st) {
  if (m == 0) return hipSuccess;
  aex_serve_kernel<<<ax_grid(m, kAxBlock / a.L, 65536), kAxBlock, 0, st>>>(a, in, m, resp);
  return hipGetLastError();
}

namespace {
template <bool STATS>
void stats_l(const AexArgs& a, const uint32_t* R, hipStream_t st) {
  // 1024 blocks (each wave walks ~32 chunks): every block ends in ~20 same-address atomics on
  // the partials, which at 8192 blocks cost as much as the rows (2^23 rows: 157 us min)
  const uint32_t g = ax_grid((a.nown + 63) / 64, kAxBlock / 64, kAxStatsGrid);
  switch (a.L) {
    case 1: aex_stats_kernel<1, STATS><<<g, kAxBlock, 0, st>>>(a, R); break;
    case 2: aex_stats_kernel<2, STATS><<<g, kAxBlock, 0, st>>>(a, R); break;
    case 4: aex_stats_kernel<4, STATS><<<g, kAxBlock, 0, st>>>(a, R); break;
    case 8: aex_stats_kernel<8, STATS><<<g, kAxBlock, 0, st>>>(a, R); break;
    case 16: aex_stats_kernel<16, STATS><<<g, kAxBlock, 0, st>>>(a, R); break;
    case 32: aex_stats_kernel<32, STATS><<<g, kAxBlock, 0, st>>>(a, R); break;
    default: aex_stats_kernel<64, STATS><<<g, kAxBlock, 0, st>>>(a, R); break;
  }
}
}  // namespace

hipError_t launch_aex_finish(const AexArgs& a, const uint32_t* resp, uint64_t nreq, uint64_t nloc, bool inc,
                             hipStream_t st) {
  if (nreq + nloc)
    aex_merge_kernel<<<ax_grid(nreq + nloc, kAxBlock / a.L, 65536), kAxBlock, 0, st>>>(a, resp, nreq, nloc);
  if (!inc || !a.dirty) {
    stats_l<true>(a, a.Vn, st);
    return hipGetLastError();
  }
  const uint32_t g = ax_grid((a.nown + 63) / 64, kAxBlock / 64, kAxStatsGrid);
  switch (a.L) {
    case 1: aex_stats_inc_kernel<1><<<g, kAxBlock, 0, st>>>(a); break;
    case 2: aex_stats_inc_kernel<2><<<g, kAxBlock, 0, st>>>(a); break;
    case 4: aex_stats_inc_kernel<4><<<g, kAxBlock, 0, st>>>(a); break;
    case 8: aex_stats_inc_kernel<8><<<g, kAxBlock, 0, st>>>(a); break;
    case 16: aex_stats_inc_kernel<16><<<g, kAxBlock, 0, st>>>(a); break;
    case 32: aex_stats_inc_kernel<32><<<g, kAxBlock, 0, st>>>(a); break;
    default: aex_stats_inc_kernel<64><<<g, kAxBlock, 0, st>>>(a); break;
  }
  return hipGetLastError();
}

hipError_t launch_aex_stale(const AexArgs& a, const uint32_t* V, hipStream_t st) {
  stats_l<false>(a, V, st);
  return hipGetLastError();
}

hipError_t launch_aex_seed_next(AexArgs a, uint64_t* dirty, bool patch, hipStream_t st) {
  a.dirty = dirty;  // (the round's own args may not track it)
  const uint64_t nw = (a.nown + 63) / 64;
  if (!patch) {
    hipError_t e = hipMemcpyAsync(a.Vn, a.V, (size_t)a.nown * a.K * 4, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipMemsetAsync(a.dirty, 0, std::max<uint64_t>(nw, 1) * 8, st);
    return e;
  }
  if (nw == 0) return hipSuccess;
  const uint32_t g = ax_grid(nw, kAxBlock / 64, 512);  // mostly clean words: few waves suffice
  switch (a.L) {
    case 1: aex_patch_kernel<1><<<g, kAxBlock, 0, st>>>(a); break;
    case 2: aex_patch_kernel<2><<<g, kAxBlock, 0, st>>>(a); break;
    case 4: aex_patch_kernel<4><<<g, kAxBlock, 0, st>>>(a); break;
    case 8: aex_patch_kernel<8><<<g, kAxBlock, 0, st>>>(a); break;
    case 16: aex_patch_kernel<16><<<g, kAxBlock, 0, st>>>(a); break;
    case 32: aex_patch_kernel<32><<<g, kAxBlock, 0, st>>>(a); break;
    default: aex_patch_kernel<64><<<g, kAxBlock, 0, st>>>(a); break;
  }
  return hipGetLastError();
}

hipError_t launch_aex_init(uint32_t* V, uint64_t lo, uint64_t nown, uint32_t K, uint32_t k0, uint32_t k1,
                           hipStream_t st) {
  if (nown == 0) return hipSuccess;
  aex_init_kernel<<<ax_grid(nown * ((K + 3) / 4), kAxBlock, 65536), kAxBlock, 0, st>>>(V, lo, nown, K, k0, k1);
  return hipGetLastError();
}

hipError_t launch_aex_fill_alive(const AexArgs& a, hipStream_t st) {
  if (a.nown == 0) return hipSuccess;
  aex_fill_alive_kernel<<<ax_grid((a.nown + 63) / 64, kAxBlock, 1024), kAxBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_aex_local_max(const uint32_t* V, uint64_t nown, uint32_t K, uint32_t* out, hipStream_t st) {
  hipError_t e = hipMemsetAsync(out, 0, K * 4, st);
  if (e != hipSuccess || nown == 0) return e;
  aex_max_kernel<<<ax_grid(nown * K, kAxBlock, 4096), kAxBlock, 0, st>>>(V, nown, K, out);
  return hipGetLastError();
}

}  // namespace gossip
