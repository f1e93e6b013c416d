// sharded.hip — sparse rounds across G shards (sharded.h).
//
// Reference hot path: (*NodeState).Gossip, main.go:65-89, whose only
// cross-node traffic is the per-neighbour SyncRPC (main.go:81).  Here a sparse
// round's cross-shard traffic is the rare list (all-gather) and the pushes
// that land on another shard (all-to-all); everything else stays on the GPU
// that owns the node.  The scan follows frontier.hip's (same tests, same
// batching of loads before stores), with peers drawn over the global id space.
#include <hipcub/hipcub.hpp>

#include "philox.h"
#include "sharded.h"
#include "wave.h"

namespace gossip {

namespace {

constexpr int kScanThreads = 1024;
constexpr uint32_t kScanGrid = 256;  // one block per CU: the summary takes 128 KiB of LDS
constexpr uint32_t kRwWords = 512;   // own rare-bitmap words staged per chunk (32K nodes; LDS room for the queues)
constexpr int kScanUnroll = 2;
constexpr uint32_t kMsgShift = 40;   // message node word: owner << 40 | node at the owner
// up to this many rare nodes (all shards), the index skips the per-word ranks and the
// summary pass over all N nodes: a value is found by binary search in its owner's list
constexpr uint64_t kSmallIndex = 1ull << 16;

__device__ __forceinline__ uint64_t word_valid(uint64_t w, uint64_t n) {
  const uint64_t lo = w << 6;
  return n >= lo + 64 ? ~0ull : ((1ull << (n - lo)) - 1ull);
}

// own rare word w: maj 0 -> nonzero nodes, maj 1 -> nodes not yet full
__device__ __forceinline__ uint64_t own_rare(const FrontierBufs& f, uint64_t w, uint64_t nown, uint32_t maj) {
  return maj ? (~f.fullb[w] & word_valid(w, nown)) : f.nzb[w];
}

__global__ __launch_bounds__(256) void wcount_kernel(FrontierBufs f, uint64_t nown, uint32_t maj, uint32_t* wcount) {
  const uint64_t nw = (nown + 63) >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w < nw) wcount[w] = (uint32_t)__popcll(own_rare(f, w, nown, maj));
  else if (w == nw) wcount[w] = 0;
}

// One wave per 64 bitmap words: lane i loads word i, the wave then visits only
// the nonzero words (lane b writes node b of the word), so empty stretches of
// the bitmap cost one load per 64 words.
__global__ __launch_bounds__(256) void list_kernel(FrontierBufs f, const uint64_t* __restrict__ S, uint64_t nown,
                                                    uint64_t lo, uint32_t maj, const uint32_t* __restrict__ wpos,
                                                    SxItem* __restrict__ out) {
  const uint64_t nw = (nown + 63) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u));  // this wave's first word
  const uint64_t wl = w0 + lane;
  const uint64_t x = wl < nw ? own_rare(f, wl, nown, maj) : 0ull;
  const uint32_t pl = wl < nw ? wpos[wl] : 0u;
  uint64_t nzw = __ballot(x != 0);
  while (nzw) {
    const uint32_t src = (uint32_t)__builtin_ctzll(nzw);
    nzw &= nzw - 1;
    const uint64_t xw = __shfl(x, src, 64);
    const uint32_t pos0 = __shfl(pl, src, 64);
    if ((xw >> lane) & 1ull) {
      const uint64_t i = ((w0 + src) << 6) + lane;
      out[pos0 + (uint32_t)__popcll(xw & ((1ull << lane) - 1ull))] = SxItem{lo + i, S[i]};
    }
  }
}

// Lists are in id order (and shards in rank order), so the items of one bitmap
// word sit in consecutive lanes: a segmented OR across the wave leaves one
// atomic per word a wave touches instead of one per item.
template <bool SUMM>
__global__ __launch_bounds__(256) void setbits_kernel(const SxItem* __restrict__ recv, uint64_t stride, uint32_t G,
                                                       const uint64_t* __restrict__ cbase, uint64_t* __restrict__ grb,
                                                       uint32_t* __restrict__ summ, uint32_t glog) {
  const uint64_t total = stride * G;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t step = (uint64_t)gridDim.x * 256;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256; i0 < total; i0 += step) {  // whole waves iterate together
    const uint64_t i = i0 + threadIdx.x;
    bool valid = i < total;
    uint64_t p = 0;
    if (valid) {
      const uint32_t q = (uint32_t)(i / stride);
      valid = i - q * stride < cbase[q + 1] - cbase[q];  // else padding of a shorter list
      if (valid) p = recv[i].node;
    }
    const uint64_t w = valid ? p >> 6 : ~0ull;
    uint64_t m = valid ? 1ull << (p & 63) : 0ull;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_down(m, o, 64), wy = __shfl_down(w, o, 64);
      if (lane + o < 64 && wy == w) m |= y;
    }
    const uint64_t wprev = __shfl_up(w, 1, 64);
    if (valid && (lane == 0 || wprev != w)) atomicOr((unsigned long long*)&grb[w], (unsigned long long)m);
    // small lists: the LDS summary straight from the items (one bit per 2^glog nodes)
    if (SUMM && valid) {
      const uint64_t gb = p >> glog;
      atomicOr(&summ[gb >> 5], 1u << (gb & 31u));
    }
  }
}

__global__ __launch_bounds__(256) void zero_kernel(uint4* __restrict__ p, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
    p[i] = make_uint4(0, 0, 0, 0);
}

__global__ __launch_bounds__(256) void gcount_kernel(const uint64_t* __restrict__ grb, uint64_t nwg, uint32_t* gcnt) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w < nwg) gcnt[w] = (uint32_t)__popcll(grb[w]);
  else if (w == nwg) gcnt[w] = 0;
}

struct ScanArgs {
  FrontierBufs lf;
  const uint64_t* S;
  const SxItem* recv;
  uint64_t stride;
  const uint64_t* grb;
  const uint32_t* gpre;
  const uint64_t* cbase;
  const uint32_t* gsumm;
  uint32_t gglog, gsumm_words;
  const uint32_t* gsumm2;  // mid-level summary of grb (frontier.h FrontierBufs::summ2), or null
  uint32_t g2log;
  SxItem* msg;          // block b's messages at msg[b * seg_cap, ...)
  uint32_t* blk_cnt;    // [grid] messages per block
  uint64_t seg_cap;     // k * per_block: every owned node sends at most k pushes
  uint64_t N, Nl, lo, nown, per_block;
  uint32_t G, R, k, t, key0, key1, mark_d;
  Faults fa;
};

// S_t of a rare node p (global id) whose bitmap word is rw: own shard from S,
// another shard from the gathered lists (its rank among the rare nodes, minus
// the lists before its owner's, is its place in the owner's list)
// Small lists (a.gpre null, sx_index): p's place in its owner's list by binary search.
__device__ __forceinline__ uint64_t rare_value(const ScanArgs& a, uint32_t p, uint64_t rw, uint32_t pre) {
  const uint32_t q = (uint32_t)(p / a.Nl);
  if (!a.gpre) {
    const SxItem* list = a.recv + q * a.stride;
    uint64_t lo = 0, hi = a.cbase[q + 1] - a.cbase[q];
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (list[mid].node < p) lo = mid + 1;
      else hi = mid;
    }
    return list[lo].value;  // p is in the list: its grb bit is set
  }
  const uint64_t rank = (uint64_t)pre + (uint64_t)__popcll(rw & ((1ull << (p & 63u)) - 1ull));
  return a.recv[q * a.stride + (rank - a.cbase[q])].value;
}

// FAULTS: edge loss / partitions / stall active; off, none of that code exists
template <int MAJ, int MODE, bool FAULTS>
__device__ __forceinline__ void scan_body(uint4* summ4, uint64_t* rws, uint32_t* lcnt, const ScanArgs& a) {
  const uint32_t* summ = (const uint32_t*)summ4;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t n4 = (a.gsumm_words + 3) / 4;
  for (uint32_t i = tid; i < n4; i += kScanThreads) summ4[i] = ((const uint4*)a.gsumm)[i];

  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  const uint64_t fm = full_mask1(a.R), maj = MAJ ? fm : 0ull, nm1 = a.N - 1;
  const uint32_t glog = a.gglog, lo = (uint32_t)a.lo, nown = (uint32_t)a.nown, k = a.k;
  auto summ_bit = [&](uint32_t p) -> bool { return (summ[p >> (glog + 5)] >> ((p >> glog) & 31u)) & 1u; };
  const uint64_t below = (1ull << lane) - 1ull;
  // push delta d (may be 0) to global node p; every lane of the wave calls this
  // together: a wave reserves its messages' slots with one atomic
  auto push_to = [&](uint32_t p, uint64_t d) {
    const bool local = d && (p - lo < nown);
    if (local) {
      atomicOr((unsigned long long*)&a.lf.D[p - lo], (unsigned long long)d);
      if (a.mark_d) a.lf.dirtyD[(p - lo) >> 6] = 1;
    }
    const bool remote = d && !local;
    const uint64_t m = __ballot(remote);
    if (!m) return;
    const uint32_t first = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(lcnt, (uint32_t)__popcll(m));  // the block's own segment: an LDS counter
    base = __shfl(base, first, 64);
    if (remote) {
      const uint32_t q = (uint32_t)(p / a.Nl);
      a.msg[blockIdx.x * a.seg_cap + base + (uint32_t)__popcll(m & below)] =
          SxItem{((uint64_t)q << kMsgShift) | (p - (uint64_t)q * a.Nl), d};
    }
  };
  // node ids are < 2^32 (gossip_create checks N)
  const uint32_t b0 = blockIdx.x * (uint32_t)a.per_block;
  const uint32_t b1 = (uint32_t)min<uint64_t>((uint64_t)b0 + a.per_block, a.nown);
  for (uint32_t c0 = b0; c0 < b1; c0 += kRwWords * 64) {
    const uint32_t c1 = min(c0 + kRwWords * 64, b1);
    __syncthreads();  // previous chunk done with rws
    for (uint32_t i = tid; i < ((c1 - c0 + 63) >> 6); i += kScanThreads)
      rws[i] = own_rare(a.lf, (c0 >> 6) + i, a.nown, MAJ);
    __syncthreads();
    for (uint32_t base = c0; base < c1; base += kScanThreads * kScanUnroll) {
      uint32_t pp[kScanUnroll][4], hit[kScanUnroll], live[kScanUnroll];
      bool act[kScanUnroll], rn[kScanUnroll];
      // 1. draws and LDS summary tests
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t i = base + u * kScanThreads + tid;
        const bool valid = i < c1;
        const uint32_t n = lo + i;
        rn[u] = valid && ((rws[(i - c0) >> 6] >> lane) & 1ull);
        act[u] = valid && (rn[u] || !((!kPull && MAJ == 0) || (!kPush && MAJ == 1)));
        hit[u] = 0;
        live[u] = 0;  // edges not lost
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) pp[u][j] = 0;
        if (act[u] && k <= 4) {
          const u32x4 r4 = philox4x32_10(u32x4{n, a.t, 0u, 0u}, a.key0, a.key1);
          const u32x4 lw = FAULTS && a.fa.loss ? loss_draws(n, a.t, 0u, a.key0, a.key1) : u32x4{0, 0, 0, 0};
          const Reach rc = FAULTS ? reach_of(n, a.fa) : Reach{0u, 0xFFFFFFFFu};  // n's partition block (§2.8)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            if (j >= k) break;
            pp[u][j] = peer_from_word(lane_of(r4, j), nm1, n);
            const bool lost = FAULTS && edge_lost(a.fa, rc, pp[u][j], lane_of(lw, j));
            live[u] |= (lost ? 0u : 1u) << j;
            if (!lost && summ_bit(pp[u][j])) hit[u] |= 1u << j;
          }
        }
      }
      // a wave with no rare end anywhere in this batch has nothing to do (most waves in light rounds)
      {
        bool any = false;
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) any = any || rn[u] || hit[u] != 0u || (k > 4 && act[u]);  // k > 4: no hits yet
        if (!__ballot(any)) continue;
      }
      // 2. exact probes in the global rare bitmap (all issued, then consumed); in saturated
      // rounds past 2^25 nodes the L2-resident mid-level summary first
      if (a.gsumm2) {
        uint32_t sw[kScanUnroll][4];
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            sw[u][j] = ((hit[u] >> j) & 1u) ? a.gsumm2[pp[u][j] >> (a.g2log + 5)] : 0u;
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            if (!((sw[u][j] >> ((pp[u][j] >> a.g2log) & 31u)) & 1u)) hit[u] &= ~(1u << j);
      }
      uint64_t rw[kScanUnroll][4];
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) rw[u][j] = ((hit[u] >> j) & 1u) ? a.grb[pp[u][j] >> 6] : 0ull;
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
          if (!((rw[u][j] >> (pp[u][j] & 63u)) & 1ull)) hit[u] &= ~(1u << j);
      // 3. S_t of the rare ends: own shard directly, other shards through the lists
      uint32_t pre[kScanUnroll][4];
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const bool remote = ((hit[u] >> j) & 1u) && (pp[u][j] - lo >= nown);
          pre[u][j] = remote && a.gpre ? a.gpre[pp[u][j] >> 6] : 0u;
        }
      uint64_t x[kScanUnroll], vp[kScanUnroll][4];
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t i = base + u * kScanThreads + tid;
        x[u] = rn[u] ? a.S[i] : maj;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t p = pp[u][j];
          if (!((hit[u] >> j) & 1u)) vp[u][j] = maj;
          else if (p - lo < nown) vp[u][j] = a.S[p - lo];
          else vp[u][j] = rare_value(a, p, rw[u][j], pre[u][j]);
        }
      }
      // 4. deltas in registers, then the stores (frontier.hip: vmcnt retires in order)
      uint64_t accs[kScanUnroll], dpush[kScanUnroll][4];
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        accs[u] = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) dpush[u][j] = 0;
        if (!act[u] || k > 4) continue;
        uint64_t acc = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          if (j >= k) break;
          if (!((live[u] >> j) & 1u)) continue;             // lost edge
          if (!rn[u] && !((hit[u] >> j) & 1u)) continue;  // both ends majority: nothing moves
          if (kPull) acc |= vp[u][j];
          if (kPush) dpush[u][j] = x[u] & ~vp[u][j];
        }
        accs[u] = acc & ~x[u];
      }
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) push_to(pp[u][j], dpush[u][j]);
      // k > 4: the draws are redone edge by edge
      if (k > 4) {
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) {
          if (!act[u]) continue;
          const uint32_t i = base + u * kScanThreads + tid, n = lo + i;
          uint64_t acc = 0;
          u32x4 r4{0, 0, 0, 0}, lw{0, 0, 0, 0};
          const Reach rc = FAULTS ? reach_of(n, a.fa) : Reach{0u, 0xFFFFFFFFu};  // n's partition block (§2.8)
          for (uint32_t j = 0; j < k; ++j) {
            if ((j & 3u) == 0) {
              r4 = philox4x32_10(u32x4{n, a.t, 0u, j >> 2}, a.key0, a.key1);
              if (FAULTS && a.fa.loss) lw = loss_draws(n, a.t, j >> 2, a.key0, a.key1);
            }
            const uint32_t p = peer_from_word(lane_of(r4, j & 3u), nm1, n);
            const bool lost = FAULTS && edge_lost(a.fa, rc, p, lane_of(lw, j & 3u));
            uint64_t w = 0;
            bool rp = summ_bit(p);
            if (rp && a.gsumm2) rp = (a.gsumm2[p >> (a.g2log + 5)] >> ((p >> a.g2log) & 31u)) & 1u;
            if (rp) {
              w = a.grb[p >> 6];
              rp = (w >> (p & 63u)) & 1ull;
            }
            const bool moves = !lost && (rn[u] || rp);  // else lost, or both ends majority: nothing moves
            uint64_t v = maj;
            if (rp) v = (p - lo < nown) ? a.S[p - lo] : rare_value(a, p, w, a.gpre ? a.gpre[p >> 6] : 0u);
            if (kPull && moves) acc |= v;
            if (kPush) push_to(p, moves ? x[u] & ~v : 0ull);
          }
          accs[u] = acc & ~x[u];
        }
      }
      // pull deltas: ORed into D beside the pushes (frontier.hip: one delta array)
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t i = base + u * kScanThreads + tid;
        if (!accs[u]) continue;
        atomicOr((unsigned long long*)&a.lf.D[i], (unsigned long long)accs[u]);
        if (a.mark_d) a.lf.dirtyD[i >> 6] = 1;
      }
    }
  }
}

// Queued scan (frontier.hip scan_body_q; FrontierBufs::scan_q, k <= 4): the edges with a possibly
// rare end wait in a per-wave LDS queue and are resolved 128 at a time, two per lane, every
// load of the chain issued before any is used.  A queued edge: x = own index - block base
// (< 2^24) | rare(n) << 24 | summary hit(p) << 25, y = p (global id).
constexpr uint32_t kQFlush = 128;
constexpr uint32_t kQCap = kQFlush + 64;

template <int MAJ, int MODE, bool FAULTS>
__device__ __forceinline__ void scan_body_q(uint4* summ4, uint64_t* rws, uint2* qs, uint32_t* lcnt,
                                            const ScanArgs& a) {
  const uint32_t* summ = (const uint32_t*)summ4;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  uint2* qw = qs + (tid >> 6) * kQCap;  // this wave's queue
  const uint32_t n4 = (a.gsumm_words + 3) / 4;
  for (uint32_t i = tid; i < n4; i += kScanThreads) summ4[i] = ((const uint4*)a.gsumm)[i];

  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  const uint64_t maj = MAJ ? full_mask1(a.R) : 0ull, nm1 = a.N - 1;
  const uint32_t glog = a.gglog, lo = (uint32_t)a.lo, nown = (uint32_t)a.nown, k = a.k;
  auto summ_bit = [&](uint32_t p) -> bool { return (summ[p >> (glog + 5)] >> ((p >> glog) & 31u)) & 1u; };
  const uint64_t below = (1ull << lane) - 1ull;
  auto push_to = [&](uint32_t p, uint64_t d) {  // every lane of the wave together (scan_body)
    const bool local = d && (p - lo < nown);
    if (local) {
      atomicOr((unsigned long long*)&a.lf.D[p - lo], (unsigned long long)d);
      if (a.mark_d) a.lf.dirtyD[(p - lo) >> 6] = 1;
    }
    const bool remote = d && !local;
    const uint64_t m = __ballot(remote);
    if (!m) return;
    const uint32_t first = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(lcnt, (uint32_t)__popcll(m));
    base = __shfl(base, first, 64);
    if (remote) {
      const uint32_t q = (uint32_t)(p / a.Nl);
      a.msg[blockIdx.x * a.seg_cap + base + (uint32_t)__popcll(m & below)] =
          SxItem{((uint64_t)q << kMsgShift) | (p - (uint64_t)q * a.Nl), d};
    }
  };
  const uint32_t b0 = blockIdx.x * (uint32_t)a.per_block;
  const uint32_t b1 = (uint32_t)min<uint64_t>((uint64_t)b0 + a.per_block, a.nown);
  constexpr int kE = kQFlush / 64;
  auto flush = [&](uint32_t nf) {
    uint32_t i[kE], p[kE];
    bool rn[kE], hit[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const uint32_t s = lane + 64u * e;
      const uint2 q = s < nf ? qw[s] : uint2{0u, 0u};
      i[e] = b0 + (q.x & 0xFFFFFFu);
      rn[e] = (q.x >> 24) & 1u;
      hit[e] = (q.x >> 25) & 1u;
      p[e] = q.y;
    }
    if (a.gsumm2) {
      uint32_t sw[kE];
#pragma unroll
      for (int e = 0; e < kE; ++e) sw[e] = hit[e] ? a.gsumm2[p[e] >> (a.g2log + 5)] : 0u;
#pragma unroll
      for (int e = 0; e < kE; ++e) hit[e] = hit[e] && ((sw[e] >> ((p[e] >> a.g2log) & 31u)) & 1u);
    }
    uint64_t rw[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) rw[e] = hit[e] ? a.grb[p[e] >> 6] : 0ull;
#pragma unroll
    for (int e = 0; e < kE; ++e) hit[e] = hit[e] && ((rw[e] >> (p[e] & 63u)) & 1ull);
    uint32_t pre[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) pre[e] = hit[e] && (p[e] - lo >= nown) && a.gpre ? a.gpre[p[e] >> 6] : 0u;
    uint64_t x[kE], vp[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      x[e] = rn[e] ? a.S[i[e]] : maj;
      if (!hit[e]) vp[e] = maj;
      else if (p[e] - lo < nown) vp[e] = a.S[p[e] - lo];
      else vp[e] = rare_value(a, p[e], rw[e], pre[e]);
    }
    uint64_t dpush[kE], dpull[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const bool any = rn[e] || hit[e];  // both ends majority (or an empty slot): nothing moves
      dpush[e] = kPush && any ? x[e] & ~vp[e] : 0ull;
      dpull[e] = kPull && any ? vp[e] & ~x[e] : 0ull;
    }
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      push_to(p[e], dpush[e]);
      if (dpull[e]) {
        atomicOr((unsigned long long*)&a.lf.D[i[e]], (unsigned long long)dpull[e]);
        if (a.mark_d) a.lf.dirtyD[i[e] >> 6] = 1;
      }
    }
  };
  uint32_t qn = 0;  // entries in this wave's queue (wave-uniform)
  for (uint32_t c0 = b0; c0 < b1; c0 += kRwWords * 64) {
    const uint32_t c1 = min(c0 + kRwWords * 64, b1);
    __syncthreads();  // previous chunk done with rws
    for (uint32_t i = tid; i < ((c1 - c0 + 63) >> 6); i += kScanThreads)
      rws[i] = own_rare(a.lf, (c0 >> 6) + i, a.nown, MAJ);
    __syncthreads();
    for (uint32_t base = c0; base < c1; base += kScanThreads * kScanUnroll) {
      uint32_t pp[kScanUnroll][4], cand[kScanUnroll];
      bool rn[kScanUnroll];
      bool any = false;
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t i = base + u * kScanThreads + tid;
        const bool valid = i < c1;
        const uint32_t n = lo + i;
        rn[u] = valid && ((rws[(i - c0) >> 6] >> lane) & 1ull);
        const bool act = valid && (rn[u] || !((!kPull && MAJ == 0) || (!kPush && MAJ == 1)));
        cand[u] = 0;  // bit j: edge j is live and has a rare or possibly rare end
        if (act) {
          const u32x4 r4 = philox4x32_10(u32x4{n, a.t, 0u, 0u}, a.key0, a.key1);
          const u32x4 lw = FAULTS && a.fa.loss ? loss_draws(n, a.t, 0u, a.key0, a.key1) : u32x4{0, 0, 0, 0};
          const Reach rc = FAULTS ? reach_of(n, a.fa) : Reach{0u, 0xFFFFFFFFu};  // n's partition block (§2.8)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            if (j >= k) break;
            pp[u][j] = peer_from_word(lane_of(r4, j), nm1, n);
            const bool lost = FAULTS && edge_lost(a.fa, rc, pp[u][j], lane_of(lw, j));
            if (!lost && (rn[u] || summ_bit(pp[u][j]))) cand[u] |= 1u << j;
          }
        }
        any = any || cand[u] != 0u;
      }
      if (!__ballot(any)) continue;
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t i = base + u * kScanThreads + tid;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          if (j >= k) break;
          const bool c = (cand[u] >> j) & 1u;
          const uint64_t m = __ballot(c);
          if (!m) continue;
          if (c) {
            const uint32_t pos =
                qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const bool h = !rn[u] || summ_bit(pp[u][j]);  // a rare node's edges are all queued
            qw[pos] = uint2{(i - b0) | (uint32_t)rn[u] << 24 | (uint32_t)h << 25, pp[u][j]};
          }
          qn += (uint32_t)__popcll(m);
          if (qn >= kQFlush) {
            __builtin_amdgcn_wave_barrier();
            flush(kQFlush);
            qn -= kQFlush;  // (< 64 left: move them to the front)
            const uint2 rest = lane < qn ? qw[kQFlush + lane] : uint2{0u, 0u};
            __builtin_amdgcn_wave_barrier();
            if (lane < qn) qw[lane] = rest;
            __builtin_amdgcn_wave_barrier();
          }
        }
      }
    }
  }
  if (qn) {
    __builtin_amdgcn_wave_barrier();
    flush(qn);
  }
}

template <int MODE, bool FAULTS>
__global__ __launch_bounds__(kScanThreads) void sx_scan_kernel(ScanArgs a, uint32_t maj) {
  __shared__ uint4 summ4[kSummBits / 128];
  __shared__ uint64_t rws[kRwWords];
  __shared__ uint2 qs[(kScanThreads / 64) * kQCap];  // 24 KiB
  __shared__ uint32_t lcnt;
  if (threadIdx.x == 0) lcnt = 0;  // (scan_body syncs before the first use)
  if (a.lf.scan_q && a.k <= 4) {
    if (maj)
      scan_body_q<1, MODE, FAULTS>(summ4, rws, qs, &lcnt, a);
    else
      scan_body_q<0, MODE, FAULTS>(summ4, rws, qs, &lcnt, a);
  } else if (maj)
    scan_body<1, MODE, FAULTS>(summ4, rws, &lcnt, a);
  else
    scan_body<0, MODE, FAULTS>(summ4, rws, &lcnt, a);
  __syncthreads();
  if (threadIdx.x == 0) a.blk_cnt[blockIdx.x] = lcnt;
}

// Messages grouped by owner, in two passes over the scan blocks' segments
// (one group block per segment): count (LDS histogram, one global atomic per
// block and owner), then scatter (each block reserves its run per owner once,
// then places its messages).
constexpr uint32_t kMaxShards = 1024;

__global__ __launch_bounds__(256) void owner_count_kernel(const SxItem* __restrict__ msg, uint64_t seg_cap,
                                                           const uint32_t* __restrict__ blk_cnt, uint32_t* cnt,
                                                           uint32_t G) {
  __shared__ uint32_t h[kMaxShards];
  for (uint32_t q = threadIdx.x; q < G; q += 256) h[q] = 0;
  __syncthreads();
  const SxItem* seg = msg + blockIdx.x * seg_cap;
  const uint32_t n = blk_cnt[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < n; i += 256) atomicAdd(&h[(uint32_t)(seg[i].node >> kMsgShift)], 1u);
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < G; q += 256)
    if (h[q]) atomicAdd(&cnt[q], h[q]);
}

__global__ __launch_bounds__(256) void owner_scatter_kernel(const SxItem* __restrict__ msg, uint64_t seg_cap,
                                                             const uint32_t* __restrict__ blk_cnt,
                                                             SxItem* __restrict__ out, const uint32_t* __restrict__ cnt,
                                                             uint32_t* fill, uint32_t G) {
  __shared__ uint32_t h[kMaxShards], base[kMaxShards];
  for (uint32_t q = threadIdx.x; q < G; q += 256) h[q] = 0;
  __syncthreads();
  const SxItem* seg = msg + blockIdx.x * seg_cap;
  const uint32_t n = blk_cnt[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < n; i += 256) atomicAdd(&h[(uint32_t)(seg[i].node >> kMsgShift)], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {  // owner q's messages start after those of owners < q
    uint32_t off = 0;
    for (uint32_t q = 0; q < G; ++q) {
      base[q] = off + (h[q] ? atomicAdd(&fill[q], h[q]) : 0u);
      off += cnt[q];
    }
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < G; q += 256) h[q] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += 256) {
    const SxItem m = seg[i];
    const uint32_t q = (uint32_t)(m.node >> kMsgShift);
    out[base[q] + atomicAdd(&h[q], 1u)] = SxItem{m.node & ((1ull << kMsgShift) - 1ull), m.value};
  }
}

__global__ __launch_bounds__(256) void apply_kernel(FrontierBufs f, const SxItem* __restrict__ in, uint64_t n,
                                                     uint32_t mark_d) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const SxItem m = in[i];
    atomicOr((unsigned long long*)&f.D[m.node], (unsigned long long)m.value);
    if (mark_d) f.dirtyD[m.node >> 6] = 1;
  }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// scan geometry (also sizes the message buffer: one segment of k * per_block items per block)
uint32_t scan_grid(uint64_t nown) {
  const uint64_t chunks = (nown + kScanThreads - 1) / kScanThreads;
  return (uint32_t)(chunks < kScanGrid ? (chunks ? chunks : 1) : kScanGrid);
}
uint64_t scan_per_block(uint64_t nown, uint32_t grid) {
  return ((nown + grid - 1) / grid + kScanThreads - 1) / kScanThreads * kScanThreads;
}
uint64_t msg_cap(const SxGeom& g) {
  const uint32_t grid = scan_grid(g.nown);
  return (uint64_t)g.k * scan_per_block(g.nown, grid) * grid;
}

size_t scan_tmp_bytes(uint64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  return bytes;
}

uint32_t grid_for(uint64_t n, uint32_t block, uint32_t cap) {
  const uint64_t g = (n + block - 1) / block;
  return (uint32_t)(g == 0 ? 1 : (g < cap ? g : cap));
}

// --- class-coded state exchange (dense rounds on the state image) ---------------
// A node's word is 0 (empty), all ones (full) or mixed; the two occupancy bits say which,
// so a shard sends its bitmaps and the words of its mixed nodes only.

__device__ __forceinline__ uint64_t cc_mixed(uint64_t nz, uint64_t full) { return nz & ~full; }

// own mixed nodes per bitmap word
__global__ __launch_bounds__(256) void cc_wcount_kernel(const uint64_t* __restrict__ nzb,
                                                        const uint64_t* __restrict__ fullb, uint64_t nown,
                                                        uint32_t* wcount) {
  const uint64_t nw = (nown + 63) >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w < nw) wcount[w] = (uint32_t)__popcll(cc_mixed(nzb[w], fullb[w]) & word_valid(w, nown));
  else if (w == nw) wcount[w] = 0;
}

// the own mixed words in id order (a wave visits only the nonzero bitmap words, as list_kernel)
__global__ __launch_bounds__(256) void cc_list_kernel(const uint64_t* __restrict__ nzb,
                                                      const uint64_t* __restrict__ fullb,
                                                      const uint64_t* __restrict__ S, uint64_t nown,
                                                      const uint32_t* __restrict__ wpos, uint64_t* __restrict__ out) {
  const uint64_t nw = (nown + 63) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w0 = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u);
  const uint64_t wl = w0 + lane;
  const uint64_t x = wl < nw ? cc_mixed(nzb[wl], fullb[wl]) & word_valid(wl, nown) : 0ull;
  const uint32_t pl = wl < nw ? wpos[wl] : 0u;
  uint64_t nzw = __ballot(x != 0);
  while (nzw) {
    const uint32_t src = (uint32_t)__builtin_ctzll(nzw);
    nzw &= nzw - 1;
    const uint64_t xw = __shfl(x, src, 64);
    const uint32_t pos0 = __shfl(pl, src, 64);
    if ((xw >> lane) & 1ull) out[pos0 + (uint32_t)__popcll(xw & ((1ull << lane) - 1ull))] = S[((w0 + src) << 6) + lane];
  }
}

// The other shards' slices of the state image from their slots and mixed words.  A wave
// expands kCcUnroll bitmap words (64 nodes each) per step, their loads issued together.
constexpr uint32_t kCcUnroll = 4;
__global__ __launch_bounds__(256) void cc_expand_kernel(const uint64_t* __restrict__ slots, uint64_t slot_words,
                                                        const uint64_t* __restrict__ vals, uint64_t stride,
                                                        uint64_t* __restrict__ image, uint64_t N, uint64_t Nl,
                                                        uint32_t rank, uint32_t R) {
  const uint64_t q = blockIdx.y;  // one grid row per shard
  if (q == rank) return;          // the own slice is already in place
  const uint64_t nwl = (Nl + 63) >> 6, fm = full_mask1(R);
  const uint64_t nq = q * Nl < N ? min(Nl, N - q * Nl) : 0ull, nwq = (nq + 63) >> 6;
  const uint64_t* nzb = slots + q * slot_words;
  const uint64_t* fb = nzb + nwl;
  const uint32_t* pre = (const uint32_t*)(fb + nwl);
  const uint64_t* qv = vals + q * stride;
  uint64_t* img = image + q * Nl;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull, bit = 1ull << lane;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (uint64_t)gridDim.x * 4;
  for (uint64_t w0 = wave * kCcUnroll; w0 < nwq; w0 += nwaves * kCcUnroll) {
    uint64_t nz[kCcUnroll], fu[kCcUnroll];
    uint32_t pr[kCcUnroll];
#pragma unroll
    for (uint32_t u = 0; u < kCcUnroll; ++u) {
      const bool in = w0 + u < nwq;
      nz[u] = in ? nzb[w0 + u] : 0ull;
      fu[u] = in ? fb[w0 + u] : 0ull;
      pr[u] = in ? pre[w0 + u] : 0u;
    }
    uint64_t v[kCcUnroll];
#pragma unroll
    for (uint32_t u = 0; u < kCcUnroll; ++u) {
      const uint64_t mixed = cc_mixed(nz[u], fu[u]);
      v[u] = (fu[u] & bit) ? fm : (mixed & bit) ? qv[pr[u] + (uint32_t)__popcll(mixed & below)] : 0ull;
    }
#pragma unroll
    for (uint32_t u = 0; u < kCcUnroll; ++u) {
      const uint64_t i = ((w0 + u) << 6) + lane;
      if (i < nq) img[i] = v[u];
    }
  }
}

}  // namespace

hipError_t cc_compact(const SxGeom& g, const SxBufs& b, const FrontierBufs& lf, const uint64_t* S, uint64_t* out,
                      hipStream_t st) {
  const uint64_t nwl = (g.nown + 63) / 64;
  cc_wcount_kernel<<<grid_for(nwl + 1, 256, 1u << 30), 256, 0, st>>>(lf.nzb, lf.fullb, g.nown, b.wcount);
  size_t tb = b.tmp_bytes;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(b.tmp, tb, b.wcount, b.wpos, (int)(nwl + 1), st);
  if (e != hipSuccess) return e;
  cc_list_kernel<<<grid_for(nwl, 256, 1u << 30), 256, 0, st>>>(lf.nzb, lf.fullb, S, g.nown, b.wpos, out);
  return hipGetLastError();
}

hipError_t cc_expand(const SxGeom& g, const uint64_t* slots, const uint64_t* vals, uint64_t stride,
                     uint64_t* image, uint32_t R, hipStream_t st) {
  const uint64_t nwl = (g.Nl + 63) / 64;
  const dim3 grid(grid_for((nwl + kCcUnroll - 1) / kCcUnroll, 4, 2048), g.G);
  cc_expand_kernel<<<grid, 256, 0, st>>>(slots, cc_slot_words(g.Nl), vals, stride, image, g.N, g.Nl, g.rank, R);
  return hipGetLastError();
}

size_t sx_bytes(const SxGeom& g) {
  const uint64_t nwl = (g.nown + 63) / 64, nwg = (g.N + 63) / 64;
  const uint32_t glog = frontier_glog(g.N);
  const size_t sw = ((((g.N + (1ull << glog) - 1) >> glog) + 127) / 128) * 4;
  const size_t tmp = std::max(scan_tmp_bytes(nwl + 1), scan_tmp_bytes(nwg + 1));
  const uint64_t cap = msg_cap(g);
  return 2 * al256((nwl + 1) * 4) + al256(g.Nl * sizeof(SxItem)) + al256(nwg * 8) + 2 * al256((nwg + 1) * 4) +
         al256(sw * 4) + al256((size_t)frontier_summ2_words(g.N) * 4) + al256((g.G + 1) * 8) +
         2 * al256(cap * sizeof(SxItem)) + al256((g.G + 2 + kScanGrid) * 4) + al256(g.G * 4) + al256(tmp);
}

void sx_carve(const SxGeom& g, void* base, SxBufs* b) {
  const uint64_t nwl = (g.nown + 63) / 64, nwg = (g.N + 63) / 64;
  char* p = (char*)base;
  auto take = [&](size_t bytes) {
    char* r = p;
    p += al256(bytes);
    return r;
  };
  b->wcount = (uint32_t*)take((nwl + 1) * 4);
  b->wpos = (uint32_t*)take((nwl + 1) * 4);
  b->rare_send = (SxItem*)take(g.Nl * sizeof(SxItem));  // Nl >= any shard's count: the driver sends max-count items
  b->grb = (uint64_t*)take(nwg * 8);
  b->gcnt = (uint32_t*)take((nwg + 1) * 4);
  b->gpre = (uint32_t*)take((nwg + 1) * 4);
  b->gsum = FrontierBufs{};
  b->gsum.glog = frontier_glog(g.N);
  b->gsum.summ_words = (uint32_t)((((g.N + (1ull << b->gsum.glog) - 1) >> b->gsum.glog) + 127) / 128) * 4;
  b->gsum.nzb = b->grb;
  b->gsum.summ = (uint32_t*)take((size_t)b->gsum.summ_words * 4);
  b->gsum.g2log = frontier_g2log(g.N);
  b->gsum.summ2_words = frontier_summ2_words(g.N);
  b->gsum.summ2 = b->gsum.summ2_words ? (uint32_t*)take((size_t)b->gsum.summ2_words * 4) : nullptr;
  b->cbase = (uint64_t*)take((g.G + 1) * 8);
  b->cap = msg_cap(g);
  b->msg = (SxItem*)take(b->cap * sizeof(SxItem));
  b->msg_out = (SxItem*)take(b->cap * sizeof(SxItem));
  b->msg_cnt = (uint32_t*)take((g.G + 2 + kScanGrid) * 4);  // then the scan blocks' message counts
  b->msg_fill = (uint32_t*)take(g.G * 4);
  b->tmp_bytes = std::max(scan_tmp_bytes(nwl + 1), scan_tmp_bytes(nwg + 1));
  b->tmp = take(b->tmp_bytes);
}

hipError_t sx_compact(const SxGeom& g, const SxBufs& b, const FrontierBufs& lf, const uint64_t* S, uint32_t maj,
                      hipStream_t st) {
  const uint64_t nwl = (g.nown + 63) / 64;
  wcount_kernel<<<grid_for(nwl + 1, 256, 1u << 30), 256, 0, st>>>(lf, g.nown, maj, b.wcount);
  size_t tb = b.tmp_bytes;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(b.tmp, tb, b.wcount, b.wpos, (int)(nwl + 1), st);
  if (e != hipSuccess) return e;
  list_kernel<<<grid_for(nwl, 256, 1u << 30), 256, 0, st>>>(lf, S, g.nown, g.lo, maj, b.wpos, b.rare_send);
  return hipGetLastError();
}

bool sx_small_index(uint64_t rare) { return rare <= kSmallIndex; }

hipError_t sx_index(const SxGeom& g, const SxBufs& b, const SxItem* recv, uint64_t stride, uint64_t rare,
                    hipStream_t st, bool mid) {
  const uint64_t nwg = (g.N + 63) / 64;
  // grb is 256-B aligned (sx_carve) and padded to 16 B
  zero_kernel<<<grid_for((nwg + 1) / 2, 256, 2048), 256, 0, st>>>((uint4*)b.grb, (nwg + 1) / 2);
  hipError_t e;
  if (sx_small_index(rare)) {  // no per-word ranks (values by binary search), summary from the items
    const uint64_t n16 = (b.gsum.summ_words + 3) / 4;
    zero_kernel<<<grid_for(n16, 256, 2048), 256, 0, st>>>((uint4*)b.gsum.summ, n16);
    if (stride)
      setbits_kernel<true><<<grid_for(stride * g.G, 256, 4096), 256, 0, st>>>(recv, stride, g.G, b.cbase, b.grb,
                                                                             b.gsum.summ, b.gsum.glog);
    return hipGetLastError();
  }
  if (stride)
    setbits_kernel<false><<<grid_for(stride * g.G, 256, 4096), 256, 0, st>>>(recv, stride, g.G, b.cbase, b.grb,
                                                                            nullptr, 0u);
  gcount_kernel<<<grid_for(nwg + 1, 256, 1u << 30), 256, 0, st>>>(b.grb, nwg, b.gcnt);
  size_t tb = b.tmp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(b.tmp, tb, b.gcnt, b.gpre, (int)(nwg + 1), st);
  if (e != hipSuccess) return e;
  FrontierBufs gs = b.gsum;
  if (!mid) gs.summ2 = nullptr;
  return launch_frontier_summary(gs, g.N, 0, st);
}

hipError_t sx_scan(const SxGeom& g, const SxBufs& b, const FrontierBufs& lf, const uint64_t* S, const SxItem* recv,
                   uint64_t stride, uint64_t rare, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode,
                   uint32_t maj, bool all_d, const Faults& fa, hipStream_t st, bool mid) {
  hipError_t e = hipMemsetAsync(b.msg_cnt, 0, (g.G + 2) * 4, st);
  if (e == hipSuccess) e = hipMemsetAsync(b.msg_fill, 0, g.G * 4, st);
  if (e != hipSuccess || g.nown == 0) return e;  // a shard without nodes sends nothing
  ScanArgs a{};
  a.lf = lf;
  a.S = S;
  a.recv = recv;
  a.stride = stride;
  a.grb = b.grb;
  a.gpre = sx_small_index(rare) ? nullptr : b.gpre;
  a.cbase = b.cbase;
  a.gsumm = b.gsum.summ;
  a.gglog = b.gsum.glog;
  a.gsumm_words = b.gsum.summ_words;
  // (small indexes build their summary from the items and no mid-level one: few rare nodes)
  a.gsumm2 = mid && !sx_small_index(rare) ? b.gsum.summ2 : nullptr;
  a.g2log = b.gsum.g2log;
  a.msg = b.msg;
  a.blk_cnt = b.msg_cnt + g.G + 2;
  a.N = g.N;
  a.Nl = g.Nl;
  a.lo = g.lo;
  a.nown = g.nown;
  a.G = g.G;
  a.R = g.R;
  a.k = g.k;
  a.t = t;
  a.key0 = key0;
  a.key1 = key1;
  a.mark_d = all_d ? 0u : 1u;
  a.fa = fa;
  const uint32_t grid = scan_grid(g.nown);
  a.per_block = scan_per_block(g.nown, grid);
  a.seg_cap = (uint64_t)g.k * a.per_block;  // grid * seg_cap <= k * (nown rounded up): sx_carve's cap
#define GOSSIP_SX_SCAN(M)                                                     \
  if (fa.any()) sx_scan_kernel<M, true><<<grid, kScanThreads, 0, st>>>(a, maj); \
  else sx_scan_kernel<M, false><<<grid, kScanThreads, 0, st>>>(a, maj);
  switch (mode) {
    case 1: GOSSIP_SX_SCAN(1) break;
    case 2: GOSSIP_SX_SCAN(2) break;
    case 3: GOSSIP_SX_SCAN(3) break;
    default: return hipErrorInvalidValue;
  }
#undef GOSSIP_SX_SCAN
  const uint32_t* blk = b.msg_cnt + g.G + 2;
  owner_count_kernel<<<grid, 256, 0, st>>>(b.msg, a.seg_cap, blk, b.msg_cnt, g.G);
  owner_scatter_kernel<<<grid, 256, 0, st>>>(b.msg, a.seg_cap, blk, b.msg_out, b.msg_cnt, b.msg_fill, g.G);
  return hipGetLastError();
}

hipError_t sx_apply(const FrontierBufs& lf, const SxItem* in, uint64_t n, bool all_d, hipStream_t st) {
  if (n == 0) return hipSuccess;
  apply_kernel<<<grid_for(n, 256, 4096), 256, 0, st>>>(lf, in, n, all_d ? 0u : 1u);
  return hipGetLastError();
}

}  // namespace gossip
