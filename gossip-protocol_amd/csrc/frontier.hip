// frontier.hip — sparse rounds (frontier path) of PUSH / PULL / PUSH-PULL for gfx950.
//
// Reference hot path: (*NodeState).Gossip, main.go:65-89.  The reference only
// sends when a node has just learned a value (the dedupe at main.go:113 stops
// everything else); the synchronous-round restatement sends on every edge
// every round, but an edge whose two ends are both empty (early rounds) or
// both full (late rounds) cannot change a bit.  In those rounds the work is
// proportional to the rare set, not to N:
//
//   K0 frontier_summary  coarse bitmap of the rare set (1 bit per g nodes,
//                        <= 128 KiB) built from the exact occupancy bitmaps.
//   K1 frontier_scan     every node draws its Philox peers (the only O(N)
//                        compute); an edge is kept only if one end is rare —
//                        own end from the exact bitmap word (one broadcast load
//                        per wave), peer end from the LDS summary, confirmed in
//                        the exact bitmap (L2) on a summary hit.  Kept edges
//                        read S_t of their rare ends only (a majority node's
//                        value is known: 0 or the full mask) and OR exactly the
//                        missing bits into D with global atomics.
//   K2 frontier_commit   streams D; where a 64-node group has a delta, updates
//                        S in place, clears D, rewrites the two bitmap words
//                        and adds the stats deltas (counts, full, nonzero,
//                        hash telescoping) to the running totals.
//
// Every read of K1 is of S_t (S is only written by K2), so results equal the
// dense round bit for bit.  K2 in rebuild mode computes absolute stats and
// both bitmaps from S (after inject/reset or a direct-path round).
#include "frontier.h"
#include "binned.h"

#include <algorithm>
#include "philox.h"
#include "round.h"
#include "wave.h"

namespace gossip {

namespace {

constexpr int kScanThreads = 1024;
// (non-temporal hints on the scan's S gathers: equal)
template <typename T>
__device__ __forceinline__ T scan_ld(const T* p) {
  return *p;
}
#ifndef GOSSIP_SCAN_BPC
#define GOSSIP_SCAN_BPC 1
#endif
constexpr uint32_t kScanGrid = 256 * GOSSIP_SCAN_BPC;  // one block per CU: the summary takes 128 KiB of LDS
constexpr uint32_t kScanWaves = 4 * GOSSIP_SCAN_BPC;   // waves per SIMD (launch bounds)
// commit / rebuild blocks of 1024 threads, at most kCommitMaxBlocks of them: each block ends in
// ~67 same-address atomics on the totals, which cost more than the waves gain past ~512 blocks
// (2^24 sparse rounds 132 -> 125 us against 256-thread blocks up to 4096; profiles/r05_cc2/)
constexpr int kCommitThreads = 1024;
constexpr uint32_t kCommitMaxBlocks = 512;
constexpr uint32_t kRwWords = 512;   // rare-bitmap words staged per scan chunk (32K nodes; LDS room for the queues)
constexpr int kScanUnroll = 2;  // nodes per lane per scan step (1: equal, 4: slower)
constexpr int kCommitUnroll = 4;     // dirty groups per wave per commit step
constexpr uint32_t kCommitChunkLog = 6;  // 64 groups per wave chunk (16 / 32: slower, profiles/r05_cc/)

// valid-node mask of bitmap word w (bits past N are zero in both bitmaps)
__device__ __forceinline__ uint64_t word_valid(uint64_t w, uint64_t N) {
  const uint64_t lo = w << 6;
  return N >= lo + 64 ? ~0ull : ((1ull << (N - lo)) - 1ull);
}

template <int MAJ>
__device__ __forceinline__ uint64_t rare_word(const FrontierBufs& f, uint64_t w, uint64_t N) {
  return MAJ ? (~f.fullb[w] & word_valid(w, N)) : f.nzb[w];
}

template <int MAJ>
__device__ __forceinline__ void summary_body(const FrontierBufs& f, uint64_t N) {
  const uint32_t s = blockIdx.x * 256 + threadIdx.x;
  if (s >= f.summ_words) return;
  const uint64_t nwords = (N + 63) >> 6;
  const uint32_t g = 1u << f.glog;
  uint32_t out = 0;
  if (g == 1) {
    const uint64_t w = s >> 1;
    if (w < nwords) out = (uint32_t)(rare_word<MAJ>(f, w, N) >> ((s & 1) * 32));
  } else if (g < 64) {
    const uint32_t per = 64 / g, nw = g / 2;  // summary bits per bitmap word, bitmap words per summary word
    const uint64_t gm = (g == 64) ? ~0ull : ((1ull << g) - 1ull);
    for (uint32_t i = 0; i < nw; ++i) {
      const uint64_t w = (uint64_t)s * nw + i;
      if (w >= nwords) break;
      const uint64_t x = rare_word<MAJ>(f, w, N);
      if (!x) continue;
      for (uint32_t q = 0; q < per; ++q)
        if ((x >> (q * g)) & gm) out |= 1u << (i * per + q);
    }
  } else {
    const uint32_t wpb = g / 64;  // bitmap words per summary bit
    for (uint32_t b = 0; b < 32; ++b) {
      const uint64_t w0 = ((uint64_t)s * 32 + b) * wpb;
      uint64_t any = 0;
      for (uint32_t i = 0; i < wpb && w0 + i < nwords; ++i) any |= rare_word<MAJ>(f, w0 + i, N);
      if (any) out |= 1u << b;
    }
  }
  f.summ[s] = out;
}

// number of rare nodes of S_t from the running totals (0: the round is a no-op)
__device__ __forceinline__ uint64_t rare_count(const uint64_t* partial, uint64_t N, uint32_t R, uint32_t maj) {
  return maj ? N - partial[0] : partial[4 + R];
}

// mid-level summary word s (32 bits of g2 <= 64 nodes each) from the exact bitmap
template <int MAJ>
__device__ __forceinline__ void summ2_body(const FrontierBufs& f, uint32_t s, uint64_t N) {
  if (s >= f.summ2_words) return;
  const uint64_t nwords = (N + 63) >> 6;
  const uint32_t g2 = 1u << f.g2log, per = 64 / g2;  // summary bits per exact word
  const uint64_t gm = g2 == 64 ? ~0ull : ((1ull << g2) - 1ull);
  const uint64_t w0 = (uint64_t)s * 32 / per;
  uint32_t out = 0;
  for (uint32_t i = 0; i < 32 / per; ++i) {
    const uint64_t w = w0 + i;
    if (w >= nwords) break;
    const uint64_t x = rare_word<MAJ>(f, w, N);
    if (!x) continue;
    for (uint32_t q = 0; q < per; ++q)
      if ((x >> (q * g2)) & gm) out |= 1u << (i * per + q);
  }
  f.summ2[s] = out;
}

// whether this round uses the mid-level summary: the share of peers that hit the LDS summary,
// 1 - (1 - r)^g for a rare fraction r, reaches mid_frac (partial null: the caller decided)
__device__ __forceinline__ bool use_mid(const FrontierBufs& f, const uint64_t* partial, uint64_t N, uint32_t R,
                                        uint32_t maj) {
  if (!f.summ2) return false;
  if (!partial) return true;
  const float r = (float)rare_count(partial, N, R, maj) / (float)N;
  return 1.0f - __expf((float)(1u << f.glog) * log1pf(-fminf(r, 0.999999f))) >= f.mid_frac;
}

// blocks [0, summ_words / 256): the LDS summary; the rest: the mid-level summary (summ2)
__global__ __launch_bounds__(256) void frontier_summary_kernel(FrontierBufs f, uint64_t N, const uint64_t* partial,
                                                                uint32_t R, uint32_t maj) {
  if (partial && rare_count(partial, N, R, maj) == 0) return;
  const uint32_t b1 = (f.summ_words + 255) / 256;
  if (blockIdx.x >= b1) {  // always built (a few us): the scan alone decides whether to use it
    const uint32_t s = (blockIdx.x - b1) * 256 + threadIdx.x;
    if (maj)
      summ2_body<1>(f, s, N);
    else
      summ2_body<0>(f, s, N);
    return;
  }
  if (maj)
    summary_body<1>(f, N);
  else
    summary_body<0>(f, N);
}

// K1.  MODE: 1 push, 2 pull, 3 push-pull.  MAJ: majority value 0 (0) or full (1).
// Each block owns a contiguous node range; the rare-bitmap words of the next
// 64K nodes are staged in LDS so the per-node test never waits on memory.
// A summary hit is confirmed in the exact rare bitmap before S_t[p] is read
// (the bitmap is L2-resident; S is not).  Pull deltas belong to the node's own
// lane and are plain stores to P; push deltas are atomic ORs into D.
template <int MAJ, int MODE, bool FAULTS>  // FAULTS: edge loss / partitions active (§2.8)
// direct (kSparseDirect, MAJ 0): pushes into majority peers go to Sw (= S) instead of D.
__device__ __forceinline__ void scan_body(uint4* summ4, uint64_t* rws, const FrontierBufs& f,
                                          const uint64_t* __restrict__ S, uint64_t* Sw, uint64_t N, uint32_t R,
                                          uint32_t k, uint32_t t, uint32_t key0, uint32_t key1, uint64_t per_block,
                                          bool mark_d, bool direct, bool mid, const Faults& fa) {
  const uint32_t* summ = (const uint32_t*)summ4;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t n4 = (f.summ_words + 3) / 4;
  for (uint32_t i = tid; i < n4; i += kScanThreads) summ4[i] = ((const uint4*)f.summ)[i];

  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  const uint64_t fm = full_mask1(R), maj = MAJ ? fm : 0ull, nm1 = N - 1;
  const uint32_t glog = f.glog;
  auto summ_bit = [&](uint32_t p) -> bool { return (summ[p >> (glog + 5)] >> ((p >> glog) & 31u)) & 1u; };
  // node ids are < 2^32 (gossip_create checks N), so all index math is 32-bit
  const uint32_t b0 = blockIdx.x * (uint32_t)per_block, b1 = (uint32_t)min<uint64_t>((uint64_t)b0 + per_block, N);
  for (uint32_t c0 = b0; c0 < b1; c0 += kRwWords * 64) {
    const uint32_t c1 = min(c0 + kRwWords * 64, b1);
    __syncthreads();  // previous chunk done with rws
    for (uint32_t i = tid; i < ((c1 - c0 + 63) >> 6); i += kScanThreads) rws[i] = rare_word<MAJ>(f, (c0 >> 6) + i, N);
    __syncthreads();
    for (uint32_t base = c0; base < c1; base += kScanThreads * kScanUnroll) {
      uint64_t x[kScanUnroll], vp[kScanUnroll][4];
      uint32_t pp[kScanUnroll][4], hit[kScanUnroll], live[kScanUnroll];
      bool act[kScanUnroll], rn[kScanUnroll];
      // 1. draws and LDS summary tests (no global memory); live = edges not lost (§2.8)
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t n = base + u * kScanThreads + tid;
        const bool valid = n < c1;
        rn[u] = valid && ((rws[(n - c0) >> 6] >> lane) & 1ull);
        // a majority node only acts through a rare peer; push from an empty node and
        // pull into a full one are no-ops, so those nodes skip the draws entirely
        act[u] = valid && (rn[u] || !((!kPull && MAJ == 0) || (!kPush && MAJ == 1)));
        hit[u] = 0;
        live[u] = 0;
        if (act[u] && k <= 4) {
          const u32x4 r4 = philox4x32_10(u32x4{n, t, 0u, 0u}, key0, key1);
          u32x4 lw{0, 0, 0, 0};
          Reach rc{0u, 0xFFFFFFFFu};
          if (FAULTS) {
            if (fa.loss) lw = loss_draws(n, t, 0u, key0, key1);
            rc = reach_of(n, fa);  // n's partition block
          }
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            if (j >= k) break;
            pp[u][j] = peer_from_word(lane_of(r4, j), nm1, n);
            const bool lost = FAULTS && edge_lost(fa, rc, pp[u][j], lane_of(lw, j));
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
      // 2. summary hits: exact test in the rare bitmap (2 MiB at 2^24 nodes, L2-resident)
      // (all probes issued before any is consumed: one wait for the lot); past 2^25 nodes
      // the L2-resident mid-level summary first, so fewer probes reach the exact bitmap
      if (glog && mid) {
        uint32_t sw[kScanUnroll][4];
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            sw[u][j] = ((hit[u] >> j) & 1u) ? f.summ2[pp[u][j] >> (f.g2log + 5)] : 0u;
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            if (!((sw[u][j] >> ((pp[u][j] >> f.g2log) & 31u)) & 1u)) hit[u] &= ~(1u << j);
      }
      if (glog) {
        uint64_t rw[kScanUnroll][4];
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)  // raw bitmap words: nothing computed on them inside the branch
            rw[u][j] = ((hit[u] >> j) & 1u) ? (MAJ ? f.fullb[pp[u][j] >> 6] : f.nzb[pp[u][j] >> 6]) : 0ull;
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            const bool bit = (rw[u][j] >> (pp[u][j] & 63u)) & 1ull;  // p < N: always a valid bit
            if (bit == (MAJ != 0)) hit[u] &= ~(1u << j);  // rare = nonzero (MAJ 0) / not full (MAJ 1)
          }
      }
      // 3. S_t of the rare ends only (a majority node's value is known)
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t n = base + u * kScanThreads + tid;
        x[u] = rn[u] ? scan_ld(&S[n]) : maj;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) vp[u][j] = ((hit[u] >> j) & 1u) ? scan_ld(&S[pp[u][j]]) : maj;
      }
      // 4. deltas, in registers: every gather above is consumed here, before
      // the first atomic or store below.  (A load consumed after a store was
      // issued waits for that store too: vmcnt retires in order, so each edge
      // would wait out the previous edge's atomic round trip.)
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
      // 5. push deltas: atomics into D and the group's dirty byte
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u)
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
          if (dpush[u][j]) {
            if (MAJ == 0 && direct && !((hit[u] >> j) & 1u)) {  // an empty peer: nobody reads its S_t
              atomicOr((unsigned long long*)&Sw[pp[u][j]], (unsigned long long)dpush[u][j]);
              continue;
            }
            atomicOr((unsigned long long*)&f.D[pp[u][j]], (unsigned long long)dpush[u][j]);
            if (mark_d) f.dirtyD[pp[u][j] >> 6] = 1;
          }
      // k > 4: the draws are redone edge by edge (no registers for them)
      if (k > 4) {
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) {
          if (!act[u]) continue;
          const uint32_t n = base + u * kScanThreads + tid;
          uint64_t acc = 0;
          u32x4 r4{0, 0, 0, 0}, lw{0, 0, 0, 0};
          const Reach rc = FAULTS ? reach_of(n, fa) : Reach{0u, 0xFFFFFFFFu};  // n's partition block (§2.8)
          for (uint32_t j = 0; j < k; ++j) {
            if ((j & 3u) == 0) {
              r4 = philox4x32_10(u32x4{n, t, 0u, j >> 2}, key0, key1);
              if (FAULTS && fa.loss) lw = loss_draws(n, t, j >> 2, key0, key1);
            }
            const uint32_t p = peer_from_word(lane_of(r4, j & 3u), nm1, n);
            if (FAULTS && edge_lost(fa, rc, p, lane_of(lw, j & 3u))) continue;
            bool rp = summ_bit(p);
            if (rp && glog && mid) rp = (f.summ2[p >> (f.g2log + 5)] >> ((p >> f.g2log) & 31u)) & 1u;
            if (rp && glog) rp = (rare_word<MAJ>(f, p >> 6, N) >> (p & 63u)) & 1ull;
            if (!rn[u] && !rp) continue;  // both ends majority: nothing moves
            const uint64_t v = rp ? S[p] : maj;
            if (kPull) acc |= v;
            if (kPush) {
              const uint64_t d = x[u] & ~v;
              if (d && MAJ == 0 && direct && !rp) {
                atomicOr((unsigned long long*)&Sw[p], (unsigned long long)d);
              } else if (d) {
                atomicOr((unsigned long long*)&f.D[p], (unsigned long long)d);
                if (mark_d) f.dirtyD[p >> 6] = 1;
              }
            }
          }
          accs[u] = acc & ~x[u];
        }
      }
      // pull deltas: ORed into D beside the pushes (a separate array written with whole
      // 8-word chunks cost the commit a second read and clear per node: sparse rounds
      // -2 % at 2^24, profiles/r04_an/).  Direct rounds: a majority (empty) node's pull
      // goes straight into its S word, which nobody reads this round (the pushes into it
      // are atomic ORs too), so the commit reads no delta for it.
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t n = base + u * kScanThreads + tid;
        if (!accs[u]) continue;
        if (MAJ == 0 && direct && !rn[u]) {
          atomicOr((unsigned long long*)&Sw[n], (unsigned long long)accs[u]);
          continue;
        }
        atomicOr((unsigned long long*)&f.D[n], (unsigned long long)accs[u]);
        if (mark_d) f.dirtyD[n >> 6] = 1;
      }
    }
  }
}

// Queued scan (round 5, FrontierBufs::scan_q, k <= 4).  In the rounds between the light and the
// heavy ones most waves of 128 nodes hold a few edges with a possibly rare end, and resolving
// them where they are drawn costs every such batch the whole chain of round trips (summary
// probes, S_t gathers, atomics) for a handful of lanes: with 16 waves per CU (the LDS summary
// allows one block) those rounds were latency-bound at 2-3x their Philox floor.  Here a wave
// appends each such edge to its own LDS queue and resolves the queue 128 edges at a time: one
// chain per 128 edges, two edges per lane, every load of the chain issued before any is used.
//
// A queued edge: x = node - block base (< 2^24) | rare(n) << 24 | summary hit(p) << 25, y = p.
// Both ends' deltas are relative to S_t, so splitting a node's pulls over queue entries (one
// OR per edge instead of one per node) changes no bit.
constexpr uint32_t kQFlush = 128;             // edges resolved per flush (2 per lane)
constexpr uint32_t kQCap = kQFlush + 64;      // a flush starts as soon as kQFlush are queued

template <int MAJ, int MODE>
__device__ __forceinline__ void scan_flush(const uint2* qw, uint32_t nf, const FrontierBufs& f,
                                           const uint64_t* __restrict__ S, uint64_t* Sw, uint32_t b0, uint64_t maj,
                                           bool mark_d, bool direct, bool mid, uint32_t lane) {
  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  constexpr int kE = kQFlush / 64;
  uint32_t n[kE], p[kE];
  bool rn[kE], hit[kE];
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    const uint32_t i = lane + 64u * e;
    const uint2 q = i < nf ? qw[i] : uint2{0u, 0u};
    n[e] = b0 + (q.x & 0xFFFFFFu);
    rn[e] = (q.x >> 24) & 1u;
    hit[e] = (q.x >> 25) & 1u;
    p[e] = q.y;
  }
  if (f.glog && mid) {
    uint32_t sw[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) sw[e] = hit[e] ? f.summ2[p[e] >> (f.g2log + 5)] : 0u;
#pragma unroll
    for (int e = 0; e < kE; ++e) hit[e] = hit[e] && ((sw[e] >> ((p[e] >> f.g2log) & 31u)) & 1u);
  }
  if (f.glog) {
    uint64_t rw[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) rw[e] = hit[e] ? (MAJ ? f.fullb[p[e] >> 6] : f.nzb[p[e] >> 6]) : 0ull;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const bool bit = (rw[e] >> (p[e] & 63u)) & 1ull;
      if (bit == (MAJ != 0)) hit[e] = false;
    }
  }
  uint64_t x[kE], vp[kE];
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    x[e] = rn[e] ? scan_ld(&S[n[e]]) : maj;
    vp[e] = hit[e] ? scan_ld(&S[p[e]]) : maj;
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
    if (dpush[e]) {
      if (MAJ == 0 && direct && !hit[e]) {  // an empty peer: nobody reads its S_t
        atomicOr((unsigned long long*)&Sw[p[e]], (unsigned long long)dpush[e]);
      } else {
        atomicOr((unsigned long long*)&f.D[p[e]], (unsigned long long)dpush[e]);
        if (mark_d) f.dirtyD[p[e] >> 6] = 1;
      }
    }
    if (dpull[e]) {
      if (MAJ == 0 && direct && !rn[e]) {
        atomicOr((unsigned long long*)&Sw[n[e]], (unsigned long long)dpull[e]);
      } else {
        atomicOr((unsigned long long*)&f.D[n[e]], (unsigned long long)dpull[e]);
        if (mark_d) f.dirtyD[n[e] >> 6] = 1;
      }
    }
  }
}

template <int MAJ, int MODE, bool FAULTS>
__device__ __forceinline__ void scan_body_q(uint4* summ4, uint64_t* rws, uint2* qs, const FrontierBufs& f,
                                            const uint64_t* __restrict__ S, uint64_t* Sw, uint64_t N, uint32_t R,
                                            uint32_t k, uint32_t t, uint32_t key0, uint32_t key1, uint64_t per_block,
                                            bool mark_d, bool direct, bool mid, const Faults& fa) {
  const uint32_t* summ = (const uint32_t*)summ4;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  uint2* qw = qs + (tid >> 6) * kQCap;  // this wave's queue
  const uint32_t n4 = (f.summ_words + 3) / 4;
  for (uint32_t i = tid; i < n4; i += kScanThreads) summ4[i] = ((const uint4*)f.summ)[i];

  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  const uint64_t maj = MAJ ? full_mask1(R) : 0ull;
  const uint32_t nm1 = (uint32_t)(N - 1), glog = f.glog;
  auto summ_bit = [&](uint32_t p) -> bool { return (summ[p >> (glog + 5)] >> ((p >> glog) & 31u)) & 1u; };
  const uint32_t b0 = blockIdx.x * (uint32_t)per_block, b1 = (uint32_t)min<uint64_t>((uint64_t)b0 + per_block, N);
  uint32_t qn = 0;  // entries in this wave's queue (wave-uniform)
  for (uint32_t c0 = b0; c0 < b1; c0 += kRwWords * 64) {
    const uint32_t c1 = min(c0 + kRwWords * 64, b1);
    __syncthreads();  // previous chunk done with rws
    for (uint32_t i = tid; i < ((c1 - c0 + 63) >> 6); i += kScanThreads) rws[i] = rare_word<MAJ>(f, (c0 >> 6) + i, N);
    __syncthreads();
    for (uint32_t base = c0; base < c1; base += kScanThreads * kScanUnroll) {
      uint32_t pp[kScanUnroll][4], cand[kScanUnroll];
      bool rn[kScanUnroll];
      bool any = false;
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t n = base + u * kScanThreads + tid;
        const bool valid = n < c1;
        rn[u] = valid && ((rws[(n - c0) >> 6] >> lane) & 1ull);
        const bool act = valid && (rn[u] || !((!kPull && MAJ == 0) || (!kPush && MAJ == 1)));
        cand[u] = 0;  // bit j: edge j is live and has a rare or possibly rare end
        if (act) {
          const u32x4 r4 = philox4x32_10(u32x4{n, t, 0u, 0u}, key0, key1);
          u32x4 lw{0, 0, 0, 0};
          Reach rc{0u, 0xFFFFFFFFu};
          if (FAULTS) {
            if (fa.loss) lw = loss_draws(n, t, 0u, key0, key1);
            rc = reach_of(n, fa);
          }
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            if (j >= k) break;
            pp[u][j] = peer_from_word(lane_of(r4, j), nm1, n);
            const bool lost = FAULTS && edge_lost(fa, rc, pp[u][j], lane_of(lw, j));
            if (!lost && (rn[u] || summ_bit(pp[u][j]))) cand[u] |= 1u << j;
          }
        }
        any = any || cand[u] != 0u;
      }
      if (!__ballot(any)) continue;  // most waves of the light rounds
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const uint32_t n = base + u * kScanThreads + tid;
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
            qw[pos] = uint2{(n - b0) | (uint32_t)rn[u] << 24 | (uint32_t)h << 25, pp[u][j]};
          }
          qn += (uint32_t)__popcll(m);
          if (qn >= kQFlush) {
            __builtin_amdgcn_wave_barrier();
            scan_flush<MAJ, MODE>(qw, kQFlush, f, S, Sw, b0, maj, mark_d, direct, mid, lane);
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
    scan_flush<MAJ, MODE>(qw, qn, f, S, Sw, b0, maj, mark_d, direct, mid, lane);
  }
}

// Binned sparse scan (round 6, FrontierBufs::brec).  In the heaviest sparse rounds at 2^27
// (1-4 % rare nodes) the LDS summary (128 nodes per bit) is saturated and every edge of a
// majority node costs a random probe of the mid-level summary in the L2 and a quarter of them
// one of the exact bitmap in the MALL: ~3.5 * 10^8 random requests, which bound the scan at
// ~2.9 ms whatever the occupancy (an LDS-free scan at 8 waves per SIMD measured the same,
// DESIGN.md §3.7).  Here the peer test moves into LDS the way the dense round moves its
// gathers: K1a draws every node's peers and bins its live edges by peer tile (2^19 nodes) into
// 4-B records {p - tile base | rare(n) << 19 | n - region base << 20}, one contiguous
// tile-sorted run list per 4096-node region plus a u16 run-start table; K1b loads one tile's
// exact rare bitmap (64 KiB) into LDS, walks that tile's run of every region of its chunk and
// resolves the edges with a rare end through the per-wave queue of the queued scan (S_t gathers
// and atomics).  Traffic: 8 B per node written and read (k = 2) instead of the probes.
constexpr uint32_t kBsRegLog = 12;                 // 4096 senders per region (n - region base: 12 bits)
#ifndef GOSSIP_BS_TILE_LOG
#define GOSSIP_BS_TILE_LOG 19
#endif
#ifndef GOSSIP_BS_TEST_WAVES
#define GOSSIP_BS_TEST_WAVES 4
#endif
constexpr uint32_t kBsTileLog = GOSSIP_BS_TILE_LOG;  // 2^19 peers per tile (p - tile base: 19 bits; 64 KiB bitmap)
constexpr uint32_t kBsTileWords = 1u << (kBsTileLog - 6);
constexpr int kBsEmitThreads = 1024;               // 4 senders per thread and region
constexpr int kBsTestThreads = 1024;
constexpr uint32_t kBsEmitGrid = 512;              // persistent emit blocks (2 per CU: 68 KiB of LDS each)
constexpr uint32_t kBsMaxTiles = kBsEmitThreads;   // one tile counter per emit thread: N <= 2^29
constexpr uint32_t kBsTestBlocks = 1024;           // K1b blocks: tiles x region chunks
#ifndef GOSSIP_BS_UNROLL
#define GOSSIP_BS_UNROLL 4
#endif
constexpr int kBsUnroll = GOSSIP_BS_UNROLL;        // K1b record windows in flight per wave

template <int MAJ, int MODE, bool FAULTS, int KM>  // KM: peers per node held in registers (>= k)
__device__ __forceinline__ void bs_emit_body(uint32_t* cnt, uint32_t* stg, const FrontierBufs& f, uint64_t N,
                                             uint32_t k, uint32_t t, uint32_t key0, uint32_t key1, const Faults& fa) {
  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  constexpr int kU = (1 << kBsRegLog) / kBsEmitThreads;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t nm1 = (uint32_t)(N - 1), ntiles = f.btiles, nreg = f.bregions, rcap = k << kBsRegLog;
  for (uint32_t i = tid; i < ntiles; i += kBsEmitThreads) cnt[i] = 0;
  for (uint32_t r = blockIdx.x; r < nreg; r += gridDim.x) {
    const uint32_t n0 = r << kBsRegLog;
    __syncthreads();  // cnt zeroed (first region) / stg drained (the previous one)
    uint32_t pp[kU][KM], rk[kU][KM], live[kU];
    bool rn[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t n = n0 + u * kBsEmitThreads + tid;
      const bool valid = n < N;
      const uint32_t w0 = __builtin_amdgcn_readfirstlane((n0 + u * kBsEmitThreads + (tid & ~63u)) >> 6);
      rn[u] = valid && ((rare_word<MAJ>(f, w0, N) >> lane) & 1ull);
      const bool act = valid && (rn[u] || !((!kPull && MAJ == 0) || (!kPush && MAJ == 1)));
      live[u] = 0;
      if (act) {
        const u32x4 r4 = philox4x32_10(u32x4{n, t, 0u, 0u}, key0, key1);
        u32x4 lw{0, 0, 0, 0};
        Reach rc{0u, 0xFFFFFFFFu};
        if (FAULTS) {
          if (fa.loss) lw = loss_draws(n, t, 0u, key0, key1);
          rc = reach_of(n, fa);
        }
#pragma unroll
        for (uint32_t j = 0; j < KM; ++j) {
          if (j >= k) break;
          pp[u][j] = peer_from_word(lane_of(r4, j), nm1, n);
          const bool lost = FAULTS && edge_lost(fa, rc, pp[u][j], lane_of(lw, j));
          if (!lost) {
            live[u] |= 1u << j;
            rk[u][j] = atomicAdd(&cnt[pp[u][j] >> kBsTileLog], 1u);  // rank inside the tile's run
          }
        }
      }
    }
    __syncthreads();
    // run starts: exclusive scan over the tiles (one counter per thread), the table row, and
    // cnt back to zero for the next region once every edge has read its start
    uint32_t total = 0;
    const uint32_t c = tid < ntiles ? cnt[tid] : 0u;
    const uint32_t st0 = block_exscan<kBsEmitThreads>(c, stg, &total);  // (stg as scratch: not yet in use)
    uint16_t* row = f.btab + (size_t)r * (ntiles + 1);
    if (tid < ntiles) {
      row[tid] = (uint16_t)st0;
      cnt[tid] = st0;
    }
    if (tid == 0) row[ntiles] = (uint16_t)total;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t nl = u * kBsEmitThreads + tid;
#pragma unroll
      for (uint32_t j = 0; j < KM; ++j)
        if ((live[u] >> j) & 1u) {
          const uint32_t p = pp[u][j];
          stg[cnt[p >> kBsTileLog] + rk[u][j]] =
              (p & ((1u << kBsTileLog) - 1u)) | (uint32_t)rn[u] << kBsTileLog | nl << (kBsTileLog + 1);
        }
    }
    __syncthreads();
    uint32_t* out = f.brec + (size_t)r * rcap;
    for (uint32_t i = tid; i < total; i += kBsEmitThreads) out[i] = stg[i];
    for (uint32_t i = tid; i < ntiles; i += kBsEmitThreads) cnt[i] = 0;
  }
}

// (k <= 2 without faults: 8 waves per SIMD, two blocks per CU overlap one region's Philox with
// another's stores; the other instances would spill at 64 VGPRs)
template <int MODE, bool FAULTS, int KM>
__global__ __launch_bounds__(kBsEmitThreads, (KM == 2 && !FAULTS) ? 8 : 4) void frontier_bs_emit_kernel(FrontierBufs f, uint64_t N, uint32_t R,
                                                                         uint32_t k, uint32_t t, uint32_t key0,
                                                                         uint32_t key1, const uint64_t* partial,
                                                                         uint32_t maj, Faults fa) {
  __shared__ uint32_t cnt[kBsMaxTiles];
  __shared__ uint32_t stg[4u << kBsRegLog];
  if (rare_count(partial, N, R, maj) == 0) return;
  if (maj)
    bs_emit_body<1, MODE, FAULTS, KM>(cnt, stg, f, N, k, t, key0, key1, fa);
  else
    bs_emit_body<0, MODE, FAULTS, KM>(cnt, stg, f, N, k, t, key0, key1, fa);
}

// a queued edge of K1b: x = n | rare(n) << 31, y = p | rare(p) << 31 (N <= 2^31: bs_path_ok)
template <int MAJ, int MODE>
__device__ __forceinline__ void bs_flush(const uint2* qw, uint32_t nf, const FrontierBufs& f,
                                         const uint64_t* __restrict__ S, uint64_t* Sw, uint64_t maj, bool mark_d,
                                         bool direct, uint32_t lane) {
  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  constexpr int kE = kQFlush / 64;
  uint32_t n[kE], p[kE];
  bool rn[kE], hit[kE];
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    const uint32_t i = lane + 64u * e;
    const uint2 q = i < nf ? qw[i] : uint2{0u, 0u};
    n[e] = q.x & 0x7FFFFFFFu;
    rn[e] = q.x >> 31;
    p[e] = q.y & 0x7FFFFFFFu;
    hit[e] = q.y >> 31;
  }
  uint64_t x[kE], vp[kE];
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    x[e] = rn[e] ? scan_ld(&S[n[e]]) : maj;
    vp[e] = hit[e] ? scan_ld(&S[p[e]]) : maj;
  }
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    const bool any = rn[e] || hit[e];  // (an empty slot: neither)
    const uint64_t dpush = kPush && any ? x[e] & ~vp[e] : 0ull;
    const uint64_t dpull = kPull && any ? vp[e] & ~x[e] : 0ull;
    if (dpush) {
      if (MAJ == 0 && direct && !hit[e]) {
        atomicOr((unsigned long long*)&Sw[p[e]], (unsigned long long)dpush);
      } else {
        atomicOr((unsigned long long*)&f.D[p[e]], (unsigned long long)dpush);
        if (mark_d) f.dirtyD[p[e] >> 6] = 1;
      }
    }
    if (dpull) {
      if (MAJ == 0 && direct && !rn[e]) {
        atomicOr((unsigned long long*)&Sw[n[e]], (unsigned long long)dpull);
      } else {
        atomicOr((unsigned long long*)&f.D[n[e]], (unsigned long long)dpull);
        if (mark_d) f.dirtyD[n[e] >> 6] = 1;
      }
    }
  }
}

// K1b: block = (peer tile T, region chunk).  A wave takes 64 regions at a time (lane = region),
// compacts their nonempty runs of tile T and walks the concatenation lane-strided, 64 records
// per window: the run of record i0 + lane is found from the wave-uniform run starts by
// readlane (a window spans ~3 of the ~32-record runs).
template <int MAJ, int MODE>
__device__ __forceinline__ void bs_test_body(uint64_t* bm, uint2* qs, uint64_t* wbs, uint32_t* rtab, const FrontierBufs& f,
                                             const uint64_t* __restrict__ S, uint64_t* Sw, uint64_t N, uint32_t R,
                                             uint32_t k, bool mark_d, bool direct) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t ntiles = f.btiles, nreg = f.bregions, rcap = k << kBsRegLog;
  // XCD-aware: blocks b, b + 8, ... share an XCD (and its L2); give them adjacent tiles of one
  // region chunk, so that the runs of neighbouring tiles (adjacent in each region's list) share
  // their boundary lines in that L2 instead of fetching them twice
  const uint32_t nch = gridDim.x / ntiles;
  uint32_t T = blockIdx.x % ntiles, chunk = blockIdx.x / ntiles;
  if (ntiles % 8 == 0) {
    const uint32_t per_x = ntiles / 8, j = blockIdx.x / 8;
    T = (blockIdx.x % 8) * per_x + j % per_x;
    chunk = j / per_x;
  }
  const uint32_t per = (nreg + nch - 1) / nch, r0 = chunk * per, r1 = min(r0 + per, nreg);
  const uint64_t maj = MAJ ? full_mask1(R) : 0ull, nwords = (N + 63) >> 6, w0 = (uint64_t)T * kBsTileWords;
  for (uint32_t i = tid; i < kBsTileWords; i += kBsTestThreads)
    bm[i] = w0 + i < nwords ? rare_word<MAJ>(f, w0 + i, N) : 0ull;
  __syncthreads();
  uint2* qw = qs + wave * kQCap;
  uint64_t* wb = wbs + wave * 16;
  uint32_t* rbase = rtab + wave * 128;
  uint32_t* rreg = rbase + 64;
  uint32_t qn = 0;
  const uint32_t pbase = T << kBsTileLog;
  for (uint32_t rb = r0 + wave * 64; rb < r1; rb += (kBsTestThreads / 64) * 64) {
    const uint32_t r = rb + lane;
    uint32_t s = 0, len = 0;
    if (r < r1) {  // (the transposed table: a wave reads two runs of 64 consecutive u16)
      s = f.btabT[(size_t)T * nreg + r];
      len = (uint32_t)f.btabT[(size_t)(T + 1) * nreg + r] - s;
    }
    // compact the nonempty runs to the low lanes (their order kept), then exclusive starts E
    const uint64_t ne = __ballot(len != 0);
    const uint32_t m = (uint32_t)__popcll(ne);
    const uint32_t dstl = __builtin_amdgcn_mbcnt_hi((uint32_t)(ne >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ne, 0u));
    // ds_permute writes by destination lane: nonempty lanes to slots [0, m) in order, the
    // empty ones behind them (a permutation: no two lanes share a slot)
    const uint32_t dst = len ? dstl : m + (lane - dstl);
    const uint32_t cr = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4), (int)r);
    const uint32_t cs = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4), (int)s);
    const uint32_t cl = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4), (int)len);
    const uint32_t rl = lane < m ? cl : 0u;
    uint32_t inc = rl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    const uint32_t E = inc - rl;                                  // start of compacted run `lane`
    const uint32_t total = __shfl(inc, 63, 64);
    // per compacted run: its record-index base (region offset + run start - E, mod 2^32) and region
    if (lane < m) {
      rbase[lane] = cr * rcap + cs - E;
      rreg[lane] = cr;
    }
    // windows of 1024 records: the run starts inside a window as a 16-word bitmap; in step s
    // (records w + 64 s + lane) every lane reads word s, so a record's run is the count of
    // starts before the window + the starts in words < s + popcount(word s up to its lane) - 1:
    // no search and no dependence between steps
    for (uint32_t w = 0; w < total; w += 1024) {
      if (lane < 16) wb[lane] = 0ull;
      __builtin_amdgcn_wave_barrier();
      if (lane < m && E >= w && E < w + 1024) atomicOr((unsigned long long*)&wb[(E - w) >> 6], 1ull << ((E - w) & 63u));
      __builtin_amdgcn_wave_barrier();
      const uint64_t myw = lane < 16 ? wb[lane] : 0ull;
      uint32_t cu = (uint32_t)__popcll(myw);
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const uint32_t y = __shfl_up(cu, o, 64);
        if (lane >= (uint32_t)o) cu += y;
      }
      cu -= (uint32_t)__popcll(myw);  // starts in the words before this lane's
      const uint32_t before = (uint32_t)__popcll(__ballot(lane < m && E < w));
      const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
      const uint32_t nsteps = min(16u, (total - w + 63) >> 6);
      for (uint32_t s0 = 0; s0 < nsteps; s0 += kBsUnroll) {
      uint32_t rec[kBsUnroll], rrs[kBsUnroll];
#pragma unroll
      for (int u = 0; u < kBsUnroll; ++u) {
        const uint32_t st = min(s0 + u, 15u), i = w + 64u * (s0 + u) + lane;
        const uint64_t word = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(myw >> 32), (int)st) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)myw, (int)st);
        const uint32_t cus = (uint32_t)__builtin_amdgcn_readlane((int)cu, (int)st);
        const bool valid = s0 + u < nsteps && i < total;
        const uint32_t run = valid ? before + cus + (uint32_t)__popcll(word & upto) - 1u : 0u;
        rrs[u] = rreg[run];
        rec[u] = valid ? f.brec[rbase[run] + i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kBsUnroll; ++u) {
        const uint32_t pl = rec[u] & ((1u << kBsTileLog) - 1u);
        const bool valid = s0 + u < nsteps && w + 64u * (s0 + u) + lane < total;
        const bool rnb = valid && ((rec[u] >> kBsTileLog) & 1u);
        const bool hit = valid && ((bm[pl >> 6] >> (pl & 63u)) & 1ull);
        const bool c = rnb || hit;
        const uint64_t mk = __ballot(c);
        if (!mk) continue;
        if (c) {
          const uint32_t pos =
              qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
          const uint32_t n = (rrs[u] << kBsRegLog) + (rec[u] >> (kBsTileLog + 1));
          qw[pos] = uint2{n | (uint32_t)rnb << 31, (pbase + pl) | (uint32_t)hit << 31};
        }
        qn += (uint32_t)__popcll(mk);
        if (qn >= kQFlush) {
          __builtin_amdgcn_wave_barrier();
          bs_flush<MAJ, MODE>(qw, kQFlush, f, S, Sw, maj, mark_d, direct, lane);
          qn -= kQFlush;
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
    bs_flush<MAJ, MODE>(qw, qn, f, S, Sw, maj, mark_d, direct, lane);
  }
}

template <int MODE>
__global__ __launch_bounds__(kBsTestThreads, GOSSIP_BS_TEST_WAVES) void frontier_bs_test_kernel(FrontierBufs f, uint64_t* S, uint64_t N,
                                                                         uint32_t R, uint32_t k,
                                                                         const uint64_t* partial, uint32_t maj,
                                                                         uint32_t mark_d, uint32_t direct) {
  __shared__ uint64_t bm[kBsTileWords];
  __shared__ uint2 qs[(kBsTestThreads / 64) * kQCap];
  __shared__ uint64_t wbs[(kBsTestThreads / 64) * 16];
  __shared__ uint32_t rtab[(kBsTestThreads / 64) * 128];
  if (rare_count(partial, N, R, maj) == 0) return;
  if (maj)
    bs_test_body<1, MODE>(bm, qs, wbs, rtab, f, S, S, N, R, k, mark_d != 0, false);
  else
    bs_test_body<0, MODE>(bm, qs, wbs, rtab, f, S, S, N, R, k, mark_d != 0, direct != 0);
}

template <int MODE, bool FAULTS>
__global__ __launch_bounds__(kScanThreads, kScanWaves) void frontier_scan_kernel(FrontierBufs f, uint64_t* S,
                                                                      uint64_t N, uint32_t R, uint32_t k, uint32_t t,
                                                                      uint32_t key0, uint32_t key1, uint64_t per_block,
                                                                      const uint64_t* partial, uint32_t maj,
                                                                      uint32_t mark_d, uint32_t direct, Faults fa) {
  __shared__ uint4 summ4[kSummBits / 128];
  __shared__ uint64_t rws[kRwWords];
  __shared__ uint2 qs[(kScanThreads / 64) * kQCap];  // 24 KiB: 128 + 4 + 24 KiB of the CU's 160
  if (rare_count(partial, N, R, maj) == 0) return;  // converged (or nothing injected): nothing moves
  const bool mid = use_mid(f, partial, N, R, maj);  // (the summary kernel built summ2 this round)
  if (f.scan_q && k <= 4) {
    if (maj)
      scan_body_q<1, MODE, FAULTS>(summ4, rws, qs, f, S, S, N, R, k, t, key0, key1, per_block, mark_d != 0, false, mid,
                                   fa);
    else
      scan_body_q<0, MODE, FAULTS>(summ4, rws, qs, f, S, S, N, R, k, t, key0, key1, per_block, mark_d != 0,
                                   direct != 0, mid, fa);
    return;
  }
  if (maj)
    scan_body<1, MODE, FAULTS>(summ4, rws, f, S, S, N, R, k, t, key0, key1, per_block, mark_d != 0, false, mid, fa);
  else
    scan_body<0, MODE, FAULTS>(summ4, rws, f, S, S, N, R, k, t, key0, key1, per_block, mark_d != 0, direct != 0,
                               mid, fa);
}

// Stats of one 64-node group whose words went from old to nw (old == 0 in a
// rebuild), and its two bitmap words (wave-exclusive plain stores).
// Per-rumor counts are summed bit-sliced per lane (slice b = weight 2^b, up to 31 groups) and
// transposed once per slice when the slices fill up: 5 transposes per 31 groups instead of one
// per group (the transpose was most of a commit's VALU work).
struct GroupStats {
  uint64_t hash = 0;
  uint32_t full = 0, nz = 0, c_lane = 0;
  uint64_t sl[5] = {0, 0, 0, 0, 0};
  uint32_t sn = 0;  // words added to sl since the last fold (wave-uniform)

  __device__ __forceinline__ void fold(uint32_t lane) {
#pragma unroll
    for (uint32_t b = 0; b < 5; ++b) {
      if (__ballot(sl[b] != 0)) c_lane += (uint32_t)__popcll(transpose64(sl[b], lane)) << b;
      sl[b] = 0;
    }
    sn = 0;
  }

  __device__ __forceinline__ void add(const FrontierBufs& f, uint64_t g, uint64_t n, bool valid, uint64_t old,
                                      uint64_t nw, uint64_t fm, bool do_hash, uint32_t lane) {
    const uint64_t nzw = __ballot(valid && nw != 0), fw = __ballot(valid && nw == fm);
    if (lane == 0) {
      f.nzb[g] = nzw;
      f.fullb[g] = fw;
    }
    const uint64_t nb = nw & ~old;
    full += (uint32_t)__popcll(__ballot(valid && nw == fm && old != fm));
    nz += (uint32_t)__popcll(__ballot(valid && nw != 0 && old == 0));
    if (do_hash && nb) {
      hash += mix64(nw + (f.id0 + n) * kGold64);
      if (old) hash -= mix64(old + (f.id0 + n) * kGold64);
    }
    if (__ballot(nb != 0)) {
      uint64_t c = nb;  // ripple-carry add into the slices
#pragma unroll
      for (uint32_t b = 0; b < 5; ++b) {
        const uint64_t t = sl[b] & c;
        sl[b] ^= c;
        c = t;
      }
      if (++sn == 31) fold(lane);
    }
  }

  // block-level fold into the running totals
  __device__ __forceinline__ void flush(uint64_t* __restrict__ partial, uint32_t R, uint32_t* cnt,
                                        uint64_t (*red)[kCommitThreads / 64]) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (sn) fold(lane);
    if (lane < R && c_lane) atomicAdd(&cnt[lane], c_lane);
    const uint64_t h = wave_sum64(hash);
    if (lane == 0) {
      red[0][wave] = full;
      red[1][wave] = nz;
      red[2][wave] = h;
    }
    __syncthreads();
    if (tid == 0) {
      uint64_t a = 0, b = 0, hh = 0;
      for (int w = 0; w < kCommitThreads / 64; ++w) {
        a += red[0][w];
        b += red[1][w];
        hh += red[2][w];
      }
      if (a) atomicAdd((unsigned long long*)&partial[0], (unsigned long long)a);
      if (hh) atomicAdd((unsigned long long*)&partial[3], (unsigned long long)hh);
      if (b) atomicAdd((unsigned long long*)&partial[4 + R], (unsigned long long)b);
    }
    if (tid < R && cnt[tid]) atomicAdd((unsigned long long*)&partial[4 + tid], (unsigned long long)cnt[tid]);
  }
};

// Absolute stats + bitmaps of S (partial zeroed by the caller).
__global__ __launch_bounds__(kCommitThreads) void frontier_rebuild_kernel(FrontierBufs f, const uint64_t* __restrict__ S,
                                                                           uint64_t N, uint64_t* __restrict__ partial,
                                                                           uint32_t R, uint32_t flags) {
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red[3][kCommitThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 64) cnt[tid] = 0;
  __syncthreads();
  const uint64_t fm = full_mask1(R), ngroups = (N + 63) >> 6;
  GroupStats gs;
  for (uint64_t g = (uint64_t)blockIdx.x * (kCommitThreads / 64) + wave; g < ngroups;
       g += (uint64_t)gridDim.x * (kCommitThreads / 64)) {
    const uint64_t n = (g << 6) + lane;
    const bool valid = n < N;
    gs.add(f, g, n, valid, 0ull, valid ? S[n] : 0ull, fm, (flags & 1u) != 0, lane);
  }
  gs.flush(partial, R, cnt, red);
}

// K2: a wave takes 64 groups, finds the dirty ones by one coalesced load of
// their flags, and commits kCommitUnroll of them per step: S |= D in place,
// D and the flags back to zero, bitmaps and stats deltas.  dmode
// kSparseAllD: every group's D is read (the scan kept no flags);
// kSparseDirect: every group is visited (majority nodes took their deltas in S),
// D read where flagged, and the totals are absolute (partial zeroed before).
__global__ __launch_bounds__(kCommitThreads) void frontier_commit_kernel(FrontierBufs f, uint64_t* __restrict__ S,
                                                                          uint64_t N, uint64_t* __restrict__ partial,
                                                                          uint32_t R, uint32_t flags, uint32_t dmode) {
  const bool all_d = dmode == kSparseAllD, abs_t = dmode == kSparseDirect;
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red[3][kCommitThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < 64) cnt[tid] = 0;
  __syncthreads();
  const uint64_t fm = full_mask1(R), ngroups = (N + 63) >> 6;
  const bool do_hash = (flags & 1u) != 0;
  GroupStats gs;
  for (uint64_t c = (uint64_t)blockIdx.x * (kCommitThreads / 64) + wave; (c << kCommitChunkLog) < ngroups;
       c += (uint64_t)gridDim.x * (kCommitThreads / 64)) {
    const uint64_t gl = (c << kCommitChunkLog) + lane;
    const bool gv = lane < (1u << kCommitChunkLog) && gl < ngroups;
    const uint8_t fd = gv ? (all_d ? 1 : f.dirtyD[gl]) : 0;
    if (fd && !all_d) f.dirtyD[gl] = 0;
    const uint64_t mD = __ballot(fd != 0);
    uint64_t mask = abs_t ? __ballot(gv) : mD;
    while (mask) {
      uint32_t gi[kCommitUnroll];
      uint32_t cntg = 0;
#pragma unroll
      for (int u = 0; u < kCommitUnroll; ++u) {
        gi[u] = mask ? (uint32_t)__builtin_ctzll(mask) : 64u;
        if (mask) {
          mask &= mask - 1;
          ++cntg;
        }
      }
      uint64_t d[kCommitUnroll], old[kCommitUnroll], rw[kCommitUnroll];
      // direct rounds: D holds deltas of S_t's rare (nonzero) nodes only (every delta into a
      // majority node went to S), so D is read only where S_t's bitmap word has the node
#pragma unroll
      for (int u = 0; u < kCommitUnroll; ++u) rw[u] = abs_t && gi[u] < 64 ? f.nzb[(c << kCommitChunkLog) + gi[u]] : ~0ull;
#pragma unroll
      for (int u = 0; u < kCommitUnroll; ++u) {
        const uint64_t n = (((c << kCommitChunkLog) + (gi[u] & 63u)) << 6) + lane;
        const bool valid = gi[u] < 64 && n < N;
        const bool hd = gi[u] < 64 && ((mD >> gi[u]) & 1ull) && ((rw[u] >> lane) & 1ull);
        d[u] = valid && hd ? f.D[n] : 0ull;
        old[u] = valid ? S[n] : 0ull;
      }
#pragma unroll
      for (int u = 0; u < kCommitUnroll; ++u) {
        if ((uint32_t)u >= cntg) break;
        const uint64_t g = (c << kCommitChunkLog) + gi[u];
        const uint64_t n = (g << 6) + lane;
        const bool valid = n < N;
        const uint64_t nw = old[u] | d[u];
        // write whole 8-word (64 B) chunks: a partial chunk costs the HBM a read-modify-write
        const uint32_t sh = lane & ~7u;
        const uint64_t chg = __ballot(valid && nw != old[u]), dz = __ballot(d[u] != 0);
        if (valid && ((chg >> sh) & 0xFFull)) S[n] = nw;
        if (valid && ((dz >> sh) & 0xFFull)) f.D[n] = 0;
        gs.add(f, g, n, valid, abs_t ? 0ull : old[u], nw, fm, do_hash, lane);
      }
    }
  }
  gs.flush(partial, R, cnt, red);
}

// Client broadcast with exact running totals and bitmaps (atomics: two rumors
// may share an origin; each atomic's own old value makes every delta exact).
__global__ void frontier_inject_kernel(FrontierBufs f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                       uint32_t key0, uint32_t key1, int64_t node, uint32_t rumor, uint32_t flags) {
  const uint32_t r = node >= 0 ? rumor : blockIdx.x * blockDim.x + threadIdx.x;
  if (node >= 0 && (blockIdx.x | threadIdx.x)) return;
  if (r >= R) return;
  const uint64_t n = node >= 0 ? (uint64_t)node : origin_of(r, N, key0, key1);
  const uint64_t bit = 1ull << r, fm = full_mask1(R);
  const uint64_t old = atomicOr((unsigned long long*)&S[n], (unsigned long long)bit);
  if (old & bit) return;
  const uint64_t nw = old | bit;
  atomicAdd((unsigned long long*)&partial[4 + r], 1ull);
  if (old == 0) {
    atomicAdd((unsigned long long*)&partial[4 + R], 1ull);
    atomicOr((unsigned long long*)&f.nzb[n >> 6], 1ull << (n & 63));
  }
  if (nw == fm) {
    atomicAdd((unsigned long long*)&partial[0], 1ull);
    atomicOr((unsigned long long*)&f.fullb[n >> 6], 1ull << (n & 63));
  }
  if (flags & 1u)
    atomicAdd((unsigned long long*)&partial[3],
              (unsigned long long)(mix64(nw + n * kGold64) - (old ? mix64(old + n * kGold64) : 0ull)));
}

uint32_t commit_grid(uint64_t N) {
  const uint64_t groups = (N + 63) >> 6, per = kCommitThreads / 64;
  const uint64_t blocks = (groups + per - 1) / per;
  return (uint32_t)(blocks < kCommitMaxBlocks ? blocks : kCommitMaxBlocks);
}

}  // namespace

uint32_t frontier_glog(uint64_t N) {
  uint32_t glog = 0;
  while ((((N + (1ull << glog) - 1) >> glog) > kSummBits)) ++glog;
  return glog;
}

namespace {
size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

// mid-level summary: g2 (log) and u32 words; 0 words below 2^25 or past 2^30 nodes
uint32_t frontier_g2log(uint64_t N) {
  uint32_t l = 3;
  while ((N >> l) > (1ull << 24)) ++l;  // at most 2^24 bits (2 MiB)
  return l;
}
uint32_t frontier_summ2_words(uint64_t N) {
  if (N <= (1ull << 25) || N > (1ull << 30)) return 0;
  return (uint32_t)((((N + (1ull << frontier_g2log(N)) - 1) >> frontier_g2log(N)) + 31) / 32);
}

bool bs_path_ok(uint64_t N, uint32_t k) { return N > 0 && k >= 1 && k <= 4 && N <= ((uint64_t)kBsMaxTiles << kBsTileLog); }
uint32_t bs_tiles(uint64_t N) { return (uint32_t)((N + (1ull << kBsTileLog) - 1) >> kBsTileLog); }
uint32_t bs_regions(uint64_t N) { return (uint32_t)((N + (1ull << kBsRegLog) - 1) >> kBsRegLog); }
size_t bs_rec_bytes(uint64_t N, uint32_t k) { return (size_t)bs_regions(N) * ((size_t)k << kBsRegLog) * 4; }
size_t bs_tab_bytes(uint64_t N) { return 2 * (((size_t)bs_regions(N) * (bs_tiles(N) + 1) * 2 + 255) & ~(size_t)255); }

size_t frontier_bytes(uint64_t N) {
  const size_t nwords = (N + 63) / 64;
  const uint32_t glog = frontier_glog(N);
  const size_t sw = ((((N + (1ull << glog) - 1) >> glog) + 127) / 128) * 4;  // u32 words, uint4-padded
  return 2 * al256(nwords * 8) + al256(sw * 4) + al256(N * 8) + al256(nwords) +
         al256((size_t)frontier_summ2_words(N) * 4);
}

void frontier_carve(uint64_t N, void* base, FrontierBufs* f) {
  const size_t nwords = (N + 63) / 64;
  f->glog = frontier_glog(N);
  f->summ_words = (uint32_t)((((N + (1ull << f->glog) - 1) >> f->glog) + 127) / 128) * 4;
  char* p = (char*)base;
  f->nzb = (uint64_t*)p;
  p += al256(nwords * 8);
  f->fullb = (uint64_t*)p;
  p += al256(nwords * 8);
  f->summ = (uint32_t*)p;
  p += al256((size_t)f->summ_words * 4);
  f->D = (uint64_t*)p;
  p += al256(N * 8);
  f->dirtyD = (uint8_t*)p;
  p += al256(nwords);
  f->g2log = frontier_g2log(N);
  f->summ2_words = frontier_summ2_words(N);
  f->summ2 = f->summ2_words ? (uint32_t*)p : nullptr;
  f->scan_q = 1;
}

hipError_t launch_frontier_summary(const FrontierBufs& f, uint64_t N, uint32_t maj, hipStream_t st) {
  if (N == 0) return hipSuccess;  // a shard without nodes
  const uint32_t s2 = f.summ2 ? f.summ2_words : 0u;  // the mid-level summary too when f has one
  frontier_summary_kernel<<<(f.summ_words + 255) / 256 + (s2 + 255) / 256, 256, 0, st>>>(f, N, nullptr, 0, maj);
  return hipGetLastError();
}

hipError_t launch_frontier_commit(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                  uint32_t dmode, uint32_t flags, hipStream_t st) {
  if (N == 0) return hipSuccess;  // a shard without nodes
  const uint64_t wchunks = (((N + 63) >> 6) + (1u << kCommitChunkLog) - 1) >> kCommitChunkLog;  // one per wave
  const uint64_t cblocks = (wchunks + kCommitThreads / 64 - 1) / (kCommitThreads / 64);
  frontier_commit_kernel<<<(uint32_t)(cblocks < kCommitMaxBlocks ? cblocks : kCommitMaxBlocks), kCommitThreads, 0,
                           st>>>(f, S, N, partial,
                                                                                                 R, flags, dmode);
  return hipGetLastError();
}

hipError_t launch_frontier_rebuild(const FrontierBufs& f, const uint64_t* S, uint64_t N, uint64_t* partial,
                                   uint32_t R, uint32_t flags, hipStream_t st) {
  if (N == 0) return hipSuccess;  // a shard without nodes
  frontier_rebuild_kernel<<<commit_grid(N), kCommitThreads, 0, st>>>(f, S, N, partial, R, flags);
  return hipGetLastError();
}

hipError_t launch_frontier_inject(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                  uint32_t key0, uint32_t key1, int64_t node, uint32_t rumor, uint32_t flags,
                                  hipStream_t st) {
  const uint32_t grid = node >= 0 ? 1 : (R + 255) / 256;
  frontier_inject_kernel<<<grid, 256, 0, st>>>(f, S, N, partial, R, key0, key1, node, rumor, flags);
  return hipGetLastError();
}

hipError_t launch_frontier_round(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                 uint32_t k, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode, uint32_t maj,
                                 uint32_t dmode, const Faults& fa, uint32_t flags, const RoundSync& rs,
                                 hipStream_t st) {
  if (N == 0) return hipSuccess;  // a shard without nodes
  if (maj != 0 && dmode == kSparseDirect) dmode = kSparseAllD;  // (a full peer takes no push)
  const bool faults = fa.any();
  if (f.brec && f.btab && bs_path_ok(N, k)) {  // the binned sparse scan (K1a + K1b)
    const uint32_t nch = std::max(1u, std::min(f.bregions, kBsTestBlocks / f.btiles));
    const uint32_t egrid = std::min(f.bregions, kBsEmitGrid);
#define GOSSIP_BS(MODE, FAULTS)                                                                                 \
  if (k <= 2)                                                                                                    \
    frontier_bs_emit_kernel<MODE, FAULTS, 2><<<egrid, kBsEmitThreads, 0, st>>>(f, N, R, k, t, key0, key1, partial, maj, \
                                                                              fa);                              \
  else                                                                                                          \
    frontier_bs_emit_kernel<MODE, FAULTS, 4><<<egrid, kBsEmitThreads, 0, st>>>(f, N, R, k, t, key0, key1, partial, maj, \
                                                                              fa);                              \
  bin_transpose_u16(f.btab, f.btabT, f.bregions, f.btiles + 1, st);                                            \
  frontier_bs_test_kernel<MODE><<<f.btiles * nch, kBsTestThreads, 0, st>>>(f, S, N, R, k, partial, maj,          \
                                                                          dmode != kSparseAllD, dmode == kSparseDirect)
    switch (mode) {
      case 1: if (faults) { GOSSIP_BS(1, true); } else { GOSSIP_BS(1, false); } break;
      case 2: if (faults) { GOSSIP_BS(2, true); } else { GOSSIP_BS(2, false); } break;
      case 3: if (faults) { GOSSIP_BS(3, true); } else { GOSSIP_BS(3, false); } break;
      default: return hipErrorInvalidValue;
    }
#undef GOSSIP_BS
  } else {
  frontier_summary_kernel<<<(f.summ_words + 255) / 256 + (f.summ2_words + 255) / 256, 256, 0, st>>>(f, N, partial, R,
                                                                                                   maj);
  const uint64_t chunks = (N + kScanThreads - 1) / kScanThreads;
  const uint32_t grid = (uint32_t)(chunks < kScanGrid ? chunks : kScanGrid);
  // contiguous node range per block, a multiple of the block width (so lanes map to bitmap bits)
  const uint64_t per = ((N + grid - 1) / grid + kScanThreads - 1) / kScanThreads * kScanThreads;
#define GOSSIP_SCAN(MODE, FAULTS)                                                                           \
  frontier_scan_kernel<MODE, FAULTS><<<grid, kScanThreads, 0, st>>>(f, S, N, R, k, t, key0, key1, per, partial, \
                                                                    maj, dmode != kSparseAllD, dmode == kSparseDirect, fa)
  switch (mode) {
    case 1: if (faults) GOSSIP_SCAN(1, true); else GOSSIP_SCAN(1, false); break;
    case 2: if (faults) GOSSIP_SCAN(2, true); else GOSSIP_SCAN(2, false); break;
    case 3: if (faults) GOSSIP_SCAN(3, true); else GOSSIP_SCAN(3, false); break;
    default: return hipErrorInvalidValue;
  }
#undef GOSSIP_SCAN
  }
  // absolute totals: after the scan (it reads the rare count), before the commit adds to them
  if (dmode == kSparseDirect) {
    const hipError_t me = hipMemsetAsync(partial, 0, (size_t)rs.plen * 8, st);
    if (me != hipSuccess) return me;
  }
  const hipError_t ce = launch_frontier_commit(f, S, N, partial, R, dmode, flags, st);
  return ce;  // the engine enqueues the round's snapshot (round.h) after its timing event
}

}  // namespace gossip
