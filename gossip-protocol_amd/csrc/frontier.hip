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
#include "philox.h"

namespace gossip {

namespace {

constexpr int kScanThreads = 1024;
constexpr uint32_t kScanGrid = 256;  // one block per CU: the summary takes 128 KiB of LDS
constexpr int kCommitThreads = 256;

__device__ __forceinline__ uint64_t full_mask(uint32_t R) { return R >= 64 ? ~0ull : ((1ull << R) - 1ull); }

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
__global__ __launch_bounds__(256) void frontier_summary_kernel(FrontierBufs f, uint64_t N) {
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

// K1.  MODE: 1 push, 2 pull, 3 push-pull.  MAJ: majority value 0 (0) or full (1).
template <int MAJ, int MODE>
__global__ __launch_bounds__(kScanThreads) void frontier_scan_kernel(FrontierBufs f, const uint64_t* __restrict__ S,
                                                                      uint64_t N, uint32_t R, uint32_t k, uint32_t t,
                                                                      uint32_t key0, uint32_t key1) {
  __shared__ uint4 summ4[kSummBits / 128];
  const uint32_t* summ = (const uint32_t*)summ4;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t n4 = (f.summ_words + 3) / 4;
  for (uint32_t i = tid; i < n4; i += kScanThreads) summ4[i] = ((const uint4*)f.summ)[i];
  __syncthreads();

  constexpr bool kPush = (MODE & 1) != 0, kPull = (MODE & 2) != 0;
  const uint64_t fm = full_mask(R), maj = MAJ ? fm : 0ull, nm1 = N - 1;
  const uint32_t glog = f.glog;
  for (uint64_t base = (uint64_t)blockIdx.x * kScanThreads; base < N; base += (uint64_t)gridDim.x * kScanThreads) {
    const uint64_t n = base + tid;
    const bool valid = n < N;
    const uint64_t rw = rare_word<MAJ>(f, (valid ? n : N - 1) >> 6, N);  // one address per wave
    const bool rn = valid && ((rw >> lane) & 1ull);
    // a majority node only acts through a rare peer; push from an empty node and
    // pull into a full one are no-ops, so those nodes skip the draws entirely
    if (!valid || (!rn && ((!kPull && MAJ == 0) || (!kPush && MAJ == 1)))) continue;
    const uint64_t x = rn ? S[n] : maj;
    uint64_t acc = 0;
    u32x4 r4{0, 0, 0, 0};
    for (uint32_t j = 0; j < k; ++j) {
      if ((j & 3u) == 0) r4 = philox4x32_10(u32x4{(uint32_t)n, t, 0u, j >> 2}, key0, key1);
      const uint32_t p = peer_from_word(lane_of(r4, j & 3u), nm1, (uint32_t)n);
      bool rp = (summ[p >> (glog + 5)] >> ((p >> glog) & 31u)) & 1u;
      if (rp && glog) rp = (rare_word<MAJ>(f, p >> 6, N) >> (p & 63u)) & 1ull;
      if (!rn && !rp) continue;  // both ends majority: nothing moves
      const uint64_t vp = rp ? S[p] : maj;
      if (kPull) acc |= vp;
      if (kPush) {
        const uint64_t d = x & ~vp;
        if (d) atomicOr((unsigned long long*)&f.D[p], (unsigned long long)d);
      }
    }
    acc &= ~x;
    if (acc) atomicOr((unsigned long long*)&f.D[n], (unsigned long long)acc);
  }
}

__device__ __forceinline__ uint64_t transpose64(uint64_t x, uint32_t lane) {
  constexpr uint64_t kMask[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                                 0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int st = 0; st < 6; ++st) {
    const uint32_t d = 32u >> st;
    const uint64_t y = __shfl_xor(x, d, 64);
    const uint64_t m = kMask[st];
    x = (lane & d) ? ((x & ~m) | ((y & ~m) >> d)) : ((x & m) | ((y & m) << d));
  }
  return x;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// K2.  REBUILD: absolute stats + bitmaps of S (partial zeroed by the caller);
// else: apply D in place and add the deltas to the totals already in partial.
template <bool REBUILD>
__global__ __launch_bounds__(kCommitThreads) void frontier_commit_kernel(FrontierBufs f, uint64_t* __restrict__ S,
                                                                          uint64_t N, uint64_t* __restrict__ partial,
                                                                          uint32_t R, uint32_t flags) {
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red[3][kCommitThreads / 64];  // full, nonzero, hash
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t fm = full_mask(R);
  const bool do_hash = (flags & 1u) != 0;
  if (tid < 64) cnt[tid] = 0;
  __syncthreads();
  const uint64_t ngroups = (N + 63) >> 6;
  uint64_t hash = 0;
  uint32_t full = 0, nz = 0, c_lane = 0;
  for (uint64_t g = (uint64_t)blockIdx.x * (kCommitThreads / 64) + wave; g < ngroups;
       g += (uint64_t)gridDim.x * (kCommitThreads / 64)) {
    const uint64_t n = (g << 6) + lane;
    const bool valid = n < N;
    uint64_t old, nw;
    if (REBUILD) {
      old = 0;
      nw = valid ? S[n] : 0ull;
    } else {
      const uint64_t d = valid ? f.D[n] : 0ull;
      if (__ballot(d != 0) == 0) continue;
      old = valid ? S[n] : 0ull;
      nw = old | d;
      if (d) {
        f.D[n] = 0;
        if (nw != old) S[n] = nw;
      }
    }
    const uint64_t nzw = __ballot(valid && nw != 0), fw = __ballot(valid && nw == fm);
    if (lane == 0) {
      f.nzb[g] = nzw;
      f.fullb[g] = fw;
    }
    const uint64_t nb = nw & ~old;
    full += (uint32_t)__popcll(__ballot(valid && nw == fm && old != fm));
    nz += (uint32_t)__popcll(__ballot(valid && nw != 0 && old == 0));
    if (do_hash && nb) {
      hash += mix64(nw + n * kGold64);
      if (old) hash -= mix64(old + n * kGold64);
    }
    if (__ballot(nb != 0)) c_lane += (uint32_t)__popcll(transpose64(nb, lane));
  }
  if (lane < R && c_lane) atomicAdd(&cnt[lane], c_lane);
  hash = wave_sum64(hash);
  if (lane == 0) {
    red[0][wave] = full;
    red[1][wave] = nz;
    red[2][wave] = hash;
  }
  __syncthreads();
  if (tid == 0) {
    uint64_t a = 0, b = 0, h = 0;
    for (int w = 0; w < kCommitThreads / 64; ++w) {
      a += red[0][w];
      b += red[1][w];
      h += red[2][w];
    }
    if (a) atomicAdd((unsigned long long*)&partial[0], (unsigned long long)a);
    if (h) atomicAdd((unsigned long long*)&partial[3], (unsigned long long)h);
    if (b) atomicAdd((unsigned long long*)&partial[4 + R], (unsigned long long)b);
  }
  if (tid < R && cnt[tid]) atomicAdd((unsigned long long*)&partial[4 + tid], (unsigned long long)cnt[tid]);
}

uint32_t commit_grid(uint64_t N) {
  const uint64_t groups = (N + 63) >> 6, per = kCommitThreads / 64;
  const uint64_t blocks = (groups + per - 1) / per;
  return (uint32_t)(blocks < 2048 ? blocks : 2048);
}

}  // namespace

uint32_t frontier_glog(uint64_t N) {
  uint32_t glog = 0;
  while ((((N + (1ull << glog) - 1) >> glog) > kSummBits)) ++glog;
  return glog;
}

size_t frontier_bytes(uint64_t N) {
  const size_t nwords = (N + 63) / 64;
  const uint32_t glog = frontier_glog(N);
  const size_t sw = ((((N + (1ull << glog) - 1) >> glog) + 127) / 128) * 4;  // u32 words, uint4-padded
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  return 2 * al(nwords * 8) + al(sw * 4) + al(N * 8);
}

void frontier_carve(uint64_t N, void* base, FrontierBufs* f) {
  const size_t nwords = (N + 63) / 64;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  f->glog = frontier_glog(N);
  f->summ_words = (uint32_t)((((N + (1ull << f->glog) - 1) >> f->glog) + 127) / 128) * 4;
  char* p = (char*)base;
  f->nzb = (uint64_t*)p;
  p += al(nwords * 8);
  f->fullb = (uint64_t*)p;
  p += al(nwords * 8);
  f->summ = (uint32_t*)p;
  p += al((size_t)f->summ_words * 4);
  f->D = (uint64_t*)p;
}

hipError_t launch_frontier_rebuild(const FrontierBufs& f, const uint64_t* S, uint64_t N, uint64_t* partial,
                                   uint32_t R, uint32_t flags, hipStream_t st) {
  frontier_commit_kernel<true><<<commit_grid(N), kCommitThreads, 0, st>>>(f, const_cast<uint64_t*>(S), N, partial,
                                                                          R, flags);
  return hipGetLastError();
}

hipError_t launch_frontier_round(const FrontierBufs& f, uint64_t* S, uint64_t N, uint64_t* partial, uint32_t R,
                                 uint32_t k, uint32_t t, uint32_t key0, uint32_t key1, uint32_t mode, uint32_t maj,
                                 uint32_t flags, hipStream_t st) {
  const uint32_t sg = (f.summ_words + 255) / 256;
  if (maj)
    frontier_summary_kernel<1><<<sg, 256, 0, st>>>(f, N);
  else
    frontier_summary_kernel<0><<<sg, 256, 0, st>>>(f, N);
  const uint64_t chunks = (N + kScanThreads - 1) / kScanThreads;
  const uint32_t grid = (uint32_t)(chunks < kScanGrid ? chunks : kScanGrid);
#define GOSSIP_SCAN(MJ, MD) frontier_scan_kernel<MJ, MD><<<grid, kScanThreads, 0, st>>>(f, S, N, R, k, t, key0, key1)
  switch (maj * 4 + mode) {
    case 1: GOSSIP_SCAN(0, 1); break;
    case 2: GOSSIP_SCAN(0, 2); break;
    case 3: GOSSIP_SCAN(0, 3); break;
    case 5: GOSSIP_SCAN(1, 1); break;
    case 6: GOSSIP_SCAN(1, 2); break;
    case 7: GOSSIP_SCAN(1, 3); break;
    default: return hipErrorInvalidValue;
  }
#undef GOSSIP_SCAN
  frontier_commit_kernel<false><<<commit_grid(N), kCommitThreads, 0, st>>>(f, S, N, partial, R, flags);
  return hipGetLastError();
}

}  // namespace gossip
