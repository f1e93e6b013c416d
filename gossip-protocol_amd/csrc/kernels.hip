// kernels.hip — round kernels of the gossip engine, written for gfx950 (CDNA4, wave64).
//
// Reference hot path: (*NodeState).Gossip, main.go:65-89 — one node forwarding
// one value to its topology neighbours over sequential SyncRPCs.  Here a round
// advances every node at once: S_{t+1} = S_t | pulls | pushes,
// all reads from S_t (or the gathered image of it), all writes into S_{t+1}.
// OR is commutative, associative and idempotent, so the atomics below give a
// schedule-independent, bit-exact result.
#include "kernels.h"
#include "round.h"
#include "philox.h"

namespace gossip {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// word w of global node n in the gathered [G][W][Nl] image
template <bool ONE_WORD>
__device__ __forceinline__ uint64_t gidx(uint64_t n, uint32_t w, uint64_t Nl, uint32_t W) {
  if (ONE_WORD) return n;
  const uint64_t r = n / Nl;
  return (r * W + w) * Nl + (n - r * Nl);
}

__device__ __forceinline__ uint64_t full_mask(uint32_t R, uint32_t w) {
  const uint32_t bits = R - 64u * w;
  return bits >= 64u ? ~0ull : ((1ull << bits) - 1ull);
}

// ---------------------------------------------------------------------------
// Random-peer round (PUSH / PULL / PUSHPULL).  One lane per sender s.
//  pull : S'[s] |= S[p_j(s)]            (own senders only)
//  push : S'[p_j(s)] |= S[s]            (destinations inside the owned range)
// A push whose bits the destination already holds in S_t is dropped: it cannot
// change S_{t+1} ⊇ S_t, so the filter is exact.
// ---------------------------------------------------------------------------
template <bool ONE_WORD, bool PULL, bool PUSH>
__global__ __launch_bounds__(kBlock) void round_random_kernel(RoundArgs a, uint64_t s_begin, uint64_t s_end) {
  const uint64_t nm1 = a.N - 1;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t s = s_begin + (uint64_t)blockIdx.x * kBlock + threadIdx.x; s < s_end; s += stride) {
    const uint32_t n = (uint32_t)s;
    const bool own = (s - a.lo) < a.nown;
    if (ONE_WORD) {
      const uint64_t vs = a.G[s];
      uint64_t acc = 0;
      u32x4 x{0, 0, 0, 0}, lw{0, 0, 0, 0};
      const Reach rc = reach_of(n, a.fa);  // n's partition block
      for (uint32_t j = 0; j < a.k; ++j) {
        if ((j & 3u) == 0) {
          x = philox4x32_10(u32x4{n, a.t, 0u, j >> 2}, a.key0, a.key1);
          if (a.fa.loss) lw = loss_draws(n, a.t, j >> 2, a.key0, a.key1);
        }
        const uint32_t p = peer_from_word(lane_of(x, j & 3u), nm1, n);
        if (a.fa.any() && edge_lost(a.fa, rc, p, lane_of(lw, j & 3u))) continue;
        const bool pown = ((uint64_t)p - a.lo) < a.nown;
        const bool need = (PULL && own) || (PUSH && pown && vs != 0);
        if (!need) continue;
        const uint64_t pv = a.G[p];
        if (PULL) acc |= pv;
        if (PUSH && pown) {
          const uint64_t nb = vs & ~pv;
          if (nb) atomicOr((unsigned long long*)&a.Snext[p - a.lo], (unsigned long long)nb);
        }
      }
      if (PULL && own) {
        const uint64_t nb = acc & ~vs;
        if (nb) atomicOr((unsigned long long*)&a.Snext[s - a.lo], (unsigned long long)nb);
      }
    } else {
      u32x4 x{0, 0, 0, 0}, lw{0, 0, 0, 0};
      const Reach rc = reach_of(n, a.fa);  // n's partition block
      for (uint32_t j = 0; j < a.k; ++j) {
        if ((j & 3u) == 0) {
          x = philox4x32_10(u32x4{n, a.t, 0u, j >> 2}, a.key0, a.key1);
          if (a.fa.loss) lw = loss_draws(n, a.t, j >> 2, a.key0, a.key1);
        }
        const uint32_t p = peer_from_word(lane_of(x, j & 3u), nm1, n);
        if (a.fa.any() && edge_lost(a.fa, rc, p, lane_of(lw, j & 3u))) continue;
        const bool pown = ((uint64_t)p - a.lo) < a.nown;
        for (uint32_t w = 0; w < a.W; ++w) {
          const uint64_t vs = a.G[gidx<false>(s, w, a.Nl, a.W)];
          if (!((PULL && own) || (PUSH && pown && vs != 0))) continue;
          const uint64_t pv = a.G[gidx<false>(p, w, a.Nl, a.W)];
          if (PULL && own) {
            const uint64_t nb = pv & ~vs;
            if (nb) atomicOr((unsigned long long*)&a.Snext[(uint64_t)w * a.Nl + (s - a.lo)], (unsigned long long)nb);
          }
          if (PUSH && pown) {
            const uint64_t nb = vs & ~pv;
            if (nb) atomicOr((unsigned long long*)&a.Snext[(uint64_t)w * a.Nl + (p - a.lo)], (unsigned long long)nb);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// FLOOD round — main.go:65-89 as a pull over the in-adjacency.  G holds the
// gathered frontier F_t = S_t & ~S_{t-1}: the values each node learned last
// round and now forwards once (dedupe main.go:113) to Topology[self] (:72)
// minus its sender (:73-75).  One lane per owned node v.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool in_sorted(const uint32_t* a, uint32_t len, uint32_t x) {
  uint32_t lo = 0, hi = len;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo < len && a[lo] == x;
}

__global__ __launch_bounds__(kBlock) void round_flood_kernel(RoundArgs a) {
  uint64_t msgs = 0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < a.nown; i += stride) {
    const uint32_t v = (uint32_t)(a.lo + i);
    const uint32_t ob = a.orow[v], deg = a.orow[v + 1] - ob;
    const uint32_t ib = a.irow[v], ie = a.irow[v + 1];
    for (uint32_t w = 0; w < a.W; ++w) {
      const uint64_t li = (uint64_t)w * a.Nl + i;
      const uint64_t sv = a.S[li];
      const uint64_t fv = sv & ~a.Sprev[li];
      msgs += (uint64_t)__popcll(fv) * deg - (uint64_t)__popcll(fv & a.skip[li]);
      uint64_t acc = sv;
      for (uint32_t e = ib; e < ie; ++e) acc |= a.G[gidx<false>(a.icol[e], w, a.Nl, a.W)];
      const uint64_t nw = acc & ~sv;
      uint64_t seen = 0, sk = 0;
      for (uint32_t e = ib; e < ie && seen != nw; ++e) {
        const uint32_t u = a.icol[e];
        const uint64_t c = a.G[gidx<false>(u, w, a.Nl, a.W)] & nw & ~seen;
        if (c && in_sorted(a.ocol + ob, deg, u)) sk |= c;  // sender skip, main.go:73
        seen |= c;
      }
      a.Snext[li] = acc;
      a.skip[li] = sk;
    }
  }
  msgs = wave_sum_u64(msgs);
  if ((threadIdx.x & 63) == 0 && msgs) atomicAdd((unsigned long long*)&a.partial[2], (unsigned long long)msgs);
}

// ---------------------------------------------------------------------------
// FLOOD with faults (main.go:72-87).  The reference forwards a
// value from one goroutine that walks Topology[node] in order (:72), skips the
// value's sender (:73) and blocks in SyncRPC on each neighbour until it is acked
// (:80-87); the neighbour's 2 s context (:77) expires after D lost attempts.
// One lane per (value x, node u) walk: from position c, the sender is skipped
// (no message); any other neighbour w costs a message, lost as a random-mode
// edge (partition, or Philox({u, t, 4 | x << 16, c >> 2})[c & 3] < edge_loss: one draw per
// message, i.e. per value, as each value is its own SyncRPC at main.go:81).  A lost
// attempt ends the walk's round (the later neighbours wait); a delivered one
// ORs x into S_{t+1}[w] (w's first sender: atomicMin over the lanes that
// delivered x to w this round — snd stays kWalkNone while w lacks x) and moves
// on, unless the context has expired: then the walk stays on w for good.
// Reads S_t only; S_{t+1} starts as a copy of S_t.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void round_flood_walks_kernel(RoundArgs a, FloodWalks fw) {
  uint64_t msgs = 0;
  const uint64_t total = (uint64_t)a.R * a.N, stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += stride) {
    const uint32_t x = (uint32_t)(i / a.N), u = (uint32_t)(i - (uint64_t)x * a.N);
    const uint64_t bit = 1ull << (x & 63u);
    const uint64_t* Sx = a.S + (uint64_t)(x >> 6) * a.Nl;
    if (!(Sx[u] & bit)) continue;
    const uint32_t b = a.orow[u], deg = a.orow[u + 1] - b;
    uint32_t c = fw.cur[i];
    if (c >= deg) continue;
    uint32_t at = fw.att[i];
    const uint32_t snd = fw.snd[i];
    const Reach rc = reach_of(u, a.fa);
    while (c < deg) {
      const uint32_t w = a.ocol[b + c];
      if (w == snd) {  // main.go:73
        ++c;
        continue;
      }
      ++msgs;
      const uint32_t lw = a.fa.loss ? lane_of(loss_draws(u, a.t, c >> 2, a.key0, a.key1, x), c & 3u) : 0u;
      if (edge_lost(a.fa, rc, w, lw)) {
        at = at < 255u ? at + 1u : at;
        break;
      }
      if (!(Sx[w] & bit)) {
        atomicOr((unsigned long long*)&a.Snext[(uint64_t)(x >> 6) * a.Nl + w], (unsigned long long)bit);
        atomicMin(&fw.snd[(uint64_t)x * a.N + w], u);
      }
      if (fw.D && at >= fw.D) break;  // expired context: the walk never moves on
      ++c;
      at = 0;
    }
    fw.cur[i] = c;
    fw.att[i] = (uint8_t)at;
  }
  msgs = wave_sum_u64(msgs);
  if ((threadIdx.x & 63) == 0 && msgs) atomicAdd((unsigned long long*)&a.partial[2], (unsigned long long)msgs);
}

// The values learned in round t start their walks in round t + 1 (their first sender is set).
__global__ __launch_bounds__(kBlock) void flood_walks_learn_kernel(RoundArgs a, FloodWalks fw) {
  const uint64_t total = (uint64_t)a.R * a.N, stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += stride) {
    const uint32_t x = (uint32_t)(i / a.N), w = (uint32_t)(i - (uint64_t)x * a.N);
    const uint64_t bit = 1ull << (x & 63u), wi = (uint64_t)(x >> 6) * a.Nl + w;
    if ((a.Snext[wi] & bit) && !(a.S[wi] & bit)) {
      fw.cur[i] = 0;
      fw.att[i] = 0;
    }
  }
}

// Stall streaks after round t: a node not yet stalled counts the
// round when any of its k exchanges was lost, else starts over.  Draws only: the
// streaks never depend on S.
__global__ __launch_bounds__(kBlock) void stall_update_kernel(uint8_t* __restrict__ st, uint64_t N, uint32_t k,
                                                              uint32_t t, uint32_t key0, uint32_t key1, Faults fa) {
  fa.stall = nullptr;  // the partition block of a node that is not stalled
  const uint64_t nm1 = N - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < N; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t n = (uint32_t)i;
    const uint32_t c = st[i];
    if (c >= fa.D) continue;
    const Reach rc = reach_of(n, fa);
    bool any = false;
    u32x4 x{0, 0, 0, 0}, lw{0, 0, 0, 0};
    for (uint32_t j = 0; j < k && !any; ++j) {
      if ((j & 3u) == 0) {
        x = philox4x32_10(u32x4{n, t, 0u, j >> 2}, key0, key1);
        if (fa.loss) lw = loss_draws(n, t, j >> 2, key0, key1);
      }
      any = edge_lost(fa, rc, peer_from_word(lane_of(x, j & 3u), nm1, n), lane_of(lw, j & 3u));
    }
    st[i] = (uint8_t)(any ? c + 1 : 0);
  }
}

// ---------------------------------------------------------------------------
// Stats of S_{t+1} (convergence detection): per-rumor infected counts by
// wave64 ballot + popcount, fully-informed node count, optional state hash.
// partial = [full, alive, messages, hash, infected[R]].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void stats_kernel(RoundArgs a) {
  extern __shared__ uint32_t cnt[];  // [W*64]
  __shared__ uint64_t red_hash[kBlock / 64];
  __shared__ uint32_t red_full[kBlock / 64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t r = threadIdx.x; r < a.W * 64; r += kBlock) cnt[r] = 0;
  __syncthreads();
  const bool do_hash = (a.flags & 1u) != 0;
  uint64_t hash = 0;
  uint32_t full = 0;
  for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < a.nown; base += (uint64_t)gridDim.x * kBlock) {
    const uint64_t i = base + threadIdx.x;
    const bool valid = i < a.nown;
    bool isfull = valid;
    for (uint32_t w = 0; w < a.W; ++w) {
      const uint64_t x = valid ? a.Snext[(uint64_t)w * a.Nl + i] : 0ull;
      const uint64_t fm = full_mask(a.R, w);
      isfull = isfull && ((x & fm) == fm);
      if (do_hash && x) hash += mix64(x + ((uint64_t)w * a.N + a.lo + i) * kGold64);
      const uint64_t nz = __ballot(x != 0);
      if (nz == 0) continue;
      const uint32_t nbits = a.R - 64u * w >= 64u ? 64u : a.R - 64u * w;
      const uint64_t fl = __ballot(x == fm);
      uint32_t c_lane = 0;
      if (fl == nz) {
        c_lane = (uint32_t)__popcll(nz);
      } else {
        for (uint32_t b = 0; b < nbits; ++b) {
          const uint32_t c = (uint32_t)__popcll(__ballot((x >> b) & 1ull));
          c_lane = lane == b ? c : c_lane;
        }
      }
      if (lane < nbits && c_lane) atomicAdd(&cnt[w * 64 + lane], c_lane);
    }
    full += (uint32_t)__popcll(__ballot(isfull));
  }
  hash = wave_sum_u64(hash);
  if (lane == 0) {
    red_hash[wave] = hash;
    red_full[wave] = full;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t h = 0, f = 0;
    for (int q = 0; q < kBlock / 64; ++q) {
      h += red_hash[q];
      f += red_full[q];
    }
    if (f) atomicAdd((unsigned long long*)&a.partial[0], (unsigned long long)f);
    if (h) atomicAdd((unsigned long long*)&a.partial[3], (unsigned long long)h);
  }
  for (uint32_t r = threadIdx.x; r < a.R; r += kBlock)
    if (cnt[r]) atomicAdd((unsigned long long*)&a.partial[4 + r], (unsigned long long)cnt[r]);
}

__global__ __launch_bounds__(kBlock) void frontier_kernel(const uint64_t* __restrict__ S,
                                                          const uint64_t* __restrict__ Sprev,
                                                          uint64_t* __restrict__ F, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
    F[i] = S[i] & ~Sprev[i];
}

// Client broadcast (main.go:102-117): node >= 0 sets one bit; node < 0 injects
// every rumor r < R at its Philox tag-2 origin.
__global__ void inject_kernel(uint64_t* S, uint64_t Nl, uint64_t lo, uint64_t hi, uint64_t N, uint32_t R,
                              uint32_t key0, uint32_t key1, int64_t node, uint32_t rumor, FloodWalks fw) {
  const uint32_t r = node >= 0 ? rumor : blockIdx.x * blockDim.x + threadIdx.x;
  if (node >= 0 && (blockIdx.x | threadIdx.x)) return;
  if (r >= R) return;
  const uint64_t n = node >= 0 ? (uint64_t)node : origin_of(r, N, key0, key1);
  if (n < lo || n >= hi) return;
  const uint64_t bit = 1ull << (r & 63);
  const uint64_t old = atomicOr((unsigned long long*)&S[(uint64_t)(r >> 6) * Nl + (n - lo)], (unsigned long long)bit);
  if (fw.cur && !(old & bit)) {  // a client's value (no sender): its walk starts next round
    const uint64_t i = (uint64_t)r * N + n;
    fw.cur[i] = 0;
    fw.att[i] = 0;
    fw.snd[i] = kWalkNone;
  }
}

__global__ __launch_bounds__(kBlock) void hash_kernel(const uint64_t* S, uint64_t Nl, uint64_t nown, uint32_t W,
                                                      uint64_t N, uint64_t lo, uint64_t* out) {
  uint64_t h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nown; i += (uint64_t)gridDim.x * kBlock)
    for (uint32_t w = 0; w < W; ++w) {
      const uint64_t x = S[(uint64_t)w * Nl + i];
      if (x) h += mix64(x + ((uint64_t)w * N + lo + i) * kGold64);
    }
  h = wave_sum_u64(h);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd((unsigned long long*)out, (unsigned long long)h);
}

__global__ void philox_kernel(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4 y = philox4x32_10(u32x4{ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]}, k0, k1);
  out[4 * i] = y.x;
  out[4 * i + 1] = y.y;
  out[4 * i + 2] = y.z;
  out[4 * i + 3] = y.w;
}

uint32_t grid_for(uint64_t work, uint32_t cap) {
  const uint64_t b = (work + kBlock - 1) / kBlock;
  return (uint32_t)(b == 0 ? 1 : (b < cap ? b : cap));
}

}  // namespace

hipError_t launch_round_random(const RoundArgs& a, hipStream_t st) {
  const bool pull = a.mode == 2 || a.mode == 3, push = a.mode == 1 || a.mode == 3;
  // pull-only rounds need only the owned senders; any push needs every sender
  const uint64_t sb = push ? 0 : a.lo, se = push ? a.N : a.lo + a.nown;
  const uint32_t grid = grid_for(se - sb, 1u << 20);
  if (a.W == 1) {
    if (pull && push) round_random_kernel<true, true, true><<<grid, kBlock, 0, st>>>(a, sb, se);
    else if (pull) round_random_kernel<true, true, false><<<grid, kBlock, 0, st>>>(a, sb, se);
    else round_random_kernel<true, false, true><<<grid, kBlock, 0, st>>>(a, sb, se);
  } else {
    if (pull && push) round_random_kernel<false, true, true><<<grid, kBlock, 0, st>>>(a, sb, se);
    else if (pull) round_random_kernel<false, true, false><<<grid, kBlock, 0, st>>>(a, sb, se);
    else round_random_kernel<false, false, true><<<grid, kBlock, 0, st>>>(a, sb, se);
  }
  return hipGetLastError();
}

hipError_t launch_round_flood(const RoundArgs& a, hipStream_t st) {
  round_flood_kernel<<<grid_for(a.nown, 8192), kBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_round_flood_walks(const RoundArgs& a, const FloodWalks& fw, hipStream_t st) {
  const uint64_t walks = (uint64_t)a.R * a.N;
  round_flood_walks_kernel<<<grid_for(walks, 8192), kBlock, 0, st>>>(a, fw);
  flood_walks_learn_kernel<<<grid_for(walks, 8192), kBlock, 0, st>>>(a, fw);
  return hipGetLastError();
}

hipError_t launch_stall_update(uint8_t* stall, uint64_t N, uint32_t k, uint32_t t, uint32_t key0, uint32_t key1,
                               const Faults& fa, hipStream_t st) {
  stall_update_kernel<<<grid_for(N, 8192), kBlock, 0, st>>>(stall, N, k, t, key0, key1, fa);
  return hipGetLastError();
}

__global__ void publish_kernel(const uint64_t* __restrict__ in64, const uint32_t* __restrict__ in32,
                               uint64_t* __restrict__ out, uint32_t n, int32_t slot, uint64_t value) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) out[i] = in64 ? in64[i] : (uint64_t)in32[i];
  __syncthreads();
  if (slot >= 0 && threadIdx.x == 0) out[slot] = value;
}

hipError_t launch_publish(const uint64_t* in64, const uint32_t* in32, uint64_t* out, uint32_t n, int32_t slot,
                          uint64_t value, hipStream_t st) {
  publish_kernel<<<1, 256, 0, st>>>(in64, in32, out, n, slot, value);
  return hipGetLastError();
}

hipError_t launch_stats(const RoundArgs& a, hipStream_t st) {
  stats_kernel<<<grid_for(a.nown, 2048), kBlock, a.W * 64 * sizeof(uint32_t), st>>>(a);
  return hipGetLastError();
}

hipError_t launch_frontier(const uint64_t* S, const uint64_t* Sprev, uint64_t* F, uint64_t n, hipStream_t st) {
  frontier_kernel<<<grid_for(n, 8192), kBlock, 0, st>>>(S, Sprev, F, n);
  return hipGetLastError();
}

hipError_t launch_inject(uint64_t* S, uint64_t Nl, uint64_t lo, uint64_t hi, uint64_t N, uint32_t R, uint32_t key0,
                         uint32_t key1, int64_t node, uint32_t rumor, hipStream_t st, const FloodWalks* fw) {
  const uint32_t grid = node >= 0 ? 1 : (R + kBlock - 1) / kBlock;
  inject_kernel<<<grid, kBlock, 0, st>>>(S, Nl, lo, hi, N, R, key0, key1, node, rumor,
                                         fw ? *fw : FloodWalks{nullptr, nullptr, nullptr, 0u});
  return hipGetLastError();
}

hipError_t launch_hash(const uint64_t* S, uint64_t Nl, uint64_t nown, uint32_t W, uint64_t N, uint64_t lo,
                       uint64_t* out, hipStream_t st) {
  hash_kernel<<<grid_for(nown, 2048), kBlock, 0, st>>>(S, Nl, nown, W, N, lo, out);
  return hipGetLastError();
}

hipError_t launch_philox(const uint32_t* ctr, uint32_t k0, uint32_t k1, uint32_t* out, uint32_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  philox_kernel<<<(n + 255) / 256, 256, 0, st>>>(ctr, k0, k1, out, n);
  return hipGetLastError();
}

namespace {

__global__ __launch_bounds__(64) void round_snapshot_kernel(const uint64_t* __restrict__ partial, RoundSync rs) {
  for (uint32_t i = threadIdx.x; i < rs.plen; i += 64) rs.ring[i] = partial[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();  // totals visible to the host before the sequence word
    __atomic_store_n(&rs.ring[rs.plen], (uint64_t)rs.seq, __ATOMIC_RELEASE);
  }
}

}  // namespace

hipError_t launch_round_snapshot(const uint64_t* partial, const RoundSync& rs, hipStream_t st) {
  round_snapshot_kernel<<<1, 64, 0, st>>>(partial, rs);
  return hipGetLastError();
}

}  // namespace gossip
