// antientropy.hip — version-vector anti-entropy with churn (configs[4]).
//
// Each node holds K uint32 versions (AoS rows V[n*K + c], so a peer's whole
// vector is one contiguous K*4-byte row).  Round t: churn (ae_churn_word),
// then every alive node n exchanges with its Philox peers p_j(n,t) that are
// alive too: both take the elementwise max of the two S_t rows.  The
// reference's only failure handling is retry-until-acked (main.go:77-87);
// churn here is the build-defined fault model of SURVEY.md §5.
//
// Every kernel walks 64-node chunks, one chunk per wave.  The node phase runs
// one lane per node (Philox peer draw, the peer's alive bit from the churn
// kernel's bitmap); the row phase runs L = next power of two >= K lanes per
// node, 64/L nodes per sub-step, with the node phase's results handed over by
// shuffles.  Alive and stale bits share one [chunks][2] array (AeArgs::ab).
//
// Two round paths, chosen per round by the host (engine.hip), both after the
// churn kernel:
// - dense (binned, the default where it fits): the emit bins every alive sender's
//   exchanges by the peer's 2^14-node tile; one block per tile sorts its in-edges by
//   node in LDS and writes every row of V' = max(own row, the peers' rows, the rows
//   of the senders that picked the node) once, with the round's stats;
// - dense (atomic, the fallback): a pull pass writes every row of V' = max(V[n],
//   V[p_j]) and the per-exchange push masks; a push pass atomicMax-es V[n] into
//   V'[p_j] for the masked components only; a stats pass;
// - sparse (most of a run: once nearly every alive node holds the global max
//   vector, only exchanges touching a stale node can change anything): the
//   scan lists the exchanges with a stale end, the rows of both ends are
//   snapshotted, then merged in place, and a fix-up pass updates the stale
//   bitmap and the hash for each touched node once (claimed by epoch).
#include "antientropy.h"

#include <type_traits>

#include "philox.h"
#include "wave.h"

namespace gossip {

namespace {

constexpr int kAeBlock = 256;
constexpr int kAeWaves = kAeBlock / 64;
// fallback dense-round kernels: no minimum waves per SIMD (forcing 3-6 spilled or was no
// faster: DESIGN.md §3.7)

// pipelined sparse rounds: the previous round closed the gate (converged, overflowed, or gated off)
__device__ __forceinline__ bool ae_gated_off(const AeArgs& a) {
  return a.gate && *(volatile const uint32_t*)a.gate == 0u;
}

// alive after round t's churn, from the churn word (ae_churn_word)
__device__ __forceinline__ bool churned(bool alive, uint32_t x, uint32_t fail, uint32_t rec) {
  return alive ? !(x < fail) : (x < rec);
}

__device__ __forceinline__ uint64_t wave_id() { return (uint64_t)blockIdx.x * kAeWaves + (threadIdx.x >> 6); }
__device__ __forceinline__ uint64_t wave_count() { return (uint64_t)gridDim.x * kAeWaves; }

// block sum of one u64 per lane, added to *dst by one atomic (NW waves per block)
template <int NW = kAeWaves>
__device__ __forceinline__ void block_add(uint64_t v, uint64_t* red, uint64_t* dst) {
  v = wave_sum64(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
    for (int w = 0; w < NW; ++w) s += red[w];
    if (s) atomicAdd((unsigned long long*)dst, (unsigned long long)s);
  }
  __syncthreads();
}

__device__ __forceinline__ uint64_t hash_term(uint32_t v, uint32_t c, uint64_t n, uint64_t N) {
  return v ? mix64((uint64_t)v + ((uint64_t)c * N + n) * kGold64) : 0ull;
}

// inject_random's rows, and their componentwise max folded into target (zeroed before) in the same
// pass: a thread keeps one quad q of components (the grid stride is a multiple of (K + 3) / 4), so
// its running max is per component; one LDS max per block, one global atomicMax per component.
// K % 4 == 0: the quad is one 16-B store (the rows are 16-B aligned: 4K bytes each).
__global__ __launch_bounds__(kAeBlock) void ae_init_kernel(uint32_t* V, uint64_t N, uint32_t K, uint32_t k0,
                                                           uint32_t k1, uint32_t* target) {
  __shared__ uint32_t m[64];
  if (threadIdx.x < 64) m[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t c4 = (K + 3) / 4;
  uint32_t mx[4] = {0, 0, 0, 0}, q0 = ~0u;
  // a thread's running maxima belong to its quad q0: flushed whenever the quad changes (the grid
  // stride is not always a multiple of c4, e.g. K = 9..12 past ~5.6M nodes)
  auto flush = [&]() {
    for (uint32_t r = 0; r < 4 && 4 * q0 + r < K; ++r)
      if (mx[r]) atomicMax(&m[4 * q0 + r], mx[r]);
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) mx[r] = 0;
  };
  for (uint64_t i = (uint64_t)blockIdx.x * kAeBlock + threadIdx.x; i < N * c4; i += (uint64_t)gridDim.x * kAeBlock) {
    const uint32_t n = (uint32_t)(i / c4), q = (uint32_t)(i % c4);
    if (q != q0 && q0 != ~0u) flush();
    q0 = q;
    const u32x4 x = philox4x32_10(u32x4{n, q, 3u, 0u}, k0, k1);
    const uint32_t v[4] = {x.x & 0xFFFFu, x.y & 0xFFFFu, x.z & 0xFFFFu, x.w & 0xFFFFu};
    if ((K & 3u) == 0) {
      *reinterpret_cast<uint4*>(V + (uint64_t)n * K + 4 * q) = uint4{v[0], v[1], v[2], v[3]};
    } else {
      for (uint32_t r = 0; r < 4 && 4 * q + r < K; ++r) V[(uint64_t)n * K + 4 * q + r] = v[r];
    }
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) mx[r] = max(mx[r], v[r]);
  }
  if (q0 != ~0u) flush();
  __syncthreads();
  if (threadIdx.x < K && m[threadIdx.x]) atomicMax(&target[threadIdx.x], m[threadIdx.x]);
}

__global__ void ae_inject_kernel(uint32_t* V, uint32_t* target, uint64_t node, uint32_t K, uint32_t c) {
  const uint32_t v = ++V[node * K + c];
  atomicMax(&target[c], v);
}

__device__ __forceinline__ bool alive_bit(const uint64_t* ab, uint32_t n) { return (ab[2 * (n >> 6)] >> (n & 63)) & 1ull; }

// alive and stale bit of n with one 16-B load
__device__ __forceinline__ void alive_stale(const uint64_t* ab, uint32_t n, bool* al, bool* st) {
  const uint4 w = *reinterpret_cast<const uint4*>(ab + 2 * (n >> 6));
  const uint32_t sh = n & 31;
  const uint32_t aw = (n & 32) ? w.y : w.x, sw = (n & 32) ? w.w : w.z;
  *al = (aw >> sh) & 1u;
  *st = (sw >> sh) & 1u;
}

// peer j of node n in round t; x carries the Philox words across j
__device__ __forceinline__ uint32_t peer_j(const AeArgs& a, uint32_t n, uint32_t j, u32x4& x) {
  if ((j & 3u) == 0) x = philox4x32_10(u32x4{n, a.t, 0u, j >> 2}, a.key0, a.key1);
  return peer_from_word(lane_of(x, j & 3u), a.N - 1, n);
}

__global__ __launch_bounds__(kAeBlock) void ae_fill_alive_kernel(uint64_t* ab, uint64_t N) {
  const uint64_t nw = (N + 63) / 64;
  for (uint64_t w = (uint64_t)blockIdx.x * kAeBlock + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * kAeBlock) {
    ab[2 * w] = (w + 1) * 64 <= N ? ~0ull : ((1ull << (N & 63)) - 1ull);
    ab[2 * w + 1] = 0;
  }
}

// churn of round t, one lane per node: ab -> abn (bits past N stay 0), stale bits carried
__global__ __launch_bounds__(kAeBlock) void ae_churn_kernel(AeArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t chunks = (a.N + 63) / 64;
  for (uint64_t ch = wave_id(); ch < chunks; ch += wave_count()) {
    const uint64_t n = ch * 64 + lane;
    bool al = false;
    if (n < a.N) {
      const u32x4 x0 = ae_first_draw((uint32_t)n, a.t, a.k, a.key0, a.key1);
      al = churned((a.ab[2 * ch] >> lane) & 1ull, ae_churn_word(x0, (uint32_t)n, a.t, a.k, a.key0, a.key1), a.fail,
                   a.rec);
    }
    const uint64_t b = __ballot(al);
    if (lane == 0) a.abn[2 * ch] = b;
    if (lane == 1) a.abn[2 * ch + 1] = a.ab[2 * ch + 1];
  }
}

// ---------------------------------------------------------------- dense round
// Row phase layout: sub-step i of a chunk covers nodes i*per .. i*per+per-1, lane
// (sub, c) holds component c of node i*per + sub.  Each lane keeps its L values
// in registers across the exchanges.

template <uint32_t L>
struct MaskOf {  // one bit per lane of a node's group
  using T = typename std::conditional<L <= 8, uint8_t,
            typename std::conditional<L <= 16, uint16_t,
            typename std::conditional<L <= 32, uint32_t, uint64_t>::type>::type>::type;
};

// pull pass: Vn[n] = max(V[n], V[p_j] for every exchange j of n) — plain stores of
// every row — and, per exchange, the mask of components where V[n] > V[p_j]: the
// push pass then needs neither the peer's row nor its alive bit
template <uint32_t L>
__global__ __launch_bounds__(kAeBlock) void ae_pull_kernel(AeArgs a) {
  using MT = typename MaskOf<L>::T;
  constexpr uint32_t per = 64 / L;
  constexpr uint64_t gmask = L >= 64 ? ~0ull : ((1ull << L) - 1ull);
  __shared__ uint64_t red[kAeWaves];
  const uint32_t lane = threadIdx.x & 63, sub = lane / L, c = lane % L;
  const uint32_t* __restrict__ V = a.V;
  uint32_t* __restrict__ Vn = a.Vn;
  MT* __restrict__ pm = reinterpret_cast<MT*>(a.pmask);
  const uint64_t chunks = (a.N + 63) / 64;
  uint64_t msgs = 0;
  for (uint64_t ch = wave_id(); ch < chunks; ch += wave_count()) {
    const uint32_t n = (uint32_t)(ch * 64 + lane);
    const bool aln = (a.abn[2 * ch] >> lane) & 1ull;
    uint32_t own[L], acc[L];
#pragma unroll
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t node = ch * 64 + i * per + sub;
      own[i] = (node < a.N && c < a.K) ? V[node * a.K + c] : 0u;
      acc[i] = own[i];
    }
    u32x4 x{0, 0, 0, 0};
    for (uint32_t j = 0; j < a.k; ++j) {
      uint32_t p = 0;
      bool ex = false;
      if (aln) {
        p = peer_j(a, n, j, x);
        ex = alive_bit(a.abn, p);
      }
      msgs += ex ? 1u : 0u;
      if (!__ballot(ex)) {
        if (ch * 64 + lane < a.N) pm[(ch * 64 + lane) * a.k + j] = 0;
        continue;
      }
      uint32_t vp[L];
      bool go[L];
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) {
        const uint32_t src = i * per + sub;
        const uint32_t pp = (uint32_t)__shfl((int)p, (int)src, 64);
        go[i] = __shfl((int)ex, (int)src, 64) && c < a.K;
        vp[i] = go[i] ? V[(uint64_t)pp * a.K + c] : 0u;
      }
      // lane (sub, 0) stores the push mask of node i*per + sub
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) {
        acc[i] = max(acc[i], vp[i]);
        const uint64_t m = __ballot(go[i] && own[i] > vp[i]);
        const uint64_t node = ch * 64 + i * per + sub;
        if (c == 0 && node < a.N) pm[node * a.k + j] = (MT)((m >> (sub * L)) & gmask);
      }
    }
#pragma unroll
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t node = ch * 64 + i * per + sub;
      if (node < a.N && c < a.K) Vn[node * a.K + c] = acc[i];
    }
  }
  block_add(msgs, red, &a.partial[2]);
}

// push pass: atomicMax(Vn[p_j][c], V[n][c]) for the components c of the pull pass's mask
template <uint32_t L>
__global__ __launch_bounds__(kAeBlock) void ae_push_kernel(AeArgs a) {
  using MT = typename MaskOf<L>::T;
  constexpr uint32_t per = 64 / L;
  const uint32_t lane = threadIdx.x & 63, sub = lane / L, c = lane % L;
  const uint32_t* __restrict__ V = a.V;
  uint32_t* __restrict__ Vn = a.Vn;
  const MT* __restrict__ pm = reinterpret_cast<const MT*>(a.pmask);
  const uint64_t chunks = (a.N + 63) / 64;
  for (uint64_t ch = wave_id(); ch < chunks; ch += wave_count()) {
    const uint64_t nl = ch * 64 + lane;
    const uint32_t n = (uint32_t)nl;
    u32x4 x{0, 0, 0, 0};
    for (uint32_t j = 0; j < a.k; ++j) {
      const uint64_t mw = nl < a.N ? (uint64_t)pm[nl * a.k + j] : 0ull;
      // Philox words for j..j+3 are drawn at j % 4 == 0 whatever the masks say
      uint32_t p = 0;
      if ((j & 3u) == 0 || mw) p = peer_j(a, n, j, x);
      if (!__ballot(mw != 0)) continue;
      // every load in flight first: the pushed component and the peer's current
      // S_{t+1} value (its pull pass is done; values only grow, so a component
      // already at or above the pushed one needs no atomic)
      uint32_t vv[L], cv[L], dst[L];
      bool on[L];
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) {
        const uint32_t src = i * per + sub;
        const uint32_t pp = (uint32_t)__shfl((int)p, (int)src, 64);
        const uint64_t m = __shfl(mw, (int)src, 64);
        on[i] = (m >> c) & 1ull;
        dst[i] = pp;
        vv[i] = on[i] ? V[(ch * 64 + src) * a.K + c] : 0u;
        cv[i] = on[i] ? Vn[(uint64_t)pp * a.K + c] : 0u;
      }
#pragma unroll
      for (uint32_t i = 0; i < L; ++i)
        if (on[i] && vv[i] > cv[i]) atomicMax(&Vn[(uint64_t)dst[i] * a.K + c], vv[i]);
    }
  }
}

// stats of (V, alive bits of ab): alive count, alive nodes equal to the global max
// vector, per-component counts, optional hash; write_stale: stale bits of ab + aux[0].
// Here lane (sub, c) holds component c of nodes sub*L .. sub*L+L-1 (one per sub-step),
// so a group's "differs" bits OR-reduce across its L lanes into its nodes' stale bits.
template <uint32_t L>
__global__ __launch_bounds__(kAeBlock) void ae_stats_kernel(AeArgs a, const uint32_t* __restrict__ V, uint64_t* ab,
                                                            bool write_stale) {
  using BT = typename std::conditional<(L > 32), uint64_t, uint32_t>::type;
  constexpr uint32_t per = 64 / L;
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red[kAeWaves];
  const uint32_t lane = threadIdx.x & 63, sub = lane / L, c = lane % L;
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t tgt = c < a.K ? a.target[c] : 0u;
  const uint64_t chunks = (a.N + 63) / 64;
  uint64_t hash = 0, full = 0, nalive = 0, nstale = 0;
  uint32_t c_lane = 0;
  for (uint64_t ch = wave_id(); ch < chunks; ch += wave_count()) {
    uint32_t v[L];
#pragma unroll
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t node = ch * 64 + sub * L + i;
      v[i] = (node < a.N && c < a.K) ? V[node * a.K + c] : 0u;
    }
    const uint64_t aw = ab[2 * ch];  // bits past N are 0
    BT bad = 0;
    // hash_term's (c*N + node) * kGold64 for node = ch*64 + sub*L + i, stepped
    // by kGold64 per i (mod 2^64: one 64-bit multiply per L terms, bit-exact)
    uint64_t hb = ((uint64_t)c * a.N + ch * 64 + sub * L) * kGold64;
#pragma unroll
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t node = ch * 64 + sub * L + i;
      const bool valid = node < a.N && c < a.K;
      const bool al = (aw >> (sub * L + i)) & 1ull;
      if (a.flags & 1u) hash += valid && v[i] ? mix64((uint64_t)v[i] + hb) : 0ull;
      hb += kGold64;
      c_lane += (valid && al && v[i] == tgt) ? 1u : 0u;
      bad |= (BT)(valid && v[i] != tgt) << i;
    }
#pragma unroll
    for (uint32_t off = 1; off < L; off <<= 1) bad |= (BT)__shfl_xor(bad, (int)off, 64);
    uint64_t stale = 0;
    if (per <= L) {  // few groups: fetch each group's bits
#pragma unroll
      for (uint32_t g = 0; g < per; ++g) stale |= (uint64_t)__shfl(bad, (int)(g * L), 64) << (g * L);
    } else {  // few bits per group: one ballot per bit, over the group leaders
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) stale |= __ballot(c == 0 && ((bad >> i) & 1u)) << i;
    }
    nalive += (uint64_t)__popcll(aw);
    full += (uint64_t)__popcll(aw & ~stale);
    nstale += (uint64_t)__popcll(stale);
    if (write_stale && lane == 0) ab[2 * ch + 1] = stale;
  }
  if (c < a.K && c_lane) atomicAdd(&cnt[c], c_lane);
  // full / nalive / nstale are wave-uniform: count them once per wave
  if (lane != 0) full = nalive = nstale = 0;
  block_add(hash, red, &a.partial[3]);
  block_add(full, red, &a.partial[0]);
  block_add(nalive, red, &a.partial[1]);
  if (write_stale) block_add(nstale, red, &a.aux[0]);
  if (threadIdx.x < a.K && cnt[threadIdx.x])
    atomicAdd((unsigned long long*)&a.partial[4 + threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

// --------------------------------------------------------------- sparse round
// Scan: block b owns chunks [b*spc, (b+1)*spc) and lists, into its own segment,
// the exchanges with a stale end (LDS slot counter); past segcap only counted.
__global__ __launch_bounds__(kAeBlock) void ae_sparse_scan_kernel(AeArgs a) {
  __shared__ uint64_t red[kAeWaves];
  __shared__ uint32_t scnt;
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x == 0) scnt = 0;
  __syncthreads();
  const uint64_t chunks = (a.N + 63) / 64;
  const uint64_t c0 = (uint64_t)blockIdx.x * a.spc;
  const uint64_t c1 = c0 + a.spc < chunks ? c0 + a.spc : chunks;
  uint32_t* eid = a.eid + (size_t)blockIdx.x * a.segcap * 2;
  const uint64_t below = (1ull << lane) - 1ull;
  uint64_t msgs = 0;
  for (uint64_t ch = c0 + (threadIdx.x >> 6); ch < c1; ch += kAeWaves) {
    const uint32_t n = (uint32_t)(ch * 64 + lane);
    const bool aln = (a.abn[2 * ch] >> lane) & 1ull;
    const bool own_stale = (a.abn[2 * ch + 1] >> lane) & 1ull;
    u32x4 x{0, 0, 0, 0};
    for (uint32_t j = 0; j < a.k; ++j) {
      uint32_t p = 0;
      bool ex = false, pst = false;
      if (aln) {
        p = peer_j(a, n, j, x);
        alive_stale(a.abn, p, &ex, &pst);
      }
      msgs += ex ? 1u : 0u;
      const bool need = ex && (own_stale || pst);
      const uint64_t m = __ballot(need);
      if (!m) continue;
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&scnt, (uint32_t)__popcll(m));
      base = (uint32_t)__shfl((int)base, 0, 64);
      const uint32_t slot = base + (uint32_t)__popcll(m & below);
      if (need && slot < a.segcap) {
        eid[2 * slot] = n;
        eid[2 * slot + 1] = p;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.segn[blockIdx.x] = scnt;
    if (scnt) atomicMax((unsigned long long*)&a.aux[1], (unsigned long long)scnt);
  }
  block_add(msgs, red, &a.partial[2]);
}

// Binned scan, pass 1 (one block per region of 2^brs senders, persistent): the
// round's churn (ab -> abn), then every alive sender's exchanges counting-sorted
// by the peer's tile in LDS and
// written out as one contiguous region; the random reads of the peers' alive /
// stale bits move to pass 2, where each tile's bits sit in LDS.  A record is one
// u32 (ae_rec): 80 KiB of LDS per block, so two blocks share a CU and one's
// write-out overlaps the other's draws.
constexpr int kAeBinThreads = 1024;
constexpr uint32_t kAeBinRec = 16384;    // records per region (LDS)
constexpr uint32_t kAeBinTiles = 4032;  // (two emit blocks fit 160 KiB of LDS)
constexpr uint32_t kAeBinQ = kAeBinRec / kAeBinThreads;  // k == 1: senders per thread, peers in registers
constexpr uint32_t kAeDTiles = 4096;  // dense rounds: tiles of 2^14 nodes (N <= 2^26)

// record: p_local (btl bits) | n - region base (brs bits) << btl | stale(n) << (btl + brs)
__device__ __forceinline__ uint32_t ae_rec(uint32_t pl, uint32_t nl, uint32_t stale, uint32_t btl, uint32_t brs) {
  return pl | (nl << btl) | (stale << (btl + brs));
}

constexpr int kAeEmitWaves = 8;  // waves per SIMD: 8 = two blocks per CU (<= 64 VGPRs; 6 / 4 slower)
// k == 1 keeps the peers of pass A in registers (24 VGPRs spill at 8 waves; still 0.516 vs
// 0.568 ms per sparse round redrawing them, profiles/r02_ae_one)
// NT: LDS tile counters (kAeBinTiles for the sparse scan's tiles, two blocks per CU;
// kAeDTiles for the dense round's 2^14-node tiles, one block per CU)
template <bool K1, uint32_t NT>
__global__ __launch_bounds__(kAeBinThreads, (NT > kAeBinTiles ? 4 : kAeEmitWaves)) void ae_bin_emit_kernel(AeArgs a) {
  __shared__ uint32_t cur[NT];
  __shared__ __align__(16) uint32_t st[kAeBinRec];  // read back as uint4
  __shared__ uint32_t wsum[kAeBinThreads / 64];
  __shared__ uint32_t wpre[kAeBinThreads / 64 + 1];
  if (a.gate_out) {  // pipelined sparse round: this round's gate from the previous one (AeArgs)
    bool run = true;
    if (a.gate_prev) {
      const uint64_t* pa = a.prev_partial + a.pl;  // its aux words
      run = *(volatile const uint32_t*)a.gate_prev != 0u && pa[1] <= a.segcap &&
            a.prev_partial[0] != a.prev_partial[1];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.gate_out = run ? 1u : 0u;
    if (!run) return;
  } else if (ae_gated_off(a)) {
    return;
  }
  if (a.zero && blockIdx.x == 0)
    for (uint32_t i = threadIdx.x; i < a.nzero; i += kAeBinThreads) a.zero[i] = 0;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t rs = 1u << a.brs, rp = rs * a.k, nt = a.bnt;
  const uint32_t tmask = (1u << a.btl) - 1u;
  for (uint32_t s = blockIdx.x; s < a.bnreg; s += gridDim.x) {
    const uint64_t base = (uint64_t)s << a.brs;
    __syncthreads();  // the previous region's write-out has read st / cur
    for (uint32_t d = tid; d < nt; d += kAeBinThreads) cur[d] = 0;
    __syncthreads();
    // pass A: tile counts (k == 1: the peer and the stale bit stay in registers)
    uint32_t pr[K1 ? kAeBinQ : 1];
    uint32_t live = 0, stl = 0;
    const uint32_t nq = K1 ? kAeBinQ : rs / kAeBinThreads;  // rs is a multiple of the block (>= 1024 senders)
#pragma unroll
    for (uint32_t q = 0; q < nq; ++q) {
      // the round's churn (ae_churn_kernel's work, fused): a wave holds one 64-node chunk
      const uint64_t n = base + q * kAeBinThreads + tid;
      const uint64_t ch = n >> 6;
      const bool in = n < a.N;
      const uint64_t aw = in ? a.ab[2 * ch] : 0ull, sw = in ? a.ab[2 * ch + 1] : 0ull;
      // one cipher for the churn and the first peers (k <= 3)
      u32x4 x = ae_first_draw((uint32_t)n, a.t, a.k, a.key0, a.key1);
      const bool al =
          in && churned((aw >> lane) & 1ull, ae_churn_word(x, (uint32_t)n, a.t, a.k, a.key0, a.key1), a.fail, a.rec);
      const uint64_t nb = __ballot(al);
      if (in && lane == 0) a.abn[2 * ch] = nb;
      if (in && lane == 1) a.abn[2 * ch + 1] = sw;  // stale bits of S_t carried
      if (!al) continue;
      live |= 1u << q;
      stl |= (uint32_t)((sw >> lane) & 1ull) << q;
      for (uint32_t j = 0; j < a.k; ++j) {
        // (x already holds the draw of j < 4 when k <= 3)
        const uint32_t p =
            j == 0 && a.k <= 3 ? peer_from_word(x.x, a.N - 1, (uint32_t)n) : peer_j(a, (uint32_t)n, j, x);
        if (K1) pr[q] = p;
        atomicAdd(&cur[p >> a.btl], 1u);
      }
    }
    __syncthreads();
    // exclusive scan of cur[0, nt)
    const uint32_t per = (nt + kAeBinThreads - 1) / kAeBinThreads;
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
      uint32_t acc = 0;
      for (int w = 0; w < kAeBinThreads / 64; ++w) {
        wpre[w] = acc;
        acc += wsum[w];
      }
      wpre[kAeBinThreads / 64] = acc;
    }
    __syncthreads();
    uint32_t run = wpre[wave] + inc - mine;
    uint16_t* off = a.boff + (size_t)s * (nt + 1);
    for (uint32_t d = lo; d < hi; ++d) {
      const uint32_t c = cur[d];
      cur[d] = run;
      off[d] = (uint16_t)run;
      run += c;
    }
    const uint32_t total = wpre[kAeBinThreads / 64];
    if (tid == 0) off[nt] = (uint16_t)total;
    __syncthreads();
    // pass B: records to their slots
#pragma unroll
    for (uint32_t q = 0; q < nq; ++q) {
      if (!((live >> q) & 1u)) continue;
      const uint64_t n = base + q * kAeBinThreads + tid;
      const uint32_t nl = q * kAeBinThreads + tid, sb = (stl >> q) & 1u;
      if (K1) {
        const uint32_t p = pr[q];
        st[atomicAdd(&cur[p >> a.btl], 1u)] = ae_rec(p & tmask, nl, sb, a.btl, a.brs);
      } else {
        u32x4 x{0, 0, 0, 0};
        for (uint32_t j = 0; j < a.k; ++j) {
          const uint32_t p = peer_j(a, (uint32_t)n, j, x);
          st[atomicAdd(&cur[p >> a.btl], 1u)] = ae_rec(p & tmask, nl, sb, a.btl, a.brs);
        }
      }
    }
    __syncthreads();
    // 16-B stores (the region's slot has room for rp records; the tail past total is never read)
    uint4* out = (uint4*)(a.brec + (size_t)s * rp);
    for (uint32_t e = tid; e * 4 < total; e += kAeBinThreads) out[e] = ((const uint4*)st)[e];
  }
}

// Binned scan, pass 2 (one block per tile T): the tile's alive and stale bits in
// LDS; every record aimed at T (its run in each region, walked 64 runs per wave,
// lane-strided) counts a message when the peer is alive and lists the exchange
// into segment T when either end is stale.
constexpr uint32_t kAeBinTileLog = 17;  // tiles of up to 2^17 nodes (ae_rec's fields, 32 KiB of LDS)
constexpr uint32_t kAeBinTileWords = 1u << (kAeBinTileLog - 6);

__global__ __launch_bounds__(kAeBinThreads) void ae_bin_scan_kernel(AeArgs a) {
  __shared__ uint64_t wa[kAeBinTileWords], ws[kAeBinTileWords];
  __shared__ uint32_t scnt;
  __shared__ uint64_t red[kAeBinThreads / 64];
  if (ae_gated_off(a)) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t T = blockIdx.x, nt = a.bnt;
  const uint32_t tw = 1u << (a.btl - 6);  // words per tile
  const uint64_t w0 = (uint64_t)T * tw, nw = (a.N + 63) / 64;
  if (tid == 0) scnt = 0;
  for (uint32_t w = tid; w < tw; w += kAeBinThreads) {
    const bool in = w0 + w < nw;
    wa[w] = in ? a.abn[2 * (w0 + w)] : 0ull;
    ws[w] = in ? a.abn[2 * (w0 + w) + 1] : 0ull;
  }
  __syncthreads();
  uint32_t* eid = a.eid + (size_t)T * a.segcap * 2;
  const uint32_t rp = (1u << a.brs) * a.k;
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t tmask = (1u << a.btl) - 1u;
  uint64_t msgs = 0;
  for (uint32_t r0 = wave * 64; r0 < a.bnreg; r0 += (kAeBinThreads / 64) * 64) {
    const uint32_t r = r0 + lane;
    uint32_t be = 0, en = 0;
    if (r < a.bnreg) {
      const uint16_t* o = a.boff + (size_t)r * (nt + 1) + T;
      be = o[0];
      en = o[1];
    }
    const uint32_t len = en - be;
    uint32_t inc = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    const uint32_t exc = inc - len, total = __shfl(inc, 63, 64);
    const uint64_t rbase = (uint64_t)r * rp + be - exc;  // record of flat index f in this lane's run: rbase + f
    const uint32_t nmask = (1u << a.brs) - 1u;
    constexpr int U = 4;
    for (uint32_t f0 = 0; f0 < total; f0 += 64 * U) {
      uint32_t rec[U], reg[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t f = f0 + u * 64 + lane;
        // owner run: the last lane whose run starts at or before f (a non-empty run)
        uint32_t ow = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1) {
          const uint32_t c = ow + step;
          if (c < 64 && (uint32_t)__shfl((int)exc, (int)c, 64) <= f) ow = c;
        }
        const uint64_t rb = (uint64_t)__shfl((long long)rbase, (int)ow, 64);
        rec[u] = f < total ? a.brec[rb + f] : 0u;
        reg[u] = f < total ? r0 + ow : ~0u;  // the record's region (~0: past the end)
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool valid = reg[u] != ~0u;
        const uint32_t n = (reg[u] << a.brs) + ((rec[u] >> a.btl) & nmask);
        const uint32_t pl = rec[u] & tmask;
        const bool ex = valid && ((wa[pl >> 6] >> (pl & 63)) & 1ull);  // n is alive (pass 1)
        msgs += ex ? 1u : 0u;
        const bool need = ex && (((rec[u] >> (a.btl + a.brs)) & 1u) || ((ws[pl >> 6] >> (pl & 63)) & 1ull));
        const uint64_t m = __ballot(need);
        if (!m) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&scnt, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, 0, 64);
        const uint32_t slot = base + (uint32_t)__popcll(m & below);
        if (need && slot < a.segcap) {
          eid[2 * slot] = n;
          eid[2 * slot + 1] = (T << a.btl) | pl;
        }
      }
    }
  }
  msgs = wave_sum64(msgs);
  if (lane == 0) red[wave] = msgs;
  __syncthreads();
  if (tid == 0) {
    uint64_t sm = 0;
    for (int w = 0; w < kAeBinThreads / 64; ++w) sm += red[w];
    if (sm) atomicAdd((unsigned long long*)&a.partial[2], (unsigned long long)sm);
    a.segn[T] = scnt;
    if (scnt) atomicMax((unsigned long long*)&a.aux[1], (unsigned long long)scnt);
  }
}

// ---------------------------------------------------------------- binned dense round
// The push pass above costs ~4e8 global atomicMax per dense round at 2^26 nodes.  Here the
// exchanges are inverted instead: ae_bin_emit (churn fused) bins every alive sender's
// exchanges by the peer's tile of 2^14 nodes, and one block per tile counting-sorts the
// records aimed at it by node in LDS (in-edge lists).  Each node's S_{t+1} row is then the
// max of its own row, its peers' rows (pull) and the rows of the senders that picked it
// (push, as 64-B gathers): every row is written once with plain stores, so the stats pass
// folds into the same kernel.
constexpr uint32_t kAeDTileLog = 14;
constexpr uint32_t kAeDTile = 1u << kAeDTileLog;
constexpr uint32_t kAeDCap = 18432;    // in-edges sorted in LDS per pass (a tile's nodes in ranges)
constexpr uint32_t kAeDMaxReg = 4096;  // regions in the LDS run table
// 8 waves per block (one block per CU: the LDS): 256 VGPRs per lane for the 2L gathers in flight
constexpr uint32_t kAeDThreads = 512;

// every record of tile T (its run in each region, 64 runs per wave, lane-strided), as
// fn(record, region); rt[r] = run start | run end << 16
// (rt == nullptr: the run starts come from a.boff, L2-resident, for tile T)
template <uint32_t NW, typename F>
__device__ __forceinline__ void ae_tile_records(const AeArgs& a, const uint32_t* rt, uint32_t T, F&& fn) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t rp = (1u << a.brs) * a.k;
  for (uint32_t r0 = wave * 64; r0 < a.bnreg; r0 += NW * 64) {
    const uint32_t r = r0 + lane;
    uint32_t w = 0;
    if (r < a.bnreg) {
      if (rt) {
        w = rt[r];
      } else {
        const uint16_t* o = a.boff + (size_t)r * (a.bnt + 1) + T;
        w = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
      }
    }
    const uint32_t be = w & 0xFFFFu, len = (w >> 16) - be;
    uint32_t inc = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += y;
    }
    const uint32_t exc = inc - len, total = __shfl(inc, 63, 64);
    const uint64_t rbase = (uint64_t)r * rp + be - exc;
    constexpr int U = 4;
    for (uint32_t f0 = 0; f0 < total; f0 += 64 * U) {
      uint32_t rec[U], reg[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t f = f0 + u * 64 + lane;
        uint32_t ow = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1) {
          const uint32_t cc = ow + step;
          if (cc < 64 && (uint32_t)__shfl((int)exc, (int)cc, 64) <= f) ow = cc;
        }
        const uint64_t rb = (uint64_t)__shfl((long long)rbase, (int)ow, 64);
        rec[u] = f < total ? a.brec[rb + f] : 0u;
        reg[u] = f < total ? r0 + ow : ~0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (reg[u] != ~0u) fn(rec[u], reg[u]);
    }
  }
}


// The in-edge sort of tile T, shared by both apply kernels (NW waves per block).  pos2
// holds u16 counts, then starts, then (after a fill) ends, packed in pairs: a tile's
// records stay below 2^16 (k <= 3; a larger total sets aux[1], the host reruns the round).
struct AeSortSh {
  uint32_t* pos2;  // [kAeDTile / 2]
  uint32_t* srt;   // [cap] sender | (node & 63) << 26, sorted by node
  const uint32_t* rt;  // run table or nullptr
  uint32_t *wsum, *wpre, *rng;  // [NW], [NW + 1], [3]: range end, range base, total
  // stale filter (kAeSbValid: the stale bits of S_t in a.ab are exact): an in-edge matters only into a
  // stale node, and one from an up-to-date sender (row == target, the componentwise maximum of
  // every row) makes the node's S_{t+1} row the target whatever else it gets, so it is marked in
  // tgtb and never sorted; only stale-sender in-edges into stale nodes are gathered
  bool filt;
  uint64_t* stile;        // [kAeDTile / 64] stale bits of the tile's nodes (S_t), when filt
  uint32_t* tgtb;         // [kAeDTile / 32] node took an in-edge from an up-to-date sender, when filt
};

// the record is sorted (gathered) at all; marks tgtb for an up-to-date sender's in-edge
__device__ __forceinline__ bool ae_sort_keep(const AeArgs& a, const AeSortSh& sh, uint32_t rec, uint32_t pl,
                                             bool mark) {
  if (!sh.filt) return true;
  if (!((sh.stile[pl >> 6] >> (pl & 63u)) & 1ull)) return false;  // the node is up to date: nothing to take
  if ((rec >> (a.btl + a.brs)) & 1u) return true;           // a stale sender: its row is gathered
  if (mark) atomicOr(&sh.tgtb[pl >> 5], 1u << (pl & 31u));
  return false;
}

__device__ __forceinline__ uint32_t ae_pget(const AeSortSh& sh, uint32_t i) {
  return i >= kAeDTile ? sh.rng[2] : (sh.pos2[i >> 1] >> ((i & 1u) << 4)) & 0xFFFFu;
}

// counts and their exclusive scan (every thread; ends with a barrier)
template <uint32_t NW>
__device__ void ae_sort_count(const AeArgs& a, const AeSortSh& sh, uint32_t T) {
  constexpr uint32_t nth = NW * 64;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint32_t i = tid; i < kAeDTile / 2; i += nth) sh.pos2[i] = 0;
  if (sh.filt) {
    for (uint32_t i = tid; i < kAeDTile / 32; i += nth) sh.tgtb[i] = 0;
    const uint64_t w0 = ((uint64_t)T << kAeDTileLog) >> 6, nw = (a.N + 63) >> 6;
    for (uint32_t i = tid; i < kAeDTile / 64; i += nth) sh.stile[i] = w0 + i < nw ? a.ab[2 * (w0 + i) + 1] : 0ull;
  }
  __syncthreads();
  ae_tile_records<NW>(a, sh.rt, T, [&](uint32_t rec, uint32_t) {
      const uint32_t pl = rec & (kAeDTile - 1u);
      if (ae_sort_keep(a, sh, rec, pl, true)) atomicAdd(&sh.pos2[pl >> 1], 1u << ((pl & 1u) << 4));
    });
  __syncthreads();
  constexpr uint32_t qw = (kAeDTile / 2 + nth - 1) / nth;  // words per thread
  const uint32_t w0 = min(tid * qw, kAeDTile / 2), w1 = min(w0 + qw, kAeDTile / 2);
  uint32_t mine = 0;
  for (uint32_t i = w0; i < w1; ++i) {
    const uint32_t w = sh.pos2[i];
    mine += (w & 0xFFFFu) + (w >> 16);
  }
  uint32_t inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) sh.wsum[wave] = inc;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < NW; ++w) {
      sh.wpre[w] = t;
      t += sh.wsum[w];
    }
    sh.rng[2] = t;
    if (t > 0xFFFFu) a.aux[1] = 1ull;  // u16 positions would wrap
  }
  __syncthreads();
  uint32_t run = sh.wpre[wave] + inc - mine;
  for (uint32_t i = w0; i < w1; ++i) {
    const uint32_t w = sh.pos2[i];
    const uint32_t r0 = run, r1 = run + (w & 0xFFFFu);
    sh.pos2[i] = (r0 & 0xFFFFu) | (r1 << 16);
    run = r1 + (w >> 16);
  }
  __syncthreads();
}

// the next node range [lo, hi): whole chunks whose in-edges fit cap (at least one chunk),
// its records sorted into srt; returns hi, *base = the range's first position (barriers)
template <uint32_t NW>
__device__ uint32_t ae_sort_range(const AeArgs& a, const AeSortSh& sh, uint32_t T, uint32_t tn, uint32_t lo,
                                  uint32_t cap, uint32_t* base_out) {
  if (threadIdx.x == 0) {
    const uint32_t base = ae_pget(sh, lo), nch = (tn + 63) >> 6;
    uint32_t l = (lo >> 6) + 1, h = nch;
    while (l < h) {
      const uint32_t m = (l + h + 1) >> 1;
      if (((ae_pget(sh, min(m << 6, tn)) - base) & 0xFFFFu) <= cap) l = m;
      else h = m - 1;
    }
    const uint32_t hi = min(l << 6, tn);
    sh.rng[0] = hi;
    sh.rng[1] = base;
    if (((ae_pget(sh, hi) - base) & 0xFFFFu) > cap) a.aux[1] = 1ull;  // one chunk past the list: host reruns
  }
  __syncthreads();
  const uint32_t hi = sh.rng[0], base = sh.rng[1];
  const uint32_t nmask = (1u << a.brs) - 1u;
  if (ae_pget(sh, hi) != base) {
    ae_tile_records<NW>(a, sh.rt, T, [&](uint32_t rec, uint32_t reg) {
      const uint32_t pl = rec & (kAeDTile - 1u);
      if (pl >= lo && pl < hi && ae_sort_keep(a, sh, rec, pl, false)) {
        const uint32_t b = (pl & 1u) << 4;
        const uint32_t s = (((atomicAdd(&sh.pos2[pl >> 1], 1u << b) >> b) & 0xFFFFu) - base) & 0xFFFFu;
        if (s < cap) sh.srt[s] = ((reg << a.brs) + ((rec >> kAeDTileLog) & nmask)) | ((pl & 63u) << 26);
      }
    });
  }
  __syncthreads();
  *base_out = base;
  return hi;
}

__device__ __forceinline__ uint32_t ae_tile_of(uint32_t nt) {
  // XCD-contiguous tiles: the blocks resident on one XCD share run-start and record lines
  return (nt & 7u) ? blockIdx.x : (blockIdx.x & 7u) * (nt >> 3) + (blockIdx.x >> 3);
}

template <uint32_t L, uint32_t KJ>  // KJ = k (<= 3)
__global__ __launch_bounds__(kAeDThreads) void ae_dense_apply_kernel(AeArgs a) {
  static_assert(L <= 16, "per-wave LDS scratch of 64 x L words");
  constexpr uint32_t per = 64 / L;
  constexpr uint64_t gmask = L >= 64 ? ~0ull : ((1ull << L) - 1ull);
  constexpr uint32_t kW = kAeDThreads / 64;
  constexpr uint32_t kB = 16;  // in-edge gathers in flight per lane (per edges each)
  __shared__ uint32_t pos2[kAeDTile / 2];
  __shared__ uint32_t srt[kAeDCap];
  __shared__ uint32_t rt[kAeDMaxReg];
  __shared__ uint32_t scr[kW][64 * L];  // per wave: in-edge max-merges of its chunk, [node][component]
  __shared__ uint32_t wsum[kW], wpre[kW + 1], rng[3], cnt[64];
  __shared__ uint64_t red[kW];
  __shared__ uint64_t stile[kAeDTile / 64];
  __shared__ uint32_t tgtb[kAeDTile / 32];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, sub = lane / L, c = lane % L;
  const uint32_t T = ae_tile_of(a.bnt);
  const uint64_t t0 = (uint64_t)T << kAeDTileLog;
  const uint32_t tn = (uint32_t)((a.N - t0) < kAeDTile ? (a.N - t0) : kAeDTile);
  const uint32_t* __restrict__ V = a.V;
  uint32_t* __restrict__ Vn = a.Vn;
  for (uint32_t r = tid; r < a.bnreg; r += kAeDThreads) {
    const uint16_t* o = a.boff + (size_t)r * (a.bnt + 1) + T;
    rt[r] = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
  }
  if (tid < 64) cnt[tid] = 0;
  const bool filt = (a.flags & kAeSbValid) != 0;
  const AeSortSh sh{pos2, srt, rt, wsum, wpre, rng, filt, stile, tgtb};
  ae_sort_count<kW>(a, sh, T);
  auto pget = [&](uint32_t i) { return ae_pget(sh, i); };
  const uint32_t tgt = c < a.K ? a.target[c] : 0u;
  const bool hashing = (a.flags & 1u) != 0;
  uint64_t msgs = 0, hash = 0, full = 0, nalive = 0, nstale = 0;
  uint32_t c_lane = 0;
  const uint32_t cap = (a.dcap && a.dcap < kAeDCap) ? a.dcap : kAeDCap;  // a smaller one tests the ranges
  uint32_t* sc = scr[wave];
  for (uint32_t lo = 0; lo < tn;) {
    uint32_t base;
    const uint32_t hi = ae_sort_range<kW>(a, sh, T, tn, lo, cap, &base);
    // node p's in-edges now end at pget(p) and start at pget(p - 1) (base for p = lo)
    for (uint32_t ch = (lo >> 6) + wave; ch < (hi + 63) >> 6; ch += kW) {
      const uint64_t gch = (t0 >> 6) + ch;
      const uint64_t nb = t0 + ((uint64_t)ch << 6);
      const uint32_t n = (uint32_t)(nb + lane);
      const uint64_t aw = a.abn[2 * gch];  // alive after this round's churn (bits past N are 0)
      const bool aln = (aw >> lane) & 1ull;
      const uint32_t c0 = ch << 6;
      const uint32_t e0 = ((c0 == lo ? base : pget(c0 - 1)) - base) & 0xFFFFu;
      const uint32_t ne = ((pget(c0 + 63) - base) & 0xFFFFu) - e0;  // the chunk's in-edges (wave-uniform)
      // stale filter (as in ae_dense_apply_q_kernel)
      const bool need = aln && (!filt || ((stile[ch] >> lane) & 1ull));
      const bool totgt = filt && need && ((tgtb[(c0 >> 5) + (lane >> 5)] >> (lane & 31u)) & 1u);
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) sc[i * 64 + lane] = 0u;
      // every gather of the chunk is issued before any is used: own rows, the peers'
      // rows (before their alive bits are known), the first kB in-edge groups
      uint32_t acc[L];
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) {
        const uint64_t node = nb + i * per + sub;
        acc[i] = (node < a.N && c < a.K) ? V[node * a.K + c] : 0u;
      }
      // the peers' rows are gathered before their alive bits are known (waiting for
      // those first costs a round trip per chunk: 7.9 -> 10.4 ms per dense round)
      uint32_t pj[KJ];
      bool exj[KJ];
      u32x4 x{0, 0, 0, 0};
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j) pj[j] = aln ? peer_j(a, n, j, x) : 0u;
      uint32_t vp[KJ][L];
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j) {
#pragma unroll
        for (uint32_t i = 0; i < L; ++i) {
          const uint32_t src = i * per + sub;
          const uint32_t pp = (uint32_t)__shfl((int)pj[j], (int)src, 64);
          const bool go = __shfl((int)(need && !totgt), (int)src, 64) && c < a.K;
          vp[j][i] = go ? V[(uint64_t)pp * a.K + c] : 0u;
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j) exj[j] = aln && alive_bit(a.abn, pj[j]);
      auto in_group = [&](uint32_t f0) {
        uint32_t vi[kB], ti[kB];
#pragma unroll
        for (uint32_t b = 0; b < kB; ++b) {
          const uint32_t f = f0 + b * per + sub;
          // (clamped: after an overflow, flagged for the host, the list is cut short)
          const uint32_t m = (f < ne && c < a.K) ? srt[min(e0 + f, cap - 1u)] : 0u;
          const uint32_t po = m >> 26;
          const bool on = f < ne && c < a.K && ((aw >> po) & 1ull) && (m & 0x3FFFFFFu) < a.N;  // picked node alive
          vi[b] = on ? V[(uint64_t)(m & 0x3FFFFFFu) * a.K + c] : 0u;
          ti[b] = on ? po * L + c : ~0u;
        }
#pragma unroll
        for (uint32_t b = 0; b < kB; ++b)
          if (ti[b] != ~0u) atomicMax(&sc[ti[b]], vi[b]);
      };
      if (ne) in_group(0);
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j) {
        msgs += exj[j] ? 1u : 0u;
#pragma unroll
        for (uint32_t i = 0; i < L; ++i)
          if (__shfl((int)exj[j], (int)(i * per + sub), 64)) acc[i] = max(acc[i], vp[j][i]);
      }
      for (uint32_t f0 = per * kB; f0 < ne; f0 += per * kB) in_group(f0);
      // S_{t+1} rows and their stats (ae_stats_kernel's, in this layout)
      uint64_t stale = 0;
      uint64_t hb = ((uint64_t)c * a.N + nb + sub) * kGold64;
#pragma unroll
      for (uint32_t i = 0; i < L; ++i) {
        acc[i] = max(acc[i], sc[i * 64 + lane]);
        if (__shfl((int)totgt, (int)(i * per + sub), 64) && c < a.K) acc[i] = tgt;
        const uint64_t node = nb + i * per + sub;
        const bool valid = node < a.N && c < a.K;
        if (valid) Vn[node * a.K + c] = acc[i];
        const bool al = (aw >> (i * per + sub)) & 1ull;
        if (hashing) hash += valid && acc[i] ? mix64((uint64_t)acc[i] + hb) : 0ull;
        hb += (uint64_t)per * kGold64;
        c_lane += (valid && al && acc[i] == tgt) ? 1u : 0u;
        const uint64_t m = __ballot(valid && acc[i] != tgt);
#pragma unroll
        for (uint32_t g = 0; g < per; ++g) stale |= (uint64_t)(((m >> (g * L)) & gmask) != 0ull) << (i * per + g);
      }
      if (lane == 0) {
        a.abn[2 * gch + 1] = stale;
        nalive += (uint64_t)__popcll(aw);
        full += (uint64_t)__popcll(aw & ~stale);
        nstale += (uint64_t)__popcll(stale);
      }
    }
    __syncthreads();  // the next range's fill rewrites srt
    lo = hi;
  }
  if (c < a.K && c_lane) atomicAdd(&cnt[c], c_lane);
  block_add<kW>(msgs, red, &a.partial[2]);
  block_add<kW>(hash, red, &a.partial[3]);
  block_add<kW>(full, red, &a.partial[0]);
  block_add<kW>(nalive, red, &a.partial[1]);
  block_add<kW>(nstale, red, &a.aux[0]);
  if (tid < a.K && cnt[tid]) atomicAdd((unsigned long long*)&a.partial[4 + tid], (unsigned long long)cnt[tid]);
}

// K == 16 (configs[4]): a row is 64 B, moved as four 16-B pieces.  Lane r*4 + q holds
// components 4q .. 4q+3 of row r of a 16-row piece group, so the gathers need a quarter of
// the address registers and the kernel fits 16 waves per CU (the LDS table of run starts
// gives way to the per-wave scratch; the run starts come from L2).
constexpr uint32_t kAeQThreads = 12 * 64;  // 12 waves per CU: 168 VGPRs (16 waves: 16 spill at 128, slower)
constexpr uint32_t kAeQCap = 18432;        // sorted in-edges per pass (LDS)

__device__ __forceinline__ uint4 max4(uint4 x, uint4 y) {
  return uint4{max(x.x, y.x), max(x.y, y.y), max(x.z, y.z), max(x.w, y.w)};
}

template <uint32_t KJ>
__global__ __launch_bounds__(kAeQThreads) void ae_dense_apply_q_kernel(AeArgs a) {
  constexpr uint32_t kW = kAeQThreads / 64;
  constexpr uint32_t kBQ = 4;  // in-edge piece groups in flight (16 edges each)
  __shared__ uint32_t pos2[kAeDTile / 2];
  __shared__ uint32_t srt[kAeQCap];
  __shared__ __align__(16) uint32_t scr[kW][64 * 16];
  __shared__ uint32_t wsum[kW], wpre[kW + 1], rng[3], cnt[64];
  __shared__ uint64_t red[kW];
  __shared__ uint64_t stile[kAeDTile / 64];
  __shared__ uint32_t tgtb[kAeDTile / 32];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane >> 2, q = lane & 3;
  const uint32_t T = ae_tile_of(a.bnt);
  const uint64_t t0 = (uint64_t)T << kAeDTileLog;
  const uint32_t tn = (uint32_t)((a.N - t0) < kAeDTile ? (a.N - t0) : kAeDTile);
  const uint32_t* __restrict__ V = a.V;
  uint32_t* __restrict__ Vn = a.Vn;
  if (tid < 64) cnt[tid] = 0;
  const bool filt = (a.flags & kAeSbValid) != 0;
  const AeSortSh sh{pos2, srt, nullptr, wsum, wpre, rng, filt, stile, tgtb};
  ae_sort_count<kW>(a, sh, T);
  const uint4 tg = reinterpret_cast<const uint4*>(a.target)[q];
  const bool hashing = (a.flags & 1u) != 0;
  uint64_t msgs = 0, hash = 0, full = 0, nalive = 0, nstale = 0;
  uint32_t cq[4] = {0, 0, 0, 0};
  const uint32_t cap = (a.dcap && a.dcap < kAeQCap) ? a.dcap : kAeQCap;
  uint32_t* sc = scr[wave];
  auto row = [&](uint64_t node) { return reinterpret_cast<const uint4*>(V + node * 16 + q * 4); };
  for (uint32_t lo = 0; lo < tn;) {
    uint32_t base;
    const uint32_t hi = ae_sort_range<kW>(a, sh, T, tn, lo, cap, &base);
    for (uint32_t ch = (lo >> 6) + wave; ch < (hi + 63) >> 6; ch += kW) {
      const uint64_t gch = (t0 >> 6) + ch;
      const uint64_t nb = t0 + ((uint64_t)ch << 6);
      const uint32_t n = (uint32_t)(nb + lane);
      const uint64_t aw = a.abn[2 * gch];  // alive after this round's churn (bits past N are 0)
      const bool aln = (aw >> lane) & 1ull;
      const uint32_t c0 = ch << 6;
      const uint32_t e0 = ((c0 == lo ? base : ae_pget(sh, c0 - 1)) - base) & 0xFFFFu;
      const uint32_t ne = ((ae_pget(sh, c0 + 63) - base) & 0xFFFFu) - e0;  // the chunk's in-edges
      // stale filter: an up-to-date node keeps its row (it is the target) and gathers nothing; a
      // stale one takes the target outright from an alive up-to-date sender (tgtb).  (The peers'
      // rows are gathered before their bits are known, so an up-to-date peer saves no traffic and
      // is not probed for: its row is the target, and the max takes it.)
      const bool need = aln && (!filt || ((stile[ch] >> lane) & 1ull));
      const bool totgt = filt && need && ((tgtb[(c0 >> 5) + (lane >> 5)] >> (lane & 31u)) & 1u);
#pragma unroll
      for (uint32_t g = 0; g < 4; ++g) reinterpret_cast<uint4*>(sc)[g * 64 + lane] = uint4{0, 0, 0, 0};
      // own rows, the peers' rows (alive bits awaited after), the first in-edge groups
      uint4 o[4];
#pragma unroll
      for (uint32_t g = 0; g < 4; ++g) {
        const uint64_t node = nb + g * 16 + r;
        o[g] = node < a.N ? *row(node) : uint4{0, 0, 0, 0};
      }
      uint32_t pj[KJ];
      bool exj[KJ];
      u32x4 x{0, 0, 0, 0};
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j) pj[j] = aln ? peer_j(a, n, j, x) : 0u;
      // every peer row is gathered at once; the alive bits are checked after (awaiting them
      // first costs a round trip per chunk: DESIGN.md §3.8)
      uint4 vp[KJ][4];
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j)
#pragma unroll
        for (uint32_t g = 0; g < 4; ++g) {
          const uint32_t src = g * 16 + r;
          const uint32_t pp = (uint32_t)__shfl((int)pj[j], (int)src, 64);
          const bool go = __shfl((int)(need && !totgt), (int)src, 64);
          vp[j][g] = go ? *row(pp) : uint4{0, 0, 0, 0};
        }
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j) exj[j] = aln && alive_bit(a.abn, pj[j]);
      auto in_group = [&](uint32_t f0) {
        uint4 vi[kBQ];
        uint32_t ti[kBQ];
#pragma unroll
        for (uint32_t b = 0; b < kBQ; ++b) {
          const uint32_t f = f0 + b * 16 + r;
          // (clamped: after an overflow, flagged for the host, the list is cut short)
          const uint32_t m = f < ne ? srt[min(e0 + f, cap - 1u)] : 0u;
          const uint32_t po = m >> 26, sn = m & 0x3FFFFFFu;
          const bool on = f < ne && ((aw >> po) & 1ull) && sn < a.N;  // the picked node is alive
          vi[b] = on ? *row(sn) : uint4{0, 0, 0, 0};
          ti[b] = on ? po * 16 + q * 4 : ~0u;
        }
#pragma unroll
        for (uint32_t b = 0; b < kBQ; ++b)
          if (ti[b] != ~0u) {
            atomicMax(&sc[ti[b]], vi[b].x);
            atomicMax(&sc[ti[b] + 1], vi[b].y);
            atomicMax(&sc[ti[b] + 2], vi[b].z);
            atomicMax(&sc[ti[b] + 3], vi[b].w);
          }
      };
      if (ne) in_group(0);
#pragma unroll
      for (uint32_t j = 0; j < KJ; ++j) {
        msgs += exj[j] ? 1u : 0u;
#pragma unroll
        for (uint32_t g = 0; g < 4; ++g)
          if (__shfl((int)exj[j], (int)(g * 16 + r), 64)) o[g] = max4(o[g], vp[j][g]);
      }
      for (uint32_t f0 = 16 * kBQ; f0 < ne; f0 += 16 * kBQ) in_group(f0);
      // S_{t+1} rows and their stats (ae_stats_kernel's, in this layout)
      uint64_t stale = 0;
#pragma unroll
      for (uint32_t g = 0; g < 4; ++g) {
        const uint32_t nr = g * 16 + r;
        o[g] = max4(o[g], reinterpret_cast<const uint4*>(sc)[nr * 4 + q]);
        if (__shfl((int)totgt, (int)nr, 64)) o[g] = tg;
        const uint64_t node = nb + nr;
        const bool valid = node < a.N;
        if (valid) *reinterpret_cast<uint4*>(Vn + node * 16 + q * 4) = o[g];
        const bool al = (aw >> nr) & 1ull;
        const uint32_t v[4] = {o[g].x, o[g].y, o[g].z, o[g].w};
        const uint32_t tv[4] = {tg.x, tg.y, tg.z, tg.w};
        bool bad = false;
        // hash_term's ((4q + t) * N + node) * kGold64, stepped by N * kGold64 over t (mod 2^64)
        uint64_t hb = ((uint64_t)(q * 4) * a.N + node) * kGold64;
        const uint64_t hstep = a.N * kGold64;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t, hb += hstep) {
          if (hashing && valid && v[t]) hash += mix64((uint64_t)v[t] + hb);
          cq[t] += (valid && al && v[t] == tv[t]) ? 1u : 0u;
          bad |= valid && v[t] != tv[t];
        }
        // row nr is stale when any of its four lanes saw a differing component
        uint64_t m = __ballot(bad);
        m |= m >> 1;
        m |= m >> 2;
#pragma unroll
        for (uint32_t rr = 0; rr < 16; ++rr) stale |= ((m >> (4 * rr)) & 1ull) << (g * 16 + rr);
      }
      if (lane == 0) {
        a.abn[2 * gch + 1] = stale;
        nalive += (uint64_t)__popcll(aw);
        full += (uint64_t)__popcll(aw & ~stale);
        nstale += (uint64_t)__popcll(stale);
      }
    }
    __syncthreads();  // the next range's fill rewrites srt
    lo = hi;
  }
#pragma unroll
  for (uint32_t t = 0; t < 4; ++t)
    if (cq[t]) atomicAdd(&cnt[q * 4 + t], cq[t]);
  block_add<kW>(msgs, red, &a.partial[2]);
  block_add<kW>(hash, red, &a.partial[3]);
  block_add<kW>(full, red, &a.partial[0]);
  block_add<kW>(nalive, red, &a.partial[1]);
  block_add<kW>(nstale, red, &a.aux[0]);
  if (tid < 16 && cnt[tid]) atomicAdd((unsigned long long*)&a.partial[4 + tid], (unsigned long long)cnt[tid]);
}

// edges of this block's segment, or 0 when any segment overflowed (the host reruns the round dense)
// (a.spb blocks share a segment: block = segment * spb + sub, edges sub, sub + spb, ... of each step)
__device__ __forceinline__ uint32_t segment_edges(const AeArgs& a) {
  return a.aux[1] > a.segcap ? 0u : a.segn[blockIdx.x / a.spb];
}
__device__ __forceinline__ size_t segment_base(const AeArgs& a) { return (size_t)(blockIdx.x / a.spb) * a.segcap; }

// snapshot the S_t rows of both ends (before any in-place write)
template <uint32_t L>
__global__ __launch_bounds__(kAeBlock) void ae_sparse_gather_kernel(AeArgs a) {
  if (ae_gated_off(a)) return;
  constexpr uint32_t epb = kAeBlock / L;  // edges per block step
  const uint32_t c = threadIdx.x % L;
  const uint32_t m = segment_edges(a);
  if (c >= a.K) return;
  const size_t s0 = segment_base(a);
  for (uint32_t i = (blockIdx.x % a.spb) * epb + threadIdx.x / L; i < m; i += epb * a.spb) {
    const size_t e = s0 + i;
    const uint32_t n = a.eid[2 * e], p = a.eid[2 * e + 1];
    const uint32_t vn = a.V[(uint64_t)n * a.K + c], vp = a.V[(uint64_t)p * a.K + c];
    a.erow[(2 * e) * a.K + c] = vn;
    a.erow[(2 * e + 1) * a.K + c] = vp;
  }
}

// merge in place: both ends take the max of the two snapshots
template <uint32_t L>
__global__ __launch_bounds__(kAeBlock) void ae_sparse_apply_kernel(AeArgs a) {
  if (ae_gated_off(a)) return;
  constexpr uint32_t epb = kAeBlock / L;
  const uint32_t c = threadIdx.x % L;
  const uint32_t m = segment_edges(a);
  if (c >= a.K) return;
  const size_t s0 = segment_base(a);
  for (uint32_t i = (blockIdx.x % a.spb) * epb + threadIdx.x / L; i < m; i += epb * a.spb) {
    const size_t e = s0 + i;
    const uint32_t n = a.eid[2 * e], p = a.eid[2 * e + 1];
    const uint32_t on = a.erow[(2 * e) * a.K + c], op = a.erow[(2 * e + 1) * a.K + c];
    if (op > on) atomicMax(&a.V[(uint64_t)n * a.K + c], op);
    if (on > op) atomicMax(&a.V[(uint64_t)p * a.K + c], on);
  }
}

// each touched node once (the first end to claim it this epoch): hash delta
// old -> new row into partial[3], clear its stale bit when it reached the target
template <uint32_t L>
__global__ __launch_bounds__(kAeBlock) void ae_sparse_fix_kernel(AeArgs a) {
  constexpr uint32_t epb = kAeBlock / L;
  constexpr uint64_t gmask = L >= 64 ? ~0ull : ((1ull << L) - 1ull);
  __shared__ uint64_t red[kAeWaves];
  if (ae_gated_off(a)) return;
  const uint32_t lane = threadIdx.x & 63, c = lane % L, lead = lane - c;
  const uint32_t m = segment_edges(a);
  const uint32_t tgt = c < a.K ? a.target[c] : 0u;
  const size_t s0 = segment_base(a);
  uint64_t dh = 0;
  // the same trip count for every lane of the block, so the ballots see every lane
  for (uint32_t b = (blockIdx.x % a.spb) * epb; b < m; b += epb * a.spb) {
    const uint32_t i = b + threadIdx.x / L;
    const bool ve = i < m;
    const size_t e = s0 + i;
    for (uint32_t end = 0; end < 2; ++end) {
      const uint32_t xn = ve ? a.eid[2 * e + end] : 0u;
      int own = 0;
      if (ve && c == 0) own = atomicMax(&a.claim[xn], a.epoch) < a.epoch;
      own = __shfl(own, (int)lead, 64);
      const bool act = own && c < a.K;
      const uint32_t nv = act ? a.V[(uint64_t)xn * a.K + c] : 0u;
      const uint32_t ov = act ? a.erow[(2 * e + end) * a.K + c] : 0u;
      if ((a.flags & 1u) && act) dh += hash_term(nv, c, xn, a.N) - hash_term(ov, c, xn, a.N);
      const uint64_t bad = __ballot(act && nv != tgt);
      if (own && c == 0 && !((bad >> lead) & gmask))
        atomicAnd((unsigned long long*)&a.abn[2 * (xn >> 6) + 1], ~(1ull << (xn & 63)));
    }
  }
  block_add(dh, red, &a.partial[3]);
}

// stats of the sparse round's result from the bitmaps, one lane per 64-node word:
// full = alive and not stale; per-component counts add the matching components of
// the (few) alive stale rows
__global__ __launch_bounds__(kAeBlock) void ae_sparse_stats_kernel(AeArgs a) {
  __shared__ uint32_t cnt[64], tgt[64];
  __shared__ uint64_t red[kAeWaves];
  if (ae_gated_off(a)) return;
  if (threadIdx.x < 64) {
    cnt[threadIdx.x] = 0;
    tgt[threadIdx.x] = threadIdx.x < a.K ? a.target[threadIdx.x] : 0u;
  }
  __syncthreads();
  const uint64_t words = (a.N + 63) / 64;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t ctg = lane < a.K ? tgt[lane] : 0u;
  uint64_t full = 0, nalive = 0, nstale = 0;
  uint32_t c_lane = 0;  // lane c: alive stale nodes whose component c equals the target
  // whole waves iterate together (the stale rows are read one row per wave step)
  for (uint64_t w0 = (uint64_t)blockIdx.x * kAeBlock + (threadIdx.x & ~63u); w0 < words;
       w0 += (uint64_t)gridDim.x * kAeBlock) {
    const uint64_t w = w0 + lane;
    uint64_t aw = 0, sw = 0;
    if (w < words) {
      const uint4 q = *reinterpret_cast<const uint4*>(a.abn + 2 * w);
      aw = ((uint64_t)q.y << 32) | q.x;
      sw = ((uint64_t)q.w << 32) | q.z;
    }
    nalive += (uint64_t)__popcll(aw);
    full += (uint64_t)__popcll(aw & ~sw);
    nstale += (uint64_t)__popcll(sw);
    const uint64_t as = aw & sw;
    for (uint64_t pend = __ballot(as != 0); pend; pend &= pend - 1) {
      const int src = __builtin_ctzll(pend);
      const uint64_t ws = (uint64_t)__shfl((long long)w, src, 64);
      for (uint64_t bits = (uint64_t)__shfl((long long)as, src, 64); bits; bits &= bits - 1) {
        const uint64_t n = ws * 64 + (uint64_t)__builtin_ctzll(bits);
        if (lane < a.K && a.V[n * a.K + lane] == ctg) ++c_lane;  // one row per wave: lane = component
      }
    }
  }
  if (lane < a.K && c_lane) atomicAdd(&cnt[lane], c_lane);
  const uint64_t f = wave_sum64(full);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = f;
  __syncthreads();
  uint64_t bfull = 0;
  for (int w = 0; w < kAeWaves; ++w) bfull += red[w];
  __syncthreads();
  block_add(full, red, &a.partial[0]);
  block_add(nalive, red, &a.partial[1]);
  block_add(nstale, red, &a.aux[0]);
  if (threadIdx.x < a.K && (bfull + cnt[threadIdx.x]))
    atomicAdd((unsigned long long*)&a.partial[4 + threadIdx.x], (unsigned long long)(bfull + cnt[threadIdx.x]));
}

uint32_t ae_grid(uint64_t units, uint32_t per_block, uint32_t cap) {
  const uint64_t b = (units + per_block - 1) / per_block;
  return (uint32_t)(b == 0 ? 1 : (b < cap ? b : cap));
}

// 64-node chunks, one per wave: enough waves to fill 256 CUs several times over
uint32_t chunk_grid(uint64_t N) { return ae_grid((N + 63) / 64, kAeWaves, 8192); }

}  // namespace

uint32_t ae_lanes(uint32_t K) {
  uint32_t L = 1;
  while (L < K) L <<= 1;
  return L;
}

hipError_t launch_ae_init(uint32_t* V, uint32_t* target, uint64_t N, uint32_t K, uint32_t k0, uint32_t k1,
                          hipStream_t st) {
  hipError_t e = hipMemsetAsync(target, 0, K * 4, st);
  if (e != hipSuccess) return e;
  // (the kernel flushes a thread's maxima whenever its quad changes: any grid stride is exact)
  ae_init_kernel<<<ae_grid(N * ((K + 3) / 4), kAeBlock, 65536), kAeBlock, 0, st>>>(V, N, K, k0, k1, target);
  return hipGetLastError();
}

hipError_t launch_ae_inject(uint32_t* V, uint32_t* target, uint64_t node, uint32_t K, uint32_t c, hipStream_t st) {
  ae_inject_kernel<<<1, 1, 0, st>>>(V, target, node, K, c);
  return hipGetLastError();
}

#define AE_LAUNCH_L(KER, L, grid, st, ...)                                  \
  switch (L) {                                                               \
    case 1: KER<1><<<(grid), kAeBlock, 0, (st)>>>(__VA_ARGS__); break;       \
    case 2: KER<2><<<(grid), kAeBlock, 0, (st)>>>(__VA_ARGS__); break;       \
    case 4: KER<4><<<(grid), kAeBlock, 0, (st)>>>(__VA_ARGS__); break;       \
    case 8: KER<8><<<(grid), kAeBlock, 0, (st)>>>(__VA_ARGS__); break;       \
    case 16: KER<16><<<(grid), kAeBlock, 0, (st)>>>(__VA_ARGS__); break;     \
    case 32: KER<32><<<(grid), kAeBlock, 0, (st)>>>(__VA_ARGS__); break;     \
    default: KER<64><<<(grid), kAeBlock, 0, (st)>>>(__VA_ARGS__); break;     \
  }

hipError_t launch_ae_fill_alive(uint64_t* ab, uint64_t N, hipStream_t st) {
  ae_fill_alive_kernel<<<ae_grid((N + 63) / 64, kAeBlock, 1024), kAeBlock, 0, st>>>(ab, N);
  return hipGetLastError();
}

hipError_t launch_ae_churn(const AeArgs& a, hipStream_t st) {
  ae_churn_kernel<<<chunk_grid(a.N), kAeBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_ae_round(const AeArgs& a, hipStream_t st) {
  AE_LAUNCH_L(ae_pull_kernel, a.L, chunk_grid(a.N), st, a);
  AE_LAUNCH_L(ae_push_kernel, a.L, chunk_grid(a.N), st, a);
  return hipGetLastError();
}

hipError_t launch_ae_stats(const AeArgs& a, const uint32_t* V, uint64_t* ab, bool write_stale, hipStream_t st) {
  AE_LAUNCH_L(ae_stats_kernel, a.L, chunk_grid(a.N), st, a, V, ab, write_stale);
  return hipGetLastError();
}

hipError_t launch_ae_sparse(const AeArgs& a, hipStream_t st) {
  ae_sparse_scan_kernel<<<a.nseg, kAeBlock, 0, st>>>(a);
  AE_LAUNCH_L(ae_sparse_gather_kernel, a.L, a.nseg * a.spb, st, a);
  AE_LAUNCH_L(ae_sparse_apply_kernel, a.L, a.nseg * a.spb, st, a);
  AE_LAUNCH_L(ae_sparse_fix_kernel, a.L, a.nseg * a.spb, st, a);
  return hipGetLastError();
}

AeBinGeom ae_bin_geom(uint64_t N, uint32_t k) {
  AeBinGeom g{};
  uint32_t rs = kAeBinRec;  // 2^brs senders * k records <= kAeBinRec, at least one block of senders
  g.rs = 14;
  while (g.rs > 10 && (rs >> (14 - g.rs)) * k > kAeBinRec) --g.rs;
  g.nreg = (uint32_t)((N + (1ull << g.rs) - 1) >> g.rs);
  uint32_t lg = 0;
  while ((1ull << lg) < N) ++lg;
  g.tl = lg > 8 ? lg - 8 : 0;  // ~256 tiles, one block per CU
  if (g.tl < 12) g.tl = 12;
  if (g.tl > kAeBinTileLog) g.tl = kAeBinTileLog;  // with rs <= 14, a record's fields fill one u32 (ae_rec)
  g.nt = (uint32_t)((N + (1ull << g.tl) - 1) >> g.tl);
  return g;
}

bool ae_bin_fits(const AeBinGeom& g) { return g.nt <= kAeBinTiles; }

hipError_t launch_ae_sparse_binned(const AeArgs& a, hipStream_t st) {
  const uint32_t eg = a.bnreg < 512 ? a.bnreg : 512;  // two blocks per CU
  if (a.k == 1 && (1u << a.brs) == kAeBinRec)
    ae_bin_emit_kernel<true, kAeBinTiles><<<eg, kAeBinThreads, 0, st>>>(a);
  else
    ae_bin_emit_kernel<false, kAeBinTiles><<<eg, kAeBinThreads, 0, st>>>(a);
  ae_bin_scan_kernel<<<a.bnt, kAeBinThreads, 0, st>>>(a);
  AE_LAUNCH_L(ae_sparse_gather_kernel, a.L, a.nseg * a.spb, st, a);
  AE_LAUNCH_L(ae_sparse_apply_kernel, a.L, a.nseg * a.spb, st, a);
  AE_LAUNCH_L(ae_sparse_fix_kernel, a.L, a.nseg * a.spb, st, a);
  return hipGetLastError();
}

AeBinGeom ae_dense_geom(uint64_t N, uint32_t k) {
  AeBinGeom g = ae_bin_geom(N, k);  // the same sender regions
  g.tl = kAeDTileLog;
  g.nt = (uint32_t)((N + kAeDTile - 1) >> kAeDTileLog);
  return g;
}

// tiles and regions in the LDS tables, senders in 26 bits of a sorted entry, k <= 3
// (a tile's records below 2^16, u16 positions), K <= 16 (the per-wave scratch)
bool ae_dense_fits(const AeBinGeom& g, uint64_t N, uint32_t k, uint32_t K) {
  return g.nt <= kAeDTiles && g.nreg <= kAeDMaxReg && N <= (1ull << 26) && k <= 3 && K <= 16;
}

hipError_t launch_ae_dense_binned(const AeArgs& a, hipStream_t st) {
  const uint32_t eg = a.bnreg < 256 ? a.bnreg : 256;  // one block per CU (LDS)
  if (a.k == 1 && (1u << a.brs) == kAeBinRec)
    ae_bin_emit_kernel<true, kAeDTiles><<<eg, kAeBinThreads, 0, st>>>(a);
  else
    ae_bin_emit_kernel<false, kAeDTiles><<<eg, kAeBinThreads, 0, st>>>(a);
#define AE_DENSE_L(KJ)                                                                 \
  switch (a.L) {                                                                       \
    case 1: ae_dense_apply_kernel<1, KJ><<<a.bnt, kAeDThreads, 0, st>>>(a); break;     \
    case 2: ae_dense_apply_kernel<2, KJ><<<a.bnt, kAeDThreads, 0, st>>>(a); break;     \
    case 4: ae_dense_apply_kernel<4, KJ><<<a.bnt, kAeDThreads, 0, st>>>(a); break;     \
    case 8: ae_dense_apply_kernel<8, KJ><<<a.bnt, kAeDThreads, 0, st>>>(a); break;     \
    default: ae_dense_apply_kernel<16, KJ><<<a.bnt, kAeDThreads, 0, st>>>(a); break;   \
  }
  if (a.K == 16) {  // 16-B row pieces
    if (a.k == 1) ae_dense_apply_q_kernel<1><<<a.bnt, kAeQThreads, 0, st>>>(a);
    else if (a.k == 2) ae_dense_apply_q_kernel<2><<<a.bnt, kAeQThreads, 0, st>>>(a);
    else ae_dense_apply_q_kernel<3><<<a.bnt, kAeQThreads, 0, st>>>(a);
  } else if (a.k == 1) {
    AE_DENSE_L(1)
  } else if (a.k == 2) {
    AE_DENSE_L(2)
  } else {
    AE_DENSE_L(3)
  }
#undef AE_DENSE_L
  return hipGetLastError();
}


hipError_t launch_ae_sparse_stats(const AeArgs& a, hipStream_t st) {
  // few blocks: each adds its totals with three same-address atomics
  ae_sparse_stats_kernel<<<ae_grid((a.N + 63) / 64, kAeBlock, 256), kAeBlock, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace gossip
