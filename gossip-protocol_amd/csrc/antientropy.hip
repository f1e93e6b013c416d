// antientropy.hip — version-vector anti-entropy with churn (configs[4]).
//
// Each node holds K uint32 versions (AoS rows V[n*K + c], so a peer's whole
// vector is one contiguous K*4-byte row).  Round t: churn by Philox tag 1,
// then every alive node n exchanges with its Philox peers p_j(n,t) that are
// alive too: both take the elementwise max of the two S_t rows.  The
// reference's only failure handling is retry-until-acked (main.go:77-87);
// churn here is the build-defined fault model of SURVEY.md §5.
//
// Lanes: L = next power of two >= K lanes per node (a wave holds 64/L nodes);
// lane c of a node owns component c, the group's first lane draws the Philox
// numbers and broadcasts them.  Writes go to V' (seeded with a copy of V) by
// atomicMax, so concurrent pushes and pulls into one row commute.
#include "antientropy.h"
#include "philox.h"

namespace gossip {

namespace {

constexpr int kAeBlock = 256;

__device__ __forceinline__ bool churned(uint8_t alive, uint32_t n, uint32_t t, uint32_t k0, uint32_t k1,
                                        uint32_t fail, uint32_t rec) {
  const uint32_t x = philox4x32_10(u32x4{n, t, 1u, 0u}, k0, k1).x;
  return alive ? !(x < fail) : (x < rec);
}

__global__ __launch_bounds__(kAeBlock) void ae_init_kernel(uint32_t* V, uint64_t N, uint32_t K, uint32_t k0,
                                                           uint32_t k1) {
  const uint32_t c4 = (K + 3) / 4;
  for (uint64_t i = (uint64_t)blockIdx.x * kAeBlock + threadIdx.x; i < N * c4; i += (uint64_t)gridDim.x * kAeBlock) {
    const uint32_t n = (uint32_t)(i / c4), q = (uint32_t)(i % c4);
    const u32x4 x = philox4x32_10(u32x4{n, q, 3u, 0u}, k0, k1);
    for (uint32_t r = 0; r < 4 && 4 * q + r < K; ++r) V[(uint64_t)n * K + 4 * q + r] = lane_of(x, r) & 0xFFFFu;
  }
}

__global__ __launch_bounds__(kAeBlock) void ae_target_kernel(const uint32_t* V, uint64_t N, uint32_t K,
                                                             uint32_t* target) {
  __shared__ uint32_t m[64];
  if (threadIdx.x < 64) m[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kAeBlock + threadIdx.x; i < N * K; i += (uint64_t)gridDim.x * kAeBlock)
    atomicMax(&m[i % K], V[i]);
  __syncthreads();
  if (threadIdx.x < K && m[threadIdx.x]) atomicMax(&target[threadIdx.x], m[threadIdx.x]);
}

__global__ void ae_inject_kernel(uint32_t* V, uint32_t* target, uint64_t node, uint32_t K, uint32_t c) {
  const uint32_t v = ++V[node * K + c];
  atomicMax(&target[c], v);
}

__global__ __launch_bounds__(kAeBlock) void ae_round_kernel(AeArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t lead = lane & ~(a.L - 1);  // first lane of this node's group
  const uint32_t c = lane & (a.L - 1);
  const uint64_t nodes_per_block = kAeBlock / a.L;
  uint64_t msgs = 0;
  for (uint64_t base = (uint64_t)blockIdx.x * nodes_per_block; base < a.N; base += (uint64_t)gridDim.x * nodes_per_block) {
    const uint64_t n64 = base + threadIdx.x / a.L;
    const bool valid = n64 < a.N;
    const uint32_t n = (uint32_t)(valid ? n64 : a.N - 1);
    // churn of n (leader draws, group shares; every lane takes part in the shuffle)
    int aln = 0;
    if (c == 0) aln = churned(a.alive[n], n, a.t, a.key0, a.key1, a.fail, a.rec);
    aln = __shfl(aln, (int)lead, 64);
    if (valid && c == 0) a.alive_n[n] = (uint8_t)aln;
    const uint64_t vn_idx = (uint64_t)n * a.K + c;
    const bool mine = valid && aln && c < a.K;
    const uint32_t vn = mine ? a.V[vn_idx] : 0u;
    u32x4 x{0, 0, 0, 0};
    for (uint32_t j = 0; j < a.k; ++j) {
      uint32_t p = 0;
      int alp = 0;
      if (c == 0) {
        if ((j & 3u) == 0) x = philox4x32_10(u32x4{n, a.t, 0u, j >> 2}, a.key0, a.key1);
        p = peer_from_word(lane_of(x, j & 3u), a.N - 1, n);
        alp = churned(a.alive[p], p, a.t, a.key0, a.key1, a.fail, a.rec);
      }
      p = (uint32_t)__shfl((int)p, (int)lead, 64);
      alp = __shfl(alp, (int)lead, 64);
      if (!(mine && alp)) continue;
      if (c == 0) ++msgs;
      const uint64_t vp_idx = (uint64_t)p * a.K + c;
      const uint32_t vp = a.V[vp_idx];
      if (vp > vn) atomicMax(&a.Vn[vn_idx], vp);  // pull
      if (vn > vp) atomicMax(&a.Vn[vp_idx], vn);  // push
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) msgs += __shfl_xor(msgs, off, 64);
  if (lane == 0 && msgs) atomicAdd((unsigned long long*)&a.partial[2], (unsigned long long)msgs);
}

// stats of V_{t+1}: alive count, alive nodes equal to the global max vector,
// per-component counts (lane c of every group), optional hash
__global__ __launch_bounds__(kAeBlock) void ae_stats_kernel(AeArgs a, const uint32_t* __restrict__ V,
                                                            const uint8_t* __restrict__ alive) {
  __shared__ uint32_t cnt[64];
  __shared__ uint64_t red[3][kAeBlock / 64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t c = lane & (a.L - 1);
  const uint32_t groups = 64 / a.L;
  const uint64_t kmask = a.K >= 64 ? ~0ull : ((1ull << a.K) - 1ull);
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t tgt = c < a.K ? a.target[c] : 0u;
  uint64_t hash = 0, full = 0, nalive = 0;
  uint32_t c_lane = 0;
  const uint64_t nodes_per_block = kAeBlock / a.L;
  for (uint64_t base = (uint64_t)blockIdx.x * nodes_per_block; base < a.N; base += (uint64_t)gridDim.x * nodes_per_block) {
    const uint64_t n = base + threadIdx.x / a.L;
    const bool valid = n < a.N && c < a.K;
    const uint32_t v = valid ? V[n * a.K + c] : 0u;
    const bool al = n < a.N && alive[n];
    if ((a.flags & 1u) && v) hash += mix64((uint64_t)v + ((uint64_t)c * a.N + n) * kGold64);
    const uint64_t eq = __ballot(valid && v == tgt);
    const uint64_t ok = __ballot(valid && al && v == tgt);
    const uint64_t lead_alive = __ballot(c == 0 && al);
    nalive += (uint64_t)__popcll(lead_alive);
    for (uint32_t g = 0; g < groups; ++g) {
      const bool allk = ((eq >> (g * a.L)) & kmask) == kmask;
      full += (allk && ((lead_alive >> (g * a.L)) & 1ull)) ? 1u : 0u;
    }
    // lane c (< K) of group 0 counts component c over all groups of the wave
    if (lane < a.K) {
      uint32_t s = 0;
      for (uint32_t g = 0; g < groups; ++g) s += (uint32_t)((ok >> (g * a.L + lane)) & 1ull);
      c_lane += s;
    }
  }
  if (lane < a.K && c_lane) atomicAdd(&cnt[lane], c_lane);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) hash += __shfl_xor(hash, off, 64);
  if (lane == 0) {
    red[0][wave] = hash;
    red[1][wave] = full;
    red[2][wave] = nalive;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t h = 0, f = 0, al = 0;
    for (int w = 0; w < kAeBlock / 64; ++w) {
      h += red[0][w];
      f += red[1][w];
      al += red[2][w];
    }
    if (f) atomicAdd((unsigned long long*)&a.partial[0], (unsigned long long)f);
    if (al) atomicAdd((unsigned long long*)&a.partial[1], (unsigned long long)al);
    if (h) atomicAdd((unsigned long long*)&a.partial[3], (unsigned long long)h);
  }
  if (threadIdx.x < a.K && cnt[threadIdx.x])
    atomicAdd((unsigned long long*)&a.partial[4 + threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

uint32_t ae_grid(uint64_t units, uint32_t per_block, uint32_t cap) {
  const uint64_t b = (units + per_block - 1) / per_block;
  return (uint32_t)(b == 0 ? 1 : (b < cap ? b : cap));
}

}  // namespace

uint32_t ae_lanes(uint32_t K) {
  uint32_t L = 1;
  while (L < K) L <<= 1;
  return L;
}

hipError_t launch_ae_init(uint32_t* V, uint32_t* target, uint64_t N, uint32_t K, uint32_t k0, uint32_t k1,
                          hipStream_t st) {
  ae_init_kernel<<<ae_grid(N * ((K + 3) / 4), kAeBlock, 65536), kAeBlock, 0, st>>>(V, N, K, k0, k1);
  hipError_t e = hipMemsetAsync(target, 0, K * 4, st);
  if (e != hipSuccess) return e;
  ae_target_kernel<<<ae_grid(N * K, kAeBlock, 4096), kAeBlock, 0, st>>>(V, N, K, target);
  return hipGetLastError();
}

hipError_t launch_ae_inject(uint32_t* V, uint32_t* target, uint64_t node, uint32_t K, uint32_t c, hipStream_t st) {
  ae_inject_kernel<<<1, 1, 0, st>>>(V, target, node, K, c);
  return hipGetLastError();
}

hipError_t launch_ae_round(const AeArgs& a, hipStream_t st) {
  const uint32_t npb = kAeBlock / a.L;
  ae_round_kernel<<<ae_grid(a.N, npb, 1u << 20), kAeBlock, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_ae_stats(const AeArgs& a, const uint32_t* V, const uint8_t* alive, hipStream_t st) {
  const uint32_t npb = kAeBlock / a.L;
  ae_stats_kernel<<<ae_grid(a.N, npb, 8192), kAeBlock, 0, st>>>(a, V, alive);
  return hipGetLastError();
}

}  // namespace gossip
