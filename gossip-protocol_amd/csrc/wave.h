// wave.h — wave64 helpers shared by the round kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gossip {

__device__ __forceinline__ uint64_t full_mask1(uint32_t R) { return R >= 64 ? ~0ull : ((1ull << R) - 1ull); }

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// 64x64 bit-matrix transpose across a wave64: on entry lane i holds row i, on
// exit lane j holds column j (bit i = bit j of lane i's input word).  Popcount
// of the result = how many of the wave's 64 words have bit `lane` set.
// (A DPP / permlane-swap form with no ds_bpermute measured slower in the apply
// epilogue: DESIGN.md §3.7.)
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

// Block-wide exclusive scan of one u32 per thread (blockDim.x == NT, multiple of 64).
// scratch: NT/64 + 1 u32 in LDS.  Returns the exclusive prefix; *total gets the sum.
template <int NT>
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* scratch, uint32_t* total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) scratch[wave] = inc;
  __syncthreads();
  if (tid == 0) {
    uint32_t a = 0;
    for (int w = 0; w < NT / 64; ++w) {
      const uint32_t x = scratch[w];
      scratch[w] = a;
      a += x;
    }
    scratch[NT / 64] = a;
  }
  __syncthreads();
  const uint32_t r = scratch[wave] + inc - v;
  *total = scratch[NT / 64];
  __syncthreads();  // scratch may be reused right away
  return r;
}

}  // namespace gossip
