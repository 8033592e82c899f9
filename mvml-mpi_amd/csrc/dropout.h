// nn.Dropout's keep decision as a pure function of (seed, element index): a counter-based hash
// (splitmix64's finaliser) of (seed, i / 2), one 32-bit half per element — regenerable anywhere
// (the standalone mvml_dropout_fwd and the fused attention + conv epilogue draw the same mask for
// the same (seed, i)), no state, nothing stored.  Element i is kept iff dropout_u32 >= thr with
// thr = round(p 2^32) (dropout_threshold).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cmath>

#include <hip/hip_runtime.h>

namespace mvml {

__device__ __forceinline__ uint64_t dropout_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// the 64 bits serving elements 2 pair and 2 pair + 1 (low half, high half)
__device__ __forceinline__ uint64_t dropout_pair_bits(uint64_t seed, int64_t pair) {
  return dropout_mix64(seed + (uint64_t)(pair + 1) * 0x9E3779B97F4A7C15ull);
}

__device__ __forceinline__ uint32_t dropout_u32(uint64_t seed, int64_t i) {
  const uint64_t z = dropout_pair_bits(seed, i >> 1);
  return (i & 1) ? (uint32_t)(z >> 32) : (uint32_t)z;
}

inline uint32_t dropout_threshold(double p) {
  return (uint32_t)std::min<double>((double)std::llround(p * 4294967296.0), 4294967295.0);
}

inline float dropout_scale(double p) { return (float)(1.0 / (1.0 - p)); }

}  // namespace mvml
