// Counter-based dropout RNG shared by forward and backward kernels: the keep
// mask of element idx in stream s is a pure function of (seed, s, idx), so the
// backward regenerates it instead of storing it.  splitmix64 finaliser; the
// same function is restated in numpy by the tests (tests/torch_ref.py).
#pragma once
#include <cstdint>

enum SrfRngStream : unsigned {
  kStreamConv0a = 0,
  kStreamConv0b = 1,
  kStreamConv1a = 2,
  kStreamConv1b = 3,
  kStreamEncaps1 = 4,
  kStreamEncaps2 = 5,
  kStreamInput = 6,
  kStreamMid0 = 7,   // + routing layer index
};

__device__ __forceinline__ uint64_t srf_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in [0, 1) with 24 random bits
__device__ __forceinline__ float srf_uniform(uint64_t seed, unsigned stream, uint64_t idx) {
  const uint64_t z = srf_mix64(seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(stream + 1))) + idx * 0xD1B54A32D192ED03ull;
  return (float)(srf_mix64(z) >> 40) * (1.0f / 16777216.0f);
}

// Keras/TF inverted dropout keeps an element with probability 1 - p.
__device__ __forceinline__ bool srf_keep(uint64_t seed, unsigned stream, uint64_t idx, float p) {
  return srf_uniform(seed, stream, idx) >= p;
}
