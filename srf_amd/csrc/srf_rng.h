// Counter-based dropout RNG shared by forward and backward kernels: the keep
// mask of element idx in stream s is a pure function of (seed, s, idx), so the
// backward regenerates it instead of storing it.  32-bit arithmetic only
// (lowbias32 mixer, two rounds keyed by the seed); the same function is restated
// in numpy by the tests (tests/torch_ref.py).
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

__host__ __device__ __forceinline__ uint32_t srf_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Per-call seed mixed with the device-resident step counter of srf_set_seed_source
// (NULL: the seed alone).  A captured training step advances the counter on the
// device, so every graph replay draws fresh dropout masks.
__device__ __forceinline__ uint64_t srf_step_seed(uint64_t seed, const unsigned long long* src) {
  return src ? seed + *src * 0x9E3779B97F4A7C15ull : seed;
}

__device__ __forceinline__ uint32_t srf_stream_key(uint64_t seed, unsigned stream) {
  return srf_mix32((uint32_t)seed ^ srf_mix32((uint32_t)(seed >> 32) ^ (stream * 0x9E3779B9u + 0x7F4A7C15u)));
}

// uniform in [0, 1) with 24 random bits
__device__ __forceinline__ float srf_uniform(uint64_t seed, unsigned stream, uint64_t idx) {
  const uint32_t k = srf_stream_key(seed, stream);
  const uint32_t h = srf_mix32(srf_mix32((uint32_t)idx + k) ^ k);
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// Keras/TF inverted dropout keeps an element with probability 1 - p.
__device__ __forceinline__ bool srf_keep(uint64_t seed, unsigned stream, uint64_t idx, float p) {
  return srf_uniform(seed, stream, idx) >= p;
}

// The maxout convolutions drop both branches (streams a and a + 1) at the same
// element: one hash keyed by stream a, whose high and low 16 bits are the two
// uniforms (16-bit resolution: the keep probability is off by < 2^-16).
__device__ __forceinline__ void srf_keep2(uint64_t seed, unsigned stream_a, uint64_t idx, float p, bool& keep_a,
                                          bool& keep_b) {
  const uint32_t k = srf_stream_key(seed, stream_a);
  const uint32_t h = srf_mix32(srf_mix32((uint32_t)idx + k) ^ k);
  keep_a = (float)(h >> 16) * (1.0f / 65536.0f) >= p;
  keep_b = (float)(h & 0xFFFFu) * (1.0f / 65536.0f) >= p;
}
