// Shared helpers for the SRF HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace srf {
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
// device step counter set by srf_set_seed_source for this process (NULL: none)
const unsigned long long* seed_source();
// device word set by srf_set_fault_flag for this process (NULL: none)
unsigned* fault_flag();
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
}  // namespace srf

#define SRF_OK 0
#define SRF_EINVAL (-1)
#define SRF_EHIP (-2)
#define SRF_EUNSUPPORTED (-3)
#define SRF_EWORKSPACE (-4)

#define SRF_REQUIRE(cond, ...)                 \
  do {                                         \
    if (!(cond)) {                             \
      srf::set_error(__VA_ARGS__);             \
      return SRF_EINVAL;                       \
    }                                          \
  } while (0)

#define SRF_HIP_TRY(call)                                                      \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess) {                                                    \
      srf::set_error("%s failed: %s", #call, hipGetErrorString(e_));           \
      return SRF_EHIP;                                                         \
    }                                                                          \
  } while (0)

#define SRF_LAUNCH_CHECK(name)                                                 \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess) {                                                    \
      srf::set_error("launch of %s failed: %s", name, hipGetErrorString(e_));  \
      return SRF_EHIP;                                                         \
    }                                                                          \
  } while (0)

// Exact unsigned division by a runtime-constant divisor d >= 1 (Granlund-Montgomery):
// q = (t + ((n - t) >> 1)) >> (l - 1), t = umulhi(n, m).  Built on the host.
struct FastDiv {
  unsigned m, d;
  int l;
};
inline FastDiv make_fastdiv(unsigned d) {
  FastDiv f;
  f.d = d;
  f.l = 0;
  while ((1ull << f.l) < d) ++f.l;
  f.m = d > 1 ? (unsigned)((((1ull << 32) * ((1ull << f.l) - d)) / d) + 1) : 0u;
  if (f.l == 0) f.l = 1;
  return f;
}
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) {
  const unsigned t = __umulhi(n, f.m);
  const unsigned q = (t + ((n - t) >> 1)) >> (f.l - 1);
  return f.d == 1 ? n : q;
}

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

// v_mfma_f32_16x16x4_f32: lane l holds A[row=l&15][k=l>>4], B[k=l>>4][col=l&15];
// C/D lane l holds col = l&15, rows 4*(l>>4) + reg.
__device__ __forceinline__ f4 mfma16x16x4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Cross-row exchanges on the VALU (gfx950 v_permlane16/32_swap, no LDS round trip).
// Both lanes of an exchanged pair receive the two values in the same order, so
// symmetric combinations (sum, max) are bit-identical across the pair.
__device__ __forceinline__ void xpair16(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void xpair32(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
// v + v of lane ^ 16 / lane ^ 32
__device__ __forceinline__ float xor16_sum(float v) {
  float a, b;
  xpair16(v, a, b);
  return a + b;
}
__device__ __forceinline__ float xor32_sum(float v) {
  float a, b;
  xpair32(v, a, b);
  return a + b;
}

// Split-fp16 operands (route_fwd32.hip, cnnfe.hip): an operand scaled by 2^e with
// max|a 2^e| < 2^14 is split as a1 = f16(a'), a2 = f16(a' - a1); the MFMA products
// a1 b1 + a1 b2 + a2 b1 are exact in fp32 and miss only a2 b2 <= 2^-22 |ab|.
// 2^e as a float (|e| <= 126)
__device__ __forceinline__ float srf_exp2i(int e) { return __int_as_float((127 + e) << 23); }
// exponent that scales an operand of max magnitude m below 2^14, clamped to [-60, 60]
__device__ __forceinline__ int srf_split_exp(float m) {
  if (!(m > 0.f) || !(m < __builtin_inff())) return 0;
  int e;
  (void)frexpf(m, &e);
  return max(-60, min(60, 14 - e));
}
__device__ __forceinline__ void srf_split2h(float a, _Float16& a1, _Float16& a2) {
  a1 = (_Float16)a;
  a2 = (_Float16)(a - (float)a1);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
