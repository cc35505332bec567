// Device side of the register-resident SDR recurrence, shared by
// route_sdr_seq.hip (forward) and route_sdr_seq_bwd.hip (backward).  The design
// is described at the top of route_sdr_seq.hip.
#pragma once
#include <cmath>

#include "srf_common.h"

namespace srf_seq {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr float kSquashEps = 1e-7f;   // naive:248

// Values of one output capsule per lane for dout D and padded capsule count JP
// (the JP capsules of one input capsule fill at most one wave), and row slots.
constexpr int seq_kd(int D, int JP) { return D * JP / 64 > 4 ? D * JP / 64 : 4; }
constexpr int seq_slots(int D, int JP) { return kWaves * (64 / (JP * (D / seq_kd(D, JP)))); }

inline int pow2_at_least(int x) {
  int p = 4;
  while (p < x) p <<= 1;
  return p;
}

// (dout, JP) instances: dout * JP <= 1024 keeps a lane's slice of a capsule <= 16 values
#define SRF_SEQ_CASES(X)                                                                              \
  X(8, 4) X(8, 8) X(8, 16) X(8, 32) X(8, 64) X(16, 4) X(16, 8) X(16, 16) X(16, 32) X(16, 64) X(32, 4) \
  X(32, 8) X(32, 16) X(32, 32)

// ------------------------------------------------------------------ butterflies
// Value held by lane ^ O, O in {1, 2, 4, 8}: DPP quad_perm for 1 and 2, ds_swizzle
// (bit mode, xor mask) for 4 and 8 -- no LDS memory, no address registers.
template <int O>
__device__ __forceinline__ float partner(float v) {
  const int x = __float_as_int(v);
  if constexpr (O == 1) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
  else if constexpr (O == 2) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
  else return __int_as_float(__builtin_amdgcn_ds_swizzle(x, (O << 10) | 0x1F));
}

// v (+) value of lane ^ O; IEEE + and max are commutative, so both lanes of the
// pair hold the same bits.
template <int O>
__device__ __forceinline__ float pair_sum(float v) {
  if constexpr (O == 16) return xor16_sum(v);
  else if constexpr (O == 32) return xor32_sum(v);
  else return v + partner<O>(v);
}

template <int O>
__device__ __forceinline__ float pair_max(float v) {
  if constexpr (O == 16 || O == 32) {
    float a, b;
    if constexpr (O == 16) xpair16(v, a, b);
    else xpair32(v, a, b);
    return fmaxf(a, b);
  } else {
    return fmaxf(v, partner<O>(v));
  }
}

// value of lane (l - N) mod 16 within the lane's 16-lane row (DPP row_ror, VALU only)
template <int N>
__device__ __forceinline__ float row_ror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 | N, 0xF, 0xF, false));
}

// all-reduce over the lanes whose index differs only in bits [LO, HI).  Bits 2
// and 3 together go through two DPP row rotations (VALU) instead of two
// ds_swizzle round trips; max stays bit-identical over the group, a sum may
// differ in its last bit between lanes (different association order).
template <int LO, int HI>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (LO >= HI) {
    return v;
  } else if constexpr (LO == 4 && HI >= 16) {
    v += row_ror<4>(v);
    v += row_ror<8>(v);
    return group_sum<16, HI>(v);
  } else if constexpr (LO == 8) {
    return group_sum<16, HI>(v + row_ror<8>(v));   // (l - 8) mod 16 == l ^ 8
  } else {
    return group_sum<2 * LO, HI>(pair_sum<LO>(v));
  }
}
template <int LO, int HI>
__device__ __forceinline__ float group_max(float v) {
  if constexpr (LO >= HI) {
    return v;
  } else if constexpr (LO == 4 && HI >= 16) {
    v = fmaxf(v, row_ror<4>(v));
    v = fmaxf(v, row_ror<8>(v));
    return group_max<16, HI>(v);
  } else if constexpr (LO == 8) {
    return group_max<16, HI>(fmaxf(v, row_ror<8>(v)));
  } else {
    return group_max<2 * LO, HI>(pair_max<LO>(v));
  }
}

// ------------------------------------------------------------------ lane map
template <int D_, int JP_, int NIM_>
struct Cfg {
  static constexpr int D = D_;
  static constexpr int JP = JP_;
  static constexpr int NIM = NIM_;             // input capsules per lane (bound)
  static constexpr int KD = seq_kd(D, JP);     // values of a capsule per lane
  static constexpr int Q = D / KD;             // lanes per capsule
  static constexpr int ROWL = JP * Q;          // lanes per input capsule ("row")
  static constexpr int SUB = 64 / ROWL;        // rows per wave
  static constexpr int G = kWaves * SUB;       // row slots of the workgroup
  static_assert(KD <= 16 && D % KD == 0 && ROWL <= 64 && NIM * KD <= 80, "unsupported SDR shape");
};

struct Lane {
  int g;        // row slot: input capsules g, g + G, ...
  int j;        // output capsule (>= J: padding)
  int eoff;     // offset of the lane's KD values in a [J*D] vector
  int NI;       // input capsules of the row slot
  bool jv, jm;  // j < J; j < J and not the masked class 0 (naive:174-178, 216-220)
  bool q0;      // first of the Q lanes of its capsule
};

// gm / ng: this workgroup's member index and the group size (srf_group.h): member gm
// takes the block of ceil(in_n / ng) input capsules starting at gm * ceil(in_n / ng),
// its row slots stepping through the block by G (a compile-time stride)
template <class C>
__device__ __forceinline__ Lane lane_map(int in_n, int J, int mask_first, int gm = 0, int ng = 1) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sub = lane / C::ROWL, rl = lane % C::ROWL;
  const int blk = (in_n + ng - 1) / ng, base = gm * blk;
  const int nloc = max(0, min(in_n, base + blk) - base);
  const int gl = wv * C::SUB + sub;
  Lane L;
  L.j = rl / C::Q;
  L.g = base + gl;
  L.eoff = L.j * C::D + (rl % C::Q) * C::KD;
  L.NI = gl < nloc ? (nloc - gl + C::G - 1) / C::G : 0;
  L.jv = L.j < J;
  L.jm = L.jv && !(mask_first && L.j == 0);
  L.q0 = (rl % C::Q) == 0;
  return L;
}

// per-(input capsule, output capsule) scalars of the lane's rows <-> LDS [in_n][JP]
template <class C>
__device__ __forceinline__ void store_ij(const float (&v)[C::NIM], const Lane& L, float* __restrict__ dst) {
#pragma unroll
  for (int k = 0; k < C::NIM; ++k)
    if (k < L.NI && L.q0) dst[(L.g + k * C::G) * C::JP + L.j] = v[k];
}
template <class C>
__device__ __forceinline__ void load_ij(const float* __restrict__ src, const Lane& L, float (&v)[C::NIM]) {
#pragma unroll
  for (int k = 0; k < C::NIM; ++k) v[k] = k < L.NI ? src[(L.g + k * C::G) * C::JP + L.j] : 0.f;
}

// the lane's first KR rows of u_t -> registers, zeros for padded capsules and rows past
// the lane's: one buffer resource over the frame, and an invalid row reads an offset past
// its range, which the buffer unit returns as zeros (no branch per row)
template <class C, int KR>
__device__ __forceinline__ void load_rows(const float* __restrict__ ut, int JD, const Lane& L,
                                          float (&ur)[KR][C::KD]) {
  constexpr uint32_t kOff = 0x7FFFFF00u;   // past any frame (in_n * JD * 4 < 2^31)
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ut), 0, (int)kOff, 0x00020000);
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const bool ok = L.jv && k < L.NI;
    const uint32_t o = ok ? (uint32_t)(((L.g + k * C::G) * JD + L.eoff) * 4) : kOff;
#pragma unroll
    for (int c = 0; c < C::KD; c += 4) {
      const f4 x = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + c * 4, 0, 0));
      ur[k][c] = x.x;
      ur[k][c + 1] = x.y;
      ur[k][c + 2] = x.z;
      ur[k][c + 3] = x.w;
    }
  }
}

// the lane's rows of u_t -> registers
template <class C>
__device__ __forceinline__ void load_frame(const float* __restrict__ ut, int JD, const Lane& L,
                                           float (&ur)[C::NIM][C::KD]) {
  load_rows<C, C::NIM>(ut, JD, L, ur);
}

// sp summed over the wave's rows; the first row's lanes write it to part[wave][eoff ..]
template <class C>
__device__ __forceinline__ void partial_out(float (&sp)[C::KD], const Lane& L, int JD, float* __restrict__ part) {
#pragma unroll
  for (int d = 0; d < C::KD; ++d) sp[d] = group_sum<C::ROWL, 64>(sp[d]);
  if (L.jv && (threadIdx.x & 63) < C::ROWL) {
    float* dst = part + (threadIdx.x >> 6) * JD + L.eoff;
#pragma unroll
    for (int c = 0; c < C::KD; c += 4) *reinterpret_cast<f4*>(dst + c) = f4{sp[c], sp[c + 1], sp[c + 2], sp[c + 3]};
  }
}

// KD values at base + off: the [JP * D] LDS vectors (the padded capsules' tail zeroed
// once per launch by zero_tail), so every lane reads, no branch or select
template <int KD>
__device__ __forceinline__ void lds_slice(const float* __restrict__ base, int off, float (&w)[KD]) {
#pragma unroll
  for (int c = 0; c < KD; c += 4) {
    const f4 x = *reinterpret_cast<const f4*>(base + off + c);
    w[c] = x.x;
    w[c + 1] = x.y;
    w[c + 2] = x.z;
    w[c + 3] = x.w;
  }
}

// the padded capsules' entries [JD, JDp) of n LDS vectors of stride JDp -> 0
__device__ __forceinline__ void zero_tail(float* __restrict__ v, int n, int JD, int JDp) {
  const int w = JDp - JD;
  for (int k = threadIdx.x; k < n * w; k += kThreads) v[(k / w) * JDp + JD + k % w] = 0.f;
}

// row k of the lane's rows of u_t (a global re-read), zeros where !L.jv: one buffer
// resource over the frame, the padded capsules' lanes read past its range
template <class C>
__device__ __forceinline__ void load_row(const float* __restrict__ ut, int JD, const Lane& L, int k,
                                         float (&w)[C::KD]) {
  constexpr uint32_t kOff = 0x7FFFFF00u;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ut), 0, (int)kOff, 0x00020000);
  const uint32_t o = L.jv ? (uint32_t)(((L.g + k * C::G) * JD + L.eoff) * 4) : kOff;
#pragma unroll
  for (int c = 0; c < C::KD; c += 4) {
    const f4 x = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + c * 4, 0, 0));
    w[c] = x.x;
    w[c + 1] = x.y;
    w[c + 2] = x.z;
    w[c + 3] = x.w;
  }
}

// logits b += <u_ij, w_j> (naive:221-223 / :203-205) and c = softmax_j(b) for the
// lane's input capsules; rows past NI get c = 0
template <class C>
__device__ __forceinline__ void logits_softmax(const float (&ur)[C::NIM][C::KD], const float (&w)[C::KD],
                                               const Lane& L, float (&b)[C::NIM], float (&c)[C::NIM]) {
#pragma unroll
  for (int k = 0; k < C::NIM; ++k) {
    c[k] = 0.f;
    if (k < L.NI) {
      float p0 = 0.f, p1 = 0.f;
#pragma unroll
      for (int d = 0; d < C::KD; d += 2) {
        p0 += ur[k][d] * w[d];
        p1 += ur[k][d + 1] * w[d + 1];
      }
      b[k] += group_sum<1, C::Q>(p0 + p1);
      const float x = L.jm ? b[k] : -INFINITY;
      const float m = group_max<C::Q, C::ROWL>(x);
      const float e = __expf(x - m);
      c[k] = e * __builtin_amdgcn_rcpf(group_sum<C::Q, C::ROWL>(e));
    }
  }
}

// sum over the lane's input capsules of a[k] * u[k][:], summed over the wave's
// rows; the first row's lanes write it to part[wave][eoff ..]
template <class C>
__device__ __forceinline__ void row_partial(const float (&a)[C::NIM], const float (&ur)[C::NIM][C::KD],
                                            const Lane& L, int JD, float* __restrict__ part) {
  float sp[C::KD];
#pragma unroll
  for (int d = 0; d < C::KD; ++d) sp[d] = 0.f;
#pragma unroll
  for (int k = 0; k < C::NIM; ++k)
#pragma unroll
    for (int d = 0; d < C::KD; ++d) sp[d] += a[k] * ur[k][d];
#pragma unroll
  for (int d = 0; d < C::KD; ++d) sp[d] = group_sum<C::ROWL, 64>(sp[d]);
  if (L.jv && (threadIdx.x & 63) < C::ROWL) {
    float* dst = part + (threadIdx.x >> 6) * JD + L.eoff;
#pragma unroll
    for (int c = 0; c < C::KD; c += 4) *reinterpret_cast<f4*>(dst + c) = f4{sp[c], sp[c + 1], sp[c + 2], sp[c + 3]};
  }
}

// element e of the workgroup sum of the 16 wave partials
__device__ __forceinline__ float sum_parts(const float* __restrict__ part, int JD, int e) {
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) s += part[w * JD + e];
  return s;
}

// ------------------------------------------------------------------ stamps
// Diagnostic builds only (-DSRF_SEQ_STAMP=1, scripts/seq_stamps.py): per-phase
// cycle sums of waves 0 and 15 of every workgroup, stored once at the end into a
// buffer of their own (never read by the kernel, never an output).  The shipped
// build compiles every mark to nothing.
#ifndef SRF_SEQ_STAMP
#define SRF_SEQ_STAMP 0
#endif
constexpr int kStampPh = 8;
#if SRF_SEQ_STAMP
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
struct Stamps {
  unsigned long long last, sum[kStampPh];
  __device__ void start() {
    for (int p = 0; p < kStampPh; ++p) sum[p] = 0;
    last = stamp_now();
  }
  __device__ void mark(int p) {
    const unsigned long long t = stamp_now();
    sum[p] += t - last;
    last = t;
  }
  __device__ void flush(unsigned long long* out) {
    const int wv = threadIdx.x >> 6;
    if (out == nullptr || (threadIdx.x & 63) != 0 || (wv != 0 && wv != kWaves - 1)) return;
    unsigned long long* o = out + ((size_t)blockIdx.x * 2 + (wv ? 1 : 0)) * kStampPh;
    for (int p = 0; p < kStampPh; ++p) o[p] = sum[p];
  }
};
#define SEQ_STAMP_DECL Stamps st_; st_.start();
#define SEQ_MARK(p) st_.mark(p)
#define SEQ_FLUSH(buf) st_.flush(buf)
#else
#define SEQ_STAMP_DECL
#define SEQ_MARK(p) ((void)0)
#define SEQ_FLUSH(buf) ((void)(buf))
#endif

// squash over the D consecutive owner lanes of a capsule (naive:247-252); the
// recurrence is VALU-issue bound, so 1-ulp v_rcp / v_rsq replace IEEE div / sqrt
template <int D>
__device__ __forceinline__ float squash_elem(float s) {
  const float n2 = group_sum<1, D>(s * s);
  return s * (n2 * __builtin_amdgcn_rcpf(1.f + n2) * __builtin_amdgcn_rsqf(n2 + kSquashEps));
}

}  // namespace srf_seq
