// Streaming SDR recurrence for layers whose frame exceeds a workgroup's registers,
// gfx950: BASELINE C5 (in_n = 16*41 = 656 input capsules, J = 16 | 32 output
// capsules of D = 64, five iterations; u_t = 2.7 | 5.4 MB per frame).
//
// Same recurrence as route_sdr_seq*.hip (sequence_router_naive.py:162-170 with
// body_context :231-245 / pad_body_context :212-229, and its autodiff), one
// 512-thread workgroup per utterance walking its frames in order (forward) or in
// reverse (backward), but u_t is streamed from HBM once per routing iteration
// instead of held in registers:
//   lane map: an input capsule's u_ij (J*D floats) is one wave-wide slice, lane l
//   holds the KD = J*D/64 consecutive floats [l*KD, l*KD + KD), i.e. output capsule
//   j = l / RQ, dims q*KD .. q*KD + KD - 1 (RQ = D/KD lanes per capsule);
//   wave w takes input capsules i = w, w + 8, ... (NMp per pass, a multiple of PD,
//   the tail predicated off), PD capsules in flight per wave in a register ring that
//   runs ahead across iterations and frames;
//   per capsule: logit = KD FMAs + a butterfly over the RQ lanes, softmax over j =
//   butterflies over the J capsule groups (DPP / permlane, VALU only), then
//   s_j += c_ij u_ij in the lane's KD accumulators;
//   per iteration: the 8 wave partials through LDS, thread e owns s_e, the squash is
//   a butterfly over the D owner lanes, Vc (v_{t-1} + sum_{k<r} v^k, b^r = <u, Vc^r>
//   by linearity of b += <u, v>) goes back through LDS.  Two barriers per iteration.
// The forward stores each frame's couplings c^r [R][in_n][J] and pre-squash s^r
// [R][J*D] (sdr_stream_cs_floats per frame); the backward reads them and runs only
// the adjoint (same algebra as route_sdr_seq_bwd.hip):
//   gs^r = squash'(s^r)^T a^r,  q_ij = <u_ij, gs^r_j>,  sigma_i = sum_j c_ij q_ij,
//   gL_ij = c_ij (q_ij - sigma_i) (kept in a per-utterance L2 scratch),
//   gVc^r = sum_i gL_ij u_ij  (one streamed pass of u_t per iteration),
//   gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j  (a pass without u: the lane's
//   gs^r / Vc^r slices in registers, the 2R scalars of (i, j) per capsule).
// HBM per frame: forward R reads of u_t; backward R reads of u_t + one write of gu_t.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "route_sdr_seq.h"
#include "route_sdr_seq_dev.h"
#include "srf_group.h"

namespace {

using srf_seq::group_max;
using srf_seq::group_sum;

// Register-ring depths in capsules per wave (forward fp32 | bf16 u, backward), by
// 16- or 32-capsule-row shapes.  Measured (C5 step): forward fp32 (6, 3) 990 ms, (6, 2)
// 959, (6, 1) 955, (3, 2) 951, (2, 3) 980, (8, 3) 1065, (6, 4) 1131 -- deeper rings only
// add register pressure once the eight layers share HBM; with u in bf16 (packed slots,
// half the registers) a deeper forward ring pays (C5 fp8: (3, 2) 598 ms, (6, 3) 588);
// the backward's bf16 ring at the fp32 depths ((6, 3) 599 ms and (8, 4) 602 against
// (4, 2) 596).
constexpr int kPdF16 = 3, kPdF32 = 2;       // forward, fp32 u
constexpr int kPdF16Bf = 6, kPdF32Bf = 3;   // forward, bf16 u
constexpr int kPdB16 = 4, kPdB32 = 2;       // backward (fp32 and bf16 u)
constexpr int kNT = 512;          // threads per workgroup (two waves per SIMD, 256 VGPRs each)
constexpr int kNW = kNT / 64;
constexpr int kRM = 5;            // iteration bound (check_sgeom)
constexpr float kEps = 1e-7f;     // naive:248

template <int D_, int KD_>
struct SC {
  static constexpr int D = D_;
  static constexpr int KD = KD_;              // floats of a capsule per lane
  static constexpr int JD = 64 * KD;          // floats of one input capsule's u
  static constexpr int J = JD / D;
  static constexpr int RQ = D / KD;           // lanes per output capsule
  static constexpr int NE = JD / kNT;         // elements per thread in the element phases
  // capsules in flight per wave in the forward / backward register ring
  static constexpr int PDF = KD <= 8 ? 8 : KD <= 16 ? kPdF16 : kPdF32;
  static constexpr int PDF_BF = KD <= 8 ? 8 : KD <= 16 ? kPdF16Bf : kPdF32Bf;
  template <class TU>
  static constexpr int pdf() { return std::is_same<TU, float>::value ? PDF : PDF_BF; }
  static constexpr int PDB = KD <= 16 ? kPdB16 : kPdB32;
  static constexpr int PDB_BF = KD <= 16 ? kPdB16 : kPdB32;
  template <class TU>
  static constexpr int pdb() { return std::is_same<TU, float>::value ? PDB : PDB_BF; }
  static constexpr int HD = 8;                 // gu outputs per lane per sub-pass (registers: 2R*HD)
  static_assert(D % KD == 0 && NE >= 1 && KD % 4 == 0 && KD % HD == 0, "unsupported stream shape");
};

// floats per frame of the coupling record: c^r [R][in_n][J], s^r [R][JD], padded to 256 B
__host__ __device__ inline size_t cs_rec(int in_n, int J, int D, int R) {
  return ((size_t)R * ((size_t)in_n * J + (size_t)J * D) + 63) / 64 * 64;
}

// position in a wave's capsule stream: frame t, pass p of the frame, capsule slot m
// (branch-free: selects, so that the compiler's vmcnt waits on the ring stay exact)
struct Cur {
  int t, p, m;
  __device__ __forceinline__ void adv(int NMp, int NP, int dt) {
    const bool wm = m + 1 == NMp;
    m = wm ? 0 : m + 1;
    const bool wp = wm && p + 1 == NP;
    p = wp ? 0 : p + (wm ? 1 : 0);
    t += wp ? dt : 0;
  }
};

// buffer resource over n floats (n = 0: every access dropped); an offset of
// kDrop bytes is out of range, so a store predicated off is a dropped store, not a branch
__device__ __forceinline__ __amdgpu_buffer_rsrc_t float_rsrc(const float* p, size_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, p ? (int)(n * 4) : 0, 0x00020000);
}
constexpr uint32_t kDrop = 0x80000000u;
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t rs, float v, uint32_t off) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, off, 0, 0);
}

// KD consecutive bf16 values (u stored in bf16 by the fp8 pose), widened exactly to fp32
template <int KD>
__device__ __forceinline__ void load_slice(const unsigned short* __restrict__ p, float (&x)[KD]) {
  static_assert(KD % 8 == 0, "bf16 slices load 8 values per 16 bytes");
#pragma unroll
  for (int c = 0; c < KD; c += 8) {
    const auto q = *reinterpret_cast<const unsigned __attribute__((ext_vector_type(4)))*>(p + c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[c + 2 * k] = __uint_as_float(q[k] << 16);
      x[c + 2 * k + 1] = __uint_as_float(q[k] & 0xffff0000u);
    }
  }
}

template <int KD>
__device__ __forceinline__ void load_slice(const float* __restrict__ p, float (&x)[KD]) {
#pragma unroll
  for (int c = 0; c < KD; c += 4) {
    const f4 q = *reinterpret_cast<const f4*>(p + c);
    x[c] = q.x;
    x[c + 1] = q.y;
    x[c + 2] = q.z;
    x[c + 3] = q.w;
  }
}

// A ring slot: the raw words of a u_ij slice as loaded (bf16 pairs stay packed, so the
// load is not waited for at issue) and their fp32 values at the use
template <class TU, int KD>
struct Slot;
template <int KD>
struct Slot<float, KD> {
  float w[KD];
  __device__ __forceinline__ void load(const float* __restrict__ p) { load_slice<KD>(p, w); }
  __device__ __forceinline__ void widen(float (&x)[KD]) const {
#pragma unroll
    for (int d = 0; d < KD; ++d) x[d] = w[d];
  }
};
template <int KD>
struct Slot<unsigned short, KD> {
  static_assert(KD % 8 == 0, "bf16 slices load 8 values per 16 bytes");
  unsigned w[KD / 2];
  __device__ __forceinline__ void load(const unsigned short* __restrict__ p) {
#pragma unroll
    for (int c = 0; c < KD / 2; c += 4) {
      const auto q = *reinterpret_cast<const unsigned __attribute__((ext_vector_type(4)))*>(p + 2 * c);
#pragma unroll
      for (int k = 0; k < 4; ++k) w[c + k] = q[k];
    }
  }
  __device__ __forceinline__ void widen(float (&x)[KD]) const {
#pragma unroll
    for (int k = 0; k < KD / 2; ++k) {
      x[2 * k] = __uint_as_float(w[k] << 16);
      x[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  }
};

template <int KD>
__device__ __forceinline__ float dot_slice(const float (&x)[KD], const float (&w)[KD]) {
  float p0 = 0.f, p1 = 0.f;
#pragma unroll
  for (int d = 0; d < KD; d += 2) {
    p0 += x[d] * w[d];
    p1 += x[d + 1] * w[d + 1];
  }
  return p0 + p1;
}

// Workgroup groups (srf_group.h): G > 1 workgroups per utterance take capsules
// (member * kNW + wave) + kNW * G * m and add their partial sums inside the launch.
using srf_grp::Grp;
using srf_grp::kMaxGroup;
// floats of the stream backward's gL scratch [B][R][in_n][J] at the item workspace's start
__host__ __device__ inline size_t gl_floats(int B, int in_n, int J, int R) { return (size_t)B * R * in_n * J; }

// Workgroup barrier that orders LDS only (no vmcnt(0)), so the register ring's loads stay
// in flight across it; for barriers with no global data exchanged between waves of the
// kernel (the grouped launches exchange through srf_group.h and keep __syncthreads)
template <bool LDS_ONLY>
__device__ __forceinline__ void wg_bar() {
  if constexpr (LDS_ONLY) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    __syncthreads();
  }
}

// the accumulators computed here: no sinking of their updates past this point (IR or
// scheduler), and no global load hoisted above it
template <int K>
__device__ __forceinline__ void pin(float (&a)[K]) {
#pragma unroll
  for (int d = 0; d < K; ++d) asm volatile("" : "+v"(a[d]));
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float squash_fac(float n2) {
  return n2 * __builtin_amdgcn_rcpf(1.f + n2) * __builtin_amdgcn_rsqf(n2 + kEps);
}

// gs = squash'(s)^T a over the D owner lanes of a capsule (sdr_bwd_kernel's algebra)
template <int D>
__device__ __forceinline__ float dsquash(float s, float a) {
  const float n2 = group_sum<1, D>(s * s);
  const float sa = group_sum<1, D>(s * a);
  const float rs = 1.f / sqrtf(n2 + kEps);
  const float ip = 1.f / (1.f + n2);
  const float gfac = n2 * ip * rs;
  const float dg2 = 2.f * rs * ip * (ip - 0.5f * n2 / (n2 + kEps)) * sa;
  return gfac * a + dg2 * s;
}

// ------------------------------------------------------------------ forward
// LDS: wl [JD] (Vc of the iteration), part [kNW][JD].
template <int D, int KD, class TU, bool GRP>
__global__ __launch_bounds__(kNT) void sdr_stream_fwd_kernel(srf::SeqItems items, int T, int in_n, int iters,
                                                             int mask_first, int NMp, Grp X) {
  using C = SC<D, KD>;
  const srf::SeqItem& I = items.it[blockIdx.y];   // the frame range of this launch item
  const TU* __restrict__ u = reinterpret_cast<const TU*>(I.u);
  float* __restrict__ v_out = I.v;
  float* __restrict__ cs = I.cs;
  const srf::SeqRange rg = I.rg;
  constexpr int JD = C::JD, J = C::J, PD = C::template pdf<TU>(), NE = C::NE;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* wl = lds;
  float* part = lds + JD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: capsule indices in SGPRs
  if (rg.t0 >= rg.t1) return;
  const int b = GRP ? blockIdx.x / X.G : blockIdx.x;
  const int gm = GRP ? blockIdx.x - b * X.G : 0;   // member of the utterance's group
  const int gw = gm * kNW + wv, cstep = GRP ? kNW * X.G : kNW;   // capsule i = gw + cstep * m
  const bool lead = gm == 0;                                    // stores s^r and v
  const int j = lane / C::RQ;
  const bool q0 = (lane % C::RQ) == 0;
  const bool jm = !(mask_first && j == 0);
  const size_t ff = (size_t)in_n * JD;
  const TU* ub = u + (size_t)b * rg.tu_n * ff + lane * KD;
  float* vo = v_out + (size_t)b * T * JD;
  const size_t csr = cs_rec(in_n, J, D, iters);

  float vc[NE];   // Vc of the thread's elements e = tid + n * kNT
#pragma unroll
  for (int n = 0; n < NE; ++n) {
    const int e = tid + n * kNT;
    vc[n] = rg.t0 > 0 ? vo[(size_t)(rg.t0 - 1) * JD + e] : 0.f;
    wl[e] = vc[n];
  }
  Slot<TU, KD> xr[PD];
  Cur lc{rg.t0, 0, 0};
  auto issue = [&](Slot<TU, KD>& x) {
    const int tc = min(lc.t, rg.t1 - 1);
    const int i = min(gw + cstep * lc.m, in_n - 1);
    x.load(ub + (size_t)(tc - rg.tu0) * ff + (size_t)i * JD);
    lc.adv(NMp, iters, 1);
  };
#pragma unroll
  for (int p = 0; p < PD; ++p) issue(xr[p]);
  wg_bar<!GRP>();

  for (int t = rg.t0; t < rg.t1; ++t) {
    const __amdgpu_buffer_rsrc_t csf = float_rsrc(cs ? cs + ((size_t)b * T + t) * csr : nullptr, csr);
    for (int r = 0; r < iters; ++r) {
      float w[KD], acc[KD];
      load_slice<KD>(wl + lane * KD, w);
#pragma unroll
      for (int d = 0; d < KD; ++d) acc[d] = 0.f;
      int m0 = 0;
      do {   // NMp >= PD (nm_padded): no zero-trip path, whose merge would wait on the ring
#pragma unroll
        for (int p = 0; p < PD; ++p) {
          const int i = gw + cstep * (m0 + p);
          const bool iv = i < in_n;
          float x[KD];
          xr[p].widen(x);
          const float lg = group_sum<1, C::RQ>(dot_slice<KD>(x, w));
          const float lj = jm ? lg : -INFINITY;
          const float mx = group_max<C::RQ, 64>(lj);
          const float ex = __expf(lj - mx);
          // tail slots masked arithmetically: a select here becomes a uniform branch around the
          // softmax, which splits the block and sinks the accumulation past the slot's reload
          const float c = ex * __builtin_amdgcn_rcpf(group_sum<C::RQ, 64>(ex)) * (iv ? 1.f : 0.f);
#pragma unroll
          for (int d = 0; d < KD; ++d) acc[d] += c * x[d];
          bstore(csf, c, q0 && iv ? (uint32_t)((r * in_n + i) * J + j) * 4 : kDrop);
          // the slot's last use before its reload, so the load lands in the same registers
          // (the accumulation sunk past it would need a second set and copies that wait)
          pin(acc);
          issue(xr[p]);
          __builtin_amdgcn_sched_barrier(0);   // keep the ring order: no hoisting across capsules
        }
        m0 += PD;
      } while (m0 < NMp);
#pragma unroll
      for (int d = 0; d < KD; d += 4)
        *reinterpret_cast<f4*>(part + wv * JD + lane * KD + d) = f4{acc[d], acc[d + 1], acc[d + 2], acc[d + 3]};
      wg_bar<!GRP>();
      if constexpr (GRP) srf_grp::allreduce<kNW, kNT>(part, JD, I.ws, X, b, gm, (unsigned)((t - rg.t0) * iters + r), tid);
#pragma unroll
      for (int n = 0; n < NE; ++n) {
        const int e = tid + n * kNT;
        float s = 0.f;
        if constexpr (GRP) {
          s = part[e];
        } else {
#pragma unroll
          for (int w2 = 0; w2 < kNW; ++w2) s += part[w2 * JD + e];
        }
        const float v = s * squash_fac(group_sum<1, D>(s * s));
        bstore(csf, s, lead ? (uint32_t)(iters * in_n * J + r * JD + e) * 4 : kDrop);
        if (r == iters - 1) {
          if (lead) vo[(size_t)t * JD + e] = v;
          vc[n] = v;   // v_t: Vc^0 of frame t + 1
        } else {
          vc[n] += v;
        }
        wl[e] = vc[n];
      }
      wg_bar<!GRP>();
    }
  }
  srf_grp::depart<GRP>(I.ws, X, b, tid);
}

// ------------------------------------------------------------------ backward
// LDS: part [kNW][JD], gsl [kRM][JD] (gs^r), vcl [kRM][JD] (Vc^r).
// gls: per-utterance scratch gL^r [R][in_n][J].
template <int D, int KD, class TU, bool GRP>
__global__ __launch_bounds__(kNT) void sdr_stream_bwd_kernel(srf::SeqItems items, int T, int in_n, int iters,
                                                             int NMp, Grp X) {
  using C = SC<D, KD>;
  const srf::SeqItem& I = items.it[blockIdx.y];   // the frame range of this launch item
  const TU* __restrict__ u = reinterpret_cast<const TU*>(I.u);
  const float* __restrict__ v_saved = I.v;
  const float* __restrict__ g_v = I.g_v;
  float* __restrict__ gu = I.gu;
  const float* __restrict__ cs = I.cs;
  float* __restrict__ gls = I.ws;
  const srf::SeqRange rg = I.rg;
  constexpr int JD = C::JD, J = C::J, PD = C::template pdb<TU>(), NE = C::NE, HD = C::HD;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* part = lds;
  float* gsl = part + kNW * JD;
  float* vcl = gsl + kRM * JD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: capsule indices in SGPRs
  if (rg.t0 >= rg.t1) return;
  const int b = GRP ? blockIdx.x / X.G : blockIdx.x;
  const int gm = GRP ? blockIdx.x - b * X.G : 0;   // member of the utterance's group
  const int gw = gm * kNW + wv, cstep = GRP ? kNW * X.G : kNW;   // capsule i = gw + cstep * m
  const bool lead = gm == 0;                                    // writes the carry out
  const int R = iters;
  const int j = lane / C::RQ;
  const bool q0 = (lane % C::RQ) == 0;
  const size_t ff = (size_t)in_n * JD;
  const size_t PJ = (size_t)in_n * J;
  const TU* ub = u + (size_t)b * rg.tu_n * ff + lane * KD;
  float* gub = gu + (size_t)b * rg.tg_n * ff + lane * KD;
  const size_t csr = cs_rec(in_n, J, D, iters);
  const float* csb = cs + (size_t)b * T * csr;
  float* gl = gls + (size_t)b * R * PJ;
  const __amdgpu_buffer_rsrc_t glr = float_rsrc(gl, (size_t)R * PJ);
  float* carry_io = rg.carry ? rg.carry + (size_t)b * JD : nullptr;

  float carry[NE];
#pragma unroll
  for (int n = 0; n < NE; ++n) carry[n] = carry_io ? carry_io[tid + n * kNT] : 0.f;

  // ring of the adjoint passes: u_t slice and c^r_ij of capsule i, pass p <-> r = R-1-p
  Slot<TU, KD> xr[PD];
  float cr[PD];
  Cur lc{rg.t1 - 1, 0, 0};
  auto issue = [&](Slot<TU, KD>& x, float& c) {
    const int tc = max(lc.t, rg.t0);
    const int i = min(gw + cstep * lc.m, in_n - 1);
    x.load(ub + (size_t)(tc - rg.tu0) * ff + (size_t)i * JD);
    c = csb[(size_t)tc * csr + (size_t)(R - 1 - lc.p) * PJ + (size_t)i * J + j];
    lc.adv(NMp, R, -1);
  };

#pragma unroll
  for (int p = 0; p < PD; ++p) issue(xr[p], cr[p]);
  for (int t = rg.t1 - 1; t >= rg.t0; --t) {
    const float* csf = csb + (size_t)t * csr;
    // ---- element phase: Vc^r from s^r, the top adjoint
    float gv[NE];
#pragma unroll
    for (int n = 0; n < NE; ++n) {
      const int e = tid + n * kNT;
      const float a = g_v[((size_t)b * T + t) * JD + e] + carry[n];
      const float vp = v_saved[((size_t)b * T + max(t - 1, 0)) * JD + e];   // unconditional (see sn)
      float vcv = t > 0 ? vp : 0.f;
      for (int r = 0; r < R; ++r) {
        const float sv = csf[(size_t)R * PJ + (size_t)r * JD + e];
        vcl[r * JD + e] = vcv;
        vcv += sv * squash_fac(group_sum<1, D>(sv * sv));
        if (r == R - 1) gsl[r * JD + e] = dsquash<D>(sv, a);
      }
      carry[n] = 0.f;
      gv[n] = 0.f;
    }
    wg_bar<!GRP>();
    // ---- adjoint passes r = R-1 .. 0 over u_t
    for (int p = 0; p < R; ++p) {
      const int r = R - 1 - p;
      float g[KD], gacc[KD], sn[NE];
      load_slice<KD>(gsl + r * JD + lane * KD, g);
#pragma unroll
      for (int n = 0; n < NE; ++n)   // s^{r-1}, for gs^{r-1} at the end of the pass (unused at r = 0:
        // loaded unconditionally, a load under a branch is waited for at the merge)
        sn[n] = csf[(size_t)R * PJ + (size_t)max(r - 1, 0) * JD + tid + n * kNT];
#pragma unroll
      for (int d = 0; d < KD; ++d) gacc[d] = 0.f;
      int m0 = 0;
      do {   // NMp >= PD, as in the forward
#pragma unroll
        for (int pp = 0; pp < PD; ++pp) {
          const int i = gw + cstep * (m0 + pp);
          const bool iv = i < in_n;
          float x[KD];
          xr[pp].widen(x);
          const float qd = group_sum<1, C::RQ>(dot_slice<KD>(x, g));
          const float c = iv ? cr[pp] : 0.f;
          const float sig = group_sum<C::RQ, 64>(c * qd);
          const float gL = c * (qd - sig);
#pragma unroll
          for (int d = 0; d < KD; ++d) gacc[d] += gL * x[d];
          bstore(glr, gL, q0 && iv ? (uint32_t)((r * in_n + i) * J + j) * 4 : kDrop);
          pin(gacc);   // reload in place (see the forward)
          issue(xr[pp], cr[pp]);   // runs on into frame t - 1 (the gu pass leaves the ring alone)
          __builtin_amdgcn_sched_barrier(0);
        }
        m0 += PD;
      } while (m0 < NMp);
#pragma unroll
      for (int d = 0; d < KD; d += 4)
        *reinterpret_cast<f4*>(part + wv * JD + lane * KD + d) = f4{gacc[d], gacc[d + 1], gacc[d + 2], gacc[d + 3]};
      wg_bar<!GRP>();
      if constexpr (GRP) srf_grp::allreduce<kNW, kNT>(part, JD, I.ws, X, b, gm, (unsigned)((rg.t1 - 1 - t) * R + p), tid);
#pragma unroll
      for (int n = 0; n < NE; ++n) {
        const int e = tid + n * kNT;
        float gvc = 0.f;
        if constexpr (GRP) {
          gvc = part[e];
        } else {
#pragma unroll
          for (int w2 = 0; w2 < kNW; ++w2) gvc += part[w2 * JD + e];
        }
        carry[n] += gvc;      // dL/dv_{t-1} = sum_r gVc^r
        gv[n] += gvc;         // dL/dv^{r-1} = sum_{r' >= r} gVc^{r'}
        if (r > 0) gsl[(r - 1) * JD + e] = dsquash<D>(sn[n], gv[n]);
      }
      // the gu pass after the last one reads the gL scratch back: there the stores drain
      if (p + 1 < R) wg_bar<!GRP>();
      else __syncthreads();
    }
    // ---- gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j, HD outputs per lane per sub-pass
    float* gut = gub + (size_t)(t - rg.tg0) * ff;
#pragma unroll
    for (int h = 0; h < KD; h += HD) {
      float gs[kRM][HD], vv[kRM][HD];
#pragma unroll
      for (int r = 0; r < kRM; ++r) {
        if (r < R) {
          load_slice<HD>(gsl + r * JD + lane * KD + h, gs[r]);
          load_slice<HD>(vcl + r * JD + lane * KD + h, vv[r]);
        } else {
#pragma unroll
          for (int d = 0; d < HD; ++d) gs[r][d] = vv[r][d] = 0.f;
        }
      }
      // scalars of capsule i for the lane's j, one capsule ahead
      float sc[2][2 * kRM];
      auto fetch = [&](int m, float(&s)[2 * kRM]) {
        const int i = min(gw + cstep * m, in_n - 1);
#pragma unroll
        for (int r = 0; r < kRM; ++r) {
          const int rr = min(r, R - 1);
          s[r] = csf[(size_t)rr * PJ + (size_t)i * J + j];
          s[kRM + r] = gl[(size_t)rr * PJ + (size_t)i * J + j];
        }
      };
      fetch(0, sc[0]);
      for (int m0 = 0; m0 < NMp; m0 += 2) {
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int m = m0 + pp;
          fetch(m + 1, sc[pp ^ 1]);
          const int i = gw + cstep * m;
          float o[HD];
#pragma unroll
          for (int d = 0; d < HD; ++d) o[d] = 0.f;
#pragma unroll
          for (int r = 0; r < kRM; ++r) {
            if (r < R) {
#pragma unroll
              for (int d = 0; d < HD; ++d) o[d] += sc[pp][r] * gs[r][d] + sc[pp][kRM + r] * vv[r][d];
            }
          }
          if (i < in_n) {
#pragma unroll
            for (int d = 0; d < HD; d += 4)
              *reinterpret_cast<f4*>(gut + (size_t)i * JD + h + d) = f4{o[d], o[d + 1], o[d + 2], o[d + 3]};
          }
        }
      }
    }
    __syncthreads();   // gsl / vcl / the gL scratch are rewritten by frame t - 1
  }
  if (carry_io && lead)
#pragma unroll
    for (int n = 0; n < NE; ++n) carry_io[tid + n * kNT] = carry[n];
  srf_grp::depart<GRP>(I.ws, X, b, tid);
}

// ------------------------------------------------------------------ host
// capsule slots per wave and pass: a multiple of the ring depth PD (the ring's slots
// are static registers) and of 2 (the gu pass walks slots in pairs)
int nm_padded(int in_n, int pd, int G) {
  const int step = pd % 2 ? 2 * pd : pd;
  const int nm = (in_n + kNW * G - 1) / (kNW * G);
  return (nm + step - 1) / step * step;
}

size_t fwd_lds(int JD) { return (size_t)(1 + kNW) * JD * sizeof(float); }
size_t bwd_lds(int JD) { return (size_t)(kNW + 2 * kRM) * JD * sizeof(float); }

template <int D, int KD>
int launch_fwd(const srf::SeqItems& items, int B, int T, int in_n, int iters, int mask_first, hipStream_t st) {
  using C = SC<D, KD>;
  const size_t lds = fwd_lds(C::JD);
  Grp X;
  if (int rc = srf_grp::setup(items, B, gl_floats(B, in_n, C::J, iters), X, st)) return rc;
  const bool bf = items.it[0].u_bf16;
  auto k = X.G > 1 ? (bf ? sdr_stream_fwd_kernel<D, KD, unsigned short, true> : sdr_stream_fwd_kernel<D, KD, float, true>)
                   : (bf ? sdr_stream_fwd_kernel<D, KD, unsigned short, false> : sdr_stream_fwd_kernel<D, KD, float, false>);
  if (lds > 64 * 1024)
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k, dim3(B * X.G, items.n), dim3(kNT), lds, st, items, T, in_n, iters, mask_first,
                     nm_padded(in_n, bf ? C::PDF_BF : C::PDF, X.G), X);
  SRF_LAUNCH_CHECK("sdr_stream_fwd");
  return SRF_OK;
}

template <int D, int KD>
int launch_bwd(const srf::SeqItems& items, int B, int T, int in_n, int iters, hipStream_t st) {
  using C = SC<D, KD>;
  const size_t lds = bwd_lds(C::JD);
  Grp X;
  if (int rc = srf_grp::setup(items, B, gl_floats(B, in_n, C::J, iters), X, st)) return rc;
  const bool bf = items.it[0].u_bf16;
  auto k = X.G > 1 ? (bf ? sdr_stream_bwd_kernel<D, KD, unsigned short, true> : sdr_stream_bwd_kernel<D, KD, float, true>)
                   : (bf ? sdr_stream_bwd_kernel<D, KD, unsigned short, false> : sdr_stream_bwd_kernel<D, KD, float, false>);
  if (lds > 64 * 1024)
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k, dim3(B * X.G, items.n), dim3(kNT), lds, st, items, T, in_n, iters,
                     nm_padded(in_n, bf ? C::PDB_BF : C::PDB, X.G), X);
  SRF_LAUNCH_CHECK("sdr_stream_bwd");
  return SRF_OK;
}

// (dout, KD = J*dout/64) instances
#define SRF_STREAM_CASES(X) X(64, 8) X(64, 16) X(64, 32) X(32, 8) X(32, 16)

}  // namespace

namespace srf {

bool sdr_stream_supported(int in_n, int J, int dout, int iters) {
  if (iters < 1 || iters > kRM || in_n < kNW) return false;
  const int JD = J * dout;
  if (JD % 64) return false;
  const int KD = JD / 64;
#define SRF_STREAM_OK(DD, KK) \
  if (dout == DD && KD == KK) return true;
  SRF_STREAM_CASES(SRF_STREAM_OK)
#undef SRF_STREAM_OK
  return false;
}

size_t sdr_stream_cs_floats(int in_n, int J, int dout, int iters) {
  return sdr_stream_supported(in_n, J, dout, iters) ? cs_rec(in_n, J, dout, iters) : 0;
}

size_t sdr_stream_pre_floats(int B, int in_n, int J, int iters) { return gl_floats(B, in_n, J, iters); }

size_t sdr_stream_workspace_floats(int B, int in_n, int J, int dout, int iters) {
  return sdr_stream_supported(in_n, J, dout, iters) ? srf_grp::floats(gl_floats(B, in_n, J, iters), B, J * dout) : 0;
}

// the items of one launch share the u element type
static int same_u_type(const SeqItems& items) {
  for (int k = 1; k < items.n; ++k)
    SRF_REQUIRE(items.it[k].u_bf16 == items.it[0].u_bf16, "sdr_stream: launch items mix fp32 and bf16 u");
  return SRF_OK;
}

int sdr_stream_fwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                   hipStream_t st) {
  if (int rc = same_u_type(items)) return rc;
  const int KD = J * dout / 64;
#define SRF_STREAM_F(DD, KK) \
  if (dout == DD && KD == KK) return launch_fwd<DD, KK>(items, B, T, in_n, iters, mask_first, st);
  SRF_STREAM_CASES(SRF_STREAM_F)
#undef SRF_STREAM_F
  srf::set_error("sdr_stream: unsupported shape J=%d dout=%d", J, dout);
  return SRF_EUNSUPPORTED;
}

int sdr_stream_bwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, hipStream_t st) {
  if (int rc = same_u_type(items)) return rc;
  for (int k = 0; k < items.n; ++k)
    if (!items.it[k].cs || !items.it[k].ws) {
      srf::set_error("sdr_stream backward needs the forward's stored couplings and its scratch workspace");
      return SRF_EINVAL;
    }
  const int KD = J * dout / 64;
#define SRF_STREAM_B(DD, KK) \
  if (dout == DD && KD == KK) return launch_bwd<DD, KK>(items, B, T, in_n, iters, st);
  SRF_STREAM_CASES(SRF_STREAM_B)
#undef SRF_STREAM_B
  srf::set_error("sdr_stream: unsupported shape J=%d dout=%d", J, dout);
  return SRF_EUNSUPPORTED;
}

}  // namespace srf
