// Windowed pose transform + sequential dynamic routing (SDR) for one capsule
// layer, gfx950.  Replaces sequence_router_naive.py:162-170 (the tf.while_loop
// over frames) with body_context :231-245 / pad_body_context :212-229, and its
// autodiff.
//
// Frame t of an utterance is routed after frame t-1: its logits start from
// <u_t, v_{t-1}> (v_{-1} = 0), then R iterations of
//   b += <u, w> (+ mask), c = softmax_j(b), s = sum_i c u, v = squash(s)
// with w = v_{t-1} in iteration 0 and the previous iteration's v after.  With
// Vc^r = v_{t-1} + sum_{k<r} v^k the logits are b^r = <u, Vc^r> + (r+1) m, so
// the backward is the DR backward of routing.hip with Vc^0 = v_{t-1} plus the
// carried gradient dL/dv_{t-1} = sum_r gVc^r.
//
// Kernels:
//   sdr_pose_kernel   u[f][i][row] = W_i x_i(f) + b_i for every frame (MFMA), the
//                     frame-parallel part, kept in HBM for the sequential pass;
//   sdr_seq_*         (route_sdr_seq*.hip) the recurrence itself: one 1024-thread
//                     workgroup per utterance holds the frame's u in registers and
//                     walks the frames in order (forward) or in reverse,
//                     recomputing each frame's iterations, writing gu (backward);
//   sdr_fwd_kernel /  the first, 256-thread LDS version of the recurrence, kept for
//   sdr_bwd_kernel    shapes outside the register budget (and SRF_SDR_SEQ=0);
//   sdr_gx_kernel     gx = W^T gu (MFMA) scattered into g_emb via the window adjoint;
//   sdr_gw_kernel     gW = sum_f gu x^T (MFMA, K = frames); gbias = column sums of gu.
// Layouts (HBM, fp32): emb [F][N][din]; W [in_n][J*Dout][din]; bias [in_n][J*Dout];
// u, gu [F][in_n][J*Dout]; v [F][J*Dout].
#include <algorithm>
#include <cmath>

#include "srf_common.h"
#include "srf_reduce.h"
#include "route_sdr_seq.h"
#include "srf_group.h"
#include "../../include/srf.h"

namespace {

constexpr float kSquashEps = 1e-7f;   // naive:248
constexpr float kMaskLogit = -1e9f;   // naive:216-217
// One workgroup per utterance for the LDS / global-state recurrence kernels: 16 waves
// keep more of the u stream in flight than 4 (C5 train step 26.8 -> 15.4 s)
constexpr int kGsThreads = 1024;

struct SGeom {
  int B, T, N, din, lpad, rpad, J, dout, iters, mask_first;
  int F() const { return B * T; }
  int in_n() const { return N * (lpad + rpad + 1); }
  int JD() const { return J * dout; }
  int NT() const { return (J * dout + 15) / 16; }
};

// ------------------------------------------------------------------ frame ranges
// Frames t in [t0, t0 + nt) of every utterance, enumerated q = b * nt + (t - t0) in
// [0, B * nt); a u / gu buffer holds frames [v0, v0 + vn) of each utterance
// ([B][vn][in_n][JD]).  The whole layer is {T, 0, T, 0, T}.
struct FrameMap {
  int T, t0, nt, v0, vn;
  __device__ __forceinline__ void frame(int q, int& b, int& t) const {
    b = q / nt;
    t = t0 + (q - b * nt);
  }
  __device__ __forceinline__ size_t view(int b, int t) const { return (size_t)b * vn + (t - v0); }
};

// One launch of the frame-parallel contractions runs up to srf::kMaxItems frame ranges
// of same-shaped layers (grid.z = item).  pose: x = emb, w = W, b = bias, o = u;
// gx: x = gu, w = W^T, o = g_emb; gW: x = gu, b = emb, o = gW, o2 = gbias, acc.
struct GemmItem {
  const float* x;
  const float* w;
  const float* b;
  float* o;
  float* o2;
  int acc, Q;
  FrameMap fm;
};
struct GemmItems {
  GemmItem it[srf::kMaxItems];
  int n;
};

// KS consecutive floats (float4 loads when KS is a multiple of 4), zeros when !ok
template <int KS>
__device__ __forceinline__ void load_ks(const float* __restrict__ p, bool ok, float (&v)[KS]) {
  if constexpr (KS % 4 == 0) {
#pragma unroll
    for (int k = 0; k < KS; k += 4) {
      f4 q = {0.f, 0.f, 0.f, 0.f};
      if (ok) q = *reinterpret_cast<const f4*>(p + k);
      v[k] = q.x;
      v[k + 1] = q.y;
      v[k + 2] = q.z;
      v[k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < KS; ++k) v[k] = ok ? p[k] : 0.f;
  }
}

// ------------------------------------------------------------------ pose
// Workgroup = 4 waves over FT frame tiles (16 frames each) and one capsule i; wave w
// takes row tiles w, w+4, ..., each W fragment (loaded as float4s) feeding the FT
// frame tiles.  Operands as in the DR pass (k-permuted MFMA: lane group g holds K
// elements g*KS .. g*KS + KS-1 of both operands).
template <int DIN, int FT>
__global__ __launch_bounds__(256) void sdr_pose_kernel(GemmItems items, int N, int lpad, int in_n, int JD) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ emb = G.x;
  const float* __restrict__ W = G.w;
  const float* __restrict__ bias = G.b;
  float* __restrict__ u = G.o;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  if (blockIdx.x * FT * 16 >= Q) return;
  constexpr int KS = DIN / 4;
  const int T = fm.T;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fl = lane & 15, g = lane >> 4;
  const int i = blockIdx.y;
  const int w = i / N, n = i - w * N;
  float x[FT][KS];
  int qq[FT], bb[FT], tt[FT];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft) {
    qq[ft] = (blockIdx.x * FT + ft) * 16 + fl;
    fm.frame(min(qq[ft], Q - 1), bb[ft], tt[ft]);
    const int ts = tt[ft] + w - lpad;
    const bool ok = qq[ft] < Q && ts >= 0 && ts < T;
    const float* xp = emb + ((size_t)(bb[ft] * T + min(max(ts, 0), T - 1)) * N + n) * DIN + g * KS;
    load_ks<KS>(xp, ok, x[ft]);
  }
  const int NT = (JD + 15) / 16;
  for (int tile = wv; tile < NT; tile += 4) {
    const int arow = min(tile * 16 + fl, JD - 1);
    const float* wp = W + ((size_t)i * JD + arow) * DIN + g * KS;
    float a[KS];
    load_ks<KS>(wp, true, a);
    const int crow = min(tile * 16 + 4 * g, JD - 4);
    const f4 b4 = *reinterpret_cast<const f4*>(bias + (size_t)i * JD + crow);
    f4 acc[FT];
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) acc[ft] = b4;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int ft = 0; ft < FT; ++ft) acc[ft] = mfma16x16x4(a[k], x[ft][k], acc[ft]);
    const int row = tile * 16 + 4 * g;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
      if (qq[ft] < Q && row < JD)
        *reinterpret_cast<f4*>(u + (fm.view(bb[ft], tt[ft]) * in_n + i) * JD + row) = acc[ft];
  }
}

// ------------------------------------------------------------------ shared helpers
// Shared-memory views of the per-frame routing state.
struct SeqSmem {
  float* v;      // [JD]   agreement vector of the current iteration (carry at r = 0)
  float* bl;     // [P]    logits b_ij (P = in_n*J)
  float* c;      // [P]    couplings
  float* s;      // [JD]
  float* red;    // [2*in_n] softmax max / 1/sum per i
};

// b += <u, w> (+ mask); c = softmax_j(b); s = sum_i c u; v = squash(s).
// On return sm.v holds v^r and sm.s holds s^r.
template <int NT>
__device__ __forceinline__ void sdr_iteration(const float* __restrict__ ut, const SeqSmem& sm, int in_n, int J,
                                              int D, int mask_first, float* c_keep, float* s_keep) {
  const int P = in_n * J, JD = J * D;
  const int tid = threadIdx.x;
  for (int p = tid; p < P; p += NT) {
    const int i = p / J, j = p - i * J;
    const float* up = ut + (size_t)i * JD + j * D;
    const float* vp = sm.v + j * D;
    float d0 = 0.f, d1 = 0.f;
    for (int d = 0; d < D; d += 4) {
      const f4 a = *reinterpret_cast<const f4*>(up + d);
      d0 += a.x * vp[d] + a.y * vp[d + 1];
      d1 += a.z * vp[d + 2] + a.w * vp[d + 3];
    }
    sm.bl[p] += (d0 + d1) + ((mask_first && j == 0) ? kMaskLogit : 0.f);
  }
  __syncthreads();
  for (int i = tid; i < in_n; i += NT) {
    float m = -INFINITY;
    for (int j = 0; j < J; ++j) m = fmaxf(m, sm.bl[i * J + j]);
    float z = 0.f;
    for (int j = 0; j < J; ++j) z += __expf(sm.bl[i * J + j] - m);
    const float iz = 1.f / z;
    for (int j = 0; j < J; ++j) {
      const float cv = __expf(sm.bl[i * J + j] - m) * iz;
      sm.c[i * J + j] = cv;
      if (c_keep) c_keep[i * J + j] = cv;
    }
  }
  __syncthreads();
  for (int e = tid; e < JD; e += NT) {
    const int j = e / D;
    float acc = 0.f;
    for (int i = 0; i < in_n; ++i) acc += sm.c[i * J + j] * ut[(size_t)i * JD + e];
    sm.s[e] = acc;
    if (s_keep) s_keep[e] = acc;
  }
  __syncthreads();
  for (int j = tid; j < J; j += NT) {
    float n2 = 0.f;
    for (int d = 0; d < D; ++d) n2 += sm.s[j * D + d] * sm.s[j * D + d];
    const float fac = n2 / (1.f + n2) / sqrtf(n2 + kSquashEps);
    for (int d = 0; d < D; ++d) sm.v[j * D + d] = sm.s[j * D + d] * fac;
  }
  __syncthreads();
}

// ------------------------------------------------------------------ forward
// One workgroup per utterance; v_out[f] = v^{R-1} of frame f.  GS: the frame state
// does not fit one CU's LDS (C5: in_n = 16*41 capsules), so it lives in a per-workgroup
// slice of global memory (gstate, stride gstride floats) instead -- L2-resident, same code.
template <int NT, bool GS>
__global__ __launch_bounds__(NT) void sdr_fwd_kernel(const float* __restrict__ u, int T, int in_n, int J,
                                                              int D, int iters, int mask_first,
                                                              float* __restrict__ v_out, float* __restrict__ gstate,
                                                              size_t gstride, srf::SeqRange rg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* smem = GS ? gstate + blockIdx.x * gstride : lds;
  const int JD = J * D, P = in_n * J;
  SeqSmem sm{smem, smem + JD, smem + JD + P, smem + JD + 2 * P, smem + 2 * JD + 2 * P};
  const int b = blockIdx.x;
  for (int e = threadIdx.x; e < JD; e += NT)   // v_{t0-1} (v_{-1} = 0)
    sm.v[e] = rg.t0 > 0 ? v_out[((size_t)b * T + rg.t0 - 1) * JD + e] : 0.f;
  __syncthreads();
  for (int t = rg.t0; t < rg.t1; ++t) {
    const size_t f = (size_t)b * T + t;
    const float* ut = u + ((size_t)b * rg.tu_n + (t - rg.tu0)) * in_n * JD;
    for (int p = threadIdx.x; p < P; p += NT) sm.bl[p] = 0.f;
    __syncthreads();
    for (int r = 0; r < iters; ++r) sdr_iteration<NT>(ut, sm, in_n, J, D, mask_first, nullptr, nullptr);
    for (int e = threadIdx.x; e < JD; e += NT) v_out[f * JD + e] = sm.v[e];
  }
}

size_t sdr_fwd_smem(int in_n, int J, int D) {
  return (size_t)(3 * J * D + 2 * in_n * J + 2 * in_n) * sizeof(float);
}

// ------------------------------------------------------------------ backward
// One workgroup per utterance, frames in reverse.  Per frame: recompute the R
// iterations from v_{t-1} (keeping c^r, s^r, Vc^r), then for r = R-1..0
//   gs^r = squash'(s^r)^T a^r with a^{R-1} = g_v[t] + carry and, below the top,
//          a^{r-1} = sum_{r' >= r} gVc^{r'} (v^{r-1} reaches the loss only via later logits),
//   q_ij = <u_ij, gs_j>, sigma_i = sum_j c_ij q_ij, gL_ij = c_ij (q_ij - sigma_i),
//   gVc^r_j = sum_i gL_ij u_ij;
// gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j, written to HBM; carry = sum_r gVc^r.
struct BwdSmem {
  float *v, *bl, *c, *s, *red;      // forward scratch (SeqSmem)
  float *ck, *gl;                   // [R][P]
  float *sk, *vck, *gsk;            // [R][JD]
  float *acc, *carry, *gv;          // [JD]
};

template <int NT, bool GS>
__global__ __launch_bounds__(NT) void sdr_bwd_kernel(const float* __restrict__ u,
                                                              const float* __restrict__ v_saved,
                                                              const float* __restrict__ g_v, int T, int in_n, int J,
                                                              int D, int iters, int mask_first,
                                                              float* __restrict__ gu, float* __restrict__ gstate,
                                                              size_t gstride, srf::SeqRange rg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* smem = GS ? gstate + blockIdx.x * gstride : lds;
  const int JD = J * D, P = in_n * J, R = iters;
  const int tid = threadIdx.x;
  BwdSmem bs;
  float* q = smem;
  bs.v = q; q += JD;
  bs.bl = q; q += P;
  bs.c = q; q += P;
  bs.s = q; q += JD;
  bs.red = q; q += 2 * in_n;
  bs.ck = q; q += (size_t)R * P;
  bs.gl = q; q += (size_t)R * P;
  bs.sk = q; q += (size_t)R * JD;
  bs.vck = q; q += (size_t)R * JD;
  bs.gsk = q; q += (size_t)R * JD;
  bs.acc = q; q += JD;
  bs.carry = q; q += JD;
  bs.gv = q; q += JD;
  const SeqSmem sm{bs.v, bs.bl, bs.c, bs.s, bs.red};
  const int b = blockIdx.x;
  float* carry_io = rg.carry ? rg.carry + (size_t)b * JD : nullptr;
  for (int e = tid; e < JD; e += NT) bs.carry[e] = carry_io ? carry_io[e] : 0.f;
  __syncthreads();
  for (int t = rg.t1 - 1; t >= rg.t0; --t) {
    const size_t f = (size_t)b * T + t;
    const float* ut = u + ((size_t)b * rg.tu_n + (t - rg.tu0)) * in_n * JD;
    // ---- recompute the frame's iterations from v_{t-1}
    for (int e = tid; e < JD; e += NT) {
      const float vp = t > 0 ? v_saved[(f - 1) * JD + e] : 0.f;
      sm.v[e] = vp;
      bs.vck[e] = vp;                               // Vc^0 = v_{t-1}
      bs.acc[e] = g_v[f * JD + e] + bs.carry[e];   // dL/dv^{R-1}
      bs.carry[e] = 0.f;
    }
    for (int p = tid; p < P; p += NT) sm.bl[p] = 0.f;
    __syncthreads();
    for (int r = 0; r < R; ++r) {
      sdr_iteration<NT>(ut, sm, in_n, J, D, mask_first, bs.ck + (size_t)r * P, bs.sk + (size_t)r * JD);
      if (r + 1 < R) {
        for (int e = tid; e < JD; e += NT) bs.vck[(size_t)(r + 1) * JD + e] = bs.vck[(size_t)r * JD + e] + sm.v[e];
        __syncthreads();
      }
    }
    // ---- backward through the iterations; bs.acc holds dL/dv^r
    for (int r = R - 1; r >= 0; --r) {
      const float* sr = bs.sk + (size_t)r * JD;
      float* gsr = bs.gsk + (size_t)r * JD;
      for (int j = tid; j < J; j += NT) {
        float n2 = 0.f, sa = 0.f;
        for (int d = 0; d < D; ++d) {
          n2 += sr[j * D + d] * sr[j * D + d];
          sa += sr[j * D + d] * bs.acc[j * D + d];
        }
        const float rs = 1.f / sqrtf(n2 + kSquashEps);
        const float ip = 1.f / (1.f + n2);
        const float gfac = n2 * ip * rs;
        const float dg2 = 2.f * rs * ip * (ip - 0.5f * n2 / (n2 + kSquashEps)) * sa;
        for (int d = 0; d < D; ++d) gsr[j * D + d] = gfac * bs.acc[j * D + d] + dg2 * sr[j * D + d];
      }
      __syncthreads();
      // q_ij = <u_ij, gs_j> into gl (temporarily)
      const float* cr = bs.ck + (size_t)r * P;
      float* glr = bs.gl + (size_t)r * P;
      for (int p = tid; p < P; p += NT) {
        const int i = p / J, j = p - i * J;
        const float* up = ut + (size_t)i * JD + j * D;
        float d0 = 0.f, d1 = 0.f;
        for (int d = 0; d < D; d += 4) {
          const f4 a = *reinterpret_cast<const f4*>(up + d);
          d0 += a.x * gsr[j * D + d] + a.y * gsr[j * D + d + 1];
          d1 += a.z * gsr[j * D + d + 2] + a.w * gsr[j * D + d + 3];
        }
        glr[p] = d0 + d1;
      }
      __syncthreads();
      for (int i = tid; i < in_n; i += NT) {
        float sg = 0.f;
        for (int j = 0; j < J; ++j) sg += cr[i * J + j] * glr[i * J + j];
        for (int j = 0; j < J; ++j) glr[i * J + j] = cr[i * J + j] * (glr[i * J + j] - sg);
      }
      __syncthreads();
      // gVc^r_j = sum_i gL_ij u_ij: the gradient of every v^k with k < r and of v_{t-1}
      for (int e = tid; e < JD; e += NT) {
        const int j = e / D;
        float g = 0.f;
        for (int i = 0; i < in_n; ++i) g += glr[i * J + j] * ut[(size_t)i * JD + e];
        bs.carry[e] += g;
        // dL/dv^{r-1} = sum_{r' >= r} gVc^{r'} (v^{R-1} only reaches the loss directly)
        bs.gv[e] = (r == R - 1) ? g : bs.gv[e] + g;
        bs.acc[e] = bs.gv[e];
      }
      __syncthreads();
    }
    // ---- gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j
    for (int idx = tid; idx < in_n * JD; idx += NT) {
      const int i = idx / JD, e = idx - i * JD, j = e / D;
      float g = 0.f;
      for (int r = 0; r < R; ++r)
        g += bs.ck[(size_t)r * P + i * J + j] * bs.gsk[(size_t)r * JD + e] +
             bs.gl[(size_t)r * P + i * J + j] * bs.vck[(size_t)r * JD + e];
      gu[((size_t)b * rg.tg_n + (t - rg.tg0)) * in_n * JD + idx] = g;
    }
    __syncthreads();
  }
  if (carry_io)
    for (int e = tid; e < JD; e += NT) carry_io[e] = bs.carry[e];
}

size_t sdr_bwd_smem(int in_n, int J, int D, int R) {
  const size_t JD = (size_t)J * D, P = (size_t)in_n * J;
  return (3 * JD + 2 * P + 2 * in_n + 2 * R * P + 3 * R * JD + 3 * JD) * sizeof(float);
}

// ------------------------------------------------------------------ gx, gW
// gx^T[e][f] = sum_row W^T[i][e][row] gu[f][i][row] for one frame tile and capsule
// (K = rows, float4 operands), scattered into g_emb through the window adjoint.
// Frames of the map fm, gu through its view.
template <int DIN>
__global__ __launch_bounds__(64) void sdr_gx_kernel(GemmItems items, int N, int lpad, int in_n, int JD) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ gu = G.x;
  const float* __restrict__ WT = G.w;
  float* __restrict__ g_emb = G.o;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  if (blockIdx.x * 16 >= Q) return;
  constexpr int NCT = (DIN + 15) / 16;
  const int T = fm.T;
  const int lane = threadIdx.x, fl = lane & 15, g = lane >> 4;
  const int i = blockIdx.y;
  const int q = blockIdx.x * 16 + fl;
  int b, t;
  fm.frame(min(q, Q - 1), b, t);
  f4 acc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct] = f4{0.f, 0.f, 0.f, 0.f};
  const float* bp = gu + (fm.view(b, t) * in_n + i) * JD + 4 * g;
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < JD; k0 += 16) {
    const bool kin = k0 + 4 * g < JD;   // JD % 4 == 0: a float4 is wholly in or out
    const f4 bv = kin ? *reinterpret_cast<const f4*>(bp + k0) : z4;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int e = min(ct * 16 + fl, DIN - 1);
      const f4 av = kin ? *reinterpret_cast<const f4*>(WT + ((size_t)i * DIN + e) * JD + k0 + 4 * g) : z4;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) acc[ct] = mfma16x16x4(av[kk], bv[kk], acc[ct]);
    }
  }
  // C layout: col = frame (fl), rows e = ct*16 + 4g + k
  const int w = i / N, n = i - w * N;
  const int ts = t + w - lpad;
  if (q >= Q || ts < 0 || ts >= T) return;
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = ct * 16 + 4 * g + k;
      if (e < DIN) atomicAdd(g_emb + ((size_t)(b * T + ts) * N + n) * DIN + e, acc[ct][k]);
    }
}

// W [in_n][JD][din] -> WT [in_n][din][JD]; the same launch zeroes g_emb.
__global__ void sdr_transpose_w_kernel(const float* __restrict__ W, int in_n, int JD, int din,
                                       float* __restrict__ WT, float* __restrict__ zero, size_t n_zero) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nw = (size_t)in_n * JD * din;
  if (idx >= nw) {
    if (idx - nw < n_zero) zero[idx - nw] = 0.f;
    return;
  }
  const int row = idx % JD;
  const size_t rest = idx / JD;
  const int e = rest % din;
  const size_t i = rest / din;
  WT[idx] = W[(i * JD + row) * din + e];
}

// gW[i][row][e] = sum_f gu[f][i][row] x_i(f)[e] and gbias[i][row] = sum_f gu[f][i][row]:
// one wave per (i, row tile); K = frames in steps of 4 (lane group g = frame), x read
// through the window.  Frames of the map fm (gu through its view); accumulate != 0
// adds to gW / gbias (a layer's frame ranges in turn, one writer per element).
template <int DIN>
__global__ __launch_bounds__(256) void sdr_gw_kernel(GemmItems items, int N, int lpad, int in_n, int JD) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ gu = G.x;
  const float* __restrict__ emb = G.b;
  float* __restrict__ gW = G.o;
  float* __restrict__ gbias = G.o2;
  const int accumulate = G.acc;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  constexpr int NCT = (DIN + 15) / 16;
  const int T = fm.T;
  const int NT = (JD + 15) / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int task = blockIdx.x * 4 + wv;
  if (task >= in_n * NT) return;
  const int i = task / NT, tg = task - i * NT;
  const int row = min(tg * 16 + l16, JD - 1);
  const int w = i / N, n = i - w * N;
  f4 acc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct] = f4{0.f, 0.f, 0.f, 0.f};
  float sb = 0.f;
  // 8 groups of 4 frames per iteration: every load of the batch is issued before the
  // first MFMA (one round trip per 32 frames); the accumulation order is unchanged
  constexpr int U = 8;
  for (int q0 = 0; q0 < Q; q0 += 4 * U) {
    float a[U], xv[U][NCT];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int q = q0 + 4 * k + g;
      int b, t;
      fm.frame(min(q, Q - 1), b, t);
      a[k] = q < Q ? gu[(fm.view(b, t) * in_n + i) * JD + row] : 0.f;
      const int ts = t + w - lpad;
      const bool ok = q < Q && ts >= 0 && ts < T;
      const float* xp = emb + ((size_t)(b * T + min(max(ts, 0), T - 1)) * N + n) * DIN;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) xv[k][ct] = ok ? xp[min(ct * 16 + l16, DIN - 1)] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      sb += a[k];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[ct] = mfma16x16x4(a[k], xv[k][ct], acc[ct]);
    }
  }
  sb += __shfl_xor(sb, 16, 64);
  sb += __shfl_xor(sb, 32, 64);
  if (g == 0 && tg * 16 + l16 < JD) {
    float* gb = gbias + (size_t)i * JD + tg * 16 + l16;
    *gb = accumulate ? *gb + sb : sb;
  }
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int e = ct * 16 + l16;
    if (e >= DIN) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = tg * 16 + 4 * g + k;
      if (r < JD) {
        float* dst = gW + ((size_t)i * JD + r) * DIN + e;
        *dst = accumulate ? *dst + acc[ct][k] : acc[ct][k];
      }
    }
  }
}

// ------------------------------------------------------------------ pose / gx / gW on 32x32 tiles
// din 32 and 64 (C3/C4/C5): the three frame-parallel contractions of the layer on
// v_mfma_f32_32x32x2_f32, 32x32 output tiles, each lane feeding one float per operand
// per MFMA.  K runs in float4 chunks: lane half h supplies k = 8c + 4h + m for
// MFMA 4c + m (the same permutation on both operands), so every operand load is a
// float4 along k.  Output lane map: col = lane % 32, row = 8 (reg / 4) + 4 h + reg % 4.
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32x32x2(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int mfma32_row(int reg, int h) { return 8 * (reg >> 2) + 4 * h + (reg & 3); }

// x_i(frame q) of the window (zeros outside the utterance / past Q), chunk c of lane half h
template <int KC>
__device__ __forceinline__ void load_window_x(const float* __restrict__ emb, const FrameMap& fm, int q, int Q, int N,
                                              int DIN, int w, int n, int lpad, int h, f4 (&x)[KC]) {
  int b, t;
  fm.frame(min(q, Q - 1), b, t);
  const int ts = t + w - lpad;
  const bool ok = q < Q && ts >= 0 && ts < fm.T;
  const float* xp = emb + ((size_t)(b * fm.T + min(max(ts, 0), fm.T - 1)) * N + n) * DIN + 4 * h;
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    x[c] = f4{0.f, 0.f, 0.f, 0.f};
    if (ok) x[c] = *reinterpret_cast<const f4*>(xp + 8 * c);
  }
}

// u[f][i][row] = W_i x_i(f) + b_i.  Workgroup = one capsule i, 128 frames x 128 rows;
// wave (wf, wr) = 64 frames x 64 rows = 2 x 2 tiles (A = x: M = frames, B = W^T: N =
// rows, so a store writes 32 consecutive rows of one frame).  K = din at once.
template <int DIN>
__global__ __launch_bounds__(256, 2) void sdr_pose32_kernel(GemmItems items, int N, int lpad, int in_n, int JD, int nrb) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ emb = G.x;
  const float* __restrict__ W = G.w;
  const float* __restrict__ bias = G.b;
  float* __restrict__ u = G.o;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  if ((int)(blockIdx.x / nrb) * 128 >= Q) return;
  constexpr int KC = DIN / 8;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int i = blockIdx.y;
  const int rb = blockIdx.x % nrb, fb = blockIdx.x / nrb;
  const int w = i / N, n = i - w * N;
  const int f0 = fb * 128 + (wv & 1) * 64, r0 = rb * 128 + (wv >> 1) * 64;
  f4 a[2][KC], bw[2][KC];
#pragma unroll
  for (int ft = 0; ft < 2; ++ft) load_window_x<KC>(emb, fm, f0 + ft * 32 + l32, Q, N, DIN, w, n, lpad, h, a[ft]);
  f16v acc[2][2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int row = min(r0 + rt * 32 + l32, JD - 1);
    const float* wp = W + ((size_t)i * JD + row) * DIN + 4 * h;
#pragma unroll
    for (int c = 0; c < KC; ++c) bw[rt][c] = *reinterpret_cast<const f4*>(wp + 8 * c);
    const float bv = bias[(size_t)i * JD + row];
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ft][rt][r] = bv;
  }
#pragma unroll
  for (int c = 0; c < KC; ++c)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int ft = 0; ft < 2; ++ft)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[ft][rt] = mfma32x32x2(a[ft][c][m], bw[rt][c][m], acc[ft][rt]);
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = f0 + ft * 32 + mfma32_row(r, h);
      if (q >= Q) continue;
      int b, t;
      fm.frame(q, b, t);
      float* up = u + (fm.view(b, t) * in_n + i) * JD;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int row = r0 + rt * 32 + l32;
        if (row < JD) up[row] = acc[ft][rt][r];
      }
    }
}

// The same pose on v_mfma_f32_32x32x16_bf16 with every fp32 operand split into three
// bf16 terms by truncation (a = t1 + t2 + t3 + e, each residual exact in fp32, |e| <
// 2^-24 |a| in the normal range): six products per 16-wide K step (t1 t1, t1 t2, t2 t1,
// t1 t3, t2 t2, t3 t1; the dropped ones are below 2^-24 of |W x|), fp32 accumulation,
// the bias in the accumulator's start as before.  Same tiles and lane maps as
// sdr_pose32_kernel; lane half h holds k = 16 s + 8 h .. + 7 of K step s on both operands.
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3_bf16(const f4& p, const f4& q, bf8 (&t)[3]) {
  const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
  unsigned h[3][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const unsigned u = __float_as_uint(v[k]);
    h[0][k] = u & 0xFFFF0000u;
    const float r1 = v[k] - __uint_as_float(h[0][k]);
    h[1][k] = __float_as_uint(r1) & 0xFFFF0000u;
    const float r2 = r1 - __uint_as_float(h[1][k]);
    h[2][k] = __float_as_uint(r2);
  }
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    u4v w;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = __builtin_amdgcn_perm(h[m][2 * j + 1], h[m][2 * j], 0x07060302u);
    t[m] = __builtin_bit_cast(bf8, w);
  }
}

__device__ __forceinline__ f16v mfma32bf(const bf8& a, const bf8& b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// FB: frames per workgroup -- 128 (waves 2 x 2 over 128 frames x 128 rows) or 64 (the
// four waves stacked over 256 rows): a frame range of B x 10 frames pads less to 64.
template <int DIN, int FB = 128>
__global__ __launch_bounds__(256, 2) void sdr_pose3b_kernel(GemmItems items, int N, int lpad, int in_n, int JD,
                                                            int nrb) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ emb = G.x;
  const float* __restrict__ W = G.w;
  const float* __restrict__ bias = G.b;
  float* __restrict__ u = G.o;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  if ((int)(blockIdx.x / nrb) * FB >= Q) return;
  constexpr int KS = DIN / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int i = blockIdx.y;
  const int rb = blockIdx.x % nrb, fb = blockIdx.x / nrb;
  const int w = i / N, n = i - w * N;
  const int f0 = FB == 128 ? fb * 128 + (wv & 1) * 64 : fb * 64;
  const int r0 = FB == 128 ? rb * 128 + (wv >> 1) * 64 : rb * 256 + wv * 64;
  bf8 xa[2][KS][3];
#pragma unroll
  for (int ft = 0; ft < 2; ++ft) {
    const int q = f0 + ft * 32 + l32;
    int b, t;
    fm.frame(min(q, Q - 1), b, t);
    const int ts = t + w - lpad;
    const bool ok = q < Q && ts >= 0 && ts < fm.T;
    const float* xp = emb + ((size_t)(b * fm.T + min(max(ts, 0), fm.T - 1)) * N + n) * DIN + 8 * h;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      f4 p = {0.f, 0.f, 0.f, 0.f}, pq = {0.f, 0.f, 0.f, 0.f};
      if (ok) {
        p = *reinterpret_cast<const f4*>(xp + 16 * s);
        pq = *reinterpret_cast<const f4*>(xp + 16 * s + 4);
      }
      split3_bf16(p, pq, xa[ft][s]);
    }
  }
  f16v acc[2][2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int row = min(r0 + rt * 32 + l32, JD - 1);
    const float* wp = W + ((size_t)i * JD + row) * DIN + 8 * h;
    const float bv = bias[(size_t)i * JD + row];
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ft][rt][r] = bv;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf8 wb[3];
      split3_bf16(*reinterpret_cast<const f4*>(wp + 16 * s), *reinterpret_cast<const f4*>(wp + 16 * s + 4), wb);
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) {
        f16v c = acc[ft][rt];
        c = mfma32bf(xa[ft][s][2], wb[0], c);   // smallest terms first
        c = mfma32bf(xa[ft][s][1], wb[1], c);
        c = mfma32bf(xa[ft][s][0], wb[2], c);
        c = mfma32bf(xa[ft][s][1], wb[0], c);
        c = mfma32bf(xa[ft][s][0], wb[1], c);
        c = mfma32bf(xa[ft][s][0], wb[0], c);
        acc[ft][rt] = c;
      }
    }
  }
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = f0 + ft * 32 + mfma32_row(r, h);
      if (q >= Q) continue;
      int b, t;
      fm.frame(q, b, t);
      float* up = u + (fm.view(b, t) * in_n + i) * JD;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int row = r0 + rt * 32 + l32;
        if (row < JD) up[row] = acc[ft][rt][r];
      }
    }
}

// gx_i(f)[e] = sum_row gu[f][i][row] W_i[row][e], added into g_emb through the window
// adjoint.  Workgroup = one capsule, 128 frames; wave = 32 frames x din (din/32 tiles);
// K = JD in chunks of 64 (A = gu rows along k, B = W^T [i][e][row] along k), the next
// chunk's operands loaded while the current one's MFMAs run.
template <int DIN>
__global__ __launch_bounds__(256, 2) void sdr_gx32_kernel(GemmItems items, int N, int lpad, int in_n, int JD) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ gu = G.x;
  const float* __restrict__ WT = G.w;
  float* __restrict__ g_emb = G.o;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  if (blockIdx.x * 128 >= Q) return;
  constexpr int NE = DIN / 32;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int i = blockIdx.y;
  const int f0 = blockIdx.x * 128 + wv * 32;
  const int qa = min(f0 + l32, Q - 1);
  int ba, ta;
  fm.frame(qa, ba, ta);
  const float* ap = gu + (fm.view(ba, ta) * in_n + i) * JD + 4 * h;
  const float* bp[NE];
#pragma unroll
  for (int et = 0; et < NE; ++et) bp[et] = WT + ((size_t)i * DIN + et * 32 + l32) * JD + 4 * h;
  f16v acc[NE];
#pragma unroll
  for (int et = 0; et < NE; ++et)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[et][r] = 0.f;
  f4 a[2][8], bv[2][NE][8];
  auto fetch = [&](int k0, f4(&ax)[8], f4(&bx)[NE][8]) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const bool kin = k0 + 8 * c < JD;   // JD % 8 == 0 (check_sgeom)
      ax[c] = kin ? *reinterpret_cast<const f4*>(ap + k0 + 8 * c) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int et = 0; et < NE; ++et)
        bx[et][c] = kin ? *reinterpret_cast<const f4*>(bp[et] + k0 + 8 * c) : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  fetch(0, a[0], bv[0]);
  for (int k0 = 0; k0 < JD; k0 += 128) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (k0 + 64 * s >= JD) break;
      fetch(k0 + 64 * (s + 1), a[s ^ 1], bv[s ^ 1]);
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int et = 0; et < NE; ++et) acc[et] = mfma32x32x2(a[s][c][m], bv[s][et][c][m], acc[et]);
    }
  }
  const int w = i / N, n = i - w * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int q = f0 + mfma32_row(r, h);
    if (q >= Q) continue;
    int b, t;
    fm.frame(q, b, t);
    const int ts = t + w - lpad;
    if (ts < 0 || ts >= fm.T) continue;
    float* gp = g_emb + ((size_t)(b * fm.T + ts) * N + n) * DIN + l32;
#pragma unroll
    for (int et = 0; et < NE; ++et) atomicAdd(gp + et * 32, acc[et][r]);
  }
}

// gW_i[row][e] (+)= sum_f gu[f][i][row] x_i(f)[e], gbias_i[row] (+)= sum_f gu[f][i][row].
// Workgroup = one capsule, 128 rows; wave = 32 rows x din; K = frames, two per MFMA
// (lane half h takes frame 2s + h), 16 frames of loads issued before their MFMAs.
template <int DIN>
__global__ __launch_bounds__(256, 2) void sdr_gw32_kernel(GemmItems items, int N, int lpad, int in_n, int JD) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ gu = G.x;
  const float* __restrict__ emb = G.b;
  float* __restrict__ gW = G.o;
  float* __restrict__ gbias = G.o2;
  const int accumulate = G.acc;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  constexpr int NE = DIN / 32, U = 8;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int i = blockIdx.y;
  const int r0 = blockIdx.x * 128 + wv * 32;
  if (r0 >= JD) return;
  const int row = min(r0 + l32, JD - 1);
  const int w = i / N, n = i - w * N;
  f16v acc[NE];
#pragma unroll
  for (int et = 0; et < NE; ++et)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[et][r] = 0.f;
  float sb = 0.f;
  for (int q0 = 0; q0 < Q; q0 += 2 * U) {
    float a[U], xv[U][NE];
#pragma unroll
    for (int s = 0; s < U; ++s) {
      const int q = q0 + 2 * s + h;
      int b, t;
      fm.frame(min(q, Q - 1), b, t);
      a[s] = q < Q ? gu[(fm.view(b, t) * in_n + i) * JD + row] : 0.f;
      const int ts = t + w - lpad;
      const bool ok = q < Q && ts >= 0 && ts < fm.T;
      const float* xp = emb + ((size_t)(b * fm.T + min(max(ts, 0), fm.T - 1)) * N + n) * DIN + l32;
#pragma unroll
      for (int et = 0; et < NE; ++et) xv[s][et] = ok ? xp[et * 32] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < U; ++s) {
      sb += a[s];
#pragma unroll
      for (int et = 0; et < NE; ++et) acc[et] = mfma32x32x2(a[s], xv[s][et], acc[et]);
    }
  }
  sb += __shfl_xor(sb, 32, 64);
  if (h == 0 && r0 + l32 < JD) {
    float* gb = gbias + (size_t)i * JD + r0 + l32;
    *gb = accumulate ? *gb + sb : sb;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rr = r0 + mfma32_row(r, h);
    if (rr >= JD) continue;
#pragma unroll
    for (int et = 0; et < NE; ++et) {
      float* dst = gW + ((size_t)i * JD + rr) * DIN + et * 32 + l32;
      *dst = accumulate ? *dst + acc[et][r] : acc[et][r];
    }
  }
}

// gx and gW of din-32 layers in one pass over gu (C3): both contract the same gu, over
// rows (gx) and over frames (gW), so one launch reads it once instead of twice.
// Workgroup = 16 waves = one capsule i x 512 rows (32 per wave) x every frame of the
// item, in tiles of 32 frames; per tile and wave, on v_mfma_f32_32x32x2_f32:
//   gW^T tile  [rows][e] += gu[f][row] x_i(f)[e]   (A: gu, lane = row, as loaded;
//                                                  B: x through the window, lane = e)
//   gx^T part  [e][f]    = W_i[row][e] gu[f][row]  (A: W, lane = e, held for the whole
//                                                  launch; B: gu, lane = frame, read
//                                                  back transposed from a per-wave LDS
//                                                  tile [f][34] -- conflict-free reads)
// the 16 waves' gx parts summed through LDS [wave][f][33] and added into g_emb through
// the window adjoint (coalesced over e); gW / gbias stored at the end, one writer per
// element (accumulate adds, as sdr_gw_kernel).
struct GxwItem {
  const float* gu;
  const float* W;
  const float* emb;
  float* g_emb;
  float* gW;
  float* gbias;
  int acc, Q;
  FrameMap fm;
};
struct GxwItems {
  GxwItem it[srf::kMaxItems];
  int n;
};
constexpr int kGxwWaves = 16;
constexpr int kGxwThreads = 64 * kGxwWaves;
constexpr int kGxwRows = 32 * kGxwWaves;   // rows per workgroup
constexpr int kGxwTS = 34;                 // row stride of a wave's transposed tile
constexpr int kGxwPS = 33;                 // row stride of a wave's gx part
constexpr size_t kGxwLds =
    (size_t)kGxwWaves * 32 * (kGxwTS + kGxwPS) * sizeof(float) + 3 * 2 * 32 * sizeof(long long) + 2 * 32 * 32 * sizeof(float);

__global__ __launch_bounds__(kGxwThreads) void sdr_gxw32_kernel(GxwItems items, int N, int lpad, int in_n, int JD) {
  const GxwItem& G = items.it[blockIdx.z];
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* tT = lds;                                  // [wave][32 frames][kGxwTS]
  float* part = tT + kGxwWaves * 32 * kGxwTS;       // [wave][32 frames][kGxwPS]
  long long* finfo = reinterpret_cast<long long*>(part + kGxwWaves * 32 * kGxwPS);   // [3][gu | x][32]
  float* xs = reinterpret_cast<float*>(finfo + 3 * 64);   // [2][32 frames][32 e]: x of a tile
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int i = blockIdx.y;
  const int r0 = blockIdx.x * kGxwRows + wv * 32;
  const bool won = r0 < JD;   // JD % 32 == 0 (host)
  const int w = i / N, n = i - w * N;
  // gx's A operand, W_i[r0 + 2s + h][e = l32], for the whole launch
  float wa[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wa[s] = won ? G.W[((size_t)i * JD + r0 + 2 * s + h) * 32 + l32] : 0.f;
  f16v agw;
#pragma unroll
  for (int r = 0; r < 16; ++r) agw[r] = 0.f;
  float sb = 0.f;
  float* tw = tT + wv * 32 * kGxwTS;
  float* pw = part + wv * 32 * kGxwPS;
  // per tile of 32 frames: row offsets of gu and x of each frame (-1: none), written by
  // 32 threads into one of three buffers (tile t's reduction still reads buffer t % 3
  // while tile t + 1's are written and its loads issued)
  auto offsets = [&](int f0, long long* fi) {
    const int q = f0 + tid;
    int b, t;
    fm.frame(min(q, Q - 1), b, t);
    const int ts = t + w - lpad;
    fi[tid] = q < Q ? (long long)(fm.view(b, t) * in_n + i) * JD : -1;
    fi[32 + tid] = (q < Q && ts >= 0 && ts < fm.T) ? ((long long)(b * fm.T + ts) * N + n) * 32 : -1;
  };
  // gu of frames f0 + 2s + h at the wave's rows (A of gW); x of the tile, one element
  // per thread (staged in LDS: every wave uses all of it).  Absent rows load a valid
  // address and are zeroed after (no branch per load: a branch merges, and waits for,
  // the loads in flight)
  const int r0c = won ? r0 : 0;
  auto load = [&](const long long* fi, float (&a)[16], float& xr) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const long long go = fi[2 * s + h];
      const float av = G.gu[(go >= 0 ? go : 0) + r0c + l32];
      a[s] = (won && go >= 0) ? av : 0.f;
    }
    const long long xo = fi[32 + (tid >> 5)];
    const float xv = G.emb[(xo >= 0 ? xo : 0) + (tid & 31)];
    xr = xo >= 0 ? xv : 0.f;
  };
  // workgroup barrier on LDS only: no global data is exchanged inside the launch, so
  // the next tile's loads stay in flight through it (__syncthreads waits for them)
  auto bar = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  float a[16], xr;
  if (tid < 32) offsets(0, finfo);
  bar();
  load(finfo, a, xr);
  xs[tid] = xr;
  for (int f0 = 0, tb = 0, xb = 0; f0 < Q; f0 += 32, tb = tb == 2 ? 0 : tb + 1, xb ^= 1) {
    long long* fi = finfo + tb * 64;
    long long* fn = finfo + (tb == 2 ? 0 : tb + 1) * 64;
    const bool more = f0 + 32 < Q;
    if (more && tid < 32) offsets(f0 + 32, fn);
    bar();   // fn and this tile's x visible; every wave is past the previous tile's part reads
    // the next tile's loads in flight through this tile (the last tile reloads itself:
    // unconditional, so no branch merges the registers early)
    float an[16], xn;
    load(more ? fn : fi, an, xn);
    const float* xt = xs + xb * 1024;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      sb += a[s];
      agw = mfma32x32x2(a[s], xt[(2 * s + h) * 32 + l32], agw);
      tw[(2 * s + h) * kGxwTS + l32] = a[s];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f16v agx;
#pragma unroll
    for (int r = 0; r < 16; ++r) agx[r] = 0.f;
#pragma unroll
    for (int s = 0; s < 16; ++s) agx = mfma32x32x2(wa[s], tw[l32 * kGxwTS + 2 * s + h], agx);
    // agx: C[m = e][n = f]: lane (f = l32, h), reg r -> e = mfma32_row(r, h)
#pragma unroll
    for (int r = 0; r < 16; ++r) pw[l32 * kGxwPS + mfma32_row(r, h)] = agx[r];
    bar();
    for (int el = tid; el < 32 * 32; el += kGxwThreads) {
      const int f = el >> 5, e = el & 31;
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < kGxwWaves; ++k) v += part[(k * 32 + f) * kGxwPS + e];
      const long long xo = fi[32 + f];
      if (xo >= 0) atomicAdd(G.g_emb + xo + e, v);
    }
    xs[(xb ^ 1) * 1024 + tid] = xn;   // the next tile's x (its bar() makes it visible)
#pragma unroll
    for (int s = 0; s < 16; ++s) a[s] = an[s];
  }
  sb += __shfl_xor(sb, 32, 64);
  if (!won) return;
  if (h == 0) {
    float* gb = G.gbias + (size_t)i * JD + r0 + l32;
    *gb = G.acc ? *gb + sb : sb;
  }
  // agw: C[m = row][n = e]: lane (e = l32, h), reg r -> row r0 + mfma32_row(r, h)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float* dst = G.gW + ((size_t)i * JD + r0 + mfma32_row(r, h)) * 32 + l32;
    *dst = G.acc ? *dst + agw[r] : agw[r];
  }
}

// gx + gW + gbias of din = dout = 32 layers from the recurrence's gu factors
// (SeqItem::fact, C3): the register backward stores per frame gL^r [R][in_n][JP], gs^r and
// Vc^r [R][JD] (55 KB at the C3 last layer instead of 320 KB of gu), and this pass forms
//   gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j        (c^r: the forward's couplings)
// in registers and contracts it at once, on the same f32 MFMAs as sdr_gxw32_kernel (exact
// fp32 products).  A workgroup takes IW input capsules x 16 output capsules (16 waves, one
// output capsule j = 32 rows each: 512 rows, as sdr_gxw32_kernel) x every frame of the
// item in tiles of 16: per tile a lane loads its row of gs^r / Vc^r for 8 frames once
// (frames 8h + s, s < 8) and forms gu for the IW capsules (gs^r / Vc^r are shared by
// every input capsule; IW = 2 halves their L2 reads where the grid stays full), R
// streamed with the next iteration's vectors in flight.  Per capsule:
//   gW^T [rows][e] += gu[f][row] x_i(f)[e]     v_mfma_f32_32x32x2_f32 (K = frames 8h + s;
//                                               x staged in LDS per tile [i][h][e][s])
//   gx^T [e][f]     = W_i[row][e] gu[f][row]   v_mfma_f32_16x16x4_f32 (K = the wave's 32
//                                               rows, lane = frame; gu transposed through
//                                               a per-wave LDS tile; W_i in registers)
// the 8 waves' gx parts add into an LDS tile [i][e][f] (LDS atomics), flushed into g_emb
// through the window adjoint one tile later; gW / gbias stored at the end (one writer per
// element; acc adds, as sdr_gxw32_kernel).  Couplings, gL^r and x of the next tile are
// staged while this one computes; frame offsets four tiles deep.
__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

struct GxwfItem {
  const float* cs;     // couplings [B][T][R (P + JD)]
  const float* fac;    // gu factors, frame view of fm ([B][gn][R (P + 2 JD)])
  const float* W;
  const float* emb;
  float* g_emb;
  float* gW;
  float* gbias;
  int acc, Q;
  FrameMap fm;
};
struct GxwfItems {
  GxwfItem it[srf::kMaxItems];
  int n;
};
constexpr int kGxfWaves = 16;
constexpr int kGxfThreads = 64 * kGxfWaves;
constexpr int kGxfJ = kGxfWaves;       // output capsules per workgroup (32 rows each)
constexpr int kGxfXS = 12;             // stride of an x row [s] in LDS (conflict-free b128 reads)
constexpr int kGxfTS = 36;             // row stride of a wave's transposed gu tile [f][row]
constexpr int kGxfGS = 20;             // frame stride of the gx tile [i][e][f]
constexpr uint32_t kGxfOff = 0x7FFFFFFFu;   // an absent frame's factor offset (buffer loads read 0)

template <int IW, int R>
constexpr size_t gxf_lds_floats() {
  return 2 * (size_t)IW * R * 2 * kGxfJ * 16      // couplings / gL^r [buf][i][r][c|gL][j][f]
         + 2 * (size_t)IW * 2 * 32 * kGxfXS       // x [buf][i][h][e][s]
         + 2 * (size_t)IW * 32 * kGxfGS           // gx [buf][i][e][f]
         + (size_t)kGxfWaves * 16 * kGxfTS        // transposed gu per wave
         + 4 * 4 * 16;                             // frame table [4][fac | cs | b*T | t][16]
}

template <int IW, int R>
__global__ __launch_bounds__(kGxfThreads) void sdr_gxw32f_kernel(GxwfItems items, int N, int lpad, int in_n, int J,
                                                                 int JP) {
  const GxwfItem& G = items.it[blockIdx.z];
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  const int T = fm.T;
  const int JD = J * 32, P = in_n * JP;
  const size_t CSF = (size_t)R * (P + JD), FF = (size_t)R * (P + 2 * JD);
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int CB = IW * R * 2 * kGxfJ * 16, XB = IW * 2 * 32 * kGxfXS, GB = IW * 32 * kGxfGS;
  float* coef = lds;                       // [2][CB]
  float* xs = coef + 2 * CB;               // [2][XB]
  float* gxb = xs + 2 * XB;                // [2][GB]
  float* tT = gxb + 2 * GB;                // [wave][16][kGxfTS]
  int* ftab = reinterpret_cast<int*>(tT + kGxfWaves * 16 * kGxfTS);   // [4][4][16]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5, l16 = lane & 15, kg = lane >> 4;
  const int j0 = blockIdx.x * kGxfJ, j = j0 + wv;
  const int i0 = blockIdx.y * IW;
  const int NTl = (Q + 15) / 16;
  for (int k = tid; k < 2 * GB; k += kGxfThreads) gxb[k] = 0.f;
  // frame table of tile tt: factor byte offset, couplings offset, b * T, t (absent: t far out)
  auto frames = [&](int tt) {
    if (tid < 16) {
      int* fb = ftab + (tt & 3) * 64;
      const int q = tt * 16 + tid;
      const bool ok = q < Q;
      int b = 0, t = 0;
      if (ok) fm.frame(q, b, t);
      fb[tid] = ok ? (int)(fm.view(b, t) * FF * 4) : (int)kGxfOff;
      fb[16 + tid] = ok ? (int)((size_t)(b * T + t) * CSF) : 0;
      fb[32 + tid] = b * T;
      fb[48 + tid] = ok ? t : -(1 << 20);
    }
  };
  // staging of a tile: couplings / gL^r of IW capsules x 8 output capsules x 16 frames (f4
  // pieces of 4 j), and x of the IW capsules through the window (f4 pieces of 4 e)
  constexpr int JQ = kGxfJ / 4;   // f4 pieces of the workgroup's j per (frame, capsule, r, kind)
  constexpr int NCP = 16 * IW * R * 2 * JQ, NCPT = (NCP + kGxfThreads - 1) / kGxfThreads;
  f4 cv[NCPT], xv;
  auto stage_load = [&](int tt) {
    const int* fb = ftab + (tt & 3) * 64;
#pragma unroll
    for (int u = 0; u < NCPT; ++u) {
      const int p = min(tid + u * kGxfThreads, NCP - 1);
      const int f = p & 15, rest = p >> 4;
      const int jq = rest % JQ, kind = (rest / JQ) & 1, ir = rest / (2 * JQ), r = ir % R, k = ir / R;
      const int i = i0 + k;
      const bool ok = fb[48 + f] > -(1 << 20) && i < in_n;
      const float* src = kind ? G.fac + (size_t)(uint32_t)fb[f] / 4 : G.cs + (size_t)(uint32_t)fb[16 + f];
      const f4 v = *reinterpret_cast<const f4*>(ok ? src + (size_t)r * P + (size_t)i * JP + j0 + 4 * jq : G.cs);
      cv[u] = ok ? v : f4{0.f, 0.f, 0.f, 0.f};
    }
    {
      const int eq = tid & 7, f = (tid >> 3) & 15, k = tid >> 7;   // IW * 16 * 8 <= threads pieces
      const int i = i0 + k;
      const int w = i / N, n = i - w * N;
      const int ts = fb[48 + f] + w - lpad;
      const bool ok = k < IW && i < in_n && ts >= 0 && ts < T;
      const f4 v = *reinterpret_cast<const f4*>(ok ? G.emb + ((size_t)(fb[32 + f] + ts) * N + n) * 32 + 4 * eq : G.emb);
      xv = ok ? v : f4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto stage_store = [&](int buf) {
    float* cb = coef + buf * CB;
#pragma unroll
    for (int u = 0; u < NCPT; ++u) {
      const int p = tid + u * kGxfThreads;
      if (NCP % kGxfThreads != 0 && p >= NCP) continue;
      const int f = p & 15, rest = p >> 4;
      const int jq = rest % JQ, kind = (rest / JQ) & 1, ir = rest / (2 * JQ);
      float* d = cb + ((ir * 2 + kind) * kGxfJ + 4 * jq) * 16 + f;
#pragma unroll
      for (int c = 0; c < 4; ++c) d[c * 16] = cv[u][c];
    }
    {
      const int eq = tid & 7, f = (tid >> 3) & 15, k = tid >> 7;
      if (k < IW) {
        float* d = xs + buf * XB + ((k * 2 + (f >> 3)) * 32 + 4 * eq) * kGxfXS + (f & 7);
#pragma unroll
        for (int c = 0; c < 4; ++c) d[c * kGxfXS] = xv[c];
      }
    }
  };
  // gs^r / Vc^r of the lane's row, frames 8h + s: buffer loads over the factors (an absent
  // frame's offset reads zeros)
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G.fac), 0, (int)0x7FFFFFFF, 0x00020000);
  const uint32_t rowb = (uint32_t)(j * 32 + l32) * 4;
  uint32_t fo[8];
  auto frame_offsets = [&](int tt) {
    const int* fb = ftab + (tt & 3) * 64 + 8 * h;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t o = (uint32_t)fb[s];
      fo[s] = o == kGxfOff ? kGxfOff : o + rowb;
    }
  };
  auto vec_load = [&](int r, float (&gsv)[8], float (&vcv)[8]) {
    const uint32_t sg = (uint32_t)((size_t)R * P + (size_t)r * JD) * 4, sv = sg + (uint32_t)(R * JD) * 4;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      gsv[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, fo[s], sg, 0));
      vcv[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, fo[s], sv, 0));
    }
  };
  // gx's A operand, W_i[32 j + 8 kg + st][e = 16 half + l16], for the whole launch
  float wr[IW][2][8];
#pragma unroll
  for (int k = 0; k < IW; ++k)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const int i = min(i0 + k, in_n - 1);
        wr[k][hf][st] = G.W[((size_t)i * JD + j * 32 + 8 * kg + st) * 32 + 16 * hf + l16];
      }
  f16v agw[IW];
  float sb[IW];
#pragma unroll
  for (int k = 0; k < IW; ++k) {
    sb[k] = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) agw[k][r] = 0.f;
  }
  float* tw = tT + wv * 16 * kGxfTS;
  auto bar = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  frames(0);
  frames(1);
  __syncthreads();
  if (NTl > 0) {
    stage_load(0);
    stage_store(0);
  }
  frame_offsets(0);
  float gsc[8], vcc[8];
  vec_load(0, gsc, vcc);
  __syncthreads();
  for (int tt = 0; tt < NTl; ++tt) {
    const int buf = tt & 1;
    const bool more = tt + 1 < NTl;
    if (tt + 2 < NTl) frames(tt + 2);
    stage_load(more ? tt + 1 : tt);
    const float* cb = coef + buf * CB;
    float gu[IW][8];
#pragma unroll
    for (int k = 0; k < IW; ++k)
#pragma unroll
      for (int s = 0; s < 8; ++s) gu[k][s] = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      __builtin_amdgcn_sched_barrier(0);   // one iteration's vectors in flight at a time
      // the next iteration's vectors in flight through this one (the next tile's first
      // ones are issued after the contractions, to their end of the tile)
      float gsn[8], vcn[8];
      if (r + 1 < R) vec_load(r + 1, gsn, vcn);
#pragma unroll
      for (int k = 0; k < IW; ++k) {
        const float* cp = cb + ((k * R + r) * 2 * kGxfJ + wv) * 16 + 8 * h;
        const float* gp = cp + kGxfJ * 16;
        const f4 c0 = ld4(cp), c1 = ld4(cp + 4), g0 = ld4(gp), g1 = ld4(gp + 4);
        const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
        for (int s = 0; s < 8; ++s) gu[k][s] = fmaf(cc[s], gsc[s], fmaf(gg[s], vcc[s], gu[k][s]));
      }
      if (r + 1 < R) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          gsc[s] = gsn[s];
          vcc[s] = vcn[s];
        }
      }
    }
    const float* xb = xs + buf * XB;
    float* gxt = gxb + buf * GB;
#pragma unroll
    for (int k = 0; k < IW; ++k) {
      __builtin_amdgcn_sched_barrier(0);
      const float* xp = xb + ((k * 2 + h) * 32 + l32) * kGxfXS;
      const f4 x0 = ld4(xp), x1 = ld4(xp + 4);
      const float xx[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        sb[k] += gu[k][s];
        agw[k] = mfma32x32x2(gu[k][s], xx[s], agw[k]);
        tw[(8 * h + s) * kGxfTS + l32] = gu[k][s];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const f4 b0 = ld4(tw + l16 * kGxfTS + 8 * kg), b1 = ld4(tw + l16 * kGxfTS + 8 * kg + 4);
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      f4 gx[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        gx[0] = mfma16x16x4(wr[k][0][st], bb[st], gx[0]);
        gx[1] = mfma16x16x4(wr[k][1][st], bb[st], gx[1]);
      }
      // C: lane (frame l16, kg) holds e = 16 half + 4 kg + c
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int c = 0; c < 4; ++c) atomicAdd(gxt + (k * 32 + 16 * hf + 4 * kg + c) * kGxfGS + l16, gx[hf][c]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();   // every lane's tile reads done before the next capsule's writes
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // the next tile's first vectors (the last tile reloads itself: no branch around a load)
    frame_offsets(more ? tt + 1 : tt);
    vec_load(0, gsc, vcc);
    if (more) stage_store(buf ^ 1);
    bar();   // this tile's gx parts complete; the next tile's staging visible
    // flush this tile's gx through the window adjoint (and zero it for tile tt + 2)
    const int* fb = ftab + (tt & 3) * 64;
    for (int idx = tid; idx < IW * 512; idx += kGxfThreads) {
      const int k = idx >> 9, f = (idx >> 5) & 15, e = idx & 31;
      float* g = gxt + (k * 32 + e) * kGxfGS + f;
      const float v = *g;
      *g = 0.f;
      const int i = i0 + k;
      const int w = i / N, n = i - w * N;
      const int ts = fb[48 + f] + w - lpad;
      if (i < in_n && ts >= 0 && ts < T && v != 0.f)
        atomicAdd(G.g_emb + ((size_t)(fb[32 + f] + ts) * N + n) * 32 + e, v);
    }
  }
  if (j >= J) return;
#pragma unroll
  for (int k = 0; k < IW; ++k) {
    const int i = i0 + k;
    if (i >= in_n) continue;
    const float sbt = sb[k] + __shfl_xor(sb[k], 32, 64);
    if (h == 0) {
      float* gb = G.gbias + (size_t)i * JD + j * 32 + l32;
      *gb = G.acc ? *gb + sbt : sbt;
    }
    // agw: C[m = row][n = e]: lane (e = l32, h), reg r -> row mfma32_row(r, h)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float* dst = G.gW + ((size_t)i * JD + j * 32 + mfma32_row(r, h)) * 32 + l32;
      *dst = G.acc ? *dst + agw[k][r] : agw[k][r];
    }
  }
}

// ---- fp8 pose (opt-in, BASELINE C5 "fp8 pose-transform MFMA"): OCP e4m3 operands on
// v_mfma_f32_32x32x16_fp8_fp8, fp32 accumulation.  Every frame's x_i(f) and every row
// of W_i gets its own power-of-two scale 2^e with max|a 2^e| in (224, 448] (e4m3's
// largest finite value is 448), applied exactly, so each product carries at most the
// two operands' e4m3 rounding (2^-4 relative each): |u - u_exact| <= 0.13 sum_k |W||x|
// plus fp32 accumulation.  The bias is added in fp32.  Same tiles as sdr_pose32_kernel;
// lane half h holds k = 16 s + 8 h .. + 7 of k-step s (8 bytes), the same on both operands.
typedef long fp8x8;

__device__ __forceinline__ int e4m3_exp(float amax) {
  if (!(amax > 0.f) || !(amax < __builtin_inff())) return 0;
  int e;
  (void)frexpf(448.f / amax, &e);   // 2^(e-1) <= 448 / amax < 2^e
  return max(-100, min(100, e - 1));
}
__device__ __forceinline__ fp8x8 pack_e4m3(const f4& a, const f4& b, float s) {
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(a.x * s, a.y * s, 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(a.z * s, a.w * s, lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(b.x * s, b.y * s, 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(b.z * s, b.w * s, hi, true);
  return (fp8x8)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float amax8(const f4& a, const f4& b) {
  return fmaxf(fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))),
               fmaxf(fmaxf(fabsf(b.x), fabsf(b.y)), fmaxf(fabsf(b.z), fabsf(b.w))));
}

__device__ __forceinline__ unsigned short bf16_rne(float v) {
  unsigned x = __float_as_uint(v);
  x += 0x7fffu + ((x >> 16) & 1u);
  return (unsigned short)(x >> 16);
}

// BF: u stored as bf16 (round to nearest even) for the streaming recurrence of the fp8
// C5 variant: half the bytes of every u read, error 2^-9 relative -- well inside the
// e4m3 operands' 2^-4.
template <int DIN, bool BF = false>
__global__ __launch_bounds__(256, 2) void sdr_pose8_kernel(GemmItems items, int N, int lpad, int in_n, int JD, int nrb) {
  const GemmItem& G = items.it[blockIdx.z];
  const float* __restrict__ emb = G.x;
  const float* __restrict__ W = G.w;
  const float* __restrict__ bias = G.b;
  float* __restrict__ u = G.o;
  const int Q = G.Q;
  const FrameMap fm = G.fm;
  if ((int)(blockIdx.x / nrb) * 128 >= Q) return;
  constexpr int KS = DIN / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int i = blockIdx.y;
  const int rb = blockIdx.x % nrb, fb = blockIdx.x / nrb;
  const int w = i / N, n = i - w * N;
  const int f0 = fb * 128 + (wv & 1) * 64, r0 = rb * 128 + (wv >> 1) * 64;
  fp8x8 aq[2][KS], bq[2][KS];
  int ex[2], ew[2];
#pragma unroll
  for (int ft = 0; ft < 2; ++ft) {
    const int q = f0 + ft * 32 + l32;
    int b, t;
    fm.frame(min(q, Q - 1), b, t);
    const int ts = t + w - lpad;
    const bool ok = q < Q && ts >= 0 && ts < fm.T;
    const float* xp = emb + ((size_t)(b * fm.T + min(max(ts, 0), fm.T - 1)) * N + n) * DIN + 8 * h;
    f4 x[KS][2];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int c = 0; c < 2; ++c) x[s][c] = ok ? *reinterpret_cast<const f4*>(xp + 16 * s + 4 * c) : f4{0.f, 0.f, 0.f, 0.f};
      mx = fmaxf(mx, amax8(x[s][0], x[s][1]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));   // the frame's other half of din
    ex[ft] = e4m3_exp(mx);
    const float sc = srf_exp2i(ex[ft]);
#pragma unroll
    for (int s = 0; s < KS; ++s) aq[ft][s] = pack_e4m3(x[s][0], x[s][1], sc);
  }
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int row = min(r0 + rt * 32 + l32, JD - 1);
    const float* wp = W + ((size_t)i * JD + row) * DIN + 8 * h;
    f4 x[KS][2];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int c = 0; c < 2; ++c) x[s][c] = *reinterpret_cast<const f4*>(wp + 16 * s + 4 * c);
      mx = fmaxf(mx, amax8(x[s][0], x[s][1]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    ew[rt] = e4m3_exp(mx);
    const float sc = srf_exp2i(ew[rt]);
#pragma unroll
    for (int s = 0; s < KS; ++s) bq[rt][s] = pack_e4m3(x[s][0], x[s][1], sc);
  }
  f16v acc[2][2];
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ft][rt][r] = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int ft = 0; ft < 2; ++ft)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        acc[ft][rt] = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(aq[ft][s], bq[rt][s], acc[ft][rt], 0, 0, 0);
  float bv[2], sw[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int row = min(r0 + rt * 32 + l32, JD - 1);
    bv[rt] = bias[(size_t)i * JD + row];
    sw[rt] = srf_exp2i(-ew[rt]);
  }
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int fr = mfma32_row(r, h);
      const float sx = srf_exp2i(-__shfl(ex[ft], fr, 64));   // the frame's scale, from the lane that loaded it
      const int q = f0 + ft * 32 + fr;
      if (q >= Q) continue;
      int b, t;
      fm.frame(q, b, t);
      const size_t uo = (fm.view(b, t) * in_n + i) * JD;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int row = r0 + rt * 32 + l32;
        const float val = acc[ft][rt][r] * sx * sw[rt] + bv[rt];
        if (row < JD) {
          if constexpr (BF) reinterpret_cast<unsigned short*>(u)[uo + row] = bf16_rne(val);
          else u[uo + row] = val;
        }
      }
    }
}

// Which contraction runs on the 32x32-tile kernels, by din (scripts/bench_sdr_gemm.py,
// one frame range alone on the GPU, us 32x32 vs 16x16): C5 din 64 pose 850 vs 973, gx
// 1228 vs 1174, gW 937 vs 1073; C3 din 32 pose 46 vs 33, gx 47 vs 53, gW 91 vs 65.
enum class SdrGemm { kPose, kGx, kGw };
constexpr int kSdrMfma32Din32 = 3;   // bit 0 pose, bit 1 gx, bit 2 gW: the 32x32 kernels at din 32 (r04q: pose + gx)
bool use_mfma32(int din, int JD, SdrGemm k) {
  if ((din != 32 && din != 64) || JD % 8) return false;
  if (din == 64) return k != SdrGemm::kGx;
  const int bit = k == SdrGemm::kPose ? 1 : k == SdrGemm::kGx ? 2 : 4;
  return (kSdrMfma32Din32 & bit) != 0;
}

// ------------------------------------------------------------------ host
int check_sgeom(const SGeom& g) {
  SRF_REQUIRE(g.B > 0 && g.T > 0 && g.N > 0 && g.J > 1, "bad shape B=%d T=%d N=%d J=%d", g.B, g.T, g.N, g.J);
  SRF_REQUIRE(g.lpad >= 0 && g.rpad >= 0, "negative window pad");
  SRF_REQUIRE(g.iters >= 1 && g.iters <= 5, "routing iterations must be in [1,5], got %d", g.iters);
  SRF_REQUIRE(g.din == 8 || g.din == 16 || g.din == 32 || g.din == 64, "unsupported in_d %d", g.din);
  SRF_REQUIRE(g.dout % 4 == 0, "out_d must be a multiple of 4");
  return SRF_OK;
}

// Frame state beyond one CU's 160 KiB LDS goes to global memory (workspace).
bool sdr_gstate(size_t bytes) { return bytes > 160 * 1024; }

// per-workgroup slice of the global frame state, in floats (256-B aligned slices)
size_t gstate_stride(size_t state_bytes) { return srf::align_up(state_bytes, 256) / sizeof(float); }

size_t gstate_bytes(const SGeom& g, size_t state_bytes) {
  return sdr_gstate(state_bytes) ? (size_t)g.B * gstate_stride(state_bytes) * sizeof(float) : 0;
}

FrameMap frame_map(int T, int t0, int t1, int v0, int vn) { return FrameMap{T, t0, t1 - t0, v0, vn}; }

// Launches of the frame-parallel contractions over it.n items (grid.z), each a frame
// range of a same-shaped layer; items with no frames are dropped by the caller.
int max_q(const GemmItems& it) {
  int q = 0;
  for (int k = 0; k < it.n; ++k) q = std::max(q, it.it[k].Q);
  return q;
}

// mode: 0 fp32 pose, 1 fp8 pose with fp32 u, 2 fp8 pose with bf16 u
int pose_n(const SGeom& g, const GemmItems& it, hipStream_t st, int mode = 0) {
  const bool fp8 = mode != 0;
  const int Q = max_q(it);
  if (it.n == 0 || Q == 0) return SRF_OK;
  const int nrb = (g.JD() + 127) / 128;
  const dim3 grid32(nrb * ((Q + 127) / 128), g.in_n(), it.n);
  if (fp8) {
    if ((g.din != 32 && g.din != 64) || g.JD() % 8) {
      srf::set_error("fp8 pose: in_d must be 32 or 64 (got %d) and J*out_d a multiple of 8", g.din);
      return SRF_EUNSUPPORTED;
    }
#define SRF_POSE8(DIN, BF) \
  hipLaunchKernelGGL((sdr_pose8_kernel<DIN, BF>), grid32, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD(), nrb)
    if (g.din == 32) {
      if (mode == 2) SRF_POSE8(32, true); else SRF_POSE8(32, false);
    } else {
      if (mode == 2) SRF_POSE8(64, true); else SRF_POSE8(64, false);
    }
#undef SRF_POSE8
    SRF_LAUNCH_CHECK("sdr_pose8");
    return SRF_OK;
  }
  if ((g.din == 32 || g.din == 64) && g.JD() % 8 == 0) {   // fp32 pose on bf16 MFMA, three-term split operands
    // 64-frame workgroups where they pad the range's frames less than 128-frame ones
    const bool f64 = (Q + 63) / 64 * 64 < (Q + 127) / 128 * 128;
    const int nrb64 = (g.JD() + 255) / 256;
    const dim3 grid64(nrb64 * ((Q + 63) / 64), g.in_n(), it.n);
#define SRF_POSE3B(DIN)                                                                                          \
  if (f64)                                                                                                       \
    hipLaunchKernelGGL((sdr_pose3b_kernel<DIN, 64>), grid64, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD(), \
                       nrb64);                                                                                   \
  else                                                                                                           \
    hipLaunchKernelGGL((sdr_pose3b_kernel<DIN, 128>), grid32, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD(), nrb)
    if (g.din == 32) {
      SRF_POSE3B(32);
    } else {
      SRF_POSE3B(64);
    }
#undef SRF_POSE3B
    SRF_LAUNCH_CHECK("sdr_pose3b");
    return SRF_OK;
  }
  if (use_mfma32(g.din, g.JD(), SdrGemm::kPose)) {
    if (g.din == 32)
      hipLaunchKernelGGL(sdr_pose32_kernel<32>, grid32, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD(), nrb);
    else
      hipLaunchKernelGGL(sdr_pose32_kernel<64>, grid32, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD(), nrb);
    SRF_LAUNCH_CHECK("sdr_pose32");
    return SRF_OK;
  }
  constexpr int FT = 2;   // frame tiles per workgroup: each W fragment feeds two MFMA chains
  const dim3 grid((Q + 16 * FT - 1) / (16 * FT), g.in_n(), it.n);
#define SRF_POSE(DIN) \
  hipLaunchKernelGGL((sdr_pose_kernel<DIN, FT>), grid, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD())
  switch (g.din) {
    case 8: SRF_POSE(8); break;
    case 16: SRF_POSE(16); break;
    case 32: SRF_POSE(32); break;
    default: SRF_POSE(64); break;
  }
#undef SRF_POSE
  SRF_LAUNCH_CHECK("sdr_pose");
  return SRF_OK;
}

int pose_range(const SGeom& g, const float* emb, const float* W, const float* bias, const FrameMap& fm, float* u,
               hipStream_t st) {
  GemmItems it{};
  it.it[0] = GemmItem{emb, W, bias, u, nullptr, 0, g.B * fm.nt, fm};
  it.n = 1;
  return pose_n(g, it, st);
}

// The recurrence over it.n frame ranges (grid.y): the register-resident kernels when the
// shape fits, else the streaming ones, else the LDS / global-state ones (one launch per
// item; gstate: the item's workspace, B slices of the state, when it exceeds LDS).
// bf16 u (the fp8 C5 variant) is read by the streaming kernels only
int u_type_ok(const SGeom& g, const srf::SeqItems& it) {
  bool bf = false;
  for (int k = 0; k < it.n; ++k) bf = bf || it.it[k].u_bf16;
  if (bf && (srf::sdr_seq_supported(g.in_n(), g.J, g.dout, g.iters) ||
             !srf::sdr_stream_supported(g.in_n(), g.J, g.dout, g.iters))) {
    srf::set_error("bf16 u: only layers on the streaming recurrence kernels (in_n=%d J=%d dout=%d)", g.in_n(), g.J,
                   g.dout);
    return SRF_EUNSUPPORTED;
  }
  return SRF_OK;
}

int recur_fwd_n(const SGeom& g, const srf::SeqItems& it, hipStream_t st) {
  if (it.n == 0) return SRF_OK;
  if (int rc = u_type_ok(g, it)) return rc;
  if (srf::sdr_seq_supported(g.in_n(), g.J, g.dout, g.iters))
    return srf::sdr_seq_fwd(it, g.B, g.T, g.in_n(), g.J, g.dout, g.iters, g.mask_first, st);
  if (srf::sdr_stream_supported(g.in_n(), g.J, g.dout, g.iters))
    return srf::sdr_stream_fwd(it, g.B, g.T, g.in_n(), g.J, g.dout, g.iters, g.mask_first, st);
  const size_t sm = sdr_fwd_smem(g.in_n(), g.J, g.dout);
  for (int k = 0; k < it.n; ++k) {
    const srf::SeqItem& I = it.it[k];
    if (sdr_gstate(sm))
      hipLaunchKernelGGL((sdr_fwd_kernel<kGsThreads, true>), dim3(g.B), dim3(kGsThreads), 0, st, I.u, g.T, g.in_n(),
                         g.J, g.dout, g.iters, g.mask_first, I.v, I.ws, gstate_stride(sm), I.rg);
    else
      hipLaunchKernelGGL((sdr_fwd_kernel<kGsThreads, false>), dim3(g.B), dim3(kGsThreads), sm, st, I.u, g.T, g.in_n(),
                         g.J, g.dout, g.iters, g.mask_first, I.v, (float*)nullptr, (size_t)0, I.rg);
    SRF_LAUNCH_CHECK("sdr_fwd");
  }
  return SRF_OK;
}

int recur_bwd_n(const SGeom& g, const srf::SeqItems& it, hipStream_t st) {
  if (it.n == 0) return SRF_OK;
  if (int rc = u_type_ok(g, it)) return rc;
  if (srf::sdr_seq_supported(g.in_n(), g.J, g.dout, g.iters))
    return srf::sdr_seq_bwd(it, g.B, g.T, g.in_n(), g.J, g.dout, g.iters, g.mask_first, st);
  if (srf::sdr_stream_supported(g.in_n(), g.J, g.dout, g.iters))
    return srf::sdr_stream_bwd(it, g.B, g.T, g.in_n(), g.J, g.dout, g.iters, st);
  const size_t sm = sdr_bwd_smem(g.in_n(), g.J, g.dout, g.iters);
  for (int k = 0; k < it.n; ++k) {
    const srf::SeqItem& I = it.it[k];
    if (sdr_gstate(sm))
      hipLaunchKernelGGL((sdr_bwd_kernel<kGsThreads, true>), dim3(g.B), dim3(kGsThreads), 0, st, I.u, I.v, I.g_v, g.T,
                         g.in_n(), g.J, g.dout, g.iters, g.mask_first, I.gu, I.ws, gstate_stride(sm), I.rg);
    else
      hipLaunchKernelGGL((sdr_bwd_kernel<kGsThreads, false>), dim3(g.B), dim3(kGsThreads), sm, st, I.u, I.v, I.g_v,
                         g.T, g.in_n(), g.J, g.dout, g.iters, g.mask_first, I.gu, (float*)nullptr, (size_t)0, I.rg);
    SRF_LAUNCH_CHECK("sdr_bwd");
  }
  return SRF_OK;
}

srf::SeqItems one_seq_item(const srf::SeqItem& I) {
  srf::SeqItems it{};
  it.it[0] = I;
  it.n = I.rg.t0 < I.rg.t1 ? 1 : 0;
  return it;
}

size_t recur_workspace(const SGeom& g) {
  // register kernels: only the exchange area of grouped launches (srf_group.h)
  if (srf::sdr_seq_supported(g.in_n(), g.J, g.dout, g.iters)) return srf_grp::floats(0, g.B, g.JD()) * sizeof(float);
  if (srf::sdr_stream_supported(g.in_n(), g.J, g.dout, g.iters))
    return srf::sdr_stream_workspace_floats(g.B, g.in_n(), g.J, g.dout, g.iters) * sizeof(float);
  return std::max(gstate_bytes(g, sdr_fwd_smem(g.in_n(), g.J, g.dout)),
                  gstate_bytes(g, sdr_bwd_smem(g.in_n(), g.J, g.dout, g.iters)));
}

int gx_n(const SGeom& g, const GemmItems& it, hipStream_t st) {
  const int Q = max_q(it);
  if (it.n == 0 || Q == 0) return SRF_OK;
  if (use_mfma32(g.din, g.JD(), SdrGemm::kGx)) {
    const dim3 grid((Q + 127) / 128, g.in_n(), it.n);
    if (g.din == 32)
      hipLaunchKernelGGL(sdr_gx32_kernel<32>, grid, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD());
    else
      hipLaunchKernelGGL(sdr_gx32_kernel<64>, grid, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD());
    SRF_LAUNCH_CHECK("sdr_gx32");
    return SRF_OK;
  }
  const dim3 grid((Q + 15) / 16, g.in_n(), it.n);
#define SRF_GX(DIN) hipLaunchKernelGGL(sdr_gx_kernel<DIN>, grid, dim3(64), 0, st, it, g.N, g.lpad, g.in_n(), g.JD())
  switch (g.din) {
    case 8: SRF_GX(8); break;
    case 16: SRF_GX(16); break;
    case 32: SRF_GX(32); break;
    default: SRF_GX(64); break;
  }
#undef SRF_GX
  SRF_LAUNCH_CHECK("sdr_gx");
  return SRF_OK;
}

int gx_range(const SGeom& g, const float* gu, const float* WT, const FrameMap& fm, float* g_emb, hipStream_t st) {
  GemmItems it{};
  it.it[0] = GemmItem{gu, WT, nullptr, g_emb, nullptr, 0, g.B * fm.nt, fm};
  it.n = 1;
  return gx_n(g, it, st);
}

// gx + gW of din-32 layers in one launch (sdr_gxw32_kernel); false: not this shape
bool gxw_supported(const SGeom& g) { return g.din == 32 && g.JD() % 32 == 0; }

int gxw_n(const SGeom& g, const GxwItems& it, hipStream_t st) {
  if (it.n == 0) return SRF_OK;
  static bool attr = false;   // one-time raise of the kernel's LDS limit (above 64 KiB)
  if (!attr) {
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)sdr_gxw32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kGxwLds));
    attr = true;
  }
  const dim3 grid((g.JD() + kGxwRows - 1) / kGxwRows, g.in_n(), it.n);
  hipLaunchKernelGGL(sdr_gxw32_kernel, grid, dim3(kGxwThreads), kGxwLds, st, it, g.N, g.lpad, g.in_n(), g.JD());
  SRF_LAUNCH_CHECK("sdr_gxw32");
  return SRF_OK;
}

// the padded capsule count of the register recurrence's [in_n][JP] records
int jp_of(int J) {
  int p = 4;
  while (p < J) p <<= 1;
  return p;
}

// gx + gW from gu factors (sdr_gxw32f_kernel): din = dout = 32, J % 16 == 0, iters <= 3
bool gxwf_supported(const SGeom& g) {
  return g.din == 32 && g.dout == 32 && g.J % kGxfJ == 0 && g.iters >= 1 && g.iters <= 3 &&
         srf::sdr_seq_fact_floats(g.in_n(), g.J, g.dout, g.iters) != 0;
}

template <int IW, int R>
int gxwf_launch(const SGeom& g, const GxwfItems& it, hipStream_t st) {
  const size_t lds = gxf_lds_floats<IW, R>() * sizeof(float);
  static bool attr = false;   // one-time raise of the kernel's LDS limit (above 64 KiB)
  if (!attr) {
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)sdr_gxw32f_kernel<IW, R>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const dim3 grid(g.J / kGxfJ, (g.in_n() + IW - 1) / IW, it.n);
  hipLaunchKernelGGL((sdr_gxw32f_kernel<IW, R>), grid, dim3(kGxfThreads), lds, st, it, g.N, g.lpad, g.in_n(), g.J,
                     jp_of(g.J));
  SRF_LAUNCH_CHECK("sdr_gxw32f");
  return SRF_OK;
}

int gxwf_n(const SGeom& g, const GxwfItems& it, hipStream_t st) {
  if (it.n == 0) return SRF_OK;
  // one input capsule per workgroup: two spill at 128 registers (16 waves)
#define SRF_GXF(RR) \
  if (g.iters == RR) return gxwf_launch<1, RR>(g, it, st);
  SRF_GXF(1)
  SRF_GXF(2)
  SRF_GXF(3)
#undef SRF_GXF
  srf::set_error("sdr_gxw32f: iters %d", g.iters);
  return SRF_EUNSUPPORTED;
}

// items with Q == 0 still run when they start the accumulation (acc == 0: zeros)
int gw_n(const SGeom& g, const GemmItems& it, hipStream_t st) {
  if (it.n == 0) return SRF_OK;
  if (use_mfma32(g.din, g.JD(), SdrGemm::kGw)) {
    const dim3 grid((g.JD() + 127) / 128, g.in_n(), it.n);
    if (g.din == 32)
      hipLaunchKernelGGL(sdr_gw32_kernel<32>, grid, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD());
    else
      hipLaunchKernelGGL(sdr_gw32_kernel<64>, grid, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD());
    SRF_LAUNCH_CHECK("sdr_gw32");
    return SRF_OK;
  }
  const int tasks = g.in_n() * g.NT();
  const dim3 grid((tasks + 3) / 4, 1, it.n);
#define SRF_GW(DIN) hipLaunchKernelGGL(sdr_gw_kernel<DIN>, grid, dim3(256), 0, st, it, g.N, g.lpad, g.in_n(), g.JD())
  switch (g.din) {
    case 8: SRF_GW(8); break;
    case 16: SRF_GW(16); break;
    case 32: SRF_GW(32); break;
    default: SRF_GW(64); break;
  }
#undef SRF_GW
  SRF_LAUNCH_CHECK("sdr_gw");
  return SRF_OK;
}

int gw_range(const SGeom& g, const float* gu, const float* emb, const FrameMap& fm, int accumulate, float* g_W,
             float* g_bias, hipStream_t st) {
  GemmItems it{};
  it.it[0] = GemmItem{gu, nullptr, emb, g_W, g_bias, accumulate, g.B * fm.nt, fm};
  it.n = (fm.nt > 0 || !accumulate) ? 1 : 0;
  return gw_n(g, it, st);
}

int transpose_w(const SGeom& g, const float* W, float* WT, float* zero, size_t n_zero, hipStream_t st) {
  const size_t total = (size_t)g.in_n() * g.JD() * g.din + n_zero;
  hipLaunchKernelGGL(sdr_transpose_w_kernel, dim3((total + 255) / 256), dim3(256), 0, st, W, g.in_n(), g.JD(), g.din,
                     WT, zero, n_zero);
  SRF_LAUNCH_CHECK("sdr_transpose_w");
  return SRF_OK;
}

// The stream recurrence (srf::sdr_stream_*) needs the forward's couplings: the
// whole-layer backward reruns its forward into cs (and a scratch v) first.
struct SdrBwdWs {
  float *u, *gu, *WT, *gstate, *cs, *v;
  size_t bytes;
};

size_t stream_cs_floats(const SGeom& g) {
  return srf::sdr_seq_supported(g.in_n(), g.J, g.dout, g.iters)
             ? 0
             : srf::sdr_stream_cs_floats(g.in_n(), g.J, g.dout, g.iters);
}

SdrBwdWs sdr_bwd_layout(const SGeom& g, void* base) {
  const size_t FU = (size_t)g.F() * g.in_n() * g.JD();
  size_t off = 0;
  auto take = [&](size_t nbytes) {
    size_t o = off;
    off += srf::align_up(nbytes, 256);
    return o;
  };
  const size_t ncs = stream_cs_floats(g);
  const size_t ou = take(FU * 4), ogu = take(FU * 4), owt = take((size_t)g.in_n() * g.JD() * g.din * 4),
               ogs = take(recur_workspace(g)), ocs = take((size_t)g.F() * ncs * 4),
               ov = take(ncs ? (size_t)g.F() * g.JD() * 4 : 0);
  char* b = static_cast<char*>(base);
  SdrBwdWs w;
  w.u = (float*)(b + ou);
  w.gu = (float*)(b + ogu);
  w.WT = (float*)(b + owt);
  w.gstate = (float*)(b + ogs);
  w.cs = ncs ? (float*)(b + ocs) : nullptr;
  w.v = ncs ? (float*)(b + ov) : nullptr;
  w.bytes = off;
  return w;
}

int range_ok(const SGeom& g, int t0, int t1, int v0, int vn) {
  SRF_REQUIRE(0 <= t0 && t0 <= t1 && t1 <= g.T, "frame range [%d, %d) outside [0, %d)", t0, t1, g.T);
  SRF_REQUIRE(t0 == t1 || (v0 <= t0 && t1 <= v0 + vn), "frame range [%d, %d) outside the buffer view [%d, %d)", t0,
              t1, v0, v0 + vn);
  return SRF_OK;
}

}  // namespace

extern "C" {

size_t srf_route_sdr_saved_floats(int B, int T, int J, int dout) { return (size_t)B * T * J * dout; }

size_t srf_route_sdr_fwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  return srf::align_up((size_t)B * T * N * (lpad + rpad + 1) * J * dout * sizeof(float), 256) +
         gstate_bytes(g, sdr_fwd_smem(g.in_n(), J, dout));
}

size_t srf_route_sdr_bwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, iters, 0};
  return sdr_bwd_layout(g, nullptr).bytes;
}

int srf_route_sdr_fwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                      int rpad, int J, int dout, int iters, int mask_first, float* v_out, float* saved,
                      void* workspace, size_t workspace_bytes, void* stream) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, iters, mask_first ? 1 : 0};
  int rc = check_sgeom(g);
  if (rc) return rc;
  SRF_REQUIRE(emb && W && bias && v_out && saved && workspace, "null pointer argument");
  if (workspace_bytes < srf_route_sdr_fwd_workspace(B, T, N, din, lpad, rpad, J, dout)) {
    srf::set_error("SDR forward workspace too small");
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* u = static_cast<float*>(workspace);
  float* gstate = u + srf::align_up((size_t)g.F() * g.in_n() * g.JD() * sizeof(float), 256) / sizeof(float);
  if ((rc = pose_range(g, emb, W, bias, frame_map(T, 0, T, 0, T), u, st))) return rc;
  if ((rc = recur_fwd_n(g, one_seq_item(srf::SeqItem{u, v_out, nullptr, nullptr, nullptr, gstate,
                                                     srf::SeqRange::whole(T)}), st)))
    return rc;
  SRF_HIP_TRY(hipMemcpyAsync(saved, v_out, (size_t)g.F() * g.JD() * sizeof(float), hipMemcpyDeviceToDevice, st));
  return SRF_OK;
}

int srf_route_sdr_bwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                      int rpad, int J, int dout, int iters, int mask_first, const float* saved, const float* g_v,
                      float* g_emb, float* g_W, float* g_bias, void* workspace, size_t workspace_bytes,
                      void* stream) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, iters, mask_first ? 1 : 0};
  int rc = check_sgeom(g);
  if (rc) return rc;
  SRF_REQUIRE(emb && W && bias && saved && g_v && g_emb && g_W && g_bias && workspace, "null pointer argument");
  const SdrBwdWs w = sdr_bwd_layout(g, workspace);
  if (workspace_bytes < w.bytes) {
    srf::set_error("SDR backward workspace too small");
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const FrameMap all = frame_map(T, 0, T, 0, T);
  if ((rc = pose_range(g, emb, W, bias, all, w.u, st))) return rc;
  if (w.cs && (rc = recur_fwd_n(g, one_seq_item(srf::SeqItem{w.u, w.v, nullptr, nullptr, w.cs, w.gstate,
                                                               srf::SeqRange::whole(T)}), st)))
    return rc;
  if ((rc = recur_bwd_n(g, one_seq_item(srf::SeqItem{w.u, const_cast<float*>(saved), g_v, w.gu, w.cs, w.gstate,
                                                     srf::SeqRange::whole(T)}), st)))
    return rc;
  if ((rc = transpose_w(g, W, w.WT, g_emb, (size_t)g.F() * N * din, st))) return rc;
  if ((rc = gx_range(g, w.gu, w.WT, all, g_emb, st))) return rc;
  return gw_range(g, w.gu, emb, all, 0, g_W, g_bias, st);
}

// ---- the same layer in frame ranges (the layer-pipelined SDR stack); the _n forms run
// up to SRF_SDR_MAX_ITEMS ranges of same-shaped layers in one launch
}  // extern "C"

namespace {

int items_ok(const SGeom& g, const srf_sdr_range* r, int n, bool use_u, bool use_g) {
  SRF_REQUIRE(r && n >= 0 && n <= SRF_SDR_MAX_ITEMS, "between 0 and %d ranges per launch, got %d", SRF_SDR_MAX_ITEMS,
              n);
  int rc;
  for (int k = 0; k < n; ++k) {
    if (use_u && (rc = range_ok(g, r[k].t0, r[k].t1, r[k].v0, r[k].vn))) return rc;
    if (use_g && (rc = range_ok(g, r[k].t0, r[k].t1, r[k].g0, r[k].gn))) return rc;
  }
  return SRF_OK;
}

srf::SeqItems seq_items(const srf_sdr_range* r, int n, int T, bool bwd, bool keep_cs) {
  srf::SeqItems it{};
  for (int k = 0; k < n; ++k) {
    if (r[k].t0 >= r[k].t1) continue;
    srf::SeqItem& I = it.it[it.n++];
    I.u = r[k].u;
    I.v = r[k].v;
    I.g_v = r[k].g_v;
    I.gu = r[k].gu;
    I.cs = keep_cs ? r[k].couplings : nullptr;
    I.ws = static_cast<float*>(r[k].workspace);
    I.rg = bwd ? srf::SeqRange{r[k].t0, r[k].t1, r[k].v0, r[k].vn, r[k].g0, r[k].gn, r[k].carry}
               : srf::SeqRange{r[k].t0, r[k].t1, r[k].v0, r[k].vn, 0, T, nullptr};
    I.u_bf16 = r[k].u_bf16;
    I.group = r[k].group;
    I.fact = bwd && I.cs != nullptr && r[k].gu_factored;
  }
  return it;
}

}  // namespace

extern "C" {

int srf_route_sdr_pose_n(const srf_sdr_range* r, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                         int dout, int fp8, void* stream) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  int rc = check_sgeom(g);
  if (rc || (rc = items_ok(g, r, n, true, false))) return rc;
  GemmItems it{};
  for (int k = 0; k < n; ++k) {
    if (r[k].t0 >= r[k].t1) continue;
    SRF_REQUIRE(r[k].emb && r[k].W && r[k].bias && r[k].u, "null pointer argument");
    it.it[it.n++] = GemmItem{r[k].emb, r[k].W, r[k].bias, r[k].u, nullptr, 0, B * (r[k].t1 - r[k].t0),
                             frame_map(T, r[k].t0, r[k].t1, r[k].v0, r[k].vn)};
  }
  SRF_REQUIRE(fp8 >= 0 && fp8 <= 2, "pose mode %d (0 fp32, 1 fp8, 2 fp8 with bf16 u)", fp8);
  return pose_n(g, it, static_cast<hipStream_t>(stream), fp8);
}

int srf_route_sdr_pose(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                       int rpad, int J, int dout, int t0, int t1, float* u, int v0, int vn, void* stream) {
  srf_sdr_range r{};
  r.t0 = t0, r.t1 = t1, r.emb = emb, r.W = W, r.bias = bias, r.u = u, r.v0 = v0, r.vn = vn;
  return srf_route_sdr_pose_n(&r, 1, B, T, N, din, lpad, rpad, J, dout, 0, stream);
}

int srf_route_sdr_pose_fp8(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                           int rpad, int J, int dout, int t0, int t1, float* u, int v0, int vn, void* stream) {
  srf_sdr_range r{};
  r.t0 = t0, r.t1 = t1, r.emb = emb, r.W = W, r.bias = bias, r.u = u, r.v0 = v0, r.vn = vn;
  return srf_route_sdr_pose_n(&r, 1, B, T, N, din, lpad, rpad, J, dout, 1, stream);
}

size_t srf_route_sdr_recur_workspace(int B, int in_n, int J, int dout, int iters) {
  SGeom g{B, 1, in_n, 8, 0, 0, J, dout, iters, 0};
  return recur_workspace(g);
}

size_t srf_route_sdr_recur_zero_range(int B, int in_n, int J, int dout, int iters, size_t* offset_bytes) {
  SGeom g{B, 1, in_n, 8, 0, 0, J, dout, iters, 0};
  size_t pre;
  if (srf::sdr_seq_supported(in_n, J, dout, iters)) {
    pre = 0;
  } else if (srf::sdr_stream_supported(in_n, J, dout, iters)) {
    pre = srf::sdr_stream_pre_floats(B, in_n, J, iters);
  } else {   // global-state kernels: the whole workspace, as before
    if (offset_bytes) *offset_bytes = 0;
    return recur_workspace(g);
  }
  if (offset_bytes) *offset_bytes = srf_grp::coff(pre) * sizeof(float);
  return (srf_grp::xoff(pre, B) - srf_grp::coff(pre)) * sizeof(float);
}

size_t srf_route_sdr_coupling_floats(int in_n, int J, int dout, int iters) {
  const size_t n = srf::sdr_seq_cs_floats(in_n, J, dout, iters);
  return n ? n : srf::sdr_stream_cs_floats(in_n, J, dout, iters);
}

size_t srf_route_sdr_fact_floats(int in_n, int J, int dout, int iters) {
  return srf::sdr_seq_fact_floats(in_n, J, dout, iters);
}

int srf_route_sdr_couplings_required(int in_n, int J, int dout, int iters) {
  return !srf::sdr_seq_supported(in_n, J, dout, iters) && srf::sdr_stream_supported(in_n, J, dout, iters);
}

int srf_route_sdr_recur_fwd_n(const srf_sdr_range* r, int n, int B, int T, int in_n, int J, int dout, int iters,
                              int mask_first, void* stream) {
  SGeom g{B, T, in_n, 8, 0, 0, J, dout, iters, mask_first ? 1 : 0};   // N = in_n, window 1: in_n() = in_n
  int rc = check_sgeom(g);
  if (rc || (rc = items_ok(g, r, n, true, false))) return rc;
  const size_t ws = recur_workspace(g);
  for (int k = 0; k < n; ++k) {
    SRF_REQUIRE(r[k].u && r[k].v, "null pointer argument");
    SRF_REQUIRE(r[k].workspace_bytes >= ws && (r[k].workspace || !ws), "SDR recurrence workspace too small");
  }
  return recur_fwd_n(g, seq_items(r, n, T, false, srf_route_sdr_coupling_floats(in_n, J, dout, iters) != 0),
                     static_cast<hipStream_t>(stream));
}

int srf_route_sdr_recur_fwd(const float* u, int v0, int vn, int B, int T, int in_n, int J, int dout, int iters,
                            int mask_first, int t0, int t1, float* v_out, float* couplings, void* workspace,
                            size_t workspace_bytes, void* stream) {
  srf_sdr_range r{};
  r.t0 = t0, r.t1 = t1, r.u = const_cast<float*>(u), r.v0 = v0, r.vn = vn, r.v = v_out, r.couplings = couplings;
  r.workspace = workspace, r.workspace_bytes = workspace_bytes;
  return srf_route_sdr_recur_fwd_n(&r, 1, B, T, in_n, J, dout, iters, mask_first, stream);
}

int srf_route_sdr_recur_bwd_n(const srf_sdr_range* r, int n, int B, int T, int in_n, int J, int dout, int iters,
                              int mask_first, void* stream) {
  SGeom g{B, T, in_n, 8, 0, 0, J, dout, iters, mask_first ? 1 : 0};
  int rc = check_sgeom(g);
  if (rc || (rc = items_ok(g, r, n, true, true))) return rc;
  const size_t ws = recur_workspace(g);
  for (int k = 0; k < n; ++k) {
    SRF_REQUIRE(r[k].u && r[k].v && r[k].g_v && r[k].carry && r[k].gu, "null pointer argument");
    SRF_REQUIRE(r[k].workspace_bytes >= ws && (r[k].workspace || !ws), "SDR recurrence workspace too small");
  }
  return recur_bwd_n(g, seq_items(r, n, T, true, srf_route_sdr_coupling_floats(in_n, J, dout, iters) != 0),
                     static_cast<hipStream_t>(stream));
}

int srf_route_sdr_recur_bwd(const float* u, int v0, int vn, const float* v_saved, const float* couplings,
                            const float* g_v, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                            int t0, int t1, float* carry, float* gu, int g0, int gn, void* workspace,
                            size_t workspace_bytes, void* stream) {
  srf_sdr_range r{};
  r.t0 = t0, r.t1 = t1, r.u = const_cast<float*>(u), r.v0 = v0, r.vn = vn, r.v = const_cast<float*>(v_saved);
  r.couplings = const_cast<float*>(couplings), r.g_v = g_v, r.carry = carry, r.gu = gu, r.g0 = g0, r.gn = gn;
  r.workspace = workspace, r.workspace_bytes = workspace_bytes;
  return srf_route_sdr_recur_bwd_n(&r, 1, B, T, in_n, J, dout, iters, mask_first, stream);
}

int srf_route_sdr_transpose_w(const float* W, int in_n, int J, int dout, int din, float* WT, void* stream) {
  SRF_REQUIRE(W && WT && in_n > 0 && J > 0 && dout > 0 && din > 0, "bad transpose arguments");
  SGeom g{1, 1, in_n, din, 0, 0, J, dout, 1, 0};
  return transpose_w(g, W, WT, nullptr, 0, static_cast<hipStream_t>(stream));
}

int srf_route_sdr_gx_n(const srf_sdr_range* r, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                       int dout, void* stream) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  int rc = check_sgeom(g);
  if (rc || (rc = items_ok(g, r, n, false, true))) return rc;
  GemmItems it{};
  for (int k = 0; k < n; ++k) {
    if (r[k].t0 >= r[k].t1) continue;
    SRF_REQUIRE(r[k].gu && r[k].WT && r[k].g_emb, "null pointer argument");
    it.it[it.n++] = GemmItem{r[k].gu, r[k].WT, nullptr, r[k].g_emb, nullptr, 0, B * (r[k].t1 - r[k].t0),
                             frame_map(T, r[k].t0, r[k].t1, r[k].g0, r[k].gn)};
  }
  return gx_n(g, it, static_cast<hipStream_t>(stream));
}

int srf_route_sdr_gx(const float* gu, int g0, int gn, const float* WT, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int t0, int t1, float* g_emb, void* stream) {
  srf_sdr_range r{};
  r.t0 = t0, r.t1 = t1, r.gu = const_cast<float*>(gu), r.g0 = g0, r.gn = gn, r.WT = WT, r.g_emb = g_emb;
  return srf_route_sdr_gx_n(&r, 1, B, T, N, din, lpad, rpad, J, dout, stream);
}

int srf_route_sdr_gw_n(const srf_sdr_range* r, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                       int dout, void* stream) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  int rc = check_sgeom(g);
  if (rc || (rc = items_ok(g, r, n, false, true))) return rc;
  GemmItems it{};
  for (int k = 0; k < n; ++k) {
    if (r[k].t0 >= r[k].t1 && r[k].accumulate) continue;   // an empty range still starts the sum
    SRF_REQUIRE(r[k].gu && r[k].emb && r[k].g_W && r[k].g_bias, "null pointer argument");
    it.it[it.n++] = GemmItem{r[k].gu, nullptr, r[k].emb, r[k].g_W, r[k].g_bias, r[k].accumulate,
                             B * (r[k].t1 - r[k].t0), frame_map(T, r[k].t0, r[k].t1, r[k].g0, r[k].gn)};
  }
  return gw_n(g, it, static_cast<hipStream_t>(stream));
}

int srf_route_sdr_gw(const float* gu, int g0, int gn, const float* emb, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int t0, int t1, int accumulate, float* g_W, float* g_bias,
                     void* stream) {
  srf_sdr_range r{};
  r.t0 = t0, r.t1 = t1, r.gu = const_cast<float*>(gu), r.g0 = g0, r.gn = gn, r.emb = emb, r.g_W = g_W;
  r.g_bias = g_bias, r.accumulate = accumulate;
  return srf_route_sdr_gw_n(&r, 1, B, T, N, din, lpad, rpad, J, dout, stream);
}

int srf_route_sdr_gx_gw_n(const srf_sdr_range* r, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                          int dout, void* stream) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  int rc = check_sgeom(g);
  if (rc || (rc = items_ok(g, r, n, false, true))) return rc;
  if (!gxw_supported(g)) {   // the two contractions' own kernels
    if ((rc = srf_route_sdr_gx_n(r, n, B, T, N, din, lpad, rpad, J, dout, stream))) return rc;
    return srf_route_sdr_gw_n(r, n, B, T, N, din, lpad, rpad, J, dout, stream);
  }
  for (int k = 0; k < n; ++k)
    SRF_REQUIRE(!r[k].gu_factored, "gx_gw_n: gu factors go through srf_route_sdr_gx_gw_fact_n");
  GxwItems it{};
  for (int k = 0; k < n; ++k) {
    if (r[k].t0 >= r[k].t1 && r[k].accumulate) continue;   // an empty range still starts the sum
    SRF_REQUIRE(r[k].gu && r[k].W && r[k].emb && r[k].g_emb && r[k].g_W && r[k].g_bias, "null pointer argument");
    it.it[it.n++] = GxwItem{r[k].gu, r[k].W, r[k].emb, r[k].g_emb, r[k].g_W, r[k].g_bias, r[k].accumulate,
                            B * std::max(0, r[k].t1 - r[k].t0), frame_map(T, r[k].t0, r[k].t1, r[k].g0, r[k].gn)};
  }
  return gxw_n(g, it, static_cast<hipStream_t>(stream));
}

int srf_route_sdr_gx_gw_fact_n(const srf_sdr_range* r, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                               int dout, int iters, void* stream) {
  SGeom g{B, T, N, din, lpad, rpad, J, dout, iters, 0};
  int rc = check_sgeom(g);
  if (rc || (rc = items_ok(g, r, n, false, true))) return rc;
  SRF_REQUIRE(gxwf_supported(g), "gu factors: din = dout = 32, J a multiple of 16, iters <= 3 (din=%d dout=%d J=%d iters=%d)",
              g.din, g.dout, g.J, iters);
  const size_t FF = srf::sdr_seq_fact_floats(g.in_n(), J, dout, iters);
  GxwfItems it{};
  for (int k = 0; k < n; ++k) {
    if (r[k].t0 >= r[k].t1 && r[k].accumulate) continue;   // an empty range still starts the sum
    SRF_REQUIRE(r[k].gu && r[k].couplings && r[k].W && r[k].emb && r[k].g_emb && r[k].g_W && r[k].g_bias,
                "null pointer argument");
    SRF_REQUIRE((size_t)B * r[k].gn * FF * 4 < 0x7FFFFF00u, "gu factors above 2 GiB per range buffer");
    SRF_REQUIRE((size_t)B * T * srf::sdr_seq_cs_floats(g.in_n(), J, dout, iters) < 0x7FFFFFFFu,
                "couplings above 2^31 floats");
    it.it[it.n++] = GxwfItem{r[k].couplings, r[k].gu, r[k].W, r[k].emb, r[k].g_emb, r[k].g_W, r[k].g_bias,
                             r[k].accumulate, B * std::max(0, r[k].t1 - r[k].t0),
                             frame_map(T, r[k].t0, r[k].t1, r[k].g0, r[k].gn)};
  }
  return gxwf_n(g, it, static_cast<hipStream_t>(stream));
}

}  // extern "C"
