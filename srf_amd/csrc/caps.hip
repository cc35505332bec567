// Capsule-side glue of SequenceRouter.call (sequence_router_naive.py:129-193):
// primary capsules, the per-layer LayerNorm + dropout, and the output head.
//
//   proj        e[f][p] = X[f][:] . Wp[:, p] + bp[p]                   (:131-132)
//   encaps      m = mask4(max(drop(conv3x3_1(e)), drop(conv3x3_2(e))))  (:133-135)
//               z = drop_in(LN_in(squash_PD(m)))                        (:137-142)
//   capsnorm    y = drop_mid(LN_mid(v)) between routing layers          (:187-191)
//   head        logits = LN_out(length_D(drop_mid(LN_mid(v))))          (:187-193)
// Every per-frame kernel is one 256-thread workgroup per frame (B*T' of them);
// the frame's vector lives in LDS, reductions are wave shuffles + LDS.
#include <algorithm>
#include <cmath>

#include "srf_common.h"
#include "srf_reduce.h"
#include "srf_rng.h"
#include "../../include/srf.h"

namespace {

constexpr float kSquashEps = 1e-7f;
constexpr float kLengthEps = 1e-7f;
constexpr float kLnEps = 1e-3f;
constexpr int kMaxVec = 4096;   // max per-frame vector (J*D or PH*PD) held in LDS

__device__ __forceinline__ int ceil_div_len(int len, int div) { return (len + div - 1) / div; }

// Sum of (a, b) over a 256-thread block; every thread gets the totals.
__device__ __forceinline__ void block_sum2(float& a, float& b, float* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) {
    red[w] = a;
    red[4 + w] = b;
  }
  __syncthreads();
  a = red[0] + red[1] + red[2] + red[3];
  b = red[4] + red[5] + red[6] + red[7];
}

__device__ __forceinline__ float drop_mult(bool on, unsigned long long seed, unsigned stream, size_t idx, float p) {
  if (!on) return 1.f;
  return srf_keep(seed, stream, idx, p) ? 1.f / (1.f - p) : 0.f;
}

// get_pos_enc (model_helper.py:30-58), evaluated in float32 like the reference:
// columns [0, PH/2) are sin(t * inv_k), [PH/2, PH) cos(t * inv_k), with
// inv_k = exp(-k * log(1e4) / (PH/2 - 1)).
__device__ __forceinline__ float pos_enc(int t, int p, int PH) {
  const int nts = PH >> 1;
  const float inc = 9.210340371976184f / (float)(nts - 1);
  const int k = p < nts ? p : p - nts;
  const float st = (float)t * expf((float)k * -inc);
  return p < nts ? sinf(st) : cosf(st);
}

// Epilogue of the projection: e = (x W + b) * scale (+ pos_enc) -- the einsum
// variant's sqrt(PH) scaling and positional encoding (sequence_router_einsum.py:129-131);
// scale = 1 and no encoding for naive / lowmemory.
__device__ __forceinline__ float proj_epilogue(float acc, int f, int T, int p, int PH, float scale, int pe) {
  const float y = acc * scale;
  return pe ? y + pos_enc(f % T, p, PH) : y;
}

// ---------------------------------------------------------------- proj
// One wave per frame, outputs in groups of 8; the K loop is unrolled 4x with
// independent loads so the wave keeps several row segments in flight.
__global__ __launch_bounds__(256) void proj_fwd_kernel(const float* __restrict__ X, int F, int K, int PH,
                                                       const float* __restrict__ Wp, const float* __restrict__ bp,
                                                       float* __restrict__ e, int T, float scale, int pe) {
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (f >= F) return;
  const float* x = X + (size_t)f * K;
  for (int p0 = 0; p0 < PH; p0 += 8) {
    const int np = min(8, PH - p0);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
#pragma unroll 4
    for (int k = l; k < K; k += 64) {
      const float xv = x[k];
      const float* w = Wp + (size_t)k * PH + p0;
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += xv * (q < np ? w[q < np ? q : 0] : 0.f);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float s = wave_sum(acc[q]);
      if (l == 0 && q < np) e[(size_t)f * PH + p0 + q] = proj_epilogue(s + bp[p0 + q], f, T, p0 + q, PH, scale, pe);
    }
  }
}

// Vectorised forms for PH in {4, 8, 16} (K % 256 == 0 is not required, K % 4 == 0 is):
// a wave owns FW frames; lane l covers k = 4l + 256j, reading X and the Wp rows as
// float4, so each Wp row fetched serves FW frames.
template <int PH, int FW>
__global__ __launch_bounds__(256) void proj_fwd_vec_kernel(const float* __restrict__ X, int F, int K,
                                                           const float* __restrict__ Wp,
                                                           const float* __restrict__ bp, float* __restrict__ e,
                                                           int T, float scale, int pe) {
  constexpr int PQ = PH / 4;
  const int l = threadIdx.x & 63;
  const int f0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * FW;
  if (f0 >= F) return;
  float acc[FW][PH];
#pragma unroll
  for (int u = 0; u < FW; ++u)
#pragma unroll
    for (int p = 0; p < PH; ++p) acc[u][p] = 0.f;
#pragma unroll 2
  for (int k0 = 4 * l; k0 < K; k0 += 256) {
    f4 x[FW], w[4][PQ];
#pragma unroll
    for (int u = 0; u < FW; ++u) x[u] = *reinterpret_cast<const f4*>(X + (size_t)min(f0 + u, F - 1) * K + k0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int q = 0; q < PQ; ++q) w[kk][q] = *reinterpret_cast<const f4*>(Wp + (size_t)(k0 + kk) * PH + 4 * q);
#pragma unroll
    for (int u = 0; u < FW; ++u)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int p = 0; p < PH; ++p) acc[u][p] += x[u][kk] * w[kk][p >> 2][p & 3];
  }
#pragma unroll
  for (int u = 0; u < FW; ++u)
#pragma unroll
    for (int p = 0; p < PH; ++p) {
      const float sum = wave_sum(acc[u][p]);
      if (l == 0 && f0 + u < F) e[(size_t)(f0 + u) * PH + p] = proj_epilogue(sum + bp[p], f0 + u, T, p, PH, scale, pe);
    }
}

// e[f][p] = proj(X[f] . Wp[:, p] + bp[p]) on v_mfma_f32_16x16x4_f32 (exact fp32): a
// workgroup = one 16-frame tile, its 16 waves split K (kProjKq each, in steps of 16:
// lane (m = l & 15, g = l >> 4) feeds X[f0 + m][k + 4g + j] and Wp[k + 4g + j][n] to
// MFMA j), then the 16 partial tiles are summed through LDS in a fixed order.
constexpr int kProjWaves = 16;
template <int PH>
__global__ __launch_bounds__(64 * kProjWaves) void proj_fwd_mfma_kernel(const float* __restrict__ X, int F, int K,
                                                                       const float* __restrict__ Wp,
                                                                       const float* __restrict__ bp,
                                                                       float* __restrict__ e, int T, float scale,
                                                                       int pe, int Kq) {
  static_assert(PH <= 16, "one 16-column output tile");
  __shared__ float part[kProjWaves][16][17];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int m = lane & 15, g = lane >> 4;
  const int f0 = blockIdx.x * 16;
  const int fm = min(f0 + m, F - 1);
  const bool fok = f0 + m < F;
  const int kb = wv * Kq, ke = min(K, kb + Kq);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int U = 4;   // k-steps of 16 in flight
  for (int k0 = kb; k0 < ke; k0 += 16 * U) {
    f4 xa[U];
    float wb[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 16 * u + 4 * g;
      const bool kok = k < ke;   // K % 4 == 0: whole float4s
      const f4 x = *reinterpret_cast<const f4*>(X + (size_t)fm * K + (kok ? k : kb));
      xa[u] = (fok && kok) ? x : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float w = Wp[(size_t)(kok ? k + j : kb) * PH + min(m, PH - 1)];
        wb[u][j] = (kok && m < PH) ? w : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma16x16x4(xa[u][j], wb[u][j], acc);
  }
  // C: lane column n = m (output p), rows 4g + v (frames)
#pragma unroll
  for (int v = 0; v < 4; ++v) part[wv][4 * g + v][m] = acc[v];
  __syncthreads();
  if (threadIdx.x < 16 * PH) {
    const int r = threadIdx.x / PH, pp = threadIdx.x % PH;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < kProjWaves; ++w) sum += part[w][r][pp];
    if (f0 + r < F) e[(size_t)(f0 + r) * PH + pp] = proj_epilogue(sum + bp[pp], f0 + r, T, pp, PH, scale, pe);
  }
}

// g_X[f][k..k+3] = sum_p g_e[f][p] Wp[k..k+3][p]: a thread writes one float4 of g_X for
// kProjXF consecutive frames, so the Wp rows it loads serve them all.
constexpr int kProjXF = 16;
template <int PH>
__global__ __launch_bounds__(256) void proj_bwd_x_vec_kernel(const float* __restrict__ g_e,
                                                             const float* __restrict__ Wp, int F, int K,
                                                             float* __restrict__ g_X) {
  constexpr int PQ = PH / 4;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int K4 = K / 4;
  const int FG = (F + kProjXF - 1) / kProjXF;
  if (idx >= (size_t)FG * K4) return;
  const int fg = (int)(idx / K4);
  const int k0 = (int)(idx - (size_t)fg * K4) * 4;
  f4 w[4][PQ];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int q = 0; q < PQ; ++q) w[kk][q] = *reinterpret_cast<const f4*>(Wp + (size_t)(k0 + kk) * PH + 4 * q);
#pragma unroll
  for (int u = 0; u < kProjXF; ++u) {
    const int f = fg * kProjXF + u;
    if (f >= F) break;
    f4 ge[PQ];
#pragma unroll
    for (int q = 0; q < PQ; ++q) ge[q] = *reinterpret_cast<const f4*>(g_e + (size_t)f * PH + 4 * q);
    f4 out;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      float sacc = 0.f;
#pragma unroll
      for (int q = 0; q < PQ; ++q)
        sacc += (w[kk][q].x * ge[q].x + w[kk][q].y * ge[q].y) + (w[kk][q].z * ge[q].z + w[kk][q].w * ge[q].w);
      out[kk] = sacc;
    }
    *reinterpret_cast<f4*>(g_X + (size_t)f * K + k0) = out;
  }
}

// g_X[f][k] = sum_p g_e[f][p] Wp[k][p]
__global__ void proj_bwd_x_kernel(const float* __restrict__ g_e, const float* __restrict__ Wp, int F, int K, int PH,
                                  float* __restrict__ g_X) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= F * K) return;
  const int k = idx % K;
  const int f = idx / K;
  float s = 0.f;
  for (int p = 0; p < PH; ++p) s += g_e[f * PH + p] * Wp[(size_t)k * PH + p];
  g_X[idx] = s;
}

// part[chunk][k*PH + p] = sum_{f in chunk} X[f][k] g_e[f][p]; row K*PH holds the bias partials.
__global__ void proj_bwd_w_kernel(const float* __restrict__ X, const float* __restrict__ g_e, int F, int K, int PH,
                                  int fchunk, float* __restrict__ part) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int ch = blockIdx.y;
  const int f0 = ch * fchunk, f1 = min(F, f0 + fchunk);
  const int cols = K * PH + PH;
  if (k < K) {
    // 16 outputs per pass: X is read once for PH <= 16 (the C2-C5 widths)
    for (int p0 = 0; p0 < PH; p0 += 16) {
      float acc[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.f;
      // frames in batches of 8: the batch's X loads are in flight together
      for (int fb = f0; fb < f1; fb += 8) {
        float xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) xv[u] = X[(size_t)min(fb + u, f1 - 1) * K + k];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (fb + u >= f1) break;
#pragma unroll
          for (int q = 0; q < 16; ++q)
            if (p0 + q < PH) acc[q] += xv[u] * g_e[(size_t)(fb + u) * PH + p0 + q];
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (p0 + q < PH) part[(size_t)ch * cols + (size_t)k * PH + p0 + q] = acc[q];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < PH) {
    float s = 0.f;
    for (int f = f0; f < f1; ++f) s += g_e[(size_t)f * PH + threadIdx.x];
    part[(size_t)ch * cols + (size_t)K * PH + threadIdx.x] = s;
  }
}

// The same partials on v_mfma_f32_16x16x4_f32 (PH <= 16): part^T[k][p] = X^T[k][f] g_e[f][p]
// with K = frames.  Wave = 16 rows k x the PH columns p over the chunk's frames, four per
// MFMA (A: lane l holds X[f0 + (l >> 4)][k0 + (l & 15)], 64-byte row pieces; B: g_e[f0 +
// (l >> 4)][l & 15]); eight K steps' loads in flight per batch.  fp32 products and
// accumulation, as the VALU kernel (the sums reassociate).
__global__ __launch_bounds__(256) void proj_bwd_w_mfma_kernel(const float* __restrict__ X,
                                                              const float* __restrict__ g_e, int F, int K, int PH,
                                                              int fchunk, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ch = blockIdx.y;
  const int k0 = (blockIdx.x * 4 + wv) * 16;
  const int f0 = ch * fchunk, f1 = min(F, f0 + fchunk);
  const int cols = K * PH + PH;
  const int kr = k0 + (lane & 15), fq = lane >> 4, pc = lane & 15;
  const bool kok = kr < K, pok = pc < PH;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  if (k0 < K) {
    constexpr int U = 8;   // K steps per batch
    for (int fb = f0; fb < f1; fb += 4 * U) {
      float a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int f = fb + 4 * u + fq;
        const bool ok = f < f1;
        const int fc = ok ? f : f0;
        const float av = X[(size_t)fc * K + (kok ? kr : 0)];
        const float bv = g_e[(size_t)fc * PH + (pok ? pc : 0)];
        a[u] = ok && kok ? av : 0.f;
        b[u] = ok && pok ? bv : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc = mfma16x16x4(a[u], b[u], acc);
    }
    // C: lane l holds column p = l & 15 of rows k0 + 4 (l >> 4) + 0..3
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 4 * fq + r;
      if (k < K && pok) part[(size_t)ch * cols + (size_t)k * PH + pc] = acc[r];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < PH) {
    float s = 0.f;
    for (int f = f0; f < f1; ++f) s += g_e[(size_t)f * PH + threadIdx.x];
    part[(size_t)ch * cols + (size_t)K * PH + threadIdx.x] = s;
  }
}

// ---------------------------------------------------------------- encaps
struct CapsDims {
  int B, T, PH, PD;   // T = T' frames per utterance
};

__device__ __forceinline__ float encaps_conv(const float* __restrict__ e3, int PH, int p, int d,
                                             const float* __restrict__ K, float bias, int PD) {
  // e3: 3 x PH neighbourhood in LDS (rows t-1, t, t+1; zero when outside [0,T))
  float v = bias;
#pragma unroll
  for (int dt = 0; dt < 3; ++dt)
#pragma unroll
    for (int dp = 0; dp < 3; ++dp) {
      const int pp = p + dp - 1;
      if (pp >= 0 && pp < PH) v += e3[dt * PH + pp] * K[(dt * 3 + dp) * PD + d];
    }
  return v;
}

__device__ __forceinline__ void load_e3(const float* __restrict__ e, int f, const CapsDims& cd, float* e3) {
  const int t = f % cd.T;
  for (int i = threadIdx.x; i < 3 * cd.PH; i += blockDim.x) {
    const int dt = i / cd.PH, p = i - dt * cd.PH;
    const int tt = t + dt - 1;
    e3[i] = (tt >= 0 && tt < cd.T) ? e[(size_t)(f + dt - 1) * cd.PH + p] : 0.f;
  }
}

// Per-frame squash factors over PD for every p (m in LDS), written to fac[p].
__device__ __forceinline__ void squash_factors(const float* m, int PH, int PD, float* fac, float* n2s) {
  for (int p = threadIdx.x; p < PH; p += blockDim.x) {
    float n2 = 0.f;
    for (int d = 0; d < PD; ++d) n2 += m[p * PD + d] * m[p * PD + d];
    fac[p] = n2 / (1.f + n2) / sqrtf(n2 + kSquashEps);
    n2s[p] = n2;
  }
}

__global__ __launch_bounds__(256) void encaps_fwd_kernel(
    const float* __restrict__ e, const int* __restrict__ inp_len, CapsDims cd, const float* __restrict__ K1,
    const float* __restrict__ b1, const float* __restrict__ K2, const float* __restrict__ b2,
    const float* __restrict__ gamma, const float* __restrict__ beta, int training, float p_caps, float p_in,
    unsigned long long seed, const unsigned long long* __restrict__ seed_src, float* __restrict__ m_out, unsigned char* __restrict__ sel,
    float* __restrict__ lnstat, float* __restrict__ z) {
  seed = srf_step_seed(seed, seed_src);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int E = cd.PH * cd.PD;
  float* m = sm;                 // E
  float* e3 = m + E;             // 3*PH
  float* fac = e3 + 3 * cd.PH;   // PH
  float* n2s = fac + cd.PH;      // PH
  float* red = n2s + cd.PH;      // 8
  const int f = blockIdx.x;
  const int b = f / cd.T, t = f - b * cd.T;
  const bool valid_t = t < ceil_div_len(inp_len[b], 4);
  load_e3(e, f, cd, e3);
  __syncthreads();
  for (int i = threadIdx.x; i < E; i += blockDim.x) {
    const int p = i / cd.PD, d = i - p * cd.PD;
    const size_t gi = (size_t)f * E + i;
    const float v1 = encaps_conv(e3, cd.PH, p, d, K1, b1[d], cd.PD) *
                     drop_mult(training && p_caps > 0.f, seed, kStreamEncaps1, gi, p_caps);
    const float v2 = encaps_conv(e3, cd.PH, p, d, K2, b2[d], cd.PD) *
                     drop_mult(training && p_caps > 0.f, seed, kStreamEncaps2, gi, p_caps);
    const bool s = v1 >= v2;
    const float mv = valid_t ? (s ? v1 : v2) : 0.f;
    m[i] = mv;
    m_out[gi] = mv;
    sel[gi] = s ? 1 : 0;
  }
  __syncthreads();
  squash_factors(m, cd.PH, cd.PD, fac, n2s);
  __syncthreads();
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < E; i += blockDim.x) {
    const float sq = m[i] * fac[i / cd.PD];
    s1 += sq;
  }
  float dummy = 0.f;
  block_sum2(s1, dummy, red);
  const float mean = s1 / E;
  for (int i = threadIdx.x; i < E; i += blockDim.x) {
    const float dv = m[i] * fac[i / cd.PD] - mean;
    s2 += dv * dv;
  }
  dummy = 0.f;
  block_sum2(s2, dummy, red);
  const float rstd = 1.f / sqrtf(s2 / E + kLnEps);
  for (int i = threadIdx.x; i < E; i += blockDim.x) {
    const size_t gi = (size_t)f * E + i;
    const float y = (m[i] * fac[i / cd.PD] - mean) * rstd * gamma[i] + beta[i];
    z[gi] = y * drop_mult(training && p_in > 0.f, seed, kStreamInput, gi, p_in);
  }
  if (threadIdx.x == 0) {
    lnstat[2 * f] = mean;
    lnstat[2 * f + 1] = rstd;
  }
}

// squash backward for one capsule: gs = g*gv + 2 g'(n2) (s.gv) s, element d.
__device__ __forceinline__ float squash_bwd_elem(float s_d, float gv_d, float n2, float sdotg) {
  const float rs = 1.f / sqrtf(n2 + kSquashEps);
  const float ip = 1.f / (1.f + n2);
  const float gfac = n2 * ip * rs;
  const float dg = rs * ip * (ip - 0.5f * n2 / (n2 + kSquashEps));
  return gfac * gv_d + 2.f * dg * sdotg * s_d;
}

// Backward part A (per frame): through input dropout, LN_in, squash, mask,
// maxout and encaps dropout to the two conv outputs g_v1, g_v2; LN gamma/beta
// and encaps kernel/bias gradient partials per frame:
//   wpart[f][0 .. 2E)                 g_gamma_in, g_beta_in contributions
//   wpart[f][2E + k*10*PD + tap*PD+d] g_K_k  (tap 9 = bias)
__global__ __launch_bounds__(256) void encaps_bwd_a_kernel(
    const float* __restrict__ g_z, const float* __restrict__ e, const float* __restrict__ m_in,
    const unsigned char* __restrict__ sel, const float* __restrict__ lnstat, const int* __restrict__ inp_len,
    CapsDims cd, const float* __restrict__ gamma, const float* __restrict__ beta, int training, float p_caps,
    float p_in, unsigned long long seed, const unsigned long long* __restrict__ seed_src, float* __restrict__ g_v1, float* __restrict__ g_v2,
    float* __restrict__ wpart) {
  seed = srf_step_seed(seed, seed_src);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int E = cd.PH * cd.PD;
  float* m = sm;                 // E
  float* gs = m + E;             // E   (grad wrt squash output, then wrt m)
  float* gv = gs + E;            // 2E  (g_v1, g_v2 for the wgrad partials)
  float* e3 = gv + 2 * E;        // 3*PH
  float* fac = e3 + 3 * cd.PH;   // PH
  float* n2s = fac + cd.PH;      // PH
  float* sdg = n2s + cd.PH;      // PH
  float* red = sdg + cd.PH;      // 8
  const int f = blockIdx.x;
  const int b = f / cd.T, t = f - b * cd.T;
  const bool valid_t = t < ceil_div_len(inp_len[b], 4);
  const float mean = lnstat[2 * f], rstd = lnstat[2 * f + 1];
  for (int i = threadIdx.x; i < E; i += blockDim.x) m[i] = m_in[(size_t)f * E + i];
  load_e3(e, f, cd, e3);
  __syncthreads();
  squash_factors(m, cd.PH, cd.PD, fac, n2s);
  __syncthreads();
  // LN backward: gy = g_z * drop; xh = (s - mean) * rstd
  float a1 = 0.f, a2 = 0.f;
  for (int i = threadIdx.x; i < E; i += blockDim.x) {
    const size_t gi = (size_t)f * E + i;
    const float gy = g_z[gi] * drop_mult(training && p_in > 0.f, seed, kStreamInput, gi, p_in);
    const float xh = (m[i] * fac[i / cd.PD] - mean) * rstd;
    wpart[(size_t)f * (2 * E + 20 * cd.PD) + i] = gy * xh;       // g_gamma
    wpart[(size_t)f * (2 * E + 20 * cd.PD) + E + i] = gy;        // g_beta
    const float gx = gy * gamma[i];
    gs[i] = gx;
    a1 += gx;
    a2 += gx * xh;
  }
  block_sum2(a1, a2, red);
  for (int i = threadIdx.x; i < E; i += blockDim.x) {
    const float xh = (m[i] * fac[i / cd.PD] - mean) * rstd;
    gs[i] = rstd * (gs[i] - a1 / E - xh * a2 / E);
  }
  __syncthreads();
  for (int p = threadIdx.x; p < cd.PH; p += blockDim.x) {
    float sg = 0.f;
    for (int d = 0; d < cd.PD; ++d) sg += m[p * cd.PD + d] * gs[p * cd.PD + d];
    sdg[p] = sg;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < E; i += blockDim.x) {
    const int p = i / cd.PD;
    const size_t gi = (size_t)f * E + i;
    float gm = valid_t ? squash_bwd_elem(m[i], gs[i], n2s[p], sdg[p]) : 0.f;
    const bool s = sel[gi] != 0;
    const float g1 = (s ? gm : 0.f) * drop_mult(training && p_caps > 0.f, seed, kStreamEncaps1, gi, p_caps);
    const float g2 = (s ? 0.f : gm) * drop_mult(training && p_caps > 0.f, seed, kStreamEncaps2, gi, p_caps);
    g_v1[gi] = g1;
    g_v2[gi] = g2;
    gv[i] = g1;
    gv[E + i] = g2;
  }
  __syncthreads();
  // kernel/bias partials: out j = (k, tap, d), tap 9 = bias
  for (int j = threadIdx.x; j < 20 * cd.PD; j += blockDim.x) {
    const int k = j / (10 * cd.PD);
    const int tap = (j / cd.PD) % 10, d = j % cd.PD;
    const float* g = gv + k * E;
    float s = 0.f;
    if (tap == 9) {
      for (int p = 0; p < cd.PH; ++p) s += g[p * cd.PD + d];
    } else {
      const int dt = tap / 3, dp = tap % 3;
      for (int p = 0; p < cd.PH; ++p) {
        const int pp = p + dp - 1;
        if (pp >= 0 && pp < cd.PH) s += g[p * cd.PD + d] * e3[dt * cd.PH + pp];
      }
    }
    wpart[(size_t)f * (2 * E + 20 * cd.PD) + 2 * E + j] = s;
  }
}

// Backward part B: g_e[t'][p'] = sum_{k,dt,dp,d} g_vk[t'-dt+1][p'-dp+1][d] K_k[dt][dp][d].
// 16 lanes per output (f, p'): lane q takes d = q, q+16, ... (coalesced along d), and
// the 16 partial sums meet in an xor butterfly.
constexpr int kEbLanes = 16;
__global__ __launch_bounds__(256) void encaps_bwd_b_kernel(const float* __restrict__ g_v1,
                                                           const float* __restrict__ g_v2, CapsDims cd,
                                                           const float* __restrict__ K1,
                                                           const float* __restrict__ K2, float* __restrict__ g_e,
                                                           float scale) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int idx = gid / kEbLanes, q = gid % kEbLanes;
  const int F = cd.B * cd.T;
  const bool live = idx < F * cd.PH;   // the whole 16-lane group agrees
  const int p = live ? idx % cd.PH : 0, f = live ? idx / cd.PH : 0;
  const int t = f % cd.T;
  const int E = cd.PH * cd.PD;
  float s = 0.f;
  if (live) {
    for (int dt = 0; dt < 3; ++dt) {
      const int tt = t - dt + 1;
      if (tt < 0 || tt >= cd.T) continue;
      const size_t fo = (size_t)(f - dt + 1) * E;
      for (int dp = 0; dp < 3; ++dp) {
        const int pp = p - dp + 1;
        if (pp < 0 || pp >= cd.PH) continue;
        for (int d = q; d < cd.PD; d += kEbLanes)
          s += g_v1[fo + pp * cd.PD + d] * K1[(dt * 3 + dp) * cd.PD + d] +
               g_v2[fo + pp * cd.PD + d] * K2[(dt * 3 + dp) * cd.PD + d];
      }
    }
  }
#pragma unroll
  for (int o = kEbLanes / 2; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (live && q == 0) g_e[idx] = s * scale;   // through the einsum variant's sqrt(PH) scaling (1 otherwise)
}

// ---------------------------------------------------------------- LN + dropout
// Frames of a row map: workgroup q handles row f = b*T + t0 + (q - b*nt), b = q / nt
// (frames [t0, t0 + nt) of every utterance; {T, 0, T} is every row, f = q).
struct RowMap {
  int T, t0, nt;
  __device__ __forceinline__ int row(int q) const {
    const int b = q / nt;
    return b * T + t0 + (q - b * nt);
  }
  static RowMap all(int F) { return RowMap{F, 0, F}; }
};

// y = drop(LN(x)) over vectors of length n (one frame per workgroup); also the
// output head: logits = LN_out(length_D(drop(LN_mid(v)))) when head != 0.
__device__ __forceinline__ void capsnorm_fwd_row(const float* __restrict__ x, int n, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, int training, float p,
                                                 unsigned long long seed, const unsigned long long* __restrict__ seed_src,
                                                 unsigned stream, float* __restrict__ y, float* __restrict__ stat,
                                                 int head, int J, int D, const float* __restrict__ gamma_o,
                                                 const float* __restrict__ beta_o, float* __restrict__ logits,
                                                 float* __restrict__ lens, float len_eps, int f) {
  seed = srf_step_seed(seed, seed_src);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* v = sm;           // n
  float* red = v + n;      // 8
  float s1 = 0.f, dummy = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float a = x[(size_t)f * n + i];
    v[i] = a;
    s1 += a;
  }
  block_sum2(s1, dummy, red);
  const float mean = s1 / n;
  float s2 = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float dv = v[i] - mean;
    s2 += dv * dv;
  }
  dummy = 0.f;
  block_sum2(s2, dummy, red);
  const float rstd = 1.f / sqrtf(s2 / n + kLnEps);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const size_t gi = (size_t)f * n + i;
    const float o = ((v[i] - mean) * rstd * gamma[i] + beta[i]) * drop_mult(training && p > 0.f, seed, stream, gi, p);
    v[i] = o;
    if (!head) y[gi] = o;
  }
  if (threadIdx.x == 0) {
    stat[4 * f] = mean;
    stat[4 * f + 1] = rstd;
  }
  if (!head) return;
  __syncthreads();
  // length over D (naive:255-258), then LN_out over the J capsules
  float* L = v + n + 8;   // J
  for (int j = threadIdx.x; j < J; j += blockDim.x) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s += v[j * D + d] * v[j * D + d];
    L[j] = sqrtf(s + len_eps);
    lens[(size_t)f * J + j] = L[j];
  }
  __syncthreads();
  float t1 = 0.f;
  dummy = 0.f;
  for (int j = threadIdx.x; j < J; j += blockDim.x) t1 += L[j];
  block_sum2(t1, dummy, red);
  const float mo = t1 / J;
  float t2 = 0.f;
  for (int j = threadIdx.x; j < J; j += blockDim.x) t2 += (L[j] - mo) * (L[j] - mo);
  dummy = 0.f;
  block_sum2(t2, dummy, red);
  const float ro = 1.f / sqrtf(t2 / J + kLnEps);
  for (int j = threadIdx.x; j < J; j += blockDim.x)
    logits[(size_t)f * J + j] = (L[j] - mo) * ro * gamma_o[j] + beta_o[j];
  if (threadIdx.x == 0) {
    stat[4 * f + 2] = mo;
    stat[4 * f + 3] = ro;
  }
}

// Backward of capsnorm_fwd.  gpart[f][0..n) = g_gamma contributions, [n..2n) g_beta;
// head: gpart[f][2n..2n+J) g_gamma_out, [2n+J..2n+2J) g_beta_out.
//   head: o = drop(LN_mid(x)), L_j = sqrt(|o_j|^2 + eps), logits = LN_out(L)
//         g_o = g_L_j * o / L_j (naive:255-258)
__device__ __forceinline__ void capsnorm_bwd_row(
    const float* __restrict__ x, int n, const float* __restrict__ gamma, const float* __restrict__ beta,
    int training, float p, unsigned long long seed, const unsigned long long* __restrict__ seed_src, unsigned stream,
    const float* __restrict__ stat, const float* __restrict__ g_in, int head, int J, int D,
    const float* __restrict__ gamma_o, const float* __restrict__ lens, float* __restrict__ g_x,
    float* __restrict__ gpart, int f) {
  seed = srf_step_seed(seed, seed_src);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* gy = sm;          // n
  float* red = gy + n;     // 8
  float* gl = red + 8;     // J
  const float mean = stat[4 * f], rstd = stat[4 * f + 1];
  const size_t stride = head ? (size_t)2 * n + 2 * J : (size_t)2 * n;
  if (head) {
    const float mo = stat[4 * f + 2], ro = stat[4 * f + 3];
    float a1 = 0.f, a2 = 0.f;
    for (int j = threadIdx.x; j < J; j += blockDim.x) {
      const float go = g_in[(size_t)f * J + j];
      const float xh = (lens[(size_t)f * J + j] - mo) * ro;
      gpart[(size_t)f * stride + 2 * n + j] = go * xh;
      gpart[(size_t)f * stride + 2 * n + J + j] = go;
      const float gx = go * gamma_o[j];
      gl[j] = gx;
      a1 += gx;
      a2 += gx * xh;
    }
    block_sum2(a1, a2, red);
    for (int j = threadIdx.x; j < J; j += blockDim.x) {
      const float xh = (lens[(size_t)f * J + j] - mo) * ro;
      gl[j] = ro * (gl[j] - a1 / J - xh * a2 / J) / lens[(size_t)f * J + j];
    }
    __syncthreads();
  }
  float a1 = 0.f, a2 = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const size_t gi = (size_t)f * n + i;
    const float xh = (x[gi] - mean) * rstd;
    const float dm = drop_mult(training && p > 0.f, seed, stream, gi, p);
    float go;
    if (head) {
      const float o = (xh * gamma[i] + beta[i]) * dm;
      go = gl[i / D] * o;
    } else {
      go = g_in[gi];
    }
    const float g = go * dm;   // gradient wrt the LN output
    gpart[(size_t)f * stride + i] = g * xh;
    gpart[(size_t)f * stride + n + i] = g;
    const float t = g * gamma[i];
    gy[i] = t;
    a1 += t;
    a2 += t * xh;
  }
  block_sum2(a1, a2, red);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const size_t gi = (size_t)f * n + i;
    const float xh = (x[gi] - mean) * rstd;
    g_x[gi] = rstd * (gy[i] - a1 / n - xh * a2 / n);
  }
}

// One wave per row for the plain LN + dropout rows (no head) of n = 64 * NPL values:
// the row in registers as float4 (NPL / 4 per lane), both moments and both backward
// sums as wave reductions -- no LDS and no barrier.  These rows are 1-4 KB: a 256-thread
// block per row spent most of its time in its block reductions.  Dropout masks are keyed
// by the element index, so they do not depend on the mapping.
template <int NPL>
__device__ __forceinline__ void capsnorm_fwd_wave(const float* __restrict__ x, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, bool drop, float p,
                                                  unsigned long long seed, unsigned stream, float* __restrict__ y,
                                                  float* __restrict__ stat, int f, int lane) {
  constexpr int n = 64 * NPL, NV = NPL / 4;
  const f4* xr = reinterpret_cast<const f4*>(x + (size_t)f * n);
  f4 v[NV];
  float s1 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    v[k] = xr[k * 64 + lane];
    s1 += (v[k].x + v[k].y) + (v[k].z + v[k].w);
  }
  const float mean = wave_sum(s1) / n;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const f4 d = v[k] - mean;
    s2 += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
  }
  const float rstd = 1.f / sqrtf(wave_sum(s2) / n + kLnEps);
  f4* yr = reinterpret_cast<f4*>(y + (size_t)f * n);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int q = k * 64 + lane;
    const f4 g = reinterpret_cast<const f4*>(gamma)[q], b = reinterpret_cast<const f4*>(beta)[q];
    const size_t gi = (size_t)f * n + 4 * q;
    f4 o;
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = ((v[k][c] - mean) * rstd * g[c] + b[c]) * drop_mult(drop, seed, stream, gi + c, p);
    yr[q] = o;
  }
  if (lane == 0) {
    stat[4 * f] = mean;
    stat[4 * f + 1] = rstd;
  }
}

// The output head on one wave per row: LN_mid + dropout as capsnorm_fwd_wave, the
// capsule lengths over groups of D / 4 lanes (capsule j = element / D; each lane's float4
// lies in one capsule), LN_out over the J lengths by wave sums (each length is held by
// its D / 4 lanes).
template <int NPL>
__device__ __forceinline__ void caps_head_fwd_wave(const float* __restrict__ x, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, bool drop, float p,
                                                   unsigned long long seed, unsigned stream,
                                                   float* __restrict__ stat, int D, const float* __restrict__ gamma_o,
                                                   const float* __restrict__ beta_o, float* __restrict__ logits,
                                                   float* __restrict__ lens, float len_eps, int f, int lane) {
  constexpr int n = 64 * NPL, NV = NPL / 4;
  const int LPC = D / 4, J = n / D;
  const f4* xr = reinterpret_cast<const f4*>(x + (size_t)f * n);
  f4 v[NV];
  float s1 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    v[k] = xr[k * 64 + lane];
    s1 += (v[k].x + v[k].y) + (v[k].z + v[k].w);
  }
  const float mean = wave_sum(s1) / n;
  float s2 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const f4 d = v[k] - mean;
    s2 += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
  }
  const float rstd = 1.f / sqrtf(wave_sum(s2) / n + kLnEps);
  float L[NV];
  float t1 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int q = k * 64 + lane;
    const f4 g = reinterpret_cast<const f4*>(gamma)[q], b = reinterpret_cast<const f4*>(beta)[q];
    const size_t gi = (size_t)f * n + 4 * q;
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float o = ((v[k][c] - mean) * rstd * g[c] + b[c]) * drop_mult(drop, seed, stream, gi + c, p);
      ss += o * o;
    }
    for (int m = 1; m < LPC; m <<= 1) ss += __shfl_xor(ss, m, 64);
    L[k] = sqrtf(ss + len_eps);
    t1 += L[k];
  }
  const float mo = wave_sum(t1) / (float)LPC / J;
  float t2 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) t2 += (L[k] - mo) * (L[k] - mo);
  const float ro = 1.f / sqrtf(wave_sum(t2) / (float)LPC / J + kLnEps);
  if (lane % LPC == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int j = (k * 64 + lane) / LPC;
      lens[(size_t)f * J + j] = L[k];
      logits[(size_t)f * J + j] = (L[k] - mo) * ro * gamma_o[j] + beta_o[j];
    }
  }
  if (lane == 0) {
    stat[4 * f] = mean;
    stat[4 * f + 1] = rstd;
    stat[4 * f + 2] = mo;
    stat[4 * f + 3] = ro;
  }
}

template <int NPL>
__global__ __launch_bounds__(256) void caps_head_fwd_wave_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, int training, float p,
                                                                 unsigned long long seed,
                                                                 const unsigned long long* __restrict__ seed_src,
                                                                 unsigned stream, float* __restrict__ stat, int D,
                                                                 const float* __restrict__ gamma_o,
                                                                 const float* __restrict__ beta_o,
                                                                 float* __restrict__ logits, float* __restrict__ lens,
                                                                 float len_eps, int rows) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= rows) return;   // whole waves: nothing below synchronises
  caps_head_fwd_wave<NPL>(x, gamma, beta, training && p > 0.f, p, srf_step_seed(seed, seed_src), stream, stat, D,
                          gamma_o, beta_o, logits, lens, len_eps, w, threadIdx.x & 63);
}

template <int NPL>
__device__ __forceinline__ void capsnorm_bwd_wave(const float* __restrict__ x, const float* __restrict__ gamma,
                                                  bool drop, float p, unsigned long long seed, unsigned stream,
                                                  const float* __restrict__ stat, const float* __restrict__ g_in,
                                                  float* __restrict__ g_x, f4 (&pgxh)[NPL / 4], f4 (&pgg)[NPL / 4],
                                                  int f, int lane) {
  constexpr int n = 64 * NPL, NV = NPL / 4;
  const float mean = stat[4 * f], rstd = stat[4 * f + 1];
  const f4* xr = reinterpret_cast<const f4*>(x + (size_t)f * n);
  const f4* gr = reinterpret_cast<const f4*>(g_in + (size_t)f * n);
  f4 xh[NV], t[NV];
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int q = k * 64 + lane;
    const f4 xv = xr[q], go = gr[q], gam = reinterpret_cast<const f4*>(gamma)[q];
    const size_t gi = (size_t)f * n + 4 * q;
    f4 gxh, gg;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      xh[k][c] = (xv[c] - mean) * rstd;
      const float g = go[c] * drop_mult(drop, seed, stream, gi + c, p);   // gradient wrt the LN output
      gxh[c] = g * xh[k][c];
      gg[c] = g;
      t[k][c] = g * gam[c];
      a1 += t[k][c];
      a2 += t[k][c] * xh[k][c];
    }
    pgxh[k] += gxh;
    pgg[k] += gg;
  }
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  f4* ox = reinterpret_cast<f4*>(g_x + (size_t)f * n);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    f4 o;
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = rstd * (t[k][c] - a1 / n - xh[k][c] * a2 / n);
    ox[k * 64 + lane] = o;
  }
}

// the parameter-gradient partials (d gamma | d beta, 2n columns) of the sum over a wave's
// rows, one partial row per wave
template <int NPL>
__device__ __forceinline__ void store_gpart(float* __restrict__ gpart, size_t row, const f4 (&pgxh)[NPL / 4],
                                            const f4 (&pgg)[NPL / 4], int lane) {
  constexpr int n = 64 * NPL;
  f4* pg = reinterpret_cast<f4*>(gpart + row * 2 * n);
#pragma unroll
  for (int k = 0; k < NPL / 4; ++k) {
    pg[k * 64 + lane] = pgxh[k];
    pg[n / 4 + k * 64 + lane] = pgg[k];
  }
}

// BWD: a wave takes rpw consecutive rows; rpw == 1 keeps one partial row per frame at the
// frame's own index (the range entry points' gpart layout), rpw > 1 writes partial row w
// (srf_capsnorm_bwd's own workspace: rpw times fewer rows for its column sum)
template <int NPL, bool BWD>
__global__ __launch_bounds__(256) void capsnorm_wave_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, int training, float p,
                                                            unsigned long long seed,
                                                            const unsigned long long* __restrict__ seed_src,
                                                            unsigned stream, float* __restrict__ y,
                                                            float* __restrict__ stat, const float* __restrict__ g_in,
                                                            float* __restrict__ gpart, RowMap rmap, int rows, int rpw) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const unsigned long long sd = srf_step_seed(seed, seed_src);
  const bool drop = training && p > 0.f;
  if constexpr (BWD) {
    const int r0 = w * rpw;
    if (r0 >= rows) return;   // whole waves: nothing below synchronises
    f4 pgxh[NPL / 4], pgg[NPL / 4];
#pragma unroll
    for (int k = 0; k < NPL / 4; ++k) pgxh[k] = pgg[k] = f4{0.f, 0.f, 0.f, 0.f};
    const int r1 = min(rows, r0 + rpw);
    for (int r = r0; r < r1; ++r)
      capsnorm_bwd_wave<NPL>(x, gamma, drop, p, sd, stream, stat, g_in, y, pgxh, pgg, rmap.row(r), lane);
    store_gpart<NPL>(gpart, rpw == 1 ? (size_t)rmap.row(r0) : (size_t)w, pgxh, pgg, lane);
  } else {
    if (w >= rows) return;
    capsnorm_fwd_wave<NPL>(x, gamma, beta, drop, p, sd, stream, y, stat, rmap.row(w), lane);
  }
}

__global__ __launch_bounds__(256) void capsnorm_fwd_kernel(
    const float* __restrict__ x, int n, const float* __restrict__ gamma, const float* __restrict__ beta, int training,
    float p, unsigned long long seed, const unsigned long long* __restrict__ seed_src, unsigned stream,
    float* __restrict__ y, float* __restrict__ stat, int head, int J, int D, const float* __restrict__ gamma_o,
    const float* __restrict__ beta_o, float* __restrict__ logits, float* __restrict__ lens, float len_eps,
    RowMap rmap) {
  capsnorm_fwd_row(x, n, gamma, beta, training, p, seed, seed_src, stream, y, stat, head, J, D, gamma_o, beta_o,
                   logits, lens, len_eps, rmap.row(blockIdx.x));
}

__global__ __launch_bounds__(256) void capsnorm_bwd_kernel(
    const float* __restrict__ x, int n, const float* __restrict__ gamma, const float* __restrict__ beta, int training,
    float p, unsigned long long seed, const unsigned long long* __restrict__ seed_src, unsigned stream,
    const float* __restrict__ stat, const float* __restrict__ g_in, int head, int J, int D,
    const float* __restrict__ gamma_o, const float* __restrict__ lens, float* __restrict__ g_x,
    float* __restrict__ gpart, RowMap rmap) {
  capsnorm_bwd_row(x, n, gamma, beta, training, p, seed, seed_src, stream, stat, g_in, head, J, D, gamma_o, lens, g_x,
                   gpart, rmap.row(blockIdx.x));
}

// The frame ranges of several same-width layers in one launch (grid.y = range): the
// layer-pipelined SDR stack's inner layers, one anti-diagonal at a time.
struct CnItems {
  srf_capsnorm_range it[SRF_CAPSNORM_MAX_ITEMS];
  int B, T, n_items;
};

template <int NPL, bool BWD>
__global__ __launch_bounds__(256) void capsnorm_range_n_wave_kernel(CnItems items, int training, float p,
                                                                    unsigned long long seed,
                                                                    const unsigned long long* __restrict__ seed_src) {
  const srf_capsnorm_range& r = items.it[blockIdx.y];
  const int nt = r.t1 - r.t0;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= items.B * nt) return;   // whole waves: nothing below synchronises
  const int f = RowMap{items.T, r.t0, nt}.row(w);
  const unsigned stream = (unsigned)(kStreamMid0 + r.layer);
  const unsigned long long sd = srf_step_seed(seed, seed_src);
  const bool drop = training && p > 0.f;
  if constexpr (BWD) {
    f4 pgxh[NPL / 4], pgg[NPL / 4];
#pragma unroll
    for (int k = 0; k < NPL / 4; ++k) pgxh[k] = pgg[k] = f4{0.f, 0.f, 0.f, 0.f};
    capsnorm_bwd_wave<NPL>(r.x, r.gamma, drop, p, sd, stream, r.stat, r.g_y, r.g_x, pgxh, pgg, f, threadIdx.x & 63);
    store_gpart<NPL>(r.gpart, (size_t)f, pgxh, pgg, threadIdx.x & 63);
  } else
    capsnorm_fwd_wave<NPL>(r.x, r.gamma, r.beta, drop, p, sd, stream, r.y, r.stat, f, threadIdx.x & 63);
}

template <bool BWD>
__global__ __launch_bounds__(256) void capsnorm_range_n_kernel(CnItems items, int n, int training, float p,
                                                               unsigned long long seed,
                                                               const unsigned long long* __restrict__ seed_src) {
  const srf_capsnorm_range& r = items.it[blockIdx.y];
  const int nt = r.t1 - r.t0;
  if ((int)blockIdx.x >= items.B * nt) return;
  const int f = RowMap{items.T, r.t0, nt}.row(blockIdx.x);
  const unsigned stream = (unsigned)(kStreamMid0 + r.layer);
  if constexpr (BWD)
    capsnorm_bwd_row(r.x, n, r.gamma, r.beta, training, p, seed, seed_src, stream, r.stat, r.g_y, 0, 0, 0, nullptr,
                     nullptr, r.g_x, r.gpart, f);
  else
    capsnorm_fwd_row(r.x, n, r.gamma, r.beta, training, p, seed, seed_src, stream, r.y, r.stat, 0, 0, 0, nullptr,
                     nullptr, nullptr, nullptr, kLengthEps, f);
}

// ---------------------------------------------------------------- host
struct CapsSaved {
  float *e, *m, *lnstat;
  unsigned char* sel;
  size_t bytes;
};

CapsSaved caps_saved_layout(int F, int PH, int PD, void* base) {
  const size_t E = (size_t)PH * PD;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += srf::align_up(bytes, 256);
    return o;
  };
  const size_t oe = take((size_t)F * PH * 4), om = take((size_t)F * E * 4), os = take((size_t)F * 2 * 4),
               osel = take((size_t)F * E);
  char* b = static_cast<char*>(base);
  CapsSaved c;
  c.e = (float*)(b + oe);
  c.m = (float*)(b + om);
  c.lnstat = (float*)(b + os);
  c.sel = (unsigned char*)(b + osel);
  c.bytes = off;
  return c;
}

struct CapsBwdWs {
  float *gv1, *gv2, *wpart, *wsum, *g_e, *ppart, *psum, *scratch;
  size_t bytes;
};

constexpr int kProjChunks = 64;

CapsBwdWs caps_bwd_layout(int F, int K, int PH, int PD, void* base) {
  const size_t E = (size_t)PH * PD;
  const size_t wcols = 2 * E + 20 * PD, pcols = (size_t)K * PH + PH;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += srf::align_up(bytes, 256);
    return o;
  };
  const size_t o1 = take((size_t)F * E * 4), o2 = take((size_t)F * E * 4), ow = take((size_t)F * wcols * 4),
               owsum = take(wcols * 4), oge = take((size_t)F * PH * 4), opp = take(kProjChunks * pcols * 4),
               ops = take(pcols * 4),
               osc = take(std::max(srf::colsum_scratch_floats(F, (int)wcols), srf::colsum_scratch_floats(kProjChunks, (int)pcols)) * 4);
  char* b = static_cast<char*>(base);
  CapsBwdWs w;
  w.gv1 = (float*)(b + o1);
  w.gv2 = (float*)(b + o2);
  w.wpart = (float*)(b + ow);
  w.wsum = (float*)(b + owsum);
  w.g_e = (float*)(b + oge);
  w.ppart = (float*)(b + opp);
  w.psum = (float*)(b + ops);
  w.scratch = (float*)(b + osc);
  w.bytes = off;
  return w;
}

int check_caps(int B, int T, int PH, int PD) {
  SRF_REQUIRE(B > 0 && T > 0 && PH > 0 && PD > 0, "bad primary capsule shape");
  SRF_REQUIRE((size_t)PH * PD <= kMaxVec, "PH*PD = %d exceeds %d", PH * PD, kMaxVec);
  return SRF_OK;
}

}  // namespace

// frames per wave of srf_capsnorm_bwd's wave kernel (4: F / 4 partial rows, a single-launch
// column sum at C4's F = 5600, and still > 256 workgroups)
constexpr int kCnRowsPerWave = 4;

// the wave-per-row kernels for n = 256, 512, 1024 (C2 / C3 / C4 / C5 widths); false: other n
template <bool BWD>
static bool capsnorm_wave(int n, int rows, RowMap rm, const float* x, const float* gamma, const float* beta,
                          int training, float p, unsigned long long seed, unsigned stream, float* y, float* stat,
                          const float* g_in, float* gpart, hipStream_t st, int rpw = 1) {
  const dim3 grid(((rows + rpw - 1) / rpw + 3) / 4);
#define SRF_CN_WAVE(NPL)                                                                                             \
  hipLaunchKernelGGL((capsnorm_wave_kernel<NPL, BWD>), grid, dim3(256), 0, st, x, gamma, beta, training, p, seed,   \
                     srf::seed_source(), stream, y, stat, g_in, gpart, rm, rows, rpw)
  if (n == 256) SRF_CN_WAVE(4);
  else if (n == 512) SRF_CN_WAVE(8);
  else if (n == 1024) SRF_CN_WAVE(16);
  else return false;
#undef SRF_CN_WAVE
  return true;
}

extern "C" {

size_t srf_primary_caps_saved_bytes(int B, int T, int PH, int PD) {
  return caps_saved_layout(B * T, PH, PD, nullptr).bytes;
}

size_t srf_primary_caps_bwd_workspace(int B, int T, int K, int PH, int PD) {
  return caps_bwd_layout(B * T, K, PH, PD, nullptr).bytes;
}

int srf_primary_caps_fwd(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                         const float* bp, const float* K1, const float* b1, const float* K2, const float* b2,
                         const float* gamma, const float* beta, int training, float p_caps, float p_in,
                         unsigned long long seed, float* z, void* saved, size_t saved_bytes, void* stream) {
  return srf_primary_caps_fwd_ex(X, inp_len, B, T, K, PH, PD, Wp, bp, K1, b1, K2, b2, gamma, beta, training, p_caps,
                                 p_in, seed, 1.f, 0, z, saved, saved_bytes, stream);
}

int srf_primary_caps_fwd_ex(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                            const float* bp, const float* K1, const float* b1, const float* K2, const float* b2,
                            const float* gamma, const float* beta, int training, float p_caps, float p_in,
                            unsigned long long seed, float proj_scale, int pos_enc, float* z, void* saved,
                            size_t saved_bytes, void* stream) {
  int rc = check_caps(B, T, PH, PD);
  if (rc) return rc;
  SRF_REQUIRE(!pos_enc || (PH >= 4 && PH % 2 == 0), "positional encoding needs an even PH >= 4, got %d", PH);
  SRF_REQUIRE(X && inp_len && Wp && bp && K1 && b1 && K2 && b2 && gamma && beta && z && saved, "null pointer");
  const int F = B * T;
  CapsSaved sv = caps_saved_layout(F, PH, PD, saved);
  if (saved_bytes < sv.bytes) {
    srf::set_error("primary caps saved buffer too small: %zu < %zu", saved_bytes, sv.bytes);
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  constexpr int FW = 2;
  const dim3 gvec((F + 4 * FW - 1) / (4 * FW));
  const int Kq = ((K + kProjWaves - 1) / kProjWaves + 15) / 16 * 16;
  if (K % 4 == 0 && (PH == 4 || PH == 8 || PH == 16)) {
    const dim3 gm((F + 15) / 16), bm(64 * kProjWaves);
    if (PH == 4)
      hipLaunchKernelGGL((proj_fwd_mfma_kernel<4>), gm, bm, 0, st, X, F, K, Wp, bp, sv.e, T, proj_scale, pos_enc, Kq);
    else if (PH == 8)
      hipLaunchKernelGGL((proj_fwd_mfma_kernel<8>), gm, bm, 0, st, X, F, K, Wp, bp, sv.e, T, proj_scale, pos_enc, Kq);
    else
      hipLaunchKernelGGL((proj_fwd_mfma_kernel<16>), gm, bm, 0, st, X, F, K, Wp, bp, sv.e, T, proj_scale, pos_enc,
                         Kq);
  } else if (K % 4 == 0 && PH == 4)
    hipLaunchKernelGGL((proj_fwd_vec_kernel<4, FW>), gvec, dim3(256), 0, st, X, F, K, Wp, bp, sv.e, T,
                       proj_scale, pos_enc);
  else if (K % 4 == 0 && PH == 8)
    hipLaunchKernelGGL((proj_fwd_vec_kernel<8, FW>), gvec, dim3(256), 0, st, X, F, K, Wp, bp, sv.e, T,
                       proj_scale, pos_enc);
  else if (K % 4 == 0 && PH == 16)
    hipLaunchKernelGGL((proj_fwd_vec_kernel<16, FW>), gvec, dim3(256), 0, st, X, F, K, Wp, bp, sv.e, T,
                       proj_scale, pos_enc);
  else
    hipLaunchKernelGGL(proj_fwd_kernel, dim3((F + 3) / 4), dim3(256), 0, st, X, F, K, PH, Wp, bp, sv.e, T, proj_scale,
                       pos_enc);
  SRF_LAUNCH_CHECK("proj_fwd");
  CapsDims cd{B, T, PH, PD};
  const size_t sh = (size_t)(PH * PD + 5 * PH + 8) * sizeof(float);
  hipLaunchKernelGGL(encaps_fwd_kernel, dim3(F), dim3(256), sh, st, sv.e, inp_len, cd, K1, b1, K2, b2, gamma, beta,
                     training, p_caps, p_in, seed, srf::seed_source(), sv.m, sv.sel, sv.lnstat, z);
  SRF_LAUNCH_CHECK("encaps_fwd");
  return SRF_OK;
}

int srf_primary_caps_bwd(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                         const float* K1, const float* K2, const float* gamma, const float* beta, int training,
                         float p_caps, float p_in, unsigned long long seed, const void* saved, const float* g_z,
                         float* g_X, float* g_Wp, float* g_bp, float* g_K1, float* g_b1, float* g_K2, float* g_b2,
                         float* g_gamma, float* g_beta, void* workspace, size_t workspace_bytes, void* stream) {
  return srf_primary_caps_bwd_ex(X, inp_len, B, T, K, PH, PD, Wp, K1, K2, gamma, beta, training, p_caps, p_in, seed,
                                 1.f, saved, g_z, g_X, g_Wp, g_bp, g_K1, g_b1, g_K2, g_b2, g_gamma, g_beta, workspace,
                                 workspace_bytes, stream);
}

int srf_primary_caps_bwd_ex(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                            const float* K1, const float* K2, const float* gamma, const float* beta, int training,
                            float p_caps, float p_in, unsigned long long seed, float proj_scale, const void* saved,
                            const float* g_z, float* g_X, float* g_Wp, float* g_bp, float* g_K1, float* g_b1,
                            float* g_K2, float* g_b2, float* g_gamma, float* g_beta, void* workspace,
                            size_t workspace_bytes, void* stream) {
  int rc = check_caps(B, T, PH, PD);
  if (rc) return rc;
  SRF_REQUIRE(X && inp_len && Wp && K1 && K2 && gamma && beta && saved && g_z && g_X && g_Wp && g_bp && g_K1 &&
                  g_b1 && g_K2 && g_b2 && g_gamma && g_beta && workspace,
              "null pointer");
  const int F = B * T, E = PH * PD;
  CapsSaved sv = caps_saved_layout(F, PH, PD, const_cast<void*>(saved));
  CapsBwdWs w = caps_bwd_layout(F, K, PH, PD, workspace);
  if (workspace_bytes < w.bytes) {
    srf::set_error("primary caps workspace too small: %zu < %zu", workspace_bytes, w.bytes);
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  CapsDims cd{B, T, PH, PD};
  const size_t sh = (size_t)(4 * E + 6 * PH + 8) * sizeof(float);
  hipLaunchKernelGGL(encaps_bwd_a_kernel, dim3(F), dim3(256), sh, st, g_z, sv.e, sv.m, sv.sel, sv.lnstat, inp_len, cd,
                     gamma, beta, training, p_caps, p_in, seed, srf::seed_source(), w.gv1, w.gv2, w.wpart);
  SRF_LAUNCH_CHECK("encaps_bwd_a");
  const int wcols = 2 * E + 20 * PD;
  // columns: gamma, beta, then per conv k its 9 taps x PD and its bias -> straight into the gradients
  if ((rc = srf::colsum(w.wpart, F, wcols, nullptr, w.scratch, st,
                        srf::ColSplit{{g_gamma, g_beta, g_K1, g_b1, g_K2, g_b2}, {E, E, 9 * PD, PD, 9 * PD, PD}})))
    return rc;
  hipLaunchKernelGGL(encaps_bwd_b_kernel, dim3(((size_t)F * PH * kEbLanes + 255) / 256), dim3(256), 0, st, w.gv1,
                     w.gv2, cd, K1, K2, w.g_e, proj_scale);
  SRF_LAUNCH_CHECK("encaps_bwd_b");
  const dim3 gx4(((size_t)((F + kProjXF - 1) / kProjXF) * (K / 4) + 255) / 256);
  if (K % 4 == 0 && PH == 4)
    hipLaunchKernelGGL(proj_bwd_x_vec_kernel<4>, gx4, dim3(256), 0, st, w.g_e, Wp, F, K, g_X);
  else if (K % 4 == 0 && PH == 8)
    hipLaunchKernelGGL(proj_bwd_x_vec_kernel<8>, gx4, dim3(256), 0, st, w.g_e, Wp, F, K, g_X);
  else if (K % 4 == 0 && PH == 16)
    hipLaunchKernelGGL(proj_bwd_x_vec_kernel<16>, gx4, dim3(256), 0, st, w.g_e, Wp, F, K, g_X);
  else
    hipLaunchKernelGGL(proj_bwd_x_kernel, dim3(((size_t)F * K + 255) / 256), dim3(256), 0, st, w.g_e, Wp, F, K, PH,
                       g_X);
  SRF_LAUNCH_CHECK("proj_bwd_x");
  const int fchunk = (F + kProjChunks - 1) / kProjChunks;
  if (PH <= 16)
    hipLaunchKernelGGL(proj_bwd_w_mfma_kernel, dim3((K + 63) / 64, kProjChunks), dim3(256), 0, st, X, w.g_e, F, K, PH,
                       fchunk, w.ppart);
  else
    hipLaunchKernelGGL(proj_bwd_w_kernel, dim3((K + 255) / 256, kProjChunks), dim3(256), 0, st, X, w.g_e, F, K, PH,
                       fchunk, w.ppart);
  SRF_LAUNCH_CHECK("proj_bwd_w");
  const int pcols = K * PH + PH;
  if ((rc = srf::colsum(w.ppart, kProjChunks, pcols, nullptr, w.scratch, st,
                        srf::ColSplit{{g_Wp, g_bp, nullptr, nullptr}, {K * PH, PH, 0, 0}})))
    return rc;
  return SRF_OK;
}

size_t srf_capsnorm_bwd_workspace(int F, int n, int J) {
  const int cols = 2 * n + 2 * J;
  return srf::align_up((size_t)F * cols * 4, 256) + srf::align_up((size_t)cols * 4, 256) +
         srf::colsum_scratch_floats(F, cols) * 4;
}

int srf_capsnorm_fwd(const float* x, int F, int n, const float* gamma, const float* beta, int training, float p,
                     unsigned long long seed, int layer, float* y, float* stat, void* stream) {
  SRF_REQUIRE(x && gamma && beta && y && stat && F > 0 && n > 0 && n <= kMaxVec, "bad capsnorm arguments");
  if (capsnorm_wave<false>(n, F, RowMap::all(F), x, gamma, beta, training, p, seed, (unsigned)(kStreamMid0 + layer), y,
                           stat, nullptr, nullptr, static_cast<hipStream_t>(stream))) {
    SRF_LAUNCH_CHECK("capsnorm_fwd");
    return SRF_OK;
  }
  hipLaunchKernelGGL(capsnorm_fwd_kernel, dim3(F), dim3(256), (size_t)(n + 8) * 4, static_cast<hipStream_t>(stream),
                     x, n, gamma, beta, training, p, seed, srf::seed_source(), (unsigned)(kStreamMid0 + layer), y, stat, 0, 0, 0,
                     (const float*)nullptr, (const float*)nullptr, (float*)nullptr, (float*)nullptr, kLengthEps,
                     RowMap::all(F));
  SRF_LAUNCH_CHECK("capsnorm_fwd");
  return SRF_OK;
}

int srf_capsnorm_fwd_range(const float* x, int B, int T, int t0, int t1, int n, const float* gamma, const float* beta,
                           int training, float p, unsigned long long seed, int layer, float* y, float* stat,
                           void* stream) {
  SRF_REQUIRE(x && gamma && beta && y && stat && B > 0 && T > 0 && 0 <= t0 && t0 <= t1 && t1 <= T && n > 0 &&
                  n <= kMaxVec,
              "bad capsnorm range arguments");
  if (t0 == t1) return SRF_OK;
  if (capsnorm_wave<false>(n, B * (t1 - t0), RowMap{T, t0, t1 - t0}, x, gamma, beta, training, p, seed,
                           (unsigned)(kStreamMid0 + layer), y, stat, nullptr, nullptr, static_cast<hipStream_t>(stream))) {
    SRF_LAUNCH_CHECK("capsnorm_fwd_range");
    return SRF_OK;
  }
  hipLaunchKernelGGL(capsnorm_fwd_kernel, dim3(B * (t1 - t0)), dim3(256), (size_t)(n + 8) * 4,
                     static_cast<hipStream_t>(stream), x, n, gamma, beta, training, p, seed, srf::seed_source(),
                     (unsigned)(kStreamMid0 + layer), y, stat, 0, 0, 0, (const float*)nullptr, (const float*)nullptr,
                     (float*)nullptr, (float*)nullptr, kLengthEps, RowMap{T, t0, t1 - t0});
  SRF_LAUNCH_CHECK("capsnorm_fwd_range");
  return SRF_OK;
}

int srf_capsnorm_bwd_range(const float* x, int B, int T, int t0, int t1, int n, const float* gamma, const float* beta,
                           int training, float p, unsigned long long seed, int layer, const float* stat,
                           const float* g_y, float* g_x, float* gpart, void* stream) {
  SRF_REQUIRE(x && gamma && beta && stat && g_y && g_x && gpart && B > 0 && T > 0 && 0 <= t0 && t0 <= t1 && t1 <= T &&
                  n > 0 && n <= kMaxVec,
              "bad capsnorm range arguments");
  if (t0 == t1) return SRF_OK;
  if (capsnorm_wave<true>(n, B * (t1 - t0), RowMap{T, t0, t1 - t0}, x, gamma, beta, training, p, seed,
                          (unsigned)(kStreamMid0 + layer), g_x, const_cast<float*>(stat), g_y, gpart,
                          static_cast<hipStream_t>(stream))) {
    SRF_LAUNCH_CHECK("capsnorm_bwd_range");
    return SRF_OK;
  }
  hipLaunchKernelGGL(capsnorm_bwd_kernel, dim3(B * (t1 - t0)), dim3(256), (size_t)(n + 8) * 4,
                     static_cast<hipStream_t>(stream), x, n, gamma, beta, training, p, seed, srf::seed_source(),
                     (unsigned)(kStreamMid0 + layer), stat, g_y, 0, 0, 1, (const float*)nullptr, (const float*)nullptr,
                     g_x, gpart, RowMap{T, t0, t1 - t0});
  SRF_LAUNCH_CHECK("capsnorm_bwd_range");
  return SRF_OK;
}

static int capsnorm_range_n(const srf_capsnorm_range* r, int n_items, int B, int T, int n, int training, float p,
                             unsigned long long seed, void* stream, bool bwd) {
  SRF_REQUIRE(r && n_items >= 0 && n_items <= SRF_CAPSNORM_MAX_ITEMS && B > 0 && T > 0 && n > 0 && n <= kMaxVec,
              "bad capsnorm range_n arguments");
  CnItems it{};
  it.B = B, it.T = T;
  int rows = 0;
  for (int k = 0; k < n_items; ++k) {
    const srf_capsnorm_range& q = r[k];
    SRF_REQUIRE(0 <= q.t0 && q.t0 <= q.t1 && q.t1 <= T, "capsnorm range [%d, %d) outside [0, %d)", q.t0, q.t1, T);
    if (q.t0 == q.t1) continue;
    SRF_REQUIRE(q.x && q.gamma && q.beta && q.stat && (bwd ? (q.g_y && q.g_x && q.gpart) : q.y != nullptr),
                "null pointer argument");
    it.it[it.n_items++] = q;
    rows = std::max(rows, B * (q.t1 - q.t0));
  }
  if (it.n_items == 0) return SRF_OK;
  if (n == 256 || n == 512 || n == 1024) {   // one wave per row
    const dim3 gw((rows + 3) / 4, it.n_items);
    hipStream_t st = static_cast<hipStream_t>(stream);
#define SRF_CN_RANGE(NPL)                                                                                    \
  if (bwd)                                                                                                  \
    hipLaunchKernelGGL((capsnorm_range_n_wave_kernel<NPL, true>), gw, dim3(256), 0, st, it, training, p, seed,  \
                       srf::seed_source());                                                                 \
  else                                                                                                      \
    hipLaunchKernelGGL((capsnorm_range_n_wave_kernel<NPL, false>), gw, dim3(256), 0, st, it, training, p, seed, \
                       srf::seed_source())
    if (n == 256) {
      SRF_CN_RANGE(4);
    } else if (n == 512) {
      SRF_CN_RANGE(8);
    } else {
      SRF_CN_RANGE(16);
    }
#undef SRF_CN_RANGE
    SRF_LAUNCH_CHECK("capsnorm_range_n");
    return SRF_OK;
  }
  const dim3 grid(rows, it.n_items);
  if (bwd)
    hipLaunchKernelGGL(capsnorm_range_n_kernel<true>, grid, dim3(256), (size_t)(n + 8) * 4,
                       static_cast<hipStream_t>(stream), it, n, training, p, seed, srf::seed_source());
  else
    hipLaunchKernelGGL(capsnorm_range_n_kernel<false>, grid, dim3(256), (size_t)(n + 8) * 4,
                       static_cast<hipStream_t>(stream), it, n, training, p, seed, srf::seed_source());
  SRF_LAUNCH_CHECK("capsnorm_range_n");
  return SRF_OK;
}

int srf_capsnorm_fwd_range_n(const srf_capsnorm_range* r, int n_items, int B, int T, int n, int training, float p,
                             unsigned long long seed, void* stream) {
  return capsnorm_range_n(r, n_items, B, T, n, training, p, seed, stream, false);
}

int srf_capsnorm_bwd_range_n(const srf_capsnorm_range* r, int n_items, int B, int T, int n, int training, float p,
                             unsigned long long seed, void* stream) {
  return capsnorm_range_n(r, n_items, B, T, n, training, p, seed, stream, true);
}

size_t srf_capsnorm_params_workspace(int F, int n) { return srf::colsum_scratch_floats(F, 2 * n) * 4; }

int srf_capsnorm_bwd_params(const float* gpart, int F, int n, float* g_gamma, float* g_beta, void* workspace,
                            size_t workspace_bytes, void* stream) {
  SRF_REQUIRE(gpart && g_gamma && g_beta && workspace && F > 0 && n > 0, "bad capsnorm params arguments");
  if (workspace_bytes < srf_capsnorm_params_workspace(F, n)) {
    srf::set_error("capsnorm params workspace too small");
    return SRF_EWORKSPACE;
  }
  return srf::colsum(gpart, F, 2 * n, nullptr, static_cast<float*>(workspace), static_cast<hipStream_t>(stream),
                     srf::ColSplit{{g_gamma, g_beta, nullptr, nullptr}, {n, n, 0, 0}});
}

int srf_capsnorm_bwd(const float* x, int F, int n, const float* gamma, const float* beta, int training, float p,
                     unsigned long long seed, int layer, const float* stat, const float* g_y, float* g_x,
                     float* g_gamma, float* g_beta, void* workspace, size_t workspace_bytes, void* stream) {
  SRF_REQUIRE(x && gamma && beta && stat && g_y && g_x && g_gamma && g_beta && workspace && F > 0 && n > 0 &&
                  n <= kMaxVec,
              "bad capsnorm arguments");
  if (workspace_bytes < srf_capsnorm_bwd_workspace(F, n, 0)) {
    srf::set_error("capsnorm workspace too small");
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  float* sum = part + srf::align_up((size_t)F * 2 * n * 4, 256) / 4;
  float* scratch = sum + srf::align_up((size_t)2 * n * 4, 256) / 4;
  // wave kernels: kCnRowsPerWave frames per wave and one partial row per wave
  int prow = F;
  if (capsnorm_wave<true>(n, F, RowMap::all(F), x, gamma, beta, training, p, seed, (unsigned)(kStreamMid0 + layer), g_x,
                          const_cast<float*>(stat), g_y, part, st, kCnRowsPerWave))
    prow = (F + kCnRowsPerWave - 1) / kCnRowsPerWave;
  else
    hipLaunchKernelGGL(capsnorm_bwd_kernel, dim3(F), dim3(256), (size_t)(n + 8) * 4, st, x, n, gamma, beta, training,
                       p, seed, srf::seed_source(), (unsigned)(kStreamMid0 + layer), stat, g_y, 0, 0, 1,
                       (const float*)nullptr, (const float*)nullptr, g_x, part, RowMap::all(F));
  SRF_LAUNCH_CHECK("capsnorm_bwd");
  (void)sum;
  return srf::colsum(part, prow, 2 * n, nullptr, scratch, st, srf::ColSplit{{g_gamma, g_beta, nullptr, nullptr}, {n, n, 0, 0}});
}

int srf_caps_head_fwd(const float* v, int F, int J, int D, const float* gamma_mid, const float* beta_mid,
                      const float* gamma_out, const float* beta_out, int training, float p, unsigned long long seed,
                      int layer, float* logits, float* stat, float* lens, void* stream) {
  return srf_caps_head_fwd_ex(v, F, J, D, gamma_mid, beta_mid, gamma_out, beta_out, training, p, seed, layer, kLengthEps,
                              logits, stat, lens, stream);
}

int srf_caps_head_fwd_ex(const float* v, int F, int J, int D, const float* gamma_mid, const float* beta_mid,
                         const float* gamma_out, const float* beta_out, int training, float p, unsigned long long seed,
                         int layer, float length_eps, float* logits, float* stat, float* lens, void* stream) {
  const int n = J * D;
  SRF_REQUIRE(v && gamma_mid && beta_mid && gamma_out && beta_out && logits && stat && lens && F > 0 && n > 0 &&
                  n <= kMaxVec,
              "bad head arguments");
  if ((n == 256 || n == 512 || n == 1024) && D % 4 == 0 && 64 % (D / 4) == 0) {   // one wave per row
    const dim3 grid((F + 3) / 4);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const unsigned sm = (unsigned)(kStreamMid0 + layer);
#define SRF_HEAD_WAVE(NPL)                                                                                          \
  hipLaunchKernelGGL((caps_head_fwd_wave_kernel<NPL>), grid, dim3(256), 0, st, v, gamma_mid, beta_mid, training, p, \
                     seed, srf::seed_source(), sm, stat, D, gamma_out, beta_out, logits, lens, length_eps, F)
    if (n == 256) {
      SRF_HEAD_WAVE(4);
    } else if (n == 512) {
      SRF_HEAD_WAVE(8);
    } else {
      SRF_HEAD_WAVE(16);
    }
#undef SRF_HEAD_WAVE
    SRF_LAUNCH_CHECK("caps_head_fwd");
    return SRF_OK;
  }
  hipLaunchKernelGGL(capsnorm_fwd_kernel, dim3(F), dim3(256), (size_t)(n + 8 + J) * 4,
                     static_cast<hipStream_t>(stream), v, n, gamma_mid, beta_mid, training, p, seed, srf::seed_source(),
                     (unsigned)(kStreamMid0 + layer), (float*)nullptr, stat, 1, J, D, gamma_out, beta_out, logits,
                     lens, length_eps, RowMap::all(F));
  SRF_LAUNCH_CHECK("caps_head_fwd");
  return SRF_OK;
}

int srf_caps_head_bwd(const float* v, int F, int J, int D, const float* gamma_mid, const float* beta_mid,
                      const float* gamma_out, int training, float p, unsigned long long seed, int layer,
                      const float* stat, const float* lens, const float* g_logits, float* g_v, float* g_gamma_mid,
                      float* g_beta_mid, float* g_gamma_out, float* g_beta_out, void* workspace,
                      size_t workspace_bytes, void* stream) {
  const int n = J * D;
  SRF_REQUIRE(v && gamma_mid && beta_mid && gamma_out && stat && lens && g_logits && g_v && g_gamma_mid &&
                  g_beta_mid && g_gamma_out && g_beta_out && workspace && F > 0 && n <= kMaxVec,
              "bad head arguments");
  if (workspace_bytes < srf_capsnorm_bwd_workspace(F, n, J)) {
    srf::set_error("head workspace too small");
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int cols = 2 * n + 2 * J;
  float* part = static_cast<float*>(workspace);
  float* sum = part + srf::align_up((size_t)F * cols * 4, 256) / 4;
  float* scratch = sum + srf::align_up((size_t)cols * 4, 256) / 4;
  hipLaunchKernelGGL(capsnorm_bwd_kernel, dim3(F), dim3(256), (size_t)(n + 8 + J) * 4, st, v, n, gamma_mid, beta_mid,
                     training, p, seed, srf::seed_source(), (unsigned)(kStreamMid0 + layer), stat, g_logits, 1, J, D, gamma_out, lens,
                     g_v, part, RowMap::all(F));
  SRF_LAUNCH_CHECK("caps_head_bwd");
  (void)sum;
  return srf::colsum(part, F, cols, nullptr, scratch, st,
                     srf::ColSplit{{g_gamma_mid, g_beta_mid, g_gamma_out, g_beta_out}, {n, n, J, J}});
}

}  // extern "C"
