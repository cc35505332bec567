// Windowed pose transform + dynamic routing (DR) for one capsule layer, gfx950.
//
// Replaces sequence_router_naive.py:149-185 (window :150-151, pose :154-159,
// DR while_loop :171-185 / _loop_body :199-206) and its autodiff.
//
// Design: u_hat = W x + b is never materialised.  Every
// routing pass recomputes the u tile of (16 frames x 16 capsule rows) on the
// matrix cores (v_mfma_f32_16x16x4_f32, exact fp32) straight from the windowed
// input, and consumes it in registers:
//   * forward pass r   : s^r_j = sum_i c^r_ij u_ij with c^r = softmax_j(<u_ij, Vc^r_j>)
//                        (Vc^r = sum_{r'<r} v^r', the linearity of the logits,
//                        naive:205), partial sums over an i-chunk per workgroup;
//   * backward pass r  : gVc^r_j = sum_i gL^r_ij u_ij and the per-(frame,i)
//                        softmax statistics (logZ^r, sigma^r);
//   * gradient pass    : gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j, which only
//                        needs per-(frame,i) scalars, so j tiles are independent.
// Layouts (HBM, fp32): emb [F=B*T][N][Din]; W [in_n][J*Dout][Din] (row = j*Dout+d);
// bias [in_n][J*Dout]; per-frame vectors [F][J*Dout].
#include <algorithm>
#include <cmath>

#include "srf_common.h"
#include "../../include/srf.h"

namespace {

constexpr float kSquashEps = 1e-7f;  // naive:248
constexpr int MODE_FWD = 0;
constexpr int MODE_BWD = 1;

struct Geom {
  int B, T, N, din, lpad, rpad, J, dout, iters, mask_first;
  int F() const { return B * T; }
  int in_n() const { return N * (lpad + rpad + 1); }
  int JD() const { return J * dout; }
  int NT() const { return (J * dout + 15) / 16; }
};

// ---------------------------------------------------------------- fragments
// MFMA operand k-permutation: k-step ks of lane group g carries input element
// e = g*KS + ks, so each lane reads KS contiguous floats of x and of W.
template <int KS>
__device__ __forceinline__ void load_vec(const float* __restrict__ p, float (&v)[KS]) {
  if constexpr (KS % 4 == 0) {
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
      f4 t = *reinterpret_cast<const f4*>(p + 4 * q);
      v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
    }
  } else {
    static_assert(KS == 2, "din must be 8, 16, 32 or 64");
    f2 t = *reinterpret_cast<const f2*>(p);
    v[0] = t.x; v[1] = t.y;
  }
}

// Windowed input (naive:150-151): capsule i = w*N + n of frame (b,t) is
// emb[b, t + w - lpad, n] or zero outside [0, T).
__device__ __forceinline__ const float* window_src(const float* __restrict__ emb, int f, int F, int T,
                                                   int N, int din, int lpad, int i) {
  if (f >= F) return nullptr;
  const int w = i / N, n = i - w * N;
  const int b = f / T, t = f - b * T;
  const int ts = t + w - lpad;
  if (ts < 0 || ts >= T) return nullptr;
  return emb + ((size_t)(b * T + ts) * N + n) * din;
}

template <int DIN>
__device__ __forceinline__ void load_x(const float* __restrict__ src, int g, float (&x)[DIN / 4]) {
  constexpr int KS = DIN / 4;
  if (src) {
    load_vec<KS>(src + g * KS, x);
  } else {
#pragma unroll
    for (int k = 0; k < KS; ++k) x[k] = 0.f;
  }
}

// u tile (16 rows of (j,d) x 16 frames) for capsule i and global tile tg.
template <int DIN>
__device__ __forceinline__ f4 pose_tile(const float* __restrict__ W, const float* __restrict__ bias, int i,
                                        int JD, int tg, int lane, const float (&x)[DIN / 4]) {
  constexpr int KS = DIN / 4;
  const int arow = tg * 16 + (lane & 15);
  const int g = lane >> 4;
  float a[KS];
  if (arow < JD) {
    load_vec<KS>(W + ((size_t)i * JD + arow) * DIN + g * KS, a);
  } else {
#pragma unroll
    for (int k = 0; k < KS; ++k) a[k] = 0.f;
  }
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KS; ++k) acc = mfma16x16x4(a[k], x[k], acc);
  const int crow = tg * 16 + 4 * g;
  if (crow < JD) acc += *reinterpret_cast<const f4*>(bias + (size_t)i * JD + crow);
  return acc;
}

// Sum a per-lane partial over the rows of the output capsule j the lane's rows
// belong to.  Lane group g holds tile rows 4g..4g+3.
template <int DOUT, int TW>
__device__ __forceinline__ void jreduce(float (&p)[TW]) {
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    p[t] += __shfl_xor(p[t], 16, 64);
    if constexpr (DOUT >= 16) p[t] += __shfl_xor(p[t], 32, 64);
  }
  if constexpr (DOUT > 16) {
    constexpr int TPJ = DOUT / 16;
#pragma unroll
    for (int t0 = 0; t0 < TW; t0 += TPJ) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < TPJ; ++q) s += p[t0 + q];
#pragma unroll
      for (int q = 0; q < TPJ; ++q) p[t0 + q] = s;
    }
  }
}

template <int DOUT>
__device__ __forceinline__ int tile_j(int tg, int g) { return (tg * 16 + 4 * g) / DOUT; }

template <int DOUT>
__device__ __forceinline__ bool tile_primary(int tg) {
  if constexpr (DOUT > 16) return (tg % (DOUT / 16)) == 0;
  return true;
}

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// ---------------------------------------------------------------- routing pass
// grid: n_ftiles * n_chunks workgroups (chunk = blockIdx % n_chunks, so with
// n_chunks == 8 every XCD streams one i-chunk of W from its own L2);
// block: NW waves, wave w owns row tiles [w*TW, (w+1)*TW).
template <int DIN, int DOUT, int TW, int MODE>
__global__ __launch_bounds__(512) void route_pass_kernel(
    const float* __restrict__ emb, const float* __restrict__ W, const float* __restrict__ bias,
    int F, int T, int N, int lpad, int in_n, int J, int n_chunks, int chunk_len, int mask_first, int r,
    const float* __restrict__ vc, const float* __restrict__ gsv, float* __restrict__ slab,
    float* __restrict__ stats, int want_acc) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int JD = J * DOUT;
  const int NT = (JD + 15) / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int fl = lane & 15, g = lane >> 4;
  const int ft = blockIdx.x / n_chunks, chunk = blockIdx.x - ft * n_chunks;
  const int f = ft * 16 + fl;
  const bool fvalid = f < F;
  const int i0 = chunk * chunk_len, i1 = min(in_n, i0 + chunk_len);
  const int tbase = wv * TW;
  const int Jeff = J - (mask_first ? 1 : 0);

  float vcr[TW][4], gsr[TW][4], acc[TW][4];
  const bool use_vc = (r > 0);
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int row = (tbase + t) * 16 + 4 * g;
    const bool ok = fvalid && row < JD;
    f4 z = {0.f, 0.f, 0.f, 0.f};
    f4 a = (ok && use_vc) ? ld4(vc + (size_t)f * JD + row) : z;
    f4 b = z;
    if constexpr (MODE == MODE_BWD) b = ok ? ld4(gsv + (size_t)f * JD + row) : z;
    vcr[t][0] = a.x; vcr[t][1] = a.y; vcr[t][2] = a.z; vcr[t][3] = a.w;
    gsr[t][0] = b.x; gsr[t][1] = b.y; gsr[t][2] = b.z; gsr[t][3] = b.w;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[t][k] = 0.f;
  }

  int parity = 0;
  for (int i = i0; i < i1; ++i) {
    float x[DIN / 4];
    load_x<DIN>(window_src(emb, f, F, T, N, DIN, lpad, i), g, x);
    float u[TW][4];
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int tg = tbase + t;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (tg < NT) v = pose_tile<DIN>(W, bias, i, JD, tg, lane, x);
      u[t][0] = v.x; u[t][1] = v.y; u[t][2] = v.z; u[t][3] = v.w;
    }

    float c[TW];
    float gL[TW];
    if (MODE == MODE_FWD && r == 0) {
      // iteration 0: logits are 0 (+ the mask), so c is uniform (naive:172-181)
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int j = tile_j<DOUT>(tbase + t, g);
        const bool valid = j < J && !(mask_first && j == 0);
        c[t] = valid ? 1.f / (float)Jeff : 0.f;
      }
    } else {
      float p[TW], q[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        float s = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s += u[t][k] * vcr[t][k];
          s2 += u[t][k] * gsr[t][k];
        }
        p[t] = s;
        q[t] = s2;
      }
      jreduce<DOUT, TW>(p);
      if constexpr (MODE == MODE_BWD) jreduce<DOUT, TW>(q);
      // local softmax statistics over this lane's output capsules
      float m = -INFINITY;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int tg = tbase + t;
        const int j = tile_j<DOUT>(tg, g);
        if (tile_primary<DOUT>(tg) && j < J && !(mask_first && j == 0)) m = fmaxf(m, p[t]);
      }
      float z = 0.f, y = 0.f;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int tg = tbase + t;
        const int j = tile_j<DOUT>(tg, g);
        if (tile_primary<DOUT>(tg) && j < J && !(mask_first && j == 0)) {
          const float e = __expf(p[t] - m);
          z += e;
          if constexpr (MODE == MODE_BWD) y += e * q[t];
        }
      }
      if constexpr (DOUT == 8) {
        // lane groups {0,1} and {2,3} hold different capsules: combine
        const float mo = __shfl_xor(m, 32, 64), zo = __shfl_xor(z, 32, 64), yo = __shfl_xor(y, 32, 64);
        const float M = fmaxf(m, mo);
        const float s1 = (m == -INFINITY) ? 0.f : __expf(m - M);
        const float s2 = (mo == -INFINITY) ? 0.f : __expf(mo - M);
        z = z * s1 + zo * s2;
        y = y * s1 + yo * s2;
        m = M;
      }
      if (NW > 1) {
        float* slot = red + parity * (NW * 48);
        if (g == 0) {
          slot[wv * 48 + fl * 3 + 0] = m;
          slot[wv * 48 + fl * 3 + 1] = z;
          slot[wv * 48 + fl * 3 + 2] = y;
        }
        __syncthreads();
        float M = -INFINITY;
        for (int w = 0; w < NW; ++w) M = fmaxf(M, slot[w * 48 + fl * 3]);
        float Z = 0.f, Y = 0.f;
        for (int w = 0; w < NW; ++w) {
          const float mw = slot[w * 48 + fl * 3];
          if (mw != -INFINITY) {
            const float s = __expf(mw - M);
            Z += slot[w * 48 + fl * 3 + 1] * s;
            Y += slot[w * 48 + fl * 3 + 2] * s;
          }
        }
        m = M; z = Z; y = Y;
        parity ^= 1;
      }
      const float invz = 1.f / z;
      const float sigma = y * invz;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int j = tile_j<DOUT>(tbase + t, g);
        const bool valid = j < J && !(mask_first && j == 0);
        c[t] = valid ? __expf(p[t] - m) * invz : 0.f;
        gL[t] = c[t] * (q[t] - sigma);
      }
      if constexpr (MODE == MODE_BWD) {
        if (wv == 0 && g == 0 && fvalid) {
          stats[((size_t)f * in_n + i) * 2 + 0] = m + __logf(z);
          stats[((size_t)f * in_n + i) * 2 + 1] = sigma;
        }
      }
    }
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const float w = (MODE == MODE_FWD) ? c[t] : gL[t];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[t][k] += w * u[t][k];
    }
  }
  if (!want_acc) return;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int row = (tbase + t) * 16 + 4 * g;
    if (fvalid && row < JD) {
      f4 v = {acc[t][0], acc[t][1], acc[t][2], acc[t][3]};
      st4(slab + ((size_t)chunk * F + f) * JD + row, v);
    }
  }
}

// ---------------------------------------------------------------- gu pass
// gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j with c^r = exp(L^r - logZ^r),
// gL^r = c^r (<gs^r_j, u_ij> - sigma^r).  One wave = 16 frames x TW row tiles x
// an i-chunk; no cross-wave traffic.
template <int DIN, int DOUT, int TW, int R>
__global__ __launch_bounds__(256) void route_gu_kernel(
    const float* __restrict__ emb, const float* __restrict__ W, const float* __restrict__ bias, int F, int T,
    int N, int lpad, int in_n, int J, int mask_first, int n_tgroups, int n_chunks, int chunk_len,
    const float* __restrict__ saved, const float* __restrict__ gs, const float* __restrict__ stats,
    float* __restrict__ gu) {
  const int JD = J * DOUT;
  const int NT = (JD + 15) / 16;
  const size_t FJD = (size_t)F * JD;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fl = lane & 15, g = lane >> 4;
  const int n_ftiles = (F + 15) / 16;
  const int task = blockIdx.x * 4 + wv;
  if (task >= n_ftiles * n_tgroups * n_chunks) return;
  const int chunk = task % n_chunks;
  const int tgrp = (task / n_chunks) % n_tgroups;
  const int ft = task / (n_chunks * n_tgroups);
  const int f = ft * 16 + fl;
  const bool fvalid = f < F;
  const int tbase = tgrp * TW;
  const int i0 = chunk * chunk_len, i1 = min(in_n, i0 + chunk_len);

  float vcr[R][TW][4], gsr[R][TW][4];
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int row = (tbase + t) * 16 + 4 * g;
      const bool ok = fvalid && row < JD;
      f4 z = {0.f, 0.f, 0.f, 0.f};
      // Vc^r (r >= 1) is stored after iteration r-1 at saved[(r-1)*2+1]
      f4 a = (ok && r > 0) ? ld4(saved + (size_t)(2 * (r - 1) + 1) * FJD + (size_t)f * JD + row) : z;
      f4 b = ok ? ld4(gs + (size_t)r * FJD + (size_t)f * JD + row) : z;
      vcr[r][t][0] = a.x; vcr[r][t][1] = a.y; vcr[r][t][2] = a.z; vcr[r][t][3] = a.w;
      gsr[r][t][0] = b.x; gsr[r][t][1] = b.y; gsr[r][t][2] = b.z; gsr[r][t][3] = b.w;
    }
  }

  for (int i = i0; i < i1; ++i) {
    float x[DIN / 4];
    load_x<DIN>(window_src(emb, f, F, T, N, DIN, lpad, i), g, x);
    float u[TW][4], ga[TW][4];
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int tg = tbase + t;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (tg < NT) v = pose_tile<DIN>(W, bias, i, JD, tg, lane, x);
      u[t][0] = v.x; u[t][1] = v.y; u[t][2] = v.z; u[t][3] = v.w;
#pragma unroll
      for (int k = 0; k < 4; ++k) ga[t][k] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float p[TW], q[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        float s = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s += u[t][k] * vcr[r][t][k];
          s2 += u[t][k] * gsr[r][t][k];
        }
        p[t] = s;
        q[t] = s2;
      }
      if (r > 0) jreduce<DOUT, TW>(p);
      jreduce<DOUT, TW>(q);
      float logz = 0.f, sigma = 0.f;
      if (fvalid) {
        logz = stats[(((size_t)r * F + f) * in_n + i) * 2 + 0];
        sigma = stats[(((size_t)r * F + f) * in_n + i) * 2 + 1];
      }
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int j = tile_j<DOUT>(tbase + t, g);
        const bool valid = j < J && !(mask_first && j == 0);
        const float c = valid ? __expf(p[t] - logz) : 0.f;
        const float gl = c * (q[t] - sigma);
#pragma unroll
        for (int k = 0; k < 4; ++k) ga[t][k] += c * gsr[r][t][k] + gl * vcr[r][t][k];
      }
    }
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int row = (tbase + t) * 16 + 4 * g;
      if (fvalid && row < JD) {
        f4 v = {ga[t][0], ga[t][1], ga[t][2], ga[t][3]};
        st4(gu + ((size_t)f * in_n + i) * JD + row, v);
      }
    }
  }
}

// ---------------------------------------------------------------- gW, gbias
// gW[i][row][e] = sum_f gu[f][i][row] x[f][i][e]  (MFMA, K = frames);
// gbias[i][row] = sum_f gu[f][i][row].  One wave per (i, row tile).
template <int DIN>
__global__ __launch_bounds__(256) void route_gw_kernel(const float* __restrict__ gu,
                                                       const float* __restrict__ emb, int F, int T, int N,
                                                       int lpad, int in_n, int JD, float* __restrict__ gW,
                                                       float* __restrict__ gbias) {
  constexpr int NCT = (DIN + 15) / 16;
  const int NT = (JD + 15) / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int task = blockIdx.x * 4 + wv;
  if (task >= in_n * NT) return;
  const int i = task / NT, tg = task - i * NT;
  const int arow = tg * 16 + l16;
  const bool rvalid = arow < JD;
  f4 acc[NCT][2];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct][0] = acc[ct][1] = f4{0.f, 0.f, 0.f, 0.f};
  float gb = 0.f;
#pragma unroll 4
  for (int f0 = 0; f0 < F; f0 += 4) {
    const int f = f0 + g;
    const float a = (f < F && rvalid) ? gu[((size_t)f * in_n + i) * JD + arow] : 0.f;
    gb += a;
    const float* src = window_src(emb, f, F, T, N, DIN, lpad, i);
    const int h = (f0 >> 2) & 1;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int e = ct * 16 + l16;
      const float bx = (src && e < DIN) ? src[e] : 0.f;
      acc[ct][h] = mfma16x16x4(a, bx, acc[ct][h]);
    }
  }
  gb += __shfl_xor(gb, 16, 64);
  gb += __shfl_xor(gb, 32, 64);
  if (g == 0 && rvalid) gbias[(size_t)i * JD + arow] = gb;
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const f4 v = acc[ct][0] + acc[ct][1];
    const int e = ct * 16 + l16;
    if (e < DIN) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = tg * 16 + 4 * g + k;
        if (row < JD) gW[((size_t)i * JD + row) * DIN + e] = v[k];
      }
    }
  }
}

// ---------------------------------------------------------------- gx
// gx[f][i][e] = sum_row gu[f][i][row] W[i][row][e]  (MFMA, K = J*Dout).
template <int DIN>
__global__ __launch_bounds__(256) void route_gx_kernel(const float* __restrict__ gu,
                                                       const float* __restrict__ W, int F, int in_n, int JD,
                                                       float* __restrict__ gx) {
  constexpr int NCT = (DIN + 15) / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int n_ftiles = (F + 15) / 16;
  const int task = blockIdx.x * 4 + wv;
  if (task >= n_ftiles * in_n) return;
  const int ft = task / in_n, i = task - ft * in_n;
  const int f = ft * 16 + l16;
  const bool fvalid = f < F;
  const int KQ = JD / 4;  // JD is a multiple of 8
  const float* arow = gu + ((size_t)f * in_n + i) * JD + g * KQ;
  const float* brow = W + ((size_t)i * JD + g * KQ) * DIN;
  f4 acc[NCT][2];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct][0] = acc[ct][1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int s = 0; s < KQ; ++s) {
    const float a = fvalid ? arow[s] : 0.f;
    const int h = s & 1;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int e = ct * 16 + l16;
      const float b = (e < DIN) ? brow[(size_t)s * DIN + e] : 0.f;
      acc[ct][h] = mfma16x16x4(a, b, acc[ct][h]);
    }
  }
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const f4 v = acc[ct][0] + acc[ct][1];
    const int e = ct * 16 + l16;
    if (e < DIN) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int fo = ft * 16 + 4 * g + k;
        if (fo < F) gx[((size_t)fo * in_n + i) * DIN + e] = v[k];
      }
    }
  }
}

// Adjoint of the window (naive:150-151): g_emb[b,t,n] = sum_w gx[b, t-w+lpad, w*N+n].
__global__ void unwindow_kernel(const float* __restrict__ gx, int F, int T, int N, int din, int lpad, int win,
                                float* __restrict__ g_emb) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)F * N * din;
  if (idx >= total) return;
  const int e = idx % din;
  const int n = (idx / din) % N;
  const int f = idx / ((size_t)din * N);
  const int b = f / T, t = f - b * T;
  const int in_n = N * win;
  float s = 0.f;
  for (int w = 0; w < win; ++w) {
    const int tc = t - w + lpad;
    if (tc >= 0 && tc < T) s += gx[((size_t)(b * T + tc) * in_n + w * N + n) * din + e];
  }
  g_emb[idx] = s;
}

// ---------------------------------------------------------------- finish kernels
// s^r = sum over i-chunks; v^r = squash(s^r) (naive:204); Vc^{r+1} = Vc^r + v^r.
template <int DOUT>
__global__ void fwd_finish_kernel(const float* __restrict__ slab, int n_chunks, int F, int J,
                                  const float* __restrict__ vc_in, float* __restrict__ s_out,
                                  float* __restrict__ vc_out, float* __restrict__ v_out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= F * J) return;
  const size_t JD = (size_t)J * DOUT;
  const size_t base = (size_t)idx * DOUT;  // = f*JD + j*DOUT
  const size_t FJD = (size_t)F * JD;
  float s[DOUT];
#pragma unroll
  for (int d = 0; d < DOUT; d += 4) {
    f4 a = ld4(slab + base + d);
    for (int c = 1; c < n_chunks; ++c) a += ld4(slab + (size_t)c * FJD + base + d);
    s[d] = a.x; s[d + 1] = a.y; s[d + 2] = a.z; s[d + 3] = a.w;
  }
  float n2 = 0.f;
#pragma unroll
  for (int d = 0; d < DOUT; ++d) n2 += s[d] * s[d];
  const float fac = n2 / (1.f + n2) / sqrtf(n2 + kSquashEps);
#pragma unroll
  for (int d = 0; d < DOUT; d += 4) {
    const f4 sv = {s[d], s[d + 1], s[d + 2], s[d + 3]};
    const f4 v = sv * fac;
    st4(s_out + base + d, sv);
    f4 vc = v;
    if (vc_in) vc += ld4(vc_in + base + d);
    st4(vc_out + base + d, vc);
    if (v_out) st4(v_out + base + d, v);
  }
}

// gs = squash'(s)^T a with a = a_init (the upstream gradient of the last
// iteration's v) or, for earlier iterations, a = A += sum of gVc slabs.
template <int DOUT>
__global__ void bwd_finish_kernel(const float* __restrict__ slab, int n_chunks, int F, int J,
                                  const float* __restrict__ a_init, float* __restrict__ A,
                                  const float* __restrict__ s, float* __restrict__ gs) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= F * J) return;
  const size_t JD = (size_t)J * DOUT;
  const size_t base = (size_t)idx * DOUT;
  const size_t FJD = (size_t)F * JD;
  float a[DOUT], sv[DOUT];
#pragma unroll
  for (int d = 0; d < DOUT; d += 4) {
    f4 v;
    if (a_init) {
      v = ld4(a_init + base + d);
    } else {
      v = ld4(A + base + d);
      for (int c = 0; c < n_chunks; ++c) v += ld4(slab + (size_t)c * FJD + base + d);
      st4(A + base + d, v);
    }
    const f4 q = ld4(s + base + d);
    a[d] = v.x; a[d + 1] = v.y; a[d + 2] = v.z; a[d + 3] = v.w;
    sv[d] = q.x; sv[d + 1] = q.y; sv[d + 2] = q.z; sv[d + 3] = q.w;
  }
  float n2 = 0.f, sa = 0.f;
#pragma unroll
  for (int d = 0; d < DOUT; ++d) {
    n2 += sv[d] * sv[d];
    sa += sv[d] * a[d];
  }
  const float rs = 1.f / sqrtf(n2 + kSquashEps);
  const float ip = 1.f / (1.f + n2);
  const float gfac = n2 * ip * rs;
  const float dg = rs * ip * (ip - 0.5f * n2 / (n2 + kSquashEps));
#pragma unroll
  for (int d = 0; d < DOUT; d += 4) {
    f4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = gfac * a[d + k] + 2.f * dg * sa * sv[d + k];
    st4(gs + base + d, o);
  }
}

// ---------------------------------------------------------------- host side
struct PassCfg {
  int TW, NW;
};

PassCfg pass_cfg(const Geom& g) {
  const int NT = g.NT();
  int TW = 8;
  int NW = (NT + TW - 1) / TW;
  if (NW > 8) {
    TW = 16;
    NW = (NT + TW - 1) / TW;
  }
  return {TW, NW};
}

int auto_chunks(const Geom& g, int NW) {
  const int n_ftiles = (g.F() + 15) / 16;
  int c = (2560 + n_ftiles * NW - 1) / (n_ftiles * NW);
  if (c >= 8) c = c / 8 * 8;
  return std::max(1, std::min(c, g.in_n()));
}

int check_geom(const Geom& g) {
  SRF_REQUIRE(g.B > 0 && g.T > 0 && g.N > 0 && g.J > 1, "bad shape B=%d T=%d N=%d J=%d", g.B, g.T, g.N, g.J);
  SRF_REQUIRE(g.lpad >= 0 && g.rpad >= 0, "negative window pad");
  SRF_REQUIRE(g.iters >= 1 && g.iters <= 5, "routing iterations must be in [1,5], got %d", g.iters);
  SRF_REQUIRE(g.din == 8 || g.din == 16 || g.din == 32 || g.din == 64, "unsupported in_d %d", g.din);
  SRF_REQUIRE(g.dout == g.din, "in_d (%d) != out_d (%d) is not supported", g.din, g.dout);
  SRF_REQUIRE((long long)g.F() * g.in_n() * g.JD() < (1LL << 40), "problem too large");
  return SRF_OK;
}

template <int D, int TW, int MODE>
void launch_pass(const Geom& g, int NW, int n_chunks, const float* emb, const float* W, const float* bias, int r,
                 const float* vc, const float* gsv, float* slab, float* stats, int want_acc, hipStream_t st) {
  const int n_ftiles = (g.F() + 15) / 16;
  const int chunk_len = (g.in_n() + n_chunks - 1) / n_chunks;
  const size_t shmem = (NW > 1) ? (size_t)2 * NW * 48 * sizeof(float) : 16;
  hipLaunchKernelGGL((route_pass_kernel<D, D, TW, MODE>), dim3(n_ftiles * n_chunks), dim3(64 * NW), shmem, st,
                     emb, W, bias, g.F(), g.T, g.N, g.lpad, g.in_n(), g.J, n_chunks, chunk_len, g.mask_first, r,
                     vc, gsv, slab, stats, want_acc);
}

template <int D, int MODE>
void dispatch_pass(const Geom& g, const PassCfg& pc, int n_chunks, const float* emb, const float* W,
                   const float* bias, int r, const float* vc, const float* gsv, float* slab, float* stats,
                   int want_acc, hipStream_t st) {
  if (pc.TW == 8)
    launch_pass<D, 8, MODE>(g, pc.NW, n_chunks, emb, W, bias, r, vc, gsv, slab, stats, want_acc, st);
  else
    launch_pass<D, 16, MODE>(g, pc.NW, n_chunks, emb, W, bias, r, vc, gsv, slab, stats, want_acc, st);
}

template <int D>
void launch_fwd_finish(const Geom& g, const float* slab, int n_chunks, const float* vc_in, float* s_out,
                       float* vc_out, float* v_out, hipStream_t st) {
  const int n = g.F() * g.J;
  hipLaunchKernelGGL((fwd_finish_kernel<D>), dim3((n + 255) / 256), dim3(256), 0, st, slab, n_chunks, g.F(), g.J,
                     vc_in, s_out, vc_out, v_out);
}

template <int D>
void launch_bwd_finish(const Geom& g, const float* slab, int n_chunks, const float* a_init, float* A,
                       const float* s, float* gs, hipStream_t st) {
  const int n = g.F() * g.J;
  hipLaunchKernelGGL((bwd_finish_kernel<D>), dim3((n + 255) / 256), dim3(256), 0, st, slab, n_chunks, g.F(), g.J,
                     a_init, A, s, gs);
}

template <int D, int R>
void launch_gu(const Geom& g, int n_chunks, const float* emb, const float* W, const float* bias, const float* saved,
               const float* gs, const float* stats, float* gu, hipStream_t st) {
  constexpr int TW = (D >= 64) ? 4 : 4;
  const int n_ftiles = (g.F() + 15) / 16;
  const int n_tgroups = (g.NT() + TW - 1) / TW;
  const int chunk_len = (g.in_n() + n_chunks - 1) / n_chunks;
  const int tasks = n_ftiles * n_tgroups * n_chunks;
  hipLaunchKernelGGL((route_gu_kernel<D, D, TW, R>), dim3((tasks + 3) / 4), dim3(256), 0, st, emb, W, bias, g.F(),
                     g.T, g.N, g.lpad, g.in_n(), g.J, g.mask_first, n_tgroups, n_chunks, chunk_len, saved, gs,
                     stats, gu);
}

template <int D>
void launch_gu_r(const Geom& g, int n_chunks, const float* emb, const float* W, const float* bias,
                 const float* saved, const float* gs, const float* stats, float* gu, hipStream_t st) {
  switch (g.iters) {
    case 1: launch_gu<D, 1>(g, n_chunks, emb, W, bias, saved, gs, stats, gu, st); break;
    case 2: launch_gu<D, 2>(g, n_chunks, emb, W, bias, saved, gs, stats, gu, st); break;
    case 3: launch_gu<D, 3>(g, n_chunks, emb, W, bias, saved, gs, stats, gu, st); break;
    case 4: launch_gu<D, 4>(g, n_chunks, emb, W, bias, saved, gs, stats, gu, st); break;
    default: launch_gu<D, 5>(g, n_chunks, emb, W, bias, saved, gs, stats, gu, st); break;
  }
}

template <int D>
int fwd_impl(const Geom& g, int n_chunks, const float* emb, const float* W, const float* bias, float* v_out,
             float* saved, float* slab, hipStream_t st) {
  const PassCfg pc = pass_cfg(g);
  const size_t FJD = (size_t)g.F() * g.JD();
  for (int r = 0; r < g.iters; ++r) {
    const float* vc = r > 0 ? saved + (size_t)(2 * (r - 1) + 1) * FJD : nullptr;
    dispatch_pass<D, MODE_FWD>(g, pc, n_chunks, emb, W, bias, r, vc, nullptr, slab, nullptr, 1, st);
    SRF_LAUNCH_CHECK("route_pass(fwd)");
    launch_fwd_finish<D>(g, slab, n_chunks, vc, saved + (size_t)(2 * r) * FJD, saved + (size_t)(2 * r + 1) * FJD,
                         r == g.iters - 1 ? v_out : nullptr, st);
    SRF_LAUNCH_CHECK("fwd_finish");
  }
  return SRF_OK;
}

struct BwdWs {
  float *A, *gs, *slab, *stats, *gu, *gx;
  size_t bytes;
};

BwdWs bwd_layout(const Geom& g, int n_chunks, void* base) {
  const size_t F = g.F(), JD = g.JD(), in_n = g.in_n();
  size_t off = 0;
  auto take = [&](size_t nfloat) {
    size_t o = off;
    off += srf::align_up(nfloat * sizeof(float), 256);
    return o;
  };
  const size_t oA = take(F * JD), ogs = take((size_t)g.iters * F * JD), oslab = take((size_t)n_chunks * F * JD),
               ostats = take((size_t)g.iters * F * in_n * 2), ogu = take(F * in_n * JD), ogx = take(F * in_n * g.din);
  char* b = static_cast<char*>(base);
  BwdWs w;
  w.A = (float*)(b + oA);
  w.gs = (float*)(b + ogs);
  w.slab = (float*)(b + oslab);
  w.stats = (float*)(b + ostats);
  w.gu = (float*)(b + ogu);
  w.gx = (float*)(b + ogx);
  w.bytes = off;
  return w;
}

template <int D>
int bwd_impl(const Geom& g, int n_chunks, const float* emb, const float* W, const float* bias, const float* saved,
             const float* g_v, float* g_emb, float* g_W, float* g_bias, const BwdWs& w, hipStream_t st) {
  const PassCfg pc = pass_cfg(g);
  const size_t FJD = (size_t)g.F() * g.JD();
  const int R = g.iters;
  // gs^{R-1} = squash'(s^{R-1}) g_v.  A accumulates sum_{r'>r} gVc^{r'}, the
  // gradient of v^r for r < R-1 (those v reach the loss only through the logits).
  SRF_HIP_TRY(hipMemsetAsync(w.A, 0, FJD * sizeof(float), st));
  launch_bwd_finish<D>(g, nullptr, n_chunks, g_v, w.A, saved + (size_t)(2 * (R - 1)) * FJD,
                       w.gs + (size_t)(R - 1) * FJD, st);
  SRF_LAUNCH_CHECK("bwd_finish");
  for (int r = R - 1; r >= 0; --r) {
    const float* vc = r > 0 ? saved + (size_t)(2 * (r - 1) + 1) * FJD : nullptr;
    float* stats_r = w.stats + (size_t)r * g.F() * g.in_n() * 2;
    dispatch_pass<D, MODE_BWD>(g, pc, n_chunks, emb, W, bias, r, vc, w.gs + (size_t)r * FJD, w.slab, stats_r,
                               r > 0 ? 1 : 0, st);
    SRF_LAUNCH_CHECK("route_pass(bwd)");
    if (r > 0) {
      launch_bwd_finish<D>(g, w.slab, n_chunks, nullptr, w.A, saved + (size_t)(2 * (r - 1)) * FJD,
                           w.gs + (size_t)(r - 1) * FJD, st);
      SRF_LAUNCH_CHECK("bwd_finish");
    }
  }
  launch_gu_r<D>(g, n_chunks, emb, W, bias, saved, w.gs, w.stats, w.gu, st);
  SRF_LAUNCH_CHECK("route_gu");
  {
    const int tasks = g.in_n() * g.NT();
    hipLaunchKernelGGL((route_gw_kernel<D>), dim3((tasks + 3) / 4), dim3(256), 0, st, w.gu, emb, g.F(), g.T, g.N,
                       g.lpad, g.in_n(), g.JD(), g_W, g_bias);
    SRF_LAUNCH_CHECK("route_gw");
  }
  {
    const int tasks = ((g.F() + 15) / 16) * g.in_n();
    hipLaunchKernelGGL((route_gx_kernel<D>), dim3((tasks + 3) / 4), dim3(256), 0, st, w.gu, W, g.F(), g.in_n(),
                       g.JD(), w.gx);
    SRF_LAUNCH_CHECK("route_gx");
  }
  {
    const size_t total = (size_t)g.F() * g.N * g.din;
    hipLaunchKernelGGL(unwindow_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w.gx, g.F(), g.T, g.N, g.din,
                       g.lpad, g.lpad + g.rpad + 1, g_emb);
    SRF_LAUNCH_CHECK("unwindow");
  }
  return SRF_OK;
}

}  // namespace

extern "C" {

int srf_route_dr_auto_chunks(int B, int T, int N, int din, int lpad, int rpad, int J, int dout) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  return auto_chunks(g, pass_cfg(g).NW);
}

size_t srf_route_dr_saved_floats(int B, int T, int J, int dout, int iters) {
  return (size_t)2 * iters * B * T * J * dout;
}

size_t srf_route_dr_fwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters,
                                  int n_chunks) {
  (void)N; (void)din; (void)lpad; (void)rpad; (void)iters;
  return (size_t)n_chunks * B * T * J * dout * sizeof(float);
}

size_t srf_route_dr_bwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters,
                                  int n_chunks) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, iters, 0};
  return bwd_layout(g, n_chunks, nullptr).bytes;
}

int srf_route_dr_fwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int iters, int mask_first, int n_chunks, float* v_out, float* saved,
                     void* workspace, size_t workspace_bytes, void* stream) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, iters, mask_first ? 1 : 0};
  int rc = check_geom(g);
  if (rc) return rc;
  SRF_REQUIRE(emb && W && bias && v_out && saved && workspace, "null pointer argument");
  SRF_REQUIRE(n_chunks >= 1 && n_chunks <= g.in_n(), "n_chunks %d out of [1, %d]", n_chunks, g.in_n());
  const size_t need = srf_route_dr_fwd_workspace(B, T, N, din, lpad, rpad, J, dout, iters, n_chunks);
  if (workspace_bytes < need) {
    srf::set_error("forward workspace too small: %zu < %zu", workspace_bytes, need);
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* slab = static_cast<float*>(workspace);
  switch (din) {
    case 8: return fwd_impl<8>(g, n_chunks, emb, W, bias, v_out, saved, slab, st);
    case 16: return fwd_impl<16>(g, n_chunks, emb, W, bias, v_out, saved, slab, st);
    case 32: return fwd_impl<32>(g, n_chunks, emb, W, bias, v_out, saved, slab, st);
    default: return fwd_impl<64>(g, n_chunks, emb, W, bias, v_out, saved, slab, st);
  }
}

int srf_route_dr_bwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int iters, int mask_first, int n_chunks, const float* saved,
                     const float* g_v, float* g_emb, float* g_W, float* g_bias, void* workspace,
                     size_t workspace_bytes, void* stream) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, iters, mask_first ? 1 : 0};
  int rc = check_geom(g);
  if (rc) return rc;
  SRF_REQUIRE(emb && W && bias && saved && g_v && g_emb && g_W && g_bias && workspace, "null pointer argument");
  SRF_REQUIRE(n_chunks >= 1 && n_chunks <= g.in_n(), "n_chunks %d out of [1, %d]", n_chunks, g.in_n());
  BwdWs w = bwd_layout(g, n_chunks, workspace);
  if (workspace_bytes < w.bytes) {
    srf::set_error("backward workspace too small: %zu < %zu", workspace_bytes, w.bytes);
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (din) {
    case 8: return bwd_impl<8>(g, n_chunks, emb, W, bias, saved, g_v, g_emb, g_W, g_bias, w, st);
    case 16: return bwd_impl<16>(g, n_chunks, emb, W, bias, saved, g_v, g_emb, g_W, g_bias, w, st);
    case 32: return bwd_impl<32>(g, n_chunks, emb, W, bias, saved, g_v, g_emb, g_W, g_bias, w, st);
    default: return bwd_impl<64>(g, n_chunks, emb, W, bias, saved, g_v, g_emb, g_W, g_bias, w, st);
  }
}

}  // extern "C"
