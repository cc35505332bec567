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
#include "route_fwd32.h"
#include "../../include/srf.h"
#include "../../include/srf_prof.h"

namespace {

constexpr float kSquashEps = 1e-7f;  // naive:248

// Opt-in profiling hook (srf_route_dr_set_timing_events): events recorded on the
// launch stream around each forward routing-pass kernel of the next
// srf_route_dr_fwd call made by this thread, then cleared.
thread_local hipEvent_t* t_ev_start = nullptr;
thread_local hipEvent_t* t_ev_stop = nullptr;
thread_local int t_ev_n = 0;
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
//
// Loads are never predicated: row indices past J*Dout (only in the last, partial
// row tile) and tile indices past NT are clamped to valid addresses.  Such rows
// belong to output capsules j >= J, whose coupling c is exactly 0, so they never
// reach a valid output; keeping every load unconditional lets hipcc batch them
// instead of serialising load -> wait -> MFMA behind exec-mask branches.
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

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// Frame coordinates of one lane, computed once per kernel.
struct FrameLoc {
  int b, t;
  bool valid;
};

__device__ __forceinline__ FrameLoc frame_loc(int f, int F, int T) {
  const int fc = min(f, F - 1);
  FrameLoc r;
  r.b = fc / T;
  r.t = fc - r.b * T;
  r.valid = f < F;
  return r;
}

// Windowed input (naive:150-151): capsule i = w*N + n of frame (b,t) is
// emb[b, t + w - lpad, n] or zero outside [0, T).
template <int DIN>
__device__ __forceinline__ void load_x(const float* __restrict__ emb, const FrameLoc& fl, int T, int N, int lpad,
                                       int i, int g, float (&x)[DIN / 4]) {
  constexpr int KS = DIN / 4;
  const int w = i / N, n = i - w * N;
  const int ts = fl.t + w - lpad;
  const bool ok = fl.valid && ts >= 0 && ts < T;
  const int tsc = min(max(ts, 0), T - 1);
  load_vec<KS>(emb + ((size_t)(fl.b * T + tsc) * N + n) * DIN + g * KS, x);
#pragma unroll
  for (int k = 0; k < KS; ++k) x[k] = ok ? x[k] : 0.f;
}

// u tile (16 rows of (j,d) x 16 frames) for capsule i and global tile tg.
template <int DIN>
__device__ __forceinline__ f4 pose_tile(const float* __restrict__ W, const float* __restrict__ bias, int i,
                                        int JD, int NT, int tg, int lane, const float (&x)[DIN / 4]) {
  constexpr int KS = DIN / 4;
  const int tc = min(tg, NT - 1);
  const int arow = min(tc * 16 + (lane & 15), JD - 1);
  const int g = lane >> 4;
  float a[KS];
  load_vec<KS>(W + ((size_t)i * JD + arow) * DIN + g * KS, a);
  const int crow = min(tc * 16 + 4 * g, JD - 4);
  f4 acc = ld4(bias + (size_t)i * JD + crow);
#pragma unroll
  for (int k = 0; k < KS; ++k) acc = mfma16x16x4(a[k], x[k], acc);
  return acc;
}

// Sum a per-lane partial over the rows of the output capsule j the lane's rows
// belong to.  Lane group g holds tile rows 4g..4g+3.
template <int DOUT, int TW>
__device__ __forceinline__ void jreduce(float (&p)[TW]) {
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    p[t] = xor16_sum(p[t]);
    if constexpr (DOUT >= 16) p[t] = xor32_sum(p[t]);
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

// Per-frame vector rows 4g..4g+3 of tile tg (zero past J*Dout or past F).
__device__ __forceinline__ void load_rows(const float* __restrict__ v, int f, bool fvalid, int JD, int tg, int g,
                                          float (&o)[4]) {
  const int row = tg * 16 + 4 * g;
  const bool ok = fvalid && row < JD;
  const f4 a = ld4(v + (size_t)(fvalid ? f : 0) * JD + min(row, JD - 4));
  o[0] = ok ? a.x : 0.f; o[1] = ok ? a.y : 0.f; o[2] = ok ? a.z : 0.f; o[3] = ok ? a.w : 0.f;
}

// ---------------------------------------------------------------- routing pass
// Operand fragments of one input capsule i for a wave's TW row tiles.
template <int DIN, int TW>
struct Frags {
  float x[DIN / 4];
  float w[TW][DIN / 4];
  f4 b[TW];
};

// NOBIAS: fragments without the bias (the accumulators start at 0); the
// iteration-0 forward pass adds the i-chunk's bias sum once at the end instead.
template <int DIN, int TW, bool NOBIAS = false>
__device__ __forceinline__ void fetch_frags(const float* __restrict__ emb, const float* __restrict__ W,
                                            const float* __restrict__ bias, const FrameLoc& loc, int T, int N,
                                            int lpad, int i, int JD, int NT, int tbase, int lane,
                                            Frags<DIN, TW>& fr) {
  constexpr int KS = DIN / 4;
  const int g = lane >> 4;
  load_x<DIN>(emb, loc, T, N, lpad, i, g, fr.x);
  // Tile bases are wave-uniform (scalar registers); one per-lane offset serves
  // every tile.  J*Dout is a multiple of 16 for Dout >= 16, so only Dout == 8
  // needs the per-lane row clamp of the last, partial tile.
  const float* Wi = W + (size_t)i * JD * DIN;
  const float* bi = bias + (size_t)i * JD;
  int lrow = lane & 15, brow = 4 * g;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int tc = __builtin_amdgcn_readfirstlane(min(tbase + t, NT - 1));
    if constexpr (DIN < 16) {
      lrow = min(tc * 16 + (lane & 15), JD - 1) - tc * 16;
      brow = min(tc * 16 + 4 * g, JD - 4) - tc * 16;
    }
    load_vec<KS>(Wi + (size_t)tc * 16 * DIN + lrow * DIN + g * KS, fr.w[t]);
    if constexpr (NOBIAS) {
      fr.b[t] = f4{0.f, 0.f, 0.f, 0.f};
    } else {
      fr.b[t] = ld4(bi + tc * 16 + brow);
    }
  }
}

template <int DIN, int TW>
__device__ __forceinline__ void pose_tiles(const Frags<DIN, TW>& fr, float (&u)[TW][4]) {
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    f4 acc = fr.b[t];
#pragma unroll
    for (int k = 0; k < DIN / 4; ++k) acc = mfma16x16x4(fr.w[t][k], fr.x[k], acc);
    u[t][0] = acc.x; u[t][1] = acc.y; u[t][2] = acc.z; u[t][3] = acc.w;
  }
}

// Per-wave state of a routing pass over one frame tile.
template <int TW>
struct PassState {
  float vcr[TW][4], gsr[TW][4], acc[TW][4];
};

// One input capsule i of a routing pass: u tile -> logits <u, Vc> -> softmax
// over all output capsules (cross-wave through LDS) -> accumulate.
template <int DIN, int DOUT, int TW, int MODE, bool FIRST>
__device__ __forceinline__ void pass_step(float (&u)[TW][4], Frags<DIN, TW>& fr, PassState<TW>& st, float* red,
                                          int& parity, int i,
                                          int r, int J, int Jeff, int mask_first, int tbase, int wv, int NW, int lane,
                                          int in_n, int f, bool fvalid, float* __restrict__ stats,
                                          const float* __restrict__ emb, const float* __restrict__ W,
                                          const float* __restrict__ bias, const FrameLoc& loc, int T, int N,
                                          int lpad, int inext, int JD, int NT) {
  const int fl = lane & 15, g = lane >> 4;
  // software pipeline: u holds capsule i; the MFMAs for capsule i+1 issue now and
  // run on the matrix cores while this capsule's softmax runs on the VALU; the
  // fragments they consumed are refilled with capsule inext (= i+2)
  // (forward only: the backward pass has no registers to spare for it)
  constexpr bool PIPE = MODE == MODE_FWD && DIN <= 16;
  float unx[TW][4];
  if constexpr (PIPE) {
    pose_tiles<DIN, TW>(fr, unx);
  } else {
    pose_tiles<DIN, TW>(fr, u);
  }
  fetch_frags<DIN, TW, MODE == MODE_FWD && FIRST>(emb, W, bias, loc, T, N, lpad, inext, JD, NT, tbase, lane, fr);
  float c[TW];
  float gL[TW];
  if constexpr (MODE == MODE_FWD && FIRST) {
    // iteration 0: logits are 0 (+ the mask), so c is uniform (naive:172-181)
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int j = tile_j<DOUT>(tbase + t, g);
      const bool valid = j < J && !(mask_first && j == 0);
      c[t] = valid ? 1.f / (float)Jeff : 0.f;
      gL[t] = 0.f;
    }
  } else {
    float p[TW], q[TW];
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      float s = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s += u[t][k] * st.vcr[t][k];
        if constexpr (MODE == MODE_BWD) s2 += u[t][k] * st.gsr[t][k];
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
      const bool ok = tile_primary<DOUT>(tg) && j < J && !(mask_first && j == 0);
      const float e = ok ? __expf(p[t] - m) : 0.f;
      z += e;
      if constexpr (MODE == MODE_BWD) y += e * q[t];
    }
    if constexpr (DOUT == 8) {
      // lane groups {0,1} and {2,3} hold different capsules: combine
      float ma, mb, za, zb, ya, yb;
      xpair32(m, ma, mb);
      xpair32(z, za, zb);
      xpair32(y, ya, yb);
      const float M = fmaxf(ma, mb);
      const float s1 = (ma == -INFINITY) ? 0.f : __expf(ma - M);
      const float s2 = (mb == -INFINITY) ? 0.f : __expf(mb - M);
      z = za * s1 + zb * s2;
      y = ya * s1 + yb * s2;
      m = M;
    }
    if constexpr (PIPE) {
      // interleave the next capsule's MFMAs with this capsule's softmax VALU work
#pragma unroll
      for (int k = 0; k < TW * DIN / 4; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      }
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
        const float sc = (mw == -INFINITY) ? 0.f : __expf(mw - M);
        Z += slot[w * 48 + fl * 3 + 1] * sc;
        Y += slot[w * 48 + fl * 3 + 2] * sc;
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
    for (int k = 0; k < 4; ++k) {
      st.acc[t][k] += w * u[t][k];
      if constexpr (PIPE) u[t][k] = unx[t][k];
    }
  }
}

// grid: n_ftiles * n_chunks workgroups (chunk = blockIdx % n_chunks, so when
// n_chunks divides 8 the workgroups of one i-chunk share an XCD and its L2);
// block: NW waves, wave w owns row tiles [w*TW, (w+1)*TW).  The fragments of
// capsule i+1 are fetched before capsule i is processed (two register sets,
// loop unrolled by 2), so the loads fly across the softmax barrier.
template <int DIN, int DOUT, int TW, int MODE, bool FIRST>
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
  const FrameLoc loc = frame_loc(f, F, T);
  const int i0 = chunk * chunk_len, i1 = min(in_n, i0 + chunk_len);
  const int tbase = __builtin_amdgcn_readfirstlane(wv * TW);
  const int Jeff = J - (mask_first ? 1 : 0);

  PassState<TW> st;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    if (r > 0) {
      load_rows(vc, f, loc.valid, JD, tbase + t, g, st.vcr[t]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) st.vcr[t][k] = 0.f;
    }
    if constexpr (MODE == MODE_BWD) {
      load_rows(gsv, f, loc.valid, JD, tbase + t, g, st.gsr[t]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) st.gsr[t][k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) st.acc[t][k] = 0.f;
  }

  int parity = 0;
  if (i0 < i1) {
    constexpr int AHEAD = (MODE == MODE_FWD && DIN <= 16) ? 2 : 1;   // capsules between a fetch and its use
    Frags<DIN, TW> fr;
    float u[TW][4];
    constexpr bool NB = MODE == MODE_FWD && FIRST;
    fetch_frags<DIN, TW, NB>(emb, W, bias, loc, T, N, lpad, i0, JD, NT, tbase, lane, fr);
    if constexpr (AHEAD == 2) {
      pose_tiles<DIN, TW>(fr, u);
      fetch_frags<DIN, TW, NB>(emb, W, bias, loc, T, N, lpad, min(i0 + 1, i1 - 1), JD, NT, tbase, lane, fr);
    }
    for (int i = i0; i < i1; ++i) {
      pass_step<DIN, DOUT, TW, MODE, FIRST>(u, fr, st, red, parity, i, r, J, Jeff, mask_first, tbase, wv, NW, lane, in_n, f,
                                     loc.valid, stats, emb, W, bias, loc, T, N, lpad, min(i + AHEAD, i1 - 1), JD, NT);
    }
  }
  if (!want_acc) return;
  if constexpr (MODE == MODE_FWD && FIRST) {
    // uniform couplings: the bias enters once, as c * (sum of the chunk's biases), gsv = that sum
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int j = tile_j<DOUT>(tbase + t, g);
      const float c0 = (j < J && !(mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
      float bs[4];
      load_rows(gsv + (size_t)chunk * JD, 0, true, JD, tbase + t, g, bs);
#pragma unroll
      for (int k = 0; k < 4; ++k) st.acc[t][k] += c0 * bs[k];
    }
  }
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int row = (tbase + t) * 16 + 4 * g;
    if (loc.valid && row < JD) {
      f4 v = {st.acc[t][0], st.acc[t][1], st.acc[t][2], st.acc[t][3]};
      st4(slab + ((size_t)chunk * F + f) * JD + row, v);
    }
  }
}

// bsum[c][row] = sum of bias[i][row] over the capsules i of i-chunk c.
__global__ void bias_chunk_sum_kernel(const float* __restrict__ bias, int in_n, int JD, int n_chunks,
                                      int chunk_len, float* __restrict__ bsum) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_chunks * JD) return;
  const int c = idx / JD, row = idx - c * JD;
  const int i0 = c * chunk_len, i1 = min(in_n, i0 + chunk_len);
  float acc = 0.f;
  for (int i = i0; i < i1; ++i) acc += bias[(size_t)i * JD + row];
  bsum[idx] = acc;
}

// ---------------------------------------------------------------- gu pass
// gu_ij = c^0_ij gs^0_j + sum_{r>=1} c^r_ij gs^r_j + gL^r_ij Vc^r_j with
// c^r = exp(L^r - logZ^r), gL^r = c^r (<gs^r_j, u_ij> - sigma^r).  Vc^0 = 0, so
// iteration 0 has uniform c^0 = 1/J_eff and no logit term.  Only per-(frame,i)
// scalars are shared across output capsules, so the waves of a workgroup (one
// frame tile, TW row tiles each) are independent.  Per input capsule i a wave
//   * stores gu for the gW pass in 16x16 blocks, gu_t[i][frame tile][row tile][f][row]
//     (one contiguous 1 KiB float4 store per block);
//   * contracts gx^T[e][f] = sum_row W^T[i][e][row] gu[row][f] on the matrix cores
//     straight from the gu registers (float4 loads of the transposed W) and adds
//     it, through the window adjoint (naive:150-151), into an LDS accumulator of
//     the workgroup's output frames (ds_add, no barrier per capsule);
// the accumulator is flushed into g_emb with one atomic add per element at the end.
// When the accumulator does not fit in LDS (wide windows) the adds go to g_emb.
// CPL: the couplings c^r and logit gradients gL^r of the 32x32 passes are given
// (cst, glst: [r-1][in_n][JP][Fs], frame-minor), so gu needs
// neither the pose nor any logit: gu_ij = c^0 gs^0_j + sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j.
//
// gx accumulator layout: a frame slot (row) holds n_per*din floats; lane 16*g + fl
// updates row w + fl at float4 column chunk g of a 16-float block with one
// ds_read_b128 + ds_write_b128.  A ds_read_b128 is serviced per lane group
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) over 64 banks, a ds_write_b128 per
// 8 contiguous lanes over 32 banks.  With a plain stride no value serves both (4
// mod 64: 2-way reads; 8 mod 16: 2-way writes), so for din % 16 == 0 the row
// stride is 16 (mod 32) and chunk g of row s sits at g ^ ((s >> 1) & 3): every
// group of either instruction then covers distinct banks for any window offset w.
__host__ __device__ constexpr int gu_row_stride(int n_per, int din) {
  return din % 16 ? n_per * din + 4 : n_per * din + ((n_per * din) % 32 == 16 ? 0 : 16);
}
// float offset inside row `slot` of the row element `col`
template <int DIN>
__device__ __forceinline__ int gu_acc_col(int slot, int col) {
  if constexpr (DIN % 16 == 0) return col ^ (((slot >> 1) & 3) << 2);
  return col;
}

template <int DIN, int DOUT, int TW, int R, bool LDSACC, bool CPL = false>
__global__ __launch_bounds__(256, (DIN <= 16 ? 4 : 3)) void route_gu_kernel(
    const float* __restrict__ emb, const float* __restrict__ W, const float* __restrict__ WT,
    const float* __restrict__ bias, int F, int Fp, int T, int N, int lpad, int rpad, int in_n, int J,
    int mask_first, int n_wgroups, int n_chunks, int n_per, const float* __restrict__ saved,
    const float* __restrict__ gs, const float* __restrict__ stats, float* __restrict__ gu_t,
    float* __restrict__ g_emb, int nslots_max, const float* __restrict__ cst = nullptr,
    const float* __restrict__ glst = nullptr, int JP = 0) {
  constexpr int NCT = (DIN + 15) / 16;
  constexpr int RV = R > 1 ? R - 1 : 1;
  extern __shared__ __attribute__((aligned(16))) float gacc[];
  const int JD = J * DOUT;
  const int NT = (JD + 15) / 16;
  const size_t FJD = (size_t)F * JD;
  const int NW = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fl = lane & 15, g = lane >> 4;
  const int chunk = blockIdx.x % n_chunks;
  const int rest = blockIdx.x / n_chunks;
  const int wgrp = rest % n_wgroups;
  const int ft = rest / n_wgroups;
  const int f = ft * 16 + fl;
  const FrameLoc loc = frame_loc(f, F, T);
  const int tbase = __builtin_amdgcn_readfirstlane((wgrp * NW + wv) * TW);
  // i-chunk = input capsules (w, n) with n in [n0, n1) and every window offset w,
  // visited w-major; capsule k of the chunk is i = w*N + n.
  const int n0 = chunk * n_per, nn = min(N, n0 + n_per) - n0;
  const int Wn = in_n / N;
  const int ncap = Wn * nn;
  auto cap = [&](int k) { return (k / nn) * N + n0 + k % nn; };
  const int Jeff = J - (mask_first ? 1 : 0);
  // Per-wave gx accumulators (no LDS atomics): frame slot s <-> emb frame
  // ft*16 - lpad + s, row (n - n0, e); the stride keeps float4 rows bank-conflict free.
  const int SROW = gu_row_stride(n_per, DIN);
  const int nslots = 15 + Wn;
  float* gw_acc = gacc + (size_t)wv * nslots_max * SROW;

  if constexpr (LDSACC) {
    for (int k = threadIdx.x; k < NW * nslots_max * SROW; k += blockDim.x) gacc[k] = 0.f;
    __syncthreads();
  }

  float vcr[RV][TW][4], gsr[R][TW][4];
  float c0[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int j = tile_j<DOUT>(tbase + t, g);
    c0[t] = (j < J && !(mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r > 0) load_rows(saved + (size_t)(2 * (r - 1) + 1) * FJD, f, loc.valid, JD, tbase + t, g, vcr[r - 1][t]);
      load_rows(gs + (size_t)r * FJD, f, loc.valid, JD, tbase + t, g, gsr[r][t]);
    }
  }

  // transposed W rows for the gx contraction and the softmax stats of capsule i
  auto fetch_side = [&](int i, f4 (&wt)[NCT][TW], float (&logz)[RV], float (&sig)[RV]) {
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const int e = min(ct * 16 + fl, DIN - 1);
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int tc = min(tbase + t, NT - 1);
        wt[ct][t] = ld4(WT + ((size_t)i * DIN + e) * JD + min(tc * 16 + 4 * g, JD - 4));
      }
    }
    if constexpr (!CPL) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const f2 st = *reinterpret_cast<const f2*>(stats + (((size_t)(r - 1) * F + (loc.valid ? f : 0)) * in_n + i) * 2);
        logz[r - 1] = st.x;
        sig[r - 1] = st.y;
      }
    }
  };

  // stored couplings / logit gradients: [r-1][in_n][JP][Fs], frame-minor
  const int Fs = srf::fwd32_frame_stride(F);
  int cpos[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) cpos[t] = min(tile_j<DOUT>(tbase + t, g), J - 1);
  const size_t cblk = (size_t)in_n * JP * Fs;
  if (ncap > 0) {
    Frags<DIN, TW> fr;
    f4 wt[NCT][TW];
    float logz[RV], sig[RV];
    if constexpr (!CPL) fetch_frags<DIN, TW>(emb, W, bias, loc, T, N, lpad, cap(0), JD, NT, tbase, lane, fr);
    for (int k = 0; k < ncap; ++k) {
      const int i = cap(k);
      fetch_side(i, wt, logz, sig);
      float ga[TW][4];
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int k = 0; k < 4; ++k) ga[t][k] = c0[t] * gsr[0][t][k];
      if constexpr (CPL) {
        const size_t fi = (size_t)i * JP * Fs + (loc.valid ? f : 0);
#pragma unroll
        for (int r = 1; r < R; ++r)
#pragma unroll
          for (int t = 0; t < TW; ++t) {
            const size_t o = (size_t)(r - 1) * cblk + fi + (size_t)cpos[t] * Fs;
            const float c = cst[o];
            const float gl = glst[o];
#pragma unroll
            for (int k = 0; k < 4; ++k) ga[t][k] += c * gsr[r][t][k] + gl * vcr[r - 1][t][k];
          }
      }
      if constexpr (!CPL) {
      float u[TW][4];
      pose_tiles<DIN, TW>(fr, u);
      // operands of the next capsule are fetched now and land while this one is processed
      const int inext = cap(min(k + 1, ncap - 1));
      fetch_frags<DIN, TW>(emb, W, bias, loc, T, N, lpad, inext, JD, NT, tbase, lane, fr);
#pragma unroll
      for (int r = 1; r < R; ++r) {
        float p[TW], q[TW];
#pragma unroll
        for (int t = 0; t < TW; ++t) {
          float s = 0.f, s2 = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            s += u[t][k] * vcr[r - 1][t][k];
            s2 += u[t][k] * gsr[r][t][k];
          }
          p[t] = s;
          q[t] = s2;
        }
        jreduce<DOUT, TW>(p);
        jreduce<DOUT, TW>(q);
#pragma unroll
        for (int t = 0; t < TW; ++t) {
          const float c = c0[t] != 0.f ? __expf(p[t] - logz[r - 1]) : 0.f;
          const float gl = c * (q[t] - sig[r - 1]);
#pragma unroll
          for (int k = 0; k < 4; ++k) ga[t][k] += c * gsr[r][t][k] + gl * vcr[r - 1][t][k];
        }
      }
      }
      // gu blocks (rows past JD and frames past F carry 0); with stored scalars the
      // gW pass (route_gw2_kernel) forms gu itself and nothing is stored
      if constexpr (!CPL) {
        float* blk = gu_t + (((size_t)i * (Fp >> 4) + ft) * NT) * 256 + fl * 16 + 4 * g;
#pragma unroll
        for (int t = 0; t < TW; ++t)
          if (tbase + t < NT) st4(blk + (tbase + t) * 256, f4{ga[t][0], ga[t][1], ga[t][2], ga[t][3]});
      }
      // gx^T[e][f] over this wave's rows (rows past JD carry ga == 0)
      f4 gx[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        gx[ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int k = 0; k < 4; ++k) gx[ct] = mfma16x16x4(wt[ct][t][k], ga[t][k], gx[ct]);
      }
      const int w = i / N, n = i - w * N;
      const int ts = loc.t + w - lpad;
      if (loc.valid && ts >= 0 && ts < T) {
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          if (ct * 16 + 4 * g >= DIN) continue;
          if constexpr (LDSACC) {
            float* a = gw_acc + (fl + w) * SROW + gu_acc_col<DIN>(fl + w, (n - n0) * DIN + ct * 16 + 4 * g);
            st4(a, ld4(a) + gx[ct]);
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              atomicAdd(g_emb + ((size_t)(f + w - lpad) * N + n) * DIN + ct * 16 + 4 * g + k, gx[ct][k]);
          }
        }
      }
    }
  }
  if constexpr (LDSACC) {
    __syncthreads();
    const int f0 = ft * 16 - lpad;
    const int row = nn * DIN;
    for (int k = threadIdx.x; k < nslots * row; k += blockDim.x) {
      const int slot = k / row, rem = k - slot * row;
      const int fo = f0 + slot;
      float v = 0.f;
      const int pos = gu_acc_col<DIN>(slot, rem);
      for (int q = 0; q < NW; ++q) v += gacc[((size_t)q * nslots_max + slot) * SROW + pos];
      if (fo >= 0 && fo < F && v != 0.f) atomicAdd(g_emb + ((size_t)fo * N + n0) * DIN + rem, v);
    }
  }
}

// gu pass from stored couplings (the CPL case of route_gu_kernel) as a software
// pipeline: the transposed W rows and the per-(i, j, f) scalars c^r, gL^r of
// capsule k+1 are in flight (buffer loads, SGPR capsule offsets) while capsule k
// is formed and contracted.  gu is not stored (route_gw2_kernel forms it again).
template <int DIN, int TW, int R>
__global__ __launch_bounds__(256, DIN >= 32 ? (R >= 4 ? 2 : 3) : (R >= 4 ? 3 : 4)) void route_gux_kernel(
    const float* __restrict__ WT, int F, int T, int N, int lpad, int in_n, int J, int mask_first, int n_wgroups,
    int n_chunks, int n_per, const float* __restrict__ saved, const float* __restrict__ gs, float* __restrict__ g_emb,
    int nslots_max, const float* __restrict__ cst, const float* __restrict__ glst, int JP) {
  static_assert(R >= 2, "stored couplings exist for iters >= 2");
  constexpr int NCT = (DIN + 15) / 16;
  constexpr int RV = R - 1;
  extern __shared__ __attribute__((aligned(16))) float gacc[];
  const int JD = J * DIN;
  const int NT = (JD + 15) / 16;
  const size_t FJD = (size_t)F * JD;
  const int NW = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fl = lane & 15, g = lane >> 4;
  const int chunk = blockIdx.x % n_chunks;
  const int rest = blockIdx.x / n_chunks;
  const int wgrp = rest % n_wgroups;
  const int ft = rest / n_wgroups;
  const int f = ft * 16 + fl;
  const FrameLoc loc = frame_loc(f, F, T);
  const int tbase = __builtin_amdgcn_readfirstlane((wgrp * NW + wv) * TW);
  const int n0 = chunk * n_per, nn = min(N, n0 + n_per) - n0;
  const int Wn = in_n / N;
  const int ncap = Wn * nn;
  const int Jeff = J - (mask_first ? 1 : 0);
  const int SROW = gu_row_stride(n_per, DIN);
  const int nslots = 15 + Wn;
  float* gw_acc = gacc + (size_t)wv * nslots_max * SROW;
  for (int k = threadIdx.x; k < NW * nslots_max * SROW; k += blockDim.x) gacc[k] = 0.f;
  __syncthreads();

  float vcr[RV][TW][4], gsr[R][TW][4];
  float c0[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int j = tile_j<DIN>(tbase + t, g);
    c0[t] = (j < J && !(mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r > 0) load_rows(saved + (size_t)(2 * (r - 1) + 1) * FJD, f, loc.valid, JD, tbase + t, g, vcr[r - 1][t]);
      load_rows(gs + (size_t)r * FJD, f, loc.valid, JD, tbase + t, g, gsr[r][t]);
    }
  }
  // lane byte offsets (capsule-independent) and per-capsule SGPR offsets
  const int Fs = srf::fwd32_frame_stride(F);
  const uint32_t cblk_b = (uint32_t)in_n * JP * Fs * 4;
  // W^T in fragment order [i][tile][row quad g][e][4 rows] (prep32_kernel): a wave's
  // float4 loads of one tile are 1 KiB contiguous
  const auto rs_w = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(WT), 0, (int)((size_t)in_n * NT * 16 * DIN * 4),
                                                       0x00020000);
  const auto rs_c = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(cst), 0, (int)(cblk_b * RV), 0x00020000);
  const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(glst), 0, (int)(cblk_b * RV), 0x00020000);
  uint32_t wo[NCT][TW], co[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int tc = min(tbase + t, NT - 1);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
      wo[ct][t] = (uint32_t)(((tc * 4 + g) * DIN + min(ct * 16 + fl, DIN - 1)) * 4) * 4;
    co[t] = (uint32_t)(min(tile_j<DIN>(tbase + t, g), J - 1) * Fs + (loc.valid ? f : 0)) * 4;
  }
  // three operand sets in a ring: capsule k+2 is fetched while capsule k is formed
  constexpr int NB = 3;
  f4 wt_b[NB][NCT][TW];
  float c_b[NB][RV][TW], g_b[NB][RV][TW];
  auto fetch = [&](auto slot, int i) {
    constexpr int sl = decltype(slot)::value;
    const uint32_t sw = (uint32_t)i * NT * 16 * DIN * 4;
    const uint32_t sc = (uint32_t)i * JP * Fs * 4;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int t = 0; t < TW; ++t)
        wt_b[sl][ct][t] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs_w, wo[ct][t], sw, 0));
#pragma unroll
    for (int r = 0; r < RV; ++r)
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        c_b[sl][r][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_c, co[t], sc + r * cblk_b, 0));
        g_b[sl][r][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_g, co[t], sc + r * cblk_b, 0));
      }
  };
  // capsule k of the chunk is i = w*N + n0 + nl (visited w-major); (wf, nf) runs two capsules ahead
  int w = 0, nl = 0, wf = 0, nf = 0;
  auto advance = [&](int& ww, int& nn_) {
    if (++nn_ == nn) nn_ = 0, ++ww;
  };
  auto compute = [&](auto slot) {
    constexpr int sl = decltype(slot)::value;
    const int i = w * N + n0 + nl;
    // packed pairs (v_pk_fma_f32): gu rows 2h, 2h+1 of tile t
    float ga[TW][4];
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f2 a = c0[t] * f2{gsr[0][t][2 * h], gsr[0][t][2 * h + 1]};
#pragma unroll
        for (int r = 0; r < RV; ++r) {
          a = c_b[sl][r][t] * f2{gsr[r + 1][t][2 * h], gsr[r + 1][t][2 * h + 1]} + a;
          a = g_b[sl][r][t] * f2{vcr[r][t][2 * h], vcr[r][t][2 * h + 1]} + a;
        }
        ga[t][2 * h] = a.x;
        ga[t][2 * h + 1] = a.y;
      }
    f4 gx[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      gx[ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) gx[ct] = mfma16x16x4(wt_b[sl][ct][t][q], ga[t][q], gx[ct]);
    }
    const int ts = loc.t + w - lpad;
    if (loc.valid && ts >= 0 && ts < T) {
      const int n = i - w * N;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        if (ct * 16 + 4 * g >= DIN) continue;
        float* a = gw_acc + (fl + w) * SROW + gu_acc_col<DIN>(fl + w, (n - n0) * DIN + ct * 16 + 4 * g);
        st4(a, ld4(a) + gx[ct]);
      }
    }
    advance(w, nl);
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  // fetches past the chunk's last capsule re-read that capsule: no branch around a
  // load, so the wait before each compute counts exactly the two fetches in flight
  const int i_last = (Wn - 1) * N + n0 + nn - 1;
  auto next_i = [&]() {
    const int i = min(wf * N + n0 + nf, i_last);
    advance(wf, nf);
    return i;
  };
  // the fetch stays ahead of the compute it overlaps (no sinking by the scheduler)
#define SRF_GUX_FETCH(SL) \
  fetch(SL{}, next_i());  \
  __builtin_amdgcn_sched_barrier(0);
  if (ncap > 0) {
    SRF_GUX_FETCH(S0)
    SRF_GUX_FETCH(S1)
  }
  for (int k = 0; k < ncap; k += NB) {
    // capsule k + u sits in slot u; capsule k + u + 2 goes to slot (u + 2) % 3
    SRF_GUX_FETCH(S2)
    compute(S0{});
    if (k + 1 >= ncap) break;
    SRF_GUX_FETCH(S0)
    compute(S1{});
    if (k + 2 >= ncap) break;
    SRF_GUX_FETCH(S1)
    compute(S2{});
  }
#undef SRF_GUX_FETCH
  __syncthreads();
  const int f0 = ft * 16 - lpad;
  const int row = nn * DIN;
  for (int k = threadIdx.x; k < nslots * row; k += blockDim.x) {
    const int slot = k / row, rem = k - slot * row;
    const int fo = f0 + slot;
    float v = 0.f;
    const int pos = gu_acc_col<DIN>(slot, rem);
    for (int q = 0; q < NW; ++q) v += gacc[((size_t)q * nslots_max + slot) * SROW + pos];
    if (fo >= 0 && fo < F && v != 0.f) atomicAdd(g_emb + ((size_t)fo * N + n0) * DIN + rem, v);
  }
}

// gu pass from stored couplings on 32x32x16 split-fp16 MFMA (din 32, dout 32: the
// C3 / C4 DR layers).  gx^T[e][f] = sum_row W^T[e][row] gu[row][f] with
//   * W' = 2^aw W (the forward's exponent, prep header hdr[1]) and gu' = 2^eg gu, eg
//     one exponent per (wave, capsule, frame) from the frame's max |gu| over the
//     wave's 32 rows, so max|W'|, max|gu'| < 2^14;
//   * a' = a1 + a2 (fp16 each) and the tile W1 gu1 + W1 gu2 + W2 gu1 (the dropped
//     W2 gu2 <= 2^-22 |W' gu'|), three MFMAs per 16-row K step, products exact in fp32;
//   * the result scaled back by the exact 2^-(aw+eg) of the lane's frame column.
// A workgroup = 32 frames x 4 waves x 32 rows (one output capsule j per wave) x an
// n-chunk; lane l holds frame l & 31 and rows 8(l >> 5) + 0..7 of each K step (the
// MFMA's B map), and the rows 8q + 4(l >> 5) + 0..3 of e in its C map.  The window
// adjoint goes through per-wave LDS slabs [31 + window][n_per*32 + 4] (row stride 4
// mod 32: conflict-free ds_read_b128 / ds_write_b128 for every window offset) and is
// flushed into g_emb by one atomic add per element, as in route_gux_kernel.
#ifndef SRF_GUX16_XCD
#define SRF_GUX16_XCD 1
#endif
#ifndef SRF_GW16S_XCD
#define SRF_GW16S_XCD 1
#endif
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
// 4 waves, two workgroups per CU (three, with a two-slot ring, measured slower; 8 waves,
// one per CU, halving the j-group partial sums the flush adds into g_emb, also slower:
// C4 7.83-7.86 vs 7.82-7.83 ms, r06j)
constexpr int kGux16NW = 4;
constexpr int kGux16Occ = 2;

__device__ __forceinline__ f16v mfma32h(const h8& a, const h8& b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// The lane max of |gu| also goes to *gumax (one atomic max per wave; the caller zeroes
// it): route_gw16s_kernel takes its per-layer exponent from it.
template <int R>
__global__ __launch_bounds__(64 * kGux16NW, kGux16Occ) void route_gux16_kernel(
    const float* __restrict__ WT, const float* __restrict__ hdr, int F, int T, int N, int lpad, int in_n, int J,
    int mask_first, int n_wgroups, int n_chunks, int n_per, const float* __restrict__ saved,
    const float* __restrict__ gs, float* __restrict__ g_emb, const float* __restrict__ cst,
    const float* __restrict__ glst, int JP, float* __restrict__ gumax, int jgpw) {
  static_assert(R >= 2, "stored couplings exist for iters >= 2");
  constexpr int DIN = 32, RV = R - 1, NW = kGux16NW;
  extern __shared__ __attribute__((aligned(16))) float gacc[];
  const int JD = J * DIN;
  const int NT = JD / 16;
  const size_t FJD = (size_t)F * JD;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int fl = lane & 31, h = lane >> 5;
#if SRF_GUX16_XCD
  // XCD-aware task order: the grid is padded to a multiple of 8 and XCD x (= blockIdx.x
  // mod 8, the dispatcher's round robin) takes the x-th eighth of the tasks, ordered
  // n-chunk fastest, then frame tile, then output-capsule group: the n-chunks of one
  // (frame tile, group) share its gs^r / Vc^r rows through one L2 (they were spread over
  // four XCDs), and an XCD's W^T planes are its groups' only
  const int n_ft = (F + 31) / 32, n_tasks = n_ft * n_wgroups * n_chunks;
  const int task = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
  if (task >= n_tasks) return;
  const int chunk = task % n_chunks;
  const int rest = task / n_chunks;
  const int ft = rest % n_ft;
  const int wgrp = rest / n_ft;
#else
  const int chunk = blockIdx.x % n_chunks;
  const int rest = blockIdx.x / n_chunks;
  const int wgrp = rest % n_wgroups;
  const int ft = rest / n_wgroups;
#endif
  const int f = ft * 32 + fl;
  const FrameLoc loc = frame_loc(f, F, T);
  const int fv = loc.valid ? f : 0;
  const int n0 = chunk * n_per, nn = min(N, n0 + n_per) - n0;
  const int Wn = in_n / N;
  const int ncap = Wn * nn;
  const int Jeff = J - (mask_first ? 1 : 0);
  const int SROW = n_per * DIN + 4;
  const int nslots = 31 + Wn;
  float* slab = gacc + (size_t)wv * nslots * SROW;
  for (int k = threadIdx.x; k < NW * nslots * SROW / 4; k += blockDim.x) st4(gacc + 4 * k, f4{0.f, 0.f, 0.f, 0.f});
  __syncthreads();
  float gmax = 0.f;
  // jgpw output-capsule groups of NW per workgroup, one after the other: their gx parts
  // add up in the waves' slabs, so the flush below adds jgpw times fewer partial sums
  // into g_emb (one float atomic per element and group)
  for (int jg = 0; jg < jgpw; ++jg) {
  const int jw = (wgrp * jgpw + jg) * NW + wv;
  const bool wave_on = jw < J;
  const int j = __builtin_amdgcn_readfirstlane(min(jw, J - 1));

  // the lane's 16 rows j*32 + 16 ks + 8 h + 0..7 of gs^r (c^0 folded into gs^0) and Vc^r
  const float c0 = (wave_on && !(mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
  float gsr[R][16], vcr[RV][16];
  {
    const bool ok = loc.valid && wave_on;
    auto rows = [&](const float* base, float (&o)[16]) {
      const float* p = base + (size_t)fv * JD + j * DIN + 8 * h;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f4 a = ld4(p + 16 * ks + 4 * q);
          o[8 * ks + 4 * q] = ok ? a.x : 0.f;
          o[8 * ks + 4 * q + 1] = ok ? a.y : 0.f;
          o[8 * ks + 4 * q + 2] = ok ? a.z : 0.f;
          o[8 * ks + 4 * q + 3] = ok ? a.w : 0.f;
        }
    };
#pragma unroll
    for (int r = 0; r < R; ++r) {
      rows(gs + (size_t)r * FJD, gsr[r]);
      if (r > 0) rows(saved + (size_t)(2 * (r - 1) + 1) * FJD, vcr[r - 1]);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) gsr[0][k] *= c0;
  }
  const int aw = (int)hdr[1];
  // split W^T planes (prep32_kernel, wt16) [i][tile][h][e][8 rows] hi, then lo: K step
  // ks of the wave is tile 2j + ks, the lane's 16 bytes sit at (h, e = fl)
  const int Fs = srf::fwd32_frame_stride(F);
  const uint32_t cblk_b = (uint32_t)in_n * JP * Fs * 4;
  const uint32_t wplane = (uint32_t)in_n * NT * 16 * DIN * 2;   // bytes per plane
  const auto rs_w = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(WT), 0, (int)(2 * wplane), 0x00020000);
  const auto rs_c = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(cst), 0, (int)(cblk_b * RV), 0x00020000);
  const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(glst), 0, (int)(cblk_b * RV), 0x00020000);
  uint32_t wo[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int p = 0; p < 2; ++p) wo[ks][p] = (uint32_t)((((2 * j + ks) * 2 + h) * DIN + fl) * 16) + p * wplane;
  const uint32_t co = (uint32_t)(j * Fs + fv) * 4;
  constexpr int NB = 3;   // operand ring slots
  h8 wt_b[NB][2][2];   // [slot][ks][hi | lo]
  float c_b[NB][RV], g_b[NB][RV];
  auto fetch = [&](auto slot, int i) {
    constexpr int sl = decltype(slot)::value;
    const uint32_t swo = (uint32_t)i * NT * 16 * DIN * 2;
    const uint32_t sc = (uint32_t)i * JP * Fs * 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        wt_b[sl][ks][p] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rs_w, wo[ks][p], swo, 0));
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      c_b[sl][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_c, co, sc + r * cblk_b, 0));
      g_b[sl][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_g, co, sc + r * cblk_b, 0));
    }
  };
  int w = 0, nl = 0, wf = 0, nf = 0;
  auto advance = [&](int& ww, int& nn_) {
    if (++nn_ == nn) nn_ = 0, ++ww;
  };
  auto compute = [&](auto slot) {
    constexpr int sl = decltype(slot)::value;
    // gu on packed pairs (v_pk_fma_f32), the lane's max |gu| for the frame's exponent
    f2 gu[8];
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      f2 a = f2{gsr[0][2 * k], gsr[0][2 * k + 1]};
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        a = __builtin_elementwise_fma(f2{c_b[sl][r], c_b[sl][r]}, f2{gsr[r + 1][2 * k], gsr[r + 1][2 * k + 1]}, a);
        a = __builtin_elementwise_fma(f2{g_b[sl][r], g_b[sl][r]}, f2{vcr[r][2 * k], vcr[r][2 * k + 1]}, a);
      }
      gu[k] = a;
      m = fmaxf(m, fmaxf(fabsf(a[0]), fabsf(a[1])));
    }
    gmax = fmaxf(gmax, m);
    float ma, mb;
    xpair32(m, ma, mb);
    const int eg = srf_split_exp(fmaxf(ma, mb));
    const float sg = srf_exp2i(eg);
    // split by masking: hi = gu' with the low 13 mantissa bits cleared (exact in fp16),
    // lo = f16(gu' - hi); packed conversions
    h8 bh[2], bl[2];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const f2 a = gu[k] * sg;
      const f2 hi = __builtin_bit_cast(f2, __builtin_bit_cast(u2, a) & 0xFFFFE000u);
      const h2 ph = __builtin_convertvector(hi, h2), pl = __builtin_convertvector(a - hi, h2);
      bh[k >> 2][2 * (k & 3)] = ph[0];
      bh[k >> 2][2 * (k & 3) + 1] = ph[1];
      bl[k >> 2][2 * (k & 3)] = pl[0];
      bl[k >> 2][2 * (k & 3) + 1] = pl[1];
    }
    f16v acc = {};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      acc = mfma32h(wt_b[sl][ks][0], bh[ks], acc);
      acc = mfma32h(wt_b[sl][ks][0], bl[ks], acc);
      acc = mfma32h(wt_b[sl][ks][1], bh[ks], acc);
    }
    const float un = srf_exp2i(-(aw + eg));
    const int ts = loc.t + w - lpad;
    if (wave_on && loc.valid && ts >= 0 && ts < T) {
      float* a = slab + (fl + w) * SROW + nl * DIN + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f4 o = ld4(a + 8 * q);   // scale back and add in one fma per value
        st4(a + 8 * q, f4{fmaf(acc[4 * q], un, o.x), fmaf(acc[4 * q + 1], un, o.y), fmaf(acc[4 * q + 2], un, o.z),
                          fmaf(acc[4 * q + 3], un, o.w)});
      }
    }
    advance(w, nl);
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  const int i_last = (Wn - 1) * N + n0 + nn - 1;
  auto next_i = [&]() {
    const int i = min(wf * N + n0 + nf, i_last);
    advance(wf, nf);
    return i;
  };
#define SRF_GUX16_FETCH(SL) \
  fetch(SL{}, next_i());    \
  __builtin_amdgcn_sched_barrier(0);
  if (ncap > 0) {
    SRF_GUX16_FETCH(S0)
    SRF_GUX16_FETCH(S1)
  }
  for (int k = 0; k < ncap; k += NB) {
    SRF_GUX16_FETCH(S2)
    compute(S0{});
    if (k + 1 >= ncap) break;
    SRF_GUX16_FETCH(S0)
    compute(S1{});
    if (k + 2 >= ncap) break;
    SRF_GUX16_FETCH(S1)
    compute(S2{});
  }
#undef SRF_GUX16_FETCH
  }   // jg
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) gmax = fmaxf(gmax, __shfl_xor(gmax, o, 64));
  if (lane == 0) atomicMax(reinterpret_cast<unsigned*>(gumax), __float_as_uint(gmax));   // gmax >= 0
  __syncthreads();
  // flush: consecutive elements across the threads (coalesced atomics), (slot, element)
  // stepped without a division per element
  const int f0 = ft * 32 - lpad;
  const int row = nn * DIN;
  int sl = (int)threadIdx.x / row, rem = (int)threadIdx.x - sl * row;
  const int dsl = (int)blockDim.x / row, drem = (int)blockDim.x - dsl * row;
  for (int k = threadIdx.x; k < nslots * row; k += blockDim.x) {
    const int fo = f0 + sl;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += gacc[((size_t)q * nslots + sl) * SROW + rem];
    if (fo >= 0 && fo < F && v != 0.f) atomicAdd(g_emb + ((size_t)fo * N + n0) * DIN + rem, v);
    sl += dsl;
    rem += drem;
    if (rem >= row) rem -= row, ++sl;
  }
}

// W [in_n][JD][din] -> WT [in_n][din][JD] (A operand of the gx contraction); the
// same launch zeroes g_emb ([n_zero] floats), which the gu pass accumulates into.
__global__ void transpose_w_kernel(const float* __restrict__ W, int in_n, int JD, int din, float* __restrict__ WT,
                                   float* __restrict__ zero, size_t n_zero) {
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

// Windowed input, transposed and frame-padded: xT[i][e][f] (f < Fp), the B
// operand of the gW contraction.  One workgroup per (capsule i, 64-frame tile):
// the tile's 64 x din window rows are read along e (coalesced), transposed through
// LDS, and written as din runs of 64 consecutive frames.
constexpr int kXtFrames = 64;
__global__ __launch_bounds__(256) void window_xt_kernel(const float* __restrict__ emb, int F, int Fp, int T, int N,
                                                        int din, int lpad, int in_n, float* __restrict__ xT) {
  __shared__ float tile[kXtFrames][64 + 1];
  const int i = blockIdx.x / ((Fp + kXtFrames - 1) / kXtFrames);
  const int f0 = (blockIdx.x - i * ((Fp + kXtFrames - 1) / kXtFrames)) * kXtFrames;
  const int w = i / N, n = i - w * N;
  for (int k = threadIdx.x; k < kXtFrames * din; k += blockDim.x) {
    const int fl = k / din, e = k - fl * din;
    const int f = f0 + fl;
    float v = 0.f;
    if (f < F) {
      const int b = f / T, t = f - b * T;
      const int ts = t + w - lpad;
      if (ts >= 0 && ts < T) v = emb[((size_t)(b * T + ts) * N + n) * din + e];
    }
    tile[fl][e] = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < kXtFrames * din; k += blockDim.x) {
    const int e = k / kXtFrames, fl = k - e * kXtFrames;
    const int f = f0 + fl;
    if (f < Fp) xT[((size_t)i * din + e) * Fp + f] = tile[fl][e];
  }
}

// ---------------------------------------------------------------- gW, gbias
// gW[i][row][e] = sum_f gu[i][row][f] x[f][i][e]  (MFMA, K = frames) and
// gbias[i][row] = sum_f gu[i][row][f].  One wave per (i, row tile); per frame
// tile it reads one 1 KiB gu block (4 dword loads per lane, frames 4g..4g+3)
// and float4 frame runs of the transposed window xT.
template <int DIN>
__global__ __launch_bounds__(256) void route_gw_kernel(const float* __restrict__ gu_t,
                                                       const float* __restrict__ xT, int Fp, int in_n, int JD,
                                                       float* __restrict__ gW, float* __restrict__ gbias) {
  constexpr int NCT = (DIN + 15) / 16;
  const int NT = (JD + 15) / 16;
  const int NFT = Fp >> 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int task = blockIdx.x * 4 + wv;
  if (task >= in_n * NT) return;
  const int i = task / NT, tg = task - i * NT;
  const float* ap = gu_t + ((size_t)i * NFT * NT + tg) * 256 + (4 * g) * 16 + l16;
  const size_t astride = (size_t)NT * 256;   // next frame tile
  const float* bp[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) bp[ct] = xT + ((size_t)i * DIN + min(ct * 16 + l16, DIN - 1)) * Fp + 4 * g;
  f4 acc[NCT][2];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct][0] = acc[ct][1] = f4{0.f, 0.f, 0.f, 0.f};
  float gb = 0.f;
  auto step = [&](const f4& a, const f4 (&b)[NCT]) {
    gb += (a.x + a.y) + (a.z + a.w);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      acc[ct][0] = mfma16x16x4(a.x, b[ct].x, acc[ct][0]);
      acc[ct][1] = mfma16x16x4(a.y, b[ct].y, acc[ct][1]);
      acc[ct][0] = mfma16x16x4(a.z, b[ct].z, acc[ct][0]);
      acc[ct][1] = mfma16x16x4(a.w, b[ct].w, acc[ct][1]);
    }
  };
  auto load_a = [&](int ft) {
    const float* q = ap + (size_t)ft * astride;
    return f4{q[0], q[16], q[32], q[48]};
  };
  int ft = 0;
  // 4 frame tiles per trip: all loads issue before the MFMAs
  for (; ft + 4 <= NFT; ft += 4) {
    f4 a[4], b[4][NCT];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = load_a(ft + q);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) b[q][ct] = ld4(bp[ct] + (ft + q) * 16);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) step(a[q], b[q]);
  }
  for (; ft < NFT; ++ft) {
    f4 b[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) b[ct] = ld4(bp[ct] + ft * 16);
    step(load_a(ft), b);
  }
  gb = xor32_sum(xor16_sum(gb));
  const int arow = tg * 16 + l16;
  if (g == 0 && arow < JD) gbias[(size_t)i * JD + arow] = gb;
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


// ---------------------------------------------------------------- gW from stored scalars
// gW^T_i[e][row] = sum_f x_i^T[e][f] gu_i[f][row], with gu formed on the fly (never
// stored) from the per-frame vectors and the stored per-(i, j, f) scalars:
//   gu_fij = c^0_j gs^0_fj + sum_{r>=1} c^r_ijf gs^r_fj + gL^r_ijf Vc^r_fj.
// v_mfma_f32_16x16x4_f32 with K = frames: lane (row = l & 15, kk = l >> 4) builds gu
// for frames 4kk + v (v = 0..3, MFMA v) of its wave's 16-row tile; A = x^T.
// A workgroup = 4 waves (4 row tiles) x GCAP capsules x one of S frame splits; its
// gW / gbias sums stay in registers over the frame range.  Per 16-frame tile the
// workgroup stages the capsules' couplings, logit gradients and transposed window
// (xT) in LDS, one tile ahead (global loads of tile t+1 in flight during tile t),
// and each lane prefetches its per-frame vectors one tile ahead.  Partials: S slabs
// of [in_n][JD][D] (gW) + [in_n][JD] (gbias), or the gradients when S = 1.
template <int D>
constexpr int gw2_cap() { return D <= 16 ? 8 : (D == 32 ? 4 : 2); }
template <int D>
constexpr int gw2_jw() { return D >= 64 ? 1 : 64 / D; }   // capsules j per workgroup row group
template <int D, int R>
constexpr int gw2_stage_floats() {
  return gw2_cap<D>() * ((R > 1 ? R - 1 : 1) * 2 * gw2_jw<D>() * 16 + D * 16);
}

template <int D, int R>
__global__ __launch_bounds__(256) void route_gw2_kernel(
    const float* __restrict__ xT, const float* __restrict__ saved, const float* __restrict__ gs,
    const float* __restrict__ cst, const float* __restrict__ glst, int F, int Fp, int in_n, int J, int mask_first,
    int JP, int n_rt, int n_cc, int S, int ft_per, float* __restrict__ gwp, float* __restrict__ gbp, size_t pstride) {
  constexpr int NCT = (D + 15) / 16;
  constexpr int CAP = gw2_cap<D>();
  constexpr int RV = R > 1 ? R - 1 : 1;
  constexpr int JW = gw2_jw<D>();
  constexpr int CG = RV * 2 * JW * 16;             // per capsule: [r][c|gl][jw][16 frames]
  constexpr int SF = gw2_stage_floats<D, R>();     // per buffer: CAP x (CG + D x 16)
  constexpr int NQ = (SF / 4 + 255) / 256;         // float4 staging loads per thread
  __shared__ __attribute__((aligned(16))) float stg[2][SF];
  const int JD = J * D;
  const int NT = (JD + 15) / 16;
  const size_t FJD = (size_t)F * JD;
  const int Fs = srf::fwd32_frame_stride(F);
  const size_t cblk = (size_t)in_n * JP * Fs;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l16 = lane & 15, kk = lane >> 4;
  int b = blockIdx.x;
  const int s = b % S;
  b /= S;
  const int rtg = b % n_rt;
  const int cc = b / n_rt;
  const int tg = rtg * 4 + wv;                     // this wave's 16-row tile
  const int row = min(tg * 16 + l16, JD - 1);
  const bool rvalid = tg < NT && tg * 16 + l16 < JD;
  const int j = row / D;
  const int jg0 = (rtg * 64) / D;                  // first capsule j of the row group
  const int jl = min(j - jg0, JW - 1);
  const int Jeff = J - (mask_first ? 1 : 0);
  const float c0 = (rvalid && j < J && !(mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
  const int i0 = cc * CAP, ncap = min(in_n, i0 + CAP) - i0;
  const int NFT = Fp >> 4;
  const int ft0 = s * ft_per, ft1 = min(NFT, ft0 + ft_per);

  // staging: float4 q of the buffer <-> (capsule k, part) with parts
  //   [0, CG/4): couplings/logit gradients (r, c|gl, jw, frame quad)
  //   [CG/4, CG/4 + 4D): xT (e, frame quad)
  f4 sv[NQ];
  auto stage_load = [&](int ft) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = q * 256 + threadIdx.x;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (idx < SF / 4) {
        const int k = idx / (CG / 4 + 4 * D), rem = idx - k * (CG / 4 + 4 * D);
        const int i = i0 + min(k, ncap - 1);
        if (rem < CG / 4) {
          const int fq = rem & 3, jw = (rem >> 2) % JW, cg = (rem >> 2) / JW;   // cg = r * 2 + (0: c, 1: gL)
          const int r = cg >> 1;
          const int jj = min(jg0 + jw, JP - 1);
          const int f = ft * 16 + 4 * fq;
          const float* src = (cg & 1) ? glst : cst;
          if (R > 1 && f < F) v = ld4(src + (size_t)r * cblk + ((size_t)i * JP + jj) * Fs + f);
          if (f + 4 > F) {   // frames past F hold no stored scalars
            if (f + 0 >= F) v.x = 0.f;
            if (f + 1 >= F) v.y = 0.f;
            if (f + 2 >= F) v.z = 0.f;
            if (f + 3 >= F) v.w = 0.f;
          }
        } else {
          const int x = rem - CG / 4, e = x >> 2, fq = x & 3;
          v = ld4(xT + ((size_t)i * D + e) * Fp + ft * 16 + 4 * fq);
        }
        if (k >= ncap) v = f4{0.f, 0.f, 0.f, 0.f};
      }
      sv[q] = v;
    }
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = q * 256 + threadIdx.x;
      if (idx < SF / 4) st4(&stg[buf][idx * 4], sv[q]);
    }
  };
  float g0[4], gr[RV][4], vr[RV][4];
  float n0[4], nr[RV][4], nvr[RV][4];
  auto vec_load = [&](int ft) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int f = ft * 16 + 4 * kk + v;
      const bool ok = rvalid && f < F;
      const size_t o = (size_t)(ok ? f : 0) * JD + row;
      n0[v] = ok ? gs[o] : 0.f;
#pragma unroll
      for (int r = 1; r < R; ++r) {
        nr[r - 1][v] = ok ? gs[(size_t)r * FJD + o] : 0.f;
        nvr[r - 1][v] = ok ? saved[(size_t)(2 * (r - 1) + 1) * FJD + o] : 0.f;
      }
    }
  };

  f4 acc[CAP][NCT];
  float gb[CAP];
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    gb[k] = 0.f;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[k][ct] = f4{0.f, 0.f, 0.f, 0.f};
  }
  if (ft0 < ft1) {
    stage_load(ft0);
    vec_load(ft0);
    stage_store(0);
  }
  for (int ft = ft0; ft < ft1; ++ft) {
    const int buf = (ft - ft0) & 1;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      g0[v] = n0[v];
#pragma unroll
      for (int r = 0; r < RV; ++r) gr[r][v] = nr[r][v], vr[r][v] = nvr[r][v];
    }
    __syncthreads();   // buffer buf staged; the other buffer is free
    const bool more = ft + 1 < ft1;
    if (more) stage_load(ft + 1);
    vec_load(more ? ft + 1 : ft);   // unconditional: no register merge of old and new vectors
    const float* sb = stg[buf];
#pragma unroll
    for (int k = 0; k < CAP; ++k) {
      const float* ck = sb + k * (CG + D * 16);
      float gu[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) gu[v] = c0 * g0[v];
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const f4 c = ld4(ck + (((r - 1) * 2 + 0) * JW + jl) * 16 + 4 * kk);
        const f4 gl = ld4(ck + (((r - 1) * 2 + 1) * JW + jl) * 16 + 4 * kk);
#pragma unroll
        for (int v = 0; v < 4; ++v) gu[v] += c[v] * gr[r - 1][v] + gl[v] * vr[r - 1][v];
      }
      gb[k] += (gu[0] + gu[1]) + (gu[2] + gu[3]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const int e = ct * 16 + l16;
        const f4 xa = e < D ? ld4(ck + CG + min(e, D - 1) * 16 + 4 * kk) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[k][ct] = mfma16x16x4(xa[v], gu[v], acc[k][ct]);
      }
    }
    if (more) stage_store(buf ^ 1);
  }
  float* gw = gwp + (size_t)s * pstride;
  float* gbo = gbp + (size_t)s * pstride;
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    if (k >= ncap) continue;
    const int i = i0 + k;
    const float t = xor32_sum(xor16_sum(gb[k]));
    if (rvalid) {
      if (kk == 0) gbo[(size_t)i * JD + row] = t;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (ct * 16 + 4 * kk < D) st4(gw + ((size_t)i * JD + row) * D + ct * 16 + 4 * kk, acc[k][ct]);
    }
  }
}

// The same contraction, restructured for occupancy and a branch-free load path:
//   * staging sources are per-thread pointers fixed at kernel start (every staged
//     part is frame-minor, so tile ft + 1 is 16 floats further on);
//   * the per-frame vectors come in through buffer loads whose range check
//     returns 0 for frames past F (no masks);
//   * tile t + 1's staged registers are written after the barrier of tile t and the
//     loads of tile t + 2 go out right behind them (one barrier per tile);
//   * at most 168 registers, so three workgroups share a CU.
// The stored couplings and logit gradients are 0 for frames past F (the 32x32
// passes store zeros there) and x^T is 0 past F, so gu is 0 on padded frames.
template <int D, int R, int CAP>
__global__ __launch_bounds__(256, (D >= 32 && CAP >= 8) ? 2 : 3) void route_gw3_kernel(
    const float* __restrict__ xT, const float* __restrict__ saved, const float* __restrict__ gs,
    const float* __restrict__ cst, const float* __restrict__ glst, int F, int Fp, int in_n, int J, int mask_first,
    int JP, int n_rt, int S, int ft_per, float* __restrict__ gwp, float* __restrict__ gbp, size_t pstride) {
  static_assert(R >= 2, "stored couplings exist for iters >= 2");
  constexpr int NCT = (D + 15) / 16;
  constexpr int RV = R - 1;
  constexpr int JW = gw2_jw<D>();
  constexpr int CG = RV * 2 * JW * 16;   // per capsule: [r][c|gl][jw][16 frames]
  constexpr int PC = CG + D * 16;        // + x^T [e][16 frames] (in global memory order)
  // x^T rows in LDS: 16 frames, frame chunk c (4 floats) of row e at c ^ ((e >> 1) & 3).
  // A ds_read_b128 is serviced per lane group {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...
  // over 64 banks and lane kk*16+l16 reads row l16, chunk kk: unswizzled, two lanes of
  // a group share banks (padding the row to 24 floats fixes the reads but puts the two
  // rows of each 8-lane ds_write_b128 group on the same banks).  The swizzle keeps
  // both conflict-free without padding.
  constexpr int PCL = PC;                // per capsule in LDS
  constexpr int SF = CAP * PC;
  constexpr int SFL = CAP * PCL;
  constexpr int NQ = (SF / 4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float stg[2][SFL];
  const int JD = J * D;
  const int NT = (JD + 15) / 16;
  const size_t FJD = (size_t)F * JD;
  const int Fs = srf::fwd32_frame_stride(F);
  const size_t cblk = (size_t)in_n * JP * Fs;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l16 = lane & 15, kk = lane >> 4;
  int L = blockIdx.x;   // frame split fastest, then row group, then capsule chunk
  const int s = L % S;
  L /= S;
  const int rtg = L % n_rt;
  const int cc = L / n_rt;
  const int tg = rtg * 4 + wv;
  const int row = min(tg * 16 + l16, JD - 1);
  const bool rvalid = tg < NT && tg * 16 + l16 < JD;
  const int j = row / D;
  const int jg0 = (rtg * 64) / D;
  const int jl = min(j - jg0, JW - 1);
  const int Jeff = J - (mask_first ? 1 : 0);
  const float c0 = (rvalid && j < J && !(mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
  const int i0 = cc * CAP, ncap = min(in_n, i0 + CAP) - i0;
  const int NFT = Fp >> 4;
  const int ft0 = s * ft_per, ft1 = min(NFT, ft0 + ft_per);

  const float* src[NQ];
  int dst[NQ];   // LDS float offset of each staged float4
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int idx = min(q * 256 + (int)threadIdx.x, SF / 4 - 1);
    const int k = idx / (PC / 4), rem = idx - k * (PC / 4);
    const int i = i0 + min(k, ncap - 1);
    if (rem < CG / 4) {
      const int fq = rem & 3, jw = (rem >> 2) % JW, cg = (rem >> 2) / JW;
      const int jj = min(jg0 + jw, JP - 1);
      src[q] = ((cg & 1) ? glst : cst) + (size_t)(cg >> 1) * cblk + ((size_t)i * JP + jj) * Fs + 4 * fq;
      dst[q] = k * PCL + rem * 4;
    } else {
      const int x = rem - CG / 4;
      src[q] = xT + ((size_t)i * D + (x >> 2)) * Fp + 4 * (x & 3);
      const int e = x >> 2;
      dst[q] = k * PCL + CG + e * 16 + 4 * ((x & 3) ^ ((e >> 1) & 3));
    }
  }
  f4 sv[NQ];
  auto stage_load = [&](int ft) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) sv[q] = ld4(src[q] + ft * 16);
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = q * 256 + threadIdx.x;
      if ((SF / 4) % 256 == 0 || idx < SF / 4) st4(&stg[buf][dst[q]], sv[q]);
    }
  };
  // per-frame vectors: buffer loads, 0 past F (range check)
  const uint32_t nrec = (uint32_t)(FJD * 4);
  __amdgpu_buffer_rsrc_t rs_g[R], rs_v[RV];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    rs_g[r] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gs + (size_t)r * FJD), 0, (int)nrec, 0x00020000);
    if (r > 0)
      rs_v[r - 1] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(saved + (size_t)(2 * (r - 1) + 1) * FJD), 0,
                                                      (int)nrec, 0x00020000);
  }
  const uint32_t vo0 = (uint32_t)((4 * kk) * JD + row) * 4;
  float g0[4], gr[RV][4], vr[RV][4];
  float n0[4], nr[RV][4], nvr[RV][4];
  auto vec_load = [&](int ft) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const uint32_t o = vo0 + (uint32_t)((ft * 16 + v) * JD) * 4;
      n0[v] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_g[0], o, 0, 0));
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        nr[r][v] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_g[r + 1], o, 0, 0));
        nvr[r][v] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_v[r], o, 0, 0));
      }
    }
  };

  f4 acc[CAP][NCT];
  float gb[CAP];
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    gb[k] = 0.f;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[k][ct] = f4{0.f, 0.f, 0.f, 0.f};
  }
  if (ft0 < ft1) {
    stage_load(ft0);
    vec_load(ft0);
    stage_store(0);
    if (ft0 + 1 < ft1) stage_load(ft0 + 1);
  }
  for (int ft = ft0; ft < ft1; ++ft) {
    const int buf = (ft - ft0) & 1;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      g0[v] = n0[v];
#pragma unroll
      for (int r = 0; r < RV; ++r) gr[r][v] = nr[r][v], vr[r][v] = nvr[r][v];
    }
    __syncthreads();   // tile ft staged in buf; buf ^ 1 (tile ft - 1) is free
    if (ft + 1 < ft1) {
      stage_store(buf ^ 1);
      if (ft + 2 < ft1) stage_load(ft + 2);
    }
    // unconditional (the last tile reloads itself): a conditional load merges the old
    // and new vectors and costs a register copy of every vector per tile
    vec_load(ft + 1 < ft1 ? ft + 1 : ft);
    const float* sb = stg[buf];
#pragma unroll
    for (int k = 0; k < CAP; ++k) {
      const float* ck = sb + k * PCL;
      float gu[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) gu[v] = c0 * g0[v];
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        const f4 c = ld4(ck + ((r * 2 + 0) * JW + jl) * 16 + 4 * kk);
        const f4 gl = ld4(ck + ((r * 2 + 1) * JW + jl) * 16 + 4 * kk);
#pragma unroll
        for (int v = 0; v < 4; ++v) gu[v] += c[v] * gr[r][v] + gl[v] * vr[r][v];
      }
      gb[k] += (gu[0] + gu[1]) + (gu[2] + gu[3]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const int e = min(ct * 16 + l16, D - 1);
        const f4 xa = ld4(ck + CG + e * 16 + 4 * (kk ^ ((e >> 1) & 3)));
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[k][ct] = mfma16x16x4(xa[v], gu[v], acc[k][ct]);
      }
    }
  }
  float* gw = gwp + (size_t)s * pstride;
  float* gbo = gbp + (size_t)s * pstride;
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    if (k >= ncap) continue;
    const int i = i0 + k;
    const float t = xor32_sum(xor16_sum(gb[k]));
    if (rvalid) {
      if (kk == 0) gbo[(size_t)i * JD + row] = t;
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        if (ct * 16 + 4 * kk < D) st4(gw + ((size_t)i * JD + row) * D + ct * 16 + 4 * kk, acc[k][ct]);
    }
  }
}

// gW pass on 32x32x16 split-fp16 MFMA (din = dout = 32, iters 2..3 with stored
// couplings: the C3 / C4 DR layers): gW^T_i[e][row] = sum_f x_i^T[e][f] gu_i[f][row].
//   * x' = 2^bx x (the forward's exponent, hdr[2]), split by the forward's prep into
//     fp16 hi / lo planes blocked per 16 frames (xt16: [i][f/16][hi|lo][e][16]);
//   * gu' = 2^eg gu with ONE exponent for the layer, from max|gu| that the gx pass
//     (route_gux16_kernel) leaves in *gumax, so max|gu'| < 2^14; split into fp16
//     hi / lo by masking: hi = gu' with its low 13 mantissa bits cleared (exact in
//     fp16 in the normal range), lo = f16(gu' - hi).  Products of one exponent pair
//     sum straight into the fp32 accumulator: three MFMAs per capsule and 16-frame K
//     step (x1 g1 + x1 g2 + x2 g1, the dropped x2 g2 <= 2^-21 |x' gu'|), scaled back by
//     2^-(bx + eg) once at the end.  Errors are absolute at the layer's scale (below
//     2^-24 of max|x'| max|gu'| per product), as in the forward's per-tensor split.
// Workgroup = 4 waves x 32 rows (one output capsule j each) x CAP capsules x one of S
// frame splits; lane l holds row 32j + (l & 31) and frames 8(l >> 5) + 0..7 of each
// K step (B map), e = 8q + 4(l >> 5) + 0..3 of its C map.  Tile t + 1's couplings and
// x planes are staged while tile t computes (one barrier per tile), the per-frame
// vectors one tile ahead in registers.  LDS x planes: row e = 16 halves = two 8-half
// chunks, chunk c of row e at c ^ ((e >> 3) & 1): the ds_read_b128 lane groups then
// cover 64 distinct banks.
constexpr int kGw16Cap = 4;
template <int R, int CAP>
__global__ __launch_bounds__(256, 2) void route_gw16s_kernel(
    const _Float16* __restrict__ x16, const float* __restrict__ hdr, const float* __restrict__ gumax,
    const float* __restrict__ saved, const float* __restrict__ gs, const float* __restrict__ cst,
    const float* __restrict__ glst, int F, int Fp, int in_n, int J, int mask_first, int JP, int n_rt, int S,
    int ft_per, float* __restrict__ gwp, float* __restrict__ gbp, size_t pstride) {
  static_assert(R >= 2 && R <= 3, "stored couplings exist for iters >= 2; registers hold R <= 3");
  constexpr int D = 32, RV = R - 1;
  constexpr int CG = RV * 2 * 4 * 16;    // couplings per capsule: [r][c|gl][4 j][16 frames] floats
  constexpr int PQ = CG / 4 + 128;       // 16-byte pieces staged per capsule (couplings + x hi/lo)
  constexpr int PCB = CG * 4 + 2 * D * 16 * 2;   // LDS bytes per capsule: couplings, x hi, x lo
  constexpr int NQ = (CAP * PQ + 255) / 256;
  __shared__ __attribute__((aligned(16))) unsigned char stg[2][CAP * PCB];
  const int JD = J * D;
  const size_t FJD = (size_t)F * JD;
  const int Fs = srf::fwd32_frame_stride(F);
  const size_t cblk = (size_t)in_n * JP * Fs;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = lane & 31, h = lane >> 5;
#if SRF_GW16S_XCD
  // XCD-aware task order (as route_gux16_kernel): XCD x takes the x-th eighth of the
  // tasks ordered capsule group fastest, then output-capsule group, then frame split, so
  // a (split, group)'s gs^r / Vc^r rows stay on one XCD and a split's x planes on the
  // two or three XCDs that cover it (they were read on all eight)
  const int n_cc = (in_n + CAP - 1) / CAP, n_tasks = n_cc * n_rt * S;
  const int task = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
  if (task >= n_tasks) return;
  const int cc = task % n_cc;
  const int rtg = (task / n_cc) % n_rt;
  const int s = task / n_cc / n_rt;
#else
  int b = blockIdx.x;
  const int s = b % S;
  b /= S;
  const int rtg = b % n_rt;
  const int cc = b / n_rt;
#endif
  const int jw = rtg * 4 + wv;
  const bool wave_on = jw < J;
  const int j = min(jw, J - 1);
  const int row = j * D + n;
  const int Jeff = J - (mask_first ? 1 : 0);
  const float c0 = (wave_on && !(mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
  const int i0 = cc * CAP, ncap = min(in_n, i0 + CAP) - i0;
  const int NFT = Fp >> 4;
  const int ft0 = s * ft_per, ft1 = min(NFT, ft0 + ft_per);
  const int bx = (int)hdr[2];
  const int eg = srf_split_exp(*gumax);
  const float sg = srf_exp2i(eg);

  // staging: 16-byte piece q of a tile <-> (capsule k, part): couplings (r, c|gl, jq,
  // frame quad) or an x chunk (plane, e, 8-frame half); per-thread sources fixed, the
  // next tile is 64 bytes (couplings) or 2 KiB (x planes) on
  constexpr int NCPL = CAP * CG / 4;
  const char* src[NQ];
  int dst[NQ];
  int step[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int idx = min(q * 256 + (int)threadIdx.x, CAP * PQ - 1);
    if (idx < NCPL) {
      const int k = idx / (CG / 4), rem = idx - k * (CG / 4);
      const int i = i0 + min(k, ncap - 1);
      const int fq = rem & 3, jq = (rem >> 2) & 3, cg = rem >> 4;   // cg = r * 2 + (0: c, 1: gL)
      const int jj = min(rtg * 4 + jq, JP - 1);
      src[q] = reinterpret_cast<const char*>(((cg & 1) ? glst : cst) + (size_t)(cg >> 1) * cblk +
                                             ((size_t)i * JP + jj) * Fs + 4 * fq);
      dst[q] = k * PCB + rem * 16;
      step[q] = 64;
    } else {
      const int x = idx - NCPL, k = x >> 7, xr = x & 127;
      const int p = xr >> 6, e = (xr >> 1) & 31, hf = xr & 1;
      const int i = i0 + min(k, ncap - 1);
      src[q] = reinterpret_cast<const char*>(x16 + (((size_t)i * NFT * 2 + p) * 32 + e) * 16 + hf * 8);
      dst[q] = k * PCB + CG * 4 + p * (D * 16 * 2) + (e * 16 + ((hf ^ ((e >> 3) & 1)) * 8)) * 2;
      step[q] = 2 * 32 * 16 * 2;
    }
  }
  f4 sv[NQ];
  auto stage_load = [&](int ft) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) sv[q] = *reinterpret_cast<const f4*>(src[q] + (size_t)ft * step[q]);
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = q * 256 + threadIdx.x;
      if ((CAP * PQ) % 256 != 0 && idx >= CAP * PQ) continue;
      *reinterpret_cast<f4*>(&stg[buf][dst[q]]) = sv[q];
    }
  };
  // per-frame vectors of the lane's row, frames 8h + 0..7 of a tile: buffer loads, 0 past F
  const uint32_t nrec = (uint32_t)(FJD * 4);
  __amdgpu_buffer_rsrc_t rs_g[R], rs_v[RV];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    rs_g[r] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gs + (size_t)r * FJD), 0, (int)nrec, 0x00020000);
    if (r > 0)
      rs_v[r - 1] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(saved + (size_t)(2 * (r - 1) + 1) * FJD), 0,
                                                      (int)nrec, 0x00020000);
  }
  const uint32_t vo0 = (uint32_t)((8 * h) * JD + row) * 4;
  // the next tile's per-frame vectors, held as frame pairs so that the scaling below is
  // one packed multiply per pair with no register shuffles
  f2 nx[R + RV][4];
  auto vec_load = [&](int ft) {
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const uint32_t so = (uint32_t)((ft * 16 + v) * JD) * 4;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        nx[r][v >> 1][v & 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_g[r], vo0, so, 0));
        if (r > 0) nx[R + r - 1][v >> 1][v & 1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_v[r - 1], vo0, so, 0));
      }
    }
  };

  f16v acc[CAP];
  f2 gb[CAP];
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    gb[k] = f2{0.f, 0.f};
    acc[k] = f16v{};
  }
  if (ft0 < ft1) {
    stage_load(ft0);
    vec_load(ft0);
    stage_store(0);
    if (ft0 + 1 < ft1) stage_load(ft0 + 1);
  }
  const int xoff = CG * 4 + (n * 16 + ((h ^ ((n >> 3) & 1)) * 8)) * 2;
  const float s0 = c0 * sg;
  for (int ft = ft0; ft < ft1; ++ft) {
    const int buf = (ft - ft0) & 1;
    // this tile's vectors, scaled by 2^eg (c^0 folded into gs^0): frame pairs (v, v + 1)
    f2 fv[R + RV][4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      fv[0][v] = nx[0][v] * s0;
#pragma unroll
      for (int a = 1; a < R + RV; ++a) fv[a][v] = nx[a][v] * sg;
    }
    __syncthreads();   // tile ft staged in buf; buf ^ 1 (tile ft - 1) is free
    if (ft + 1 < ft1) {
      stage_store(buf ^ 1);
      if (ft + 2 < ft1) stage_load(ft + 2);
    }
    // unconditional (the last tile reloads itself): a conditional load merges the old
    // and new vectors and costs a register copy of every vector per tile
    vec_load(ft + 1 < ft1 ? ft + 1 : ft);
    const unsigned char* sb = stg[buf];
#pragma unroll
    for (int k = 0; k < CAP; ++k) {
      const unsigned char* ck = sb + k * PCB;
      const float* ckf = reinterpret_cast<const float*>(ck);
      f2 gu[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) gu[v] = fv[0][v];
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        const float* cp = ckf + ((r * 2 + 0) * 4 + wv) * 16 + 8 * h;
        const float* gp = ckf + ((r * 2 + 1) * 4 + wv) * 16 + 8 * h;
        const f4 ca = ld4(cp), cb = ld4(cp + 4), ga = ld4(gp), gbv = ld4(gp + 4);
        const f2 c2[4] = {f2{ca[0], ca[1]}, f2{ca[2], ca[3]}, f2{cb[0], cb[1]}, f2{cb[2], cb[3]}};
        const f2 g2[4] = {f2{ga[0], ga[1]}, f2{ga[2], ga[3]}, f2{gbv[0], gbv[1]}, f2{gbv[2], gbv[3]}};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          gu[v] = __builtin_elementwise_fma(c2[v], fv[r + 1][v], gu[v]);
          gu[v] = __builtin_elementwise_fma(g2[v], fv[R + r][v], gu[v]);
        }
      }
      gb[k] += (gu[0] + gu[1]) + (gu[2] + gu[3]);
      h8 bh, bl;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        // hi: the low 13 mantissa bits cleared (exact in fp16); lo = f16(gu' - hi)
        const f2 hi = __builtin_bit_cast(f2, __builtin_bit_cast(u2, gu[v]) & 0xFFFFE000u);
        const f2 lo = gu[v] - hi;
        const h2 ph = __builtin_convertvector(hi, h2);   // v_cvt_pk_f16_f32 (exact for hi)
        const h2 pl = __builtin_convertvector(lo, h2);
        bh[2 * v] = ph[0];
        bh[2 * v + 1] = ph[1];
        bl[2 * v] = pl[0];
        bl[2 * v + 1] = pl[1];
      }
      const h8 xh = *reinterpret_cast<const h8*>(ck + xoff);
      const h8 xl = *reinterpret_cast<const h8*>(ck + xoff + D * 16 * 2);
      acc[k] = mfma32h(xh, bh, acc[k]);
      acc[k] = mfma32h(xh, bl, acc[k]);
      acc[k] = mfma32h(xl, bh, acc[k]);
    }
  }
  float* gw = gwp + (size_t)s * pstride;
  float* gbo = gbp + (size_t)s * pstride;
  const float un = srf_exp2i(-(bx + eg)), ug = srf_exp2i(-eg);
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    const float a = gb[k][0] + gb[k][1];
    float pa, pb;
    xpair32(a, pa, pb);
    if (k >= ncap || !wave_on) continue;
    const int i = i0 + k;
    if (h == 0) gbo[(size_t)i * JD + row] = (pa + pb) * ug;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      st4(gw + ((size_t)i * JD + row) * D + 8 * q + 4 * h,
          f4{acc[k][4 * q] * un, acc[k][4 * q + 1] * un, acc[k][4 * q + 2] * un, acc[k][4 * q + 3] * un});
  }
}

// gW | gbias = sum of the S partial slabs (float4 per thread).
__global__ void gw_reduce_kernel(const float* __restrict__ part, int S, size_t n4, size_t stride, float* __restrict__ gW,
                                 size_t nw4, float* __restrict__ gb) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n4) return;
  f4 a = ld4(part + idx * 4);
  for (int s = 1; s < S; ++s) a += ld4(part + (size_t)s * stride + idx * 4);
  if (idx < nw4)
    st4(gW + idx * 4, a);
  else
    st4(gb + (idx - nw4) * 4, a);
}

// ---------------------------------------------------------------- finish kernels
// One thread per float4 of a capsule (Q = DOUT/4 adjacent lanes per capsule);
// squash norms are reduced across the Q lanes.
template <int Q>
__device__ __forceinline__ float qsum(float v) {
#pragma unroll
  for (int o = 1; o < Q; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ f4 sum_slab4(const float* __restrict__ slab, int n, size_t FJD, size_t off) {
  f4 a = ld4(slab + off);
#pragma unroll 4
  for (int c = 1; c < n; ++c) a += ld4(slab + (size_t)c * FJD + off);
  return a;
}

// s^r = sum over i-chunks; v^r = squash(s^r) (naive:204); Vc^{r+1} = Vc^r + v^r.
template <int DOUT>
__global__ void fwd_finish_kernel(const float* __restrict__ slab, int n_chunks, size_t FJD,
                                  const float* __restrict__ vc_in, float* __restrict__ s_out,
                                  float* __restrict__ vc_out, float* __restrict__ v_out) {
  constexpr int Q = DOUT / 4;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // float4 index; FJD/4 % Q == 0
  const bool ok = idx < FJD / 4;
  const size_t off = (ok ? idx : 0) * 4;
  const f4 sv = sum_slab4(slab, n_chunks, FJD, off);
  const float n2 = qsum<Q>((sv.x * sv.x + sv.y * sv.y) + (sv.z * sv.z + sv.w * sv.w));
  if (!ok) return;
  const float fac = n2 / (1.f + n2) / sqrtf(n2 + kSquashEps);
  const f4 v = sv * fac;
  st4(s_out + off, sv);
  st4(vc_out + off, vc_in ? v + ld4(vc_in + off) : v);
  if (v_out) st4(v_out + off, v);
}

// gs = squash'(s)^T a with a = a_init (the upstream gradient of the last
// iteration's v) or, for earlier iterations, a = A += sum of gVc slabs.
// zero4 / nz4: float4s zeroed by the same launch (the g_emb accumulator of the gu pass).
template <int DOUT>
__global__ void bwd_finish_kernel(const float* __restrict__ slab, int n_chunks, size_t FJD,
                                  const float* __restrict__ a_init, float* __restrict__ A,
                                  const float* __restrict__ s, float* __restrict__ gs, float* __restrict__ zero4,
                                  size_t nz4, float* __restrict__ zero1) {
  constexpr int Q = DOUT / 4;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < nz4) st4(zero4 + idx * 4, f4{0.f, 0.f, 0.f, 0.f});
  if (zero1 != nullptr && idx == 0) *zero1 = 0.f;
  const bool ok = idx < FJD / 4;
  const size_t off = (ok ? idx : 0) * 4;
  f4 a;
  if (a_init) {
    a = ld4(a_init + off);
    if (ok) st4(A + off, f4{0.f, 0.f, 0.f, 0.f});   // A starts at 0 (gradient via later logits)
  } else {
    a = ld4(A + off) + sum_slab4(slab, n_chunks, FJD, off);
    if (ok) st4(A + off, a);
  }
  const f4 sv = ld4(s + off);
  const float n2 = qsum<Q>((sv.x * sv.x + sv.y * sv.y) + (sv.z * sv.z + sv.w * sv.w));
  const float sa = qsum<Q>((sv.x * a.x + sv.y * a.y) + (sv.z * a.z + sv.w * a.w));
  if (!ok) return;
  const float rs = 1.f / sqrtf(n2 + kSquashEps);
  const float ip = 1.f / (1.f + n2);
  const float gfac = n2 * ip * rs;
  const float dg2 = 2.f * rs * ip * (ip - 0.5f * n2 / (n2 + kSquashEps)) * sa;
  st4(gs + off, a * gfac + sv * dg2);
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

// Pick the i-chunk count: minimise (scheduling rounds x capsules per workgroup)
// given the workgroups that fit on 256 CUs, preferring chunk counts that divide
// 8 (one i-chunk of W per XCD L2) and fewer slabs.
int auto_chunks(const Geom& g, int NW) {
  const int n_ftiles = (g.F() + 15) / 16;
  const int wg_per_cu = std::max(1, 8 / NW);   // ~2 waves per SIMD at our register budget
  const int slots = 256 * wg_per_cu;
  int best = 1;
  double best_cost = 1e30;
  for (int c = 1; c <= std::min(g.in_n(), 96); ++c) {
    const int rounds = (n_ftiles * c + slots - 1) / slots;
    const int len = (g.in_n() + c - 1) / c;
    double cost = (double)rounds * (len + 2);          // +2: per-workgroup prologue/epilogue
    if (8 % c != 0 && c % 8 != 0) cost *= 1.05;          // W chunk not XCD-local
    cost *= 1.0 + 0.002 * c;                             // slab traffic
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
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
  auto kern = r == 0 ? route_pass_kernel<D, D, TW, MODE, true> : route_pass_kernel<D, D, TW, MODE, false>;
  hipLaunchKernelGGL(kern, dim3(n_ftiles * n_chunks), dim3(64 * NW), shmem, st,
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
  const size_t FJD = (size_t)g.F() * g.JD();
  hipLaunchKernelGGL((fwd_finish_kernel<D>), dim3((FJD / 4 + 255) / 256), dim3(256), 0, st, slab, n_chunks, FJD,
                     vc_in, s_out, vc_out, v_out);
}

template <int D>
void launch_bwd_finish(const Geom& g, const float* slab, int n_chunks, const float* a_init, float* A,
                       const float* s, float* gs, hipStream_t st, float* zero = nullptr, size_t n_zero = 0,
                       float* zero1 = nullptr) {
  const size_t FJD = (size_t)g.F() * g.JD();
  const size_t nz4 = zero ? n_zero / 4 : 0;
  const size_t n = std::max(FJD / 4, nz4);
  hipLaunchKernelGGL((bwd_finish_kernel<D>), dim3((n + 255) / 256), dim3(256), 0, st, slab, n_chunks, FJD, a_init,
                     A, s, gs, zero, nz4, zero1);
}

// row tiles per wave in the gu pass (a wave must hold whole output capsules)
constexpr int gu_tw(int d) { return d >= 64 ? 4 : 2; }
constexpr int kGuNW = 4;  // waves per gu workgroup

inline int gu_wgroups(const Geom& g) { return (g.NT() + kGuNW * gu_tw(g.dout) - 1) / (kGuNW * gu_tw(g.dout)); }
inline int padded_frames(const Geom& g) { return (g.F() + 15) / 16 * 16; }
inline int gu_window(const Geom& g) { return g.lpad + g.rpad + 1; }
inline size_t gu_lds_bytes(const Geom& g, int nw, int n_per) {
  return (size_t)nw * (15 + gu_window(g)) * gu_row_stride(n_per, g.din) * sizeof(float);
}
constexpr size_t kGuLdsMax = 64 * 1024;

// gu i-chunks are ranges of n (all window offsets each): fill ~4 workgroups per CU,
// then fewest capsules per workgroup, with the gx accumulator inside kGuLdsMax.
int gu_n_per(const Geom& g, int nw) {
  const int base = (g.F() + 15) / 16 * gu_wgroups(g);
  const int slots = 256 * 4;
  int best = 1;
  double best_cost = 1e30;
  for (int n_per = 1; n_per <= g.N; ++n_per) {
    if (n_per > 1 && gu_lds_bytes(g, nw, n_per) > kGuLdsMax) break;
    const int chunks = (g.N + n_per - 1) / n_per;
    const int rounds = (base * chunks + slots - 1) / slots;
    const double cost = (double)rounds * (gu_window(g) * n_per + 4);
    if (cost < best_cost) {
      best_cost = cost;
      best = n_per;
    }
  }
  return best;
}

inline size_t gux16_lds_bytes(const Geom& g, int n_per) {
  return (size_t)kGux16NW * (31 + gu_window(g)) * (n_per * 32 + 4) * sizeof(float);
}
constexpr size_t kGux16LdsMax = (160 / kGux16Occ - 4) * 1024;   // kGux16Occ workgroups per CU
// route_gux16_kernel (split-fp16 32x32 tiles) for din = dout = 32 with stored
// couplings (route_gux_kernel otherwise).  A function of the geometry only: the
// forward's prep writes the kernel's split W^T planes in place of the fp32 W^T under
// the same test.
inline bool use_gux16(const Geom& g) {
  return g.din == 32 && g.dout == 32 && g.iters >= 2 && g.iters <= 4 &&   // R = 5 spills
         gux16_lds_bytes(g, 1) <= kGux16LdsMax;
}
// n-chunk size: fewest rounds of two workgroups per CU, then fewest capsules each
int gux16_n_per(const Geom& g, int jgpw) {
  const int base = (g.F() + 31) / 32 * ((g.J + kGux16NW - 1) / kGux16NW / jgpw);
  const int slots = 256 * kGux16Occ;
  int best = 1;
  double best_cost = 1e30;
  for (int n_per = 1; n_per <= g.N; ++n_per) {
    if (n_per > 1 && gux16_lds_bytes(g, n_per) > kGux16LdsMax) break;
    const int chunks = (g.N + n_per - 1) / n_per;
    const int rounds = (base * chunks + slots - 1) / slots;
    const double cost = (double)rounds * (gu_window(g) * n_per * jgpw + 4);
    if (cost < best_cost) {
      best_cost = cost;
      best = n_per;
    }
  }
  return best;
}

#ifndef SRF_GUX16_JGPW
#define SRF_GUX16_JGPW 2
#endif
template <int R>
void launch_gux16(const Geom& g, const float* WT, const float* hdr, const float* saved, const float* gs,
                  float* g_emb, const float* cst, const float* glst, int JP, float* gumax, hipStream_t st) {
  const int n_all = (g.J + kGux16NW - 1) / kGux16NW;   // output-capsule groups of kGux16NW
  const int jgpw = n_all % SRF_GUX16_JGPW == 0 ? SRF_GUX16_JGPW : 1;
  const int n_wgroups = n_all / jgpw;
  const int n_per = gux16_n_per(g, jgpw);
  const int n_chunks = (g.N + n_per - 1) / n_per;
  int grid = (g.F() + 31) / 32 * n_wgroups * n_chunks;
  if (SRF_GUX16_XCD) grid = (grid + 7) / 8 * 8;   // the kernel's XCD-aware task order
  hipLaunchKernelGGL((route_gux16_kernel<R>), dim3(grid), dim3(64 * kGux16NW), gux16_lds_bytes(g, n_per), st, WT, hdr,
                     g.F(), g.T, g.N, g.lpad, g.in_n(), g.J, g.mask_first, n_wgroups, n_chunks, n_per, saved, gs, g_emb,
                     cst, glst, JP, gumax, jgpw);
}

template <int D, int R>
void launch_gu(const Geom& g, const float* emb, const float* W, const float* WT, const float* bias,
               const float* saved, const float* gs, const float* stats, float* gu_t, float* g_emb, hipStream_t st,
               const float* cst, const float* glst, int JP, const float* hdr = nullptr, float* gumax = nullptr) {
  if constexpr (R >= 2 && D == 32) {
    if (cst != nullptr && hdr != nullptr && gumax != nullptr && use_gux16(g)) {
      launch_gux16<R>(g, WT, hdr, saved, gs, g_emb, cst, glst, JP, gumax, st);
      return;
    }
  }
  const int n_ftiles = (g.F() + 15) / 16;
  const int n_wgroups = gu_wgroups(g);
  constexpr int TW = gu_tw(D);
  const int nw = std::min(kGuNW, (g.NT() + TW - 1) / TW);
  const int n_per = gu_n_per(g, nw);
  const int n_chunks = (g.N + n_per - 1) / n_per;
  const int nslots = 15 + gu_window(g);
  const size_t lds = gu_lds_bytes(g, nw, n_per);
  if constexpr (R >= 2 && D <= 32) {   // couplings are stored by the 32x32 forward (din <= 32)
    if (lds <= kGuLdsMax && cst != nullptr) {
      hipLaunchKernelGGL((route_gux_kernel<D, TW, R>), dim3(n_ftiles * n_wgroups * n_chunks), dim3(64 * nw), lds, st,
                         WT, g.F(), g.T, g.N, g.lpad, g.in_n(), g.J, g.mask_first, n_wgroups, n_chunks, n_per, saved,
                         gs, g_emb, nslots, cst, glst, JP);
      return;
    }
  }
  if (lds <= kGuLdsMax)
    hipLaunchKernelGGL((route_gu_kernel<D, D, TW, R, true>), dim3(n_ftiles * n_wgroups * n_chunks),
                       dim3(64 * nw), lds, st, emb, W, WT, bias, g.F(), padded_frames(g), g.T, g.N, g.lpad, g.rpad,
                       g.in_n(), g.J, g.mask_first, n_wgroups, n_chunks, n_per, saved, gs, stats, gu_t, g_emb, nslots,
                       nullptr, nullptr, 0);
  else
    hipLaunchKernelGGL((route_gu_kernel<D, D, TW, R, false>), dim3(n_ftiles * n_wgroups * n_chunks),
                       dim3(64 * nw), 0, st, emb, W, WT, bias, g.F(), padded_frames(g), g.T, g.N, g.lpad, g.rpad,
                       g.in_n(), g.J, g.mask_first, n_wgroups, n_chunks, n_per, saved, gs, stats, gu_t, g_emb, nslots,
                       nullptr, nullptr, 0);
}

template <int D>
void launch_gu_r(const Geom& g, const float* emb, const float* W, const float* WT, const float* bias,
                 const float* saved, const float* gs, const float* stats, float* gu_t, float* g_emb, hipStream_t st,
                 const float* cst = nullptr, const float* glst = nullptr, int JP = 0, const float* hdr = nullptr,
                 float* gumax = nullptr) {
  switch (g.iters) {
    case 1: launch_gu<D, 1>(g, emb, W, WT, bias, saved, gs, stats, gu_t, g_emb, st, nullptr, nullptr, 0); break;
    case 2: launch_gu<D, 2>(g, emb, W, WT, bias, saved, gs, stats, gu_t, g_emb, st, cst, glst, JP, hdr, gumax); break;
    case 3: launch_gu<D, 3>(g, emb, W, WT, bias, saved, gs, stats, gu_t, g_emb, st, cst, glst, JP, hdr, gumax); break;
    case 4: launch_gu<D, 4>(g, emb, W, WT, bias, saved, gs, stats, gu_t, g_emb, st, cst, glst, JP, hdr, gumax); break;
    default: launch_gu<D, 5>(g, emb, W, WT, bias, saved, gs, stats, gu_t, g_emb, st, cst, glst, JP, hdr, gumax); break;
  }
}


// gW-from-scalars plan: capsule chunk, frame splits.  SRF_GW2_SPLITS forces S.
struct Gw2Plan {
  int cap, n_rt, n_cc, S, ft_per;
  size_t pstride;
};

inline int gw2_cap_rt(int d) { return d <= 16 ? 8 : (d == 32 ? 4 : 2); }

// route_gw3_kernel (iters 2..3, din <= 32): 8 capsules per workgroup for din <= 16,
// 4 for din 32 (two 16-column accumulators per capsule; 8 measured the same at C4);
// 0: route_gw2_kernel (deeper routing spills at 168 registers, din 64).
inline int gw3_cap(const Geom& g) {
  if (g.iters > 3) return 0;
  return g.din <= 16 ? 8 : g.din == 32 ? 4 : 0;
}

// route_gw16s_kernel (split-fp16 32x32 tiles, one gu exponent per layer from the gx
// pass) wherever route_gux16_kernel runs and the routing has at most 3 iterations: the
// C3 / C4 DR layers.  A function of the geometry only: the forward's prep writes the
// x^T planes this kernel reads (xt16) under the same test.
inline bool use_gw16s(const Geom& g) { return use_gux16(g) && g.iters <= 3; }

Gw2Plan gw2_plan(const Geom& g) {
  const bool g16 = use_gw16s(g);
  Gw2Plan p{};
  const int NT = g.NT();
  const int NCT = g16 ? 2 : (g.din + 15) / 16;
  p.n_rt = g16 ? (g.J + 3) / 4 : (NT + 3) / 4;
  p.cap = g16 ? kGw16Cap : gw3_cap(g) ? gw3_cap(g) : gw2_cap_rt(g.din);
  // workgroups resident at once; route_gw3_kernel (latency-bound) is planned for two
  // resident rounds: at C4 S = 8 frame splits (1280 workgroups) beat S = 4 (640, one
  // round) by 2 %, at C2 the slab term keeps S = 5; route_gw16s_kernel: two per CU
  const int slots = g16 ? 512 : gw3_cap(g) ? 2 * 768 : 512;
  const double per_tile = g16 ? 120.0 : 200.0;   // cycles per capsule, K step and column tile
  p.n_cc = (g.in_n() + p.cap - 1) / p.cap;
  const int NFT = padded_frames(g) / 16;
  p.pstride = (size_t)g.in_n() * g.JD() * (g.din + 1);
  const int base = p.n_rt * p.n_cc;
  double best = 1e30;
  for (int S0 = 1; S0 <= NFT; ++S0) {
    const int ft_per = (NFT + S0 - 1) / S0;
    const int S = (NFT + ft_per - 1) / ft_per;
    const int rounds = (base * S + slots - 1) / slots;
    const double work = (double)rounds * ft_per * p.cap * NCT * per_tile / 2.4e9;
    const double slab = S > 1 ? 2.0 * S * p.pstride * 4 / 4e12 : 0.0;
    if (work + slab < best) {
      best = work + slab;
      p.S = S;
      p.ft_per = ft_per;
    }
  }
  return p;
}
size_t gw2_part_floats(const Geom& g) { return (size_t)gw2_plan(g).S * gw2_plan(g).pstride; }

template <int D>
int launch_gw2(const Geom& g, const Gw2Plan& p, const float* xT, const float* saved, const float* gs,
               const float* cst, const float* glst, int JP, float* gwp, float* gbp, hipStream_t st,
               const float* hdr = nullptr, const float* gumax = nullptr) {
  const int grid = p.n_rt * p.n_cc * p.S;
  if constexpr (D == 32) {
    if (use_gw16s(g)) {
      const int grid16 = SRF_GW16S_XCD ? (grid + 7) / 8 * 8 : grid;   // the kernel's XCD-aware task order
      SRF_REQUIRE(hdr != nullptr && gumax != nullptr, "route_gw16s: needs the forward's header and the gx pass's max");
      const _Float16* x16 = reinterpret_cast<const _Float16*>(xT);
#define SRF_GW16S(R_)                                                                                              \
  hipLaunchKernelGGL((route_gw16s_kernel<R_, kGw16Cap>), dim3(grid16), dim3(256), 0, st, x16, hdr, gumax, saved, gs, \
                     cst, glst, g.F(), padded_frames(g), g.in_n(), g.J, g.mask_first, JP, p.n_rt, p.S, p.ft_per, gwp, \
                     gbp, p.pstride)
      if (g.iters == 2)
        SRF_GW16S(2);
      else
        SRF_GW16S(3);
#undef SRF_GW16S
      SRF_LAUNCH_CHECK("route_gw16s");
      return SRF_OK;
    }
  }
  if constexpr (D <= 32) {
    if (gw3_cap(g)) {
#define SRF_GW3(R_, C_)                                                                                           \
  hipLaunchKernelGGL((route_gw3_kernel<D, R_, C_>), dim3(grid), dim3(256), 0, st, xT, saved, gs, cst, glst, g.F(), \
                     padded_frames(g), g.in_n(), g.J, g.mask_first, JP, p.n_rt, p.S, p.ft_per, gwp, gbp, p.pstride)
#define SRF_GW3C(R_) \
  if (p.cap == 4) SRF_GW3(R_, 4); else SRF_GW3(R_, 8);
      switch (g.iters) {   // gw3_cap() is 0 past 3 iterations
        case 2: SRF_GW3C(2) break;
        default: SRF_GW3C(3) break;
      }
#undef SRF_GW3C
#undef SRF_GW3
      SRF_LAUNCH_CHECK("route_gw3");
      return SRF_OK;
    }
  }
#define SRF_GW2(R_)                                                                                              \
  hipLaunchKernelGGL((route_gw2_kernel<D, R_>), dim3(grid), dim3(256), 0, st, xT, saved, gs, cst, glst, g.F(),    \
                     padded_frames(g), g.in_n(), g.J, g.mask_first, JP, p.n_rt, p.n_cc, p.S, p.ft_per, gwp, gbp,   \
                     p.pstride)
  switch (g.iters) {
    case 2: SRF_GW2(2); break;
    case 3: SRF_GW2(3); break;
    case 4: SRF_GW2(4); break;
    default: SRF_GW2(5); break;
  }
#undef SRF_GW2
  SRF_LAUNCH_CHECK("route_gw2");
  return SRF_OK;
}

// The 32x32 split-fp16 passes (route_fwd32.hip) serve the shapes they support,
// route_pass_kernel (exact fp32 16x16x4 tiles) the others (din 64, J*dout > 1024).
inline bool use_fwd32(const Geom& g) { return srf::fwd32_supported(g.din, g.dout, g.J); }

// Coupling storage is used when the split-bf16 forward runs and the gu pass from
// stored couplings (route_gux_kernel) fits its window accumulator in LDS; otherwise
// the forward keeps nothing and the backward recomputes (round-1 kernels).
// The coupling readers address their blocks through buffer descriptors with 32-bit
// byte ranges and 32-bit offsets (route_gux_kernel's c / gL blocks over all
// iterations, route_gw3_kernel's per-iteration s and gs slices, the forward's
// c / logZ stores): past 2^31 bytes the forward stores nothing and the backward
// recomputes the logits instead of reading wrapped offsets.
inline bool coupling_sizes_fit(const Geom& g) {
  constexpr size_t kLim = size_t(1) << 31;
  const srf::Fwd32Plan plan = srf::fwd32_plan(g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout);
  const size_t total = srf::fwd32_cpl_layout(plan, g.F(), g.in_n(), g.din, g.dout, g.J, g.iters).total;
  return total * 4 < kLim && (size_t)g.F() * g.JD() * 4 * g.iters < kLim;
}

inline bool couplings_ok(const Geom& g) {
  if (!use_fwd32(g) || g.iters < 2 || g.din > 32) return false;
  const int TW = gu_tw(g.dout);
  const int nw = std::min(kGuNW, (g.NT() + TW - 1) / TW);
  return gu_lds_bytes(g, nw, 1) <= kGuLdsMax && coupling_sizes_fit(g);
}


template <int D>
int fwd_impl(const Geom& g, int n_chunks, const float* emb, const float* W, const float* bias, float* v_out,
             float* saved, float* couplings, float* slab, hipStream_t st) {
  const PassCfg pc = pass_cfg(g);
  const size_t FJD = (size_t)g.F() * g.JD();
  hipEvent_t* ev0 = t_ev_start;
  hipEvent_t* ev1 = t_ev_stop;
  const int nev = t_ev_n;
  t_ev_start = t_ev_stop = nullptr;
  t_ev_n = 0;
  const bool p32 = use_fwd32(g);
  srf::Fwd32Plan plan{};
  srf::Fwd32Cpl cl{};
  float* bsum = slab + (size_t)n_chunks * FJD;
  // split operand planes: in the coupling storage when the backward will reuse them
  void* planes = slab;
  void* scratch = slab;
  if (p32) {
    plan = srf::fwd32_plan(g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout, n_chunks);
    float *WT = nullptr, *xT = nullptr;
    if (couplings != nullptr) {
      cl = srf::fwd32_cpl_layout(plan, g.F(), g.in_n(), g.din, g.dout, g.J, g.iters);
      planes = couplings + cl.planes;
      WT = couplings + cl.WT;
      xT = couplings + cl.xT;
    } else {
      scratch = static_cast<char*>(static_cast<void*>(slab)) + srf::fwd32_planes_bytes(plan);
    }
    const int rc = srf::fwd32_prepare(plan, emb, W, bias, g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout, planes,
                                      scratch, WT, xT, st, WT != nullptr && use_gux16(g),
                                      xT != nullptr && use_gw16s(g));
    if (rc) return rc;
  } else {
    const int chunk_len = (g.in_n() + n_chunks - 1) / n_chunks;
    hipLaunchKernelGGL(bias_chunk_sum_kernel, dim3((n_chunks * g.JD() + 255) / 256), dim3(256), 0, st, bias,
                       g.in_n(), g.JD(), n_chunks, chunk_len, bsum);
    SRF_LAUNCH_CHECK("bias_chunk_sum");
  }
  for (int r = 0; r < g.iters; ++r) {
    const float* vc = r > 0 ? saved + (size_t)(2 * (r - 1) + 1) * FJD : nullptr;
    if (r < nev) SRF_HIP_TRY(hipEventRecord(ev0[r], st));
    if (p32 && r == 0 && srf::fwd32_first_full_supported(plan, g.din, g.dout)) {
      // iteration 0 with its finish fused: s^0, Vc^1 (and v for one iteration) directly
      const int rc = srf::fwd32_first_full(plan, planes, scratch, g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout,
                                           g.mask_first, saved, saved + FJD, g.iters == 1 ? v_out : nullptr, st);
      if (rc) return rc;
      if (r < nev) SRF_HIP_TRY(hipEventRecord(ev1[r], st));
      continue;
    }
    if (p32) {
      float *cst = nullptr, *lzst = nullptr;
      if (couplings != nullptr && r > 0) {
        const size_t blk = (size_t)srf::fwd32_frame_stride(g.F()) * g.in_n();
        cst = couplings + cl.c + (size_t)(r - 1) * blk * (plan.JDp / g.dout);
        lzst = couplings + cl.lz + (size_t)(r - 1) * blk;
      }
      const int rc = srf::fwd32_pass(plan, r == 0, planes, scratch, g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J,
                                     g.dout, g.mask_first, vc, cst, lzst, st);
      if (rc) return rc;
    } else {
      dispatch_pass<D, MODE_FWD>(g, pc, n_chunks, emb, W, bias, r, vc, r == 0 ? bsum : nullptr, slab, nullptr, 1, st);
    }
    SRF_LAUNCH_CHECK("route_pass(fwd)");
    if (r < nev) SRF_HIP_TRY(hipEventRecord(ev1[r], st));
    launch_fwd_finish<D>(g, p32 ? srf::fwd32_slab(plan, scratch) : slab,
                         p32 ? plan.n_chunks : n_chunks, vc,
                         saved + (size_t)(2 * r) * FJD, saved + (size_t)(2 * r + 1) * FJD,
                         r == g.iters - 1 ? v_out : nullptr, st);
    SRF_LAUNCH_CHECK("fwd_finish");
  }
  return SRF_OK;
}

struct BwdWs {
  float *A, *gs, *slab, *stats, *gu_t, *xT, *WT;
  void* p32;          // scratch (bias sums + partial slabs) of the B1 passes from stored couplings
  float* gl;          // gL^r of those passes [iters-1][in_n][JP][Fs], read by the gu / gW passes
  float* gwpart;      // partial gW | gbias slabs of route_gw2_kernel (S frame splits)
  float* gumax;       // max |gu| of the layer (route_gux16_kernel -> route_gw16s_kernel)
  size_t bytes;
};

BwdWs bwd_layout(const Geom& g, int n_chunks, void* base) {
  const size_t F = g.F(), JD = g.JD(), in_n = g.in_n(), Fp = padded_frames(g);
  size_t off = 0;
  auto take = [&](size_t nfloat) {
    size_t o = off;
    off += srf::align_up(nfloat * sizeof(float), 256);
    return o;
  };
  const size_t oA = take(F * JD), ogs = take((size_t)g.iters * F * JD), oslab = take((size_t)n_chunks * F * JD),
               ostats = take((size_t)(g.iters - 1) * F * in_n * 2), ogu = take(in_n * (size_t)g.NT() * 16 * Fp),
               oxt = take(in_n * g.din * Fp), owt = take(in_n * JD * g.din);
  size_t op32 = 0, ogl = 0, ogwp = 0;
  const size_t ogm = take(64);
  if (use_fwd32(g)) {
    const srf::Fwd32Plan plan = srf::fwd32_plan(g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout, n_chunks);
    op32 = take((srf::fwd32_scratch_bytes(plan) + 3) / 4);
    ogl = take((size_t)std::max(g.iters - 1, 1) * srf::fwd32_frame_stride(g.F()) * in_n * (plan.JDp / g.dout));
    ogwp = take(gw2_part_floats(g));
  }
  char* b = static_cast<char*>(base);
  BwdWs w;
  w.A = (float*)(b + oA);
  w.gs = (float*)(b + ogs);
  w.slab = (float*)(b + oslab);
  w.stats = (float*)(b + ostats);
  w.gu_t = (float*)(b + ogu);
  w.xT = (float*)(b + oxt);
  w.WT = (float*)(b + owt);
  w.p32 = op32 ? (void*)(b + op32) : nullptr;
  w.gl = ogl ? (float*)(b + ogl) : nullptr;
  w.gwpart = ogwp ? (float*)(b + ogwp) : nullptr;
  w.gumax = (float*)(b + ogm);
  w.bytes = off;
  return w;
}

// gW = gu x^T and gbias from the gu blocks the data pass left in the workspace; needs
// nothing else of the backward, so a caller may run it on a second stream (after the
// data pass, joined before g_W / g_bias or the workspace are used again).
template <int D>
int bwd_weights_impl(const Geom& g, const float* emb, float* g_W, float* g_bias, const BwdWs& w, hipStream_t st,
                     const float* saved = nullptr, const float* couplings = nullptr) {
  const int Fp = padded_frames(g);
  if (couplings != nullptr && w.gl != nullptr && g.iters > 1) {
    // gu formed from the stored couplings / logit gradients (never materialised);
    // the forward left the windowed x^T in the coupling storage
    const Gw2Plan p = gw2_plan(g);
    const srf::Fwd32Plan plan = srf::fwd32_plan(g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout);
    const srf::Fwd32Cpl cl = srf::fwd32_cpl_layout(plan, g.F(), g.in_n(), g.din, g.dout, g.J, g.iters);
    const bool direct = p.S == 1;
    float* gwp = direct ? g_W : w.gwpart;
    float* gbp = direct ? g_bias : w.gwpart + (size_t)g.in_n() * g.JD() * g.din;
    int rc = launch_gw2<D>(g, p, couplings + cl.xT, saved, w.gs, couplings + cl.c, w.gl, plan.JDp / g.dout, gwp, gbp,
                           st, srf::fwd32_hdr(plan, couplings + cl.planes), w.gumax);
    if (rc || direct) return rc;
    const size_t nw4 = (size_t)g.in_n() * g.JD() * g.din / 4, n4 = p.pstride / 4;
    hipLaunchKernelGGL(gw_reduce_kernel, dim3((n4 + 255) / 256), dim3(256), 0, st, w.gwpart, p.S, n4, p.pstride, g_W,
                       nw4, g_bias);
    SRF_LAUNCH_CHECK("gw_reduce");
    return SRF_OK;
  }
  {
    SRF_REQUIRE(g.din <= 64, "window_xt tile holds din <= 64, got %d", g.din);
    const int tiles = (Fp + kXtFrames - 1) / kXtFrames;
    hipLaunchKernelGGL(window_xt_kernel, dim3(g.in_n() * tiles), dim3(256), 0, st, emb, g.F(), Fp, g.T, g.N, g.din,
                       g.lpad, g.in_n(), w.xT);
    SRF_LAUNCH_CHECK("window_xt");
  }
  {
    const int tasks = g.in_n() * g.NT();
    hipLaunchKernelGGL((route_gw_kernel<D>), dim3((tasks + 3) / 4), dim3(256), 0, st, w.gu_t, w.xT, Fp, g.in_n(),
                       g.JD(), g_W, g_bias);
    SRF_LAUNCH_CHECK("route_gw");
  }
  return SRF_OK;
}

template <int D>
int bwd_impl(const Geom& g, int n_chunks, const float* emb, const float* W, const float* bias, const float* saved,
             const float* couplings, const float* g_v, float* g_emb, float* g_W, float* g_bias, const BwdWs& w,
             hipStream_t st, bool with_weights) {
  const PassCfg pc = pass_cfg(g);
  const size_t FJD = (size_t)g.F() * g.JD();
  const int R = g.iters;
  const int Fp = padded_frames(g);
  // gs^{R-1} = squash'(s^{R-1}) g_v.  A accumulates sum_{r'>r} gVc^{r'}, the
  // gradient of v^r for r < R-1 (those v reach the loss only through the logits).
  // Iteration 0 needs no backward pass: Vc^0 = 0, so its couplings are uniform
  // and its logits carry no gradient.
  const bool p32 = couplings != nullptr && w.p32 != nullptr && R > 1;
  const size_t n_emb = (size_t)g.F() * g.N * g.din;
  // with stored couplings this launch also zeroes g_emb (the gu pass accumulates into it)
  launch_bwd_finish<D>(g, nullptr, n_chunks, g_v, w.A, saved + (size_t)(2 * (R - 1)) * FJD,
                       w.gs + (size_t)(R - 1) * FJD, st, p32 ? g_emb : nullptr, n_emb, p32 ? w.gumax : nullptr);
  SRF_LAUNCH_CHECK("bwd_finish");
  srf::Fwd32Plan plan{};
  srf::Fwd32Cpl cl{};
  if (p32) {
    // B1 from the forward's stored couplings and operand planes on the split-bf16 32x32 tiles
    plan = srf::fwd32_plan(g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J, g.dout, n_chunks);
    cl = srf::fwd32_cpl_layout(plan, g.F(), g.in_n(), g.din, g.dout, g.J, g.iters);
  }
  for (int r = R - 1; r >= 1; --r) {
    const float* vc = saved + (size_t)(2 * (r - 1) + 1) * FJD;
    float* stats_r = w.stats + (size_t)(r - 1) * g.F() * g.in_n() * 2;
    if (p32) {
      const size_t blk = (size_t)srf::fwd32_frame_stride(g.F()) * g.in_n();
      const int JP = plan.JDp / g.dout;
      const int rc = srf::bwd32_pass(plan, couplings + cl.planes, w.p32, g.B, g.T, g.N, g.din, g.lpad, g.rpad, g.J,
                                     g.dout, couplings + cl.c + (size_t)(r - 1) * blk * JP,
                                     couplings + cl.lz + (size_t)(r - 1) * blk,
                                     w.gs + (size_t)r * FJD, stats_r, w.gl + (size_t)(r - 1) * blk * JP, st);
      if (rc) return rc;
      launch_bwd_finish<D>(g, srf::fwd32_slab(plan, w.p32), plan.n_chunks, nullptr, w.A,
                             saved + (size_t)(2 * (r - 1)) * FJD, w.gs + (size_t)(r - 1) * FJD, st);
    } else {
      dispatch_pass<D, MODE_BWD>(g, pc, n_chunks, emb, W, bias, r, vc, w.gs + (size_t)r * FJD, w.slab, stats_r, 1,
                                 st);
      SRF_LAUNCH_CHECK("route_pass(bwd)");
      launch_bwd_finish<D>(g, w.slab, n_chunks, nullptr, w.A, saved + (size_t)(2 * (r - 1)) * FJD,
                           w.gs + (size_t)(r - 1) * FJD, st);
    }
    SRF_LAUNCH_CHECK("bwd_finish");
  }
  if (!p32) {
    // W^T for the gu pass; the same launch zeroes g_emb
    const size_t total = (size_t)g.in_n() * g.JD() * g.din + n_emb;
    hipLaunchKernelGGL(transpose_w_kernel, dim3((total + 255) / 256), dim3(256), 0, st, W, g.in_n(), g.JD(), g.din,
                       w.WT, g_emb, n_emb);
    SRF_LAUNCH_CHECK("transpose_w");
  }
  if (p32) {
    // w.gumax (the gu pass's atomic max) was zeroed by the first bwd_finish launch
    launch_gu_r<D>(g, emb, W, couplings + cl.WT, bias, saved, w.gs, w.stats, w.gu_t, g_emb, st, couplings + cl.c,
                   w.gl, plan.JDp / g.dout, srf::fwd32_hdr(plan, couplings + cl.planes), w.gumax);
  } else
    launch_gu_r<D>(g, emb, W, w.WT, bias, saved, w.gs, w.stats, w.gu_t, g_emb, st);
  SRF_LAUNCH_CHECK("route_gu");
  (void)Fp;
  return with_weights ? bwd_weights_impl<D>(g, emb, g_W, g_bias, w, st, saved, p32 ? couplings : nullptr) : SRF_OK;
}

}  // namespace

extern "C" {

int srf_route_dr_set_timing_events(void* const* starts, void* const* stops, int n) {
  SRF_REQUIRE(n >= 0 && (n == 0 || (starts && stops)), "bad timing event arrays");
  t_ev_start = (hipEvent_t*)starts;
  t_ev_stop = (hipEvent_t*)stops;
  t_ev_n = n;
  return SRF_OK;
}

int srf_route_dr_auto_chunks(int B, int T, int N, int din, int lpad, int rpad, int J, int dout) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  if (use_fwd32(g)) return srf::fwd32_plan(B, T, N, din, lpad, rpad, J, dout).n_chunks;
  return auto_chunks(g, pass_cfg(g).NW);
}

size_t srf_route_dr_saved_floats(int B, int T, int J, int dout, int iters) {
  return (size_t)2 * iters * B * T * J * dout;
}

size_t srf_route_dr_fwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters,
                                  int n_chunks) {
  (void)iters;
  // partial slabs + the i-chunk bias sums of the iteration-0 pass
  size_t need = (size_t)n_chunks * ((size_t)B * T + 1) * J * dout * sizeof(float);
  Geom g{B, T, N, din, lpad, rpad, J, dout, 1, 0};
  if (use_fwd32(g))
    need = std::max(need, srf::fwd32_workspace(srf::fwd32_plan(B, T, N, din, lpad, rpad, J, dout, n_chunks)));
  return need;
}

size_t srf_route_dr_bwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters,
                                  int n_chunks) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, iters, 0};
  return bwd_layout(g, n_chunks, nullptr).bytes;
}

size_t srf_route_dr_coupling_floats(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, iters, 0};
  if (!couplings_ok(g)) return 0;
  return srf::fwd32_cpl_layout(srf::fwd32_plan(B, T, N, din, lpad, rpad, J, dout), B * T, g.in_n(), din, dout, J, iters)
      .total;
}

int srf_route_dr_fwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int iters, int mask_first, int n_chunks, float* v_out, float* saved,
                     void* workspace, size_t workspace_bytes, void* stream) {
  return srf_route_dr_fwd_ex(emb, W, bias, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks, v_out,
                             saved, nullptr, workspace, workspace_bytes, stream);
}

int srf_route_dr_fwd_ex(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                        int rpad, int J, int dout, int iters, int mask_first, int n_chunks, float* v_out,
                        float* saved, float* couplings, void* workspace, size_t workspace_bytes, void* stream) {
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
  if (couplings != nullptr && !couplings_ok(g)) couplings = nullptr;   // nothing to store
  switch (din) {
    case 8: return fwd_impl<8>(g, n_chunks, emb, W, bias, v_out, saved, couplings, slab, st);
    case 16: return fwd_impl<16>(g, n_chunks, emb, W, bias, v_out, saved, couplings, slab, st);
    case 32: return fwd_impl<32>(g, n_chunks, emb, W, bias, v_out, saved, couplings, slab, st);
    default: return fwd_impl<64>(g, n_chunks, emb, W, bias, v_out, saved, couplings, slab, st);
  }
}

namespace {
int route_dr_bwd_entry(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                       int rpad, int J, int dout, int iters, int mask_first, int n_chunks, const float* saved,
                       const float* couplings, const float* g_v, float* g_emb, float* g_W, float* g_bias,
                       void* workspace, size_t workspace_bytes, void* stream, bool with_weights) {
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
  if (couplings != nullptr && !couplings_ok(g)) couplings = nullptr;
  switch (din) {
    case 8:
      return bwd_impl<8>(g, n_chunks, emb, W, bias, saved, couplings, g_v, g_emb, g_W, g_bias, w, st, with_weights);
    case 16:
      return bwd_impl<16>(g, n_chunks, emb, W, bias, saved, couplings, g_v, g_emb, g_W, g_bias, w, st, with_weights);
    case 32:
      return bwd_impl<32>(g, n_chunks, emb, W, bias, saved, couplings, g_v, g_emb, g_W, g_bias, w, st, with_weights);
    default:
      return bwd_impl<64>(g, n_chunks, emb, W, bias, saved, couplings, g_v, g_emb, g_W, g_bias, w, st, with_weights);
  }
}
}  // namespace

int srf_route_dr_bwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int iters, int mask_first, int n_chunks, const float* saved,
                     const float* g_v, float* g_emb, float* g_W, float* g_bias, void* workspace,
                     size_t workspace_bytes, void* stream) {
  return route_dr_bwd_entry(emb, W, bias, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks, saved,
                            nullptr, g_v, g_emb, g_W, g_bias, workspace, workspace_bytes, stream, true);
}

int srf_route_dr_bwd_ex(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                        int rpad, int J, int dout, int iters, int mask_first, int n_chunks, const float* saved,
                        const float* couplings, const float* g_v, float* g_emb, float* g_W, float* g_bias,
                        void* workspace, size_t workspace_bytes, void* stream) {
  return route_dr_bwd_entry(emb, W, bias, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks, saved,
                            couplings, g_v, g_emb, g_W, g_bias, workspace, workspace_bytes, stream, true);
}

int srf_route_dr_bwd_data(const float* emb, const float* W, const float* bias, int B, int T, int N, int din,
                          int lpad, int rpad, int J, int dout, int iters, int mask_first, int n_chunks,
                          const float* saved, const float* g_v, float* g_emb, void* workspace,
                          size_t workspace_bytes, void* stream) {
  // g_W / g_bias are not touched by the data pass; the checks want non-null pointers
  float* unused = reinterpret_cast<float*>(workspace);
  return route_dr_bwd_entry(emb, W, bias, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks, saved,
                            nullptr, g_v, g_emb, unused, unused, workspace, workspace_bytes, stream, false);
}

int srf_route_dr_bwd_data_ex(const float* emb, const float* W, const float* bias, int B, int T, int N, int din,
                             int lpad, int rpad, int J, int dout, int iters, int mask_first, int n_chunks,
                             const float* saved, const float* couplings, const float* g_v, float* g_emb,
                             void* workspace, size_t workspace_bytes, void* stream) {
  float* unused = reinterpret_cast<float*>(workspace);
  return route_dr_bwd_entry(emb, W, bias, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks, saved,
                            couplings, g_v, g_emb, unused, unused, workspace, workspace_bytes, stream, false);
}

int srf_route_dr_bwd_weights(const float* emb, int B, int T, int N, int din, int lpad, int rpad, int J, int dout,
                             int iters, int mask_first, int n_chunks, float* g_W, float* g_bias, void* workspace,
                             size_t workspace_bytes, void* stream) {
  return srf_route_dr_bwd_weights_ex(emb, B, T, N, din, lpad, rpad, J, dout, iters, mask_first, n_chunks, nullptr,
                                     nullptr, g_W, g_bias, workspace, workspace_bytes, stream);
}

int srf_route_dr_bwd_weights_ex(const float* emb, int B, int T, int N, int din, int lpad, int rpad, int J, int dout,
                                int iters, int mask_first, int n_chunks, const float* saved, const float* couplings,
                                float* g_W, float* g_bias, void* workspace, size_t workspace_bytes, void* stream) {
  Geom g{B, T, N, din, lpad, rpad, J, dout, iters, mask_first ? 1 : 0};
  int rc = check_geom(g);
  if (rc) return rc;
  SRF_REQUIRE(emb && g_W && g_bias && workspace, "null pointer argument");
  SRF_REQUIRE(n_chunks >= 1 && n_chunks <= g.in_n(), "n_chunks %d out of [1, %d]", n_chunks, g.in_n());
  BwdWs w = bwd_layout(g, n_chunks, workspace);
  if (workspace_bytes < w.bytes) {
    srf::set_error("backward workspace too small: %zu < %zu", workspace_bytes, w.bytes);
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (couplings != nullptr && (!couplings_ok(g) || saved == nullptr)) couplings = nullptr;
  switch (din) {
    case 8: return bwd_weights_impl<8>(g, emb, g_W, g_bias, w, st, saved, couplings);
    case 16: return bwd_weights_impl<16>(g, emb, g_W, g_bias, w, st, saved, couplings);
    case 32: return bwd_weights_impl<32>(g, emb, g_W, g_bias, w, st, saved, couplings);
    default: return bwd_weights_impl<64>(g, emb, g_W, g_bias, w, st, saved, couplings);
  }
}

}  // extern "C"
