// CNN front end (CapsulationLayer, sequence_router.py:44-82) for gfx950.
//
// Two maxout stages over the NHWC fbank map (H = time, W = frequency):
//   y_k = mask_k( max( drop(conv_ka(x)), drop(conv_kb(x)) ) )      (:76-77)
//   x_{k+1} = mask_k( BN_k(y_k) )                                    (:78-79)
// with 3x3 stride-2 'SAME' convolutions (TF padding: pad_before = total // 2),
// mask_k zeroing frames t >= ceil(len / 2^(k+1)) (model_helper.py:125-140) and
// Keras BatchNormalization (batch statistics over every position, eps 1e-3).
//
// Kernels:
//   conv1_fwd    VALU direct conv (Cin = 1, K = 9) + maxout + dropout + mask,
//                Welford per-channel partials for BN1, argmax byte per output;
//   bn_finalize  Chan merge of the partials -> scale/shift, moving statistics;
//   conv2_fwd    MFMA implicit GEMM (M = output pixels, N = 128 = both convs,
//                K = 9 taps x 64 channels) whose A staging applies BN1 + mask1
//                and whose epilogue does bias + dropout + maxout + mask2 + BN2
//                partials;
//   bn_apply     writes the CapsulationLayer output mask2(BN2(y2)).
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdlib>

#include "srf_common.h"
#include "srf_reduce.h"
#include "srf_rng.h"
#include "../../include/srf.h"

namespace {

constexpr int C = 64;            // --model-conv-filter-num (reference default, required here)
constexpr float kBnEps = 1e-3f;   // Keras BatchNormalization default
constexpr float kBnMomentum = 0.99f;

struct Dims {
  int B, T, Fin;
  int T1, F1, T2, F2;
  int pt1, pf1, pt2, pf2;  // SAME pad_before of stage 1 / stage 2 (time, freq)
};

inline int same_out(int n) { return (n + 1) / 2; }
inline int same_pad_before(int n) {
  const int out = same_out(n);
  const int total = std::max((out - 1) * 2 + 3 - n, 0);
  return total / 2;
}

Dims make_dims(int B, int T, int Fin) {
  Dims d;
  d.B = B; d.T = T; d.Fin = Fin;
  d.T1 = same_out(T); d.F1 = same_out(Fin);
  d.T2 = same_out(d.T1); d.F2 = same_out(d.F1);
  d.pt1 = same_pad_before(T); d.pf1 = same_pad_before(Fin);
  d.pt2 = same_pad_before(d.T1); d.pf2 = same_pad_before(d.F1);
  return d;
}

__device__ __forceinline__ int ceil_div_len(int len, int div) { return (len + div - 1) / div; }

// Welford partial (count, mean, M2) merge (Chan et al.).
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  if (nb == 0.f) return;
  const float nn = n + nb;
  const float delta = meanb - mean;
  mean += delta * (nb / nn);
  m2 += m2b + delta * delta * (n * nb / nn);
  n = nn;
}

// Split-bf16 weight packing of stage 2 (defined with the split kernels below), run
// by extra blocks of the conv1 forward / conv2_bwd_prep launches.
constexpr int kPackW2Threads = 2 * C * 64;             // one wave per stage-2 output column n
constexpr int kPackW2tThreads = 9 * C * (2 * C / 8);   // (tap, cin, n/8)
__device__ __forceinline__ void pack_w2_f16_body(int idx, const float* __restrict__ ka, const float* __restrict__ kb,
                                                 _Float16* __restrict__ wp2, float* __restrict__ wsc);
__device__ __forceinline__ void pack_w2t_split_body(int idx, const float* __restrict__ ka,
                                                    const float* __restrict__ kb, __bf16* __restrict__ wq3);
__device__ __forceinline__ void pack_w2t_f16_body(int idx, const float* __restrict__ ka, const float* __restrict__ kb,
                                                  _Float16* __restrict__ wq2h, float* __restrict__ wdsc);
constexpr int kPackW2tF16Threads = C * 64;   // one wave per data-gradient output column cin

// ---------------------------------------------------------------- conv1
// A workgroup = kRows1 consecutive output rows t1 of one utterance (one wave per
// row), a lane = one output channel c.  The 2*kRows1+1 input rows the tile reads
// are staged in LDS with the SAME zero padding materialised, so each pixel's
// 3x3 window is 9 broadcast LDS reads and no bounds checks.
constexpr int kRows1 = 4;

struct Tile1 {
  int b, t1_0, fpad;   // fpad = row stride of the staged input (Fin + 2)
};

__device__ __forceinline__ Tile1 stage_rows1(const float* __restrict__ feats, const Dims& d, float* win) {
  const int tiles_per_b = (d.T1 + kRows1 - 1) / kRows1;
  Tile1 tl;
  tl.b = blockIdx.x / tiles_per_b;
  tl.t1_0 = (blockIdx.x - tl.b * tiles_per_b) * kRows1;
  tl.fpad = d.Fin + 2;
  const int nrows = 2 * kRows1 + 1;
  const int t_base = 2 * tl.t1_0 - d.pt1;
  for (int k = threadIdx.x; k < nrows * tl.fpad; k += blockDim.x) {
    const int r = k / tl.fpad, col = k - r * tl.fpad;
    const int t = t_base + r, f = col - 1;   // staged column 0 is f = -1
    const bool ok = t >= 0 && t < d.T && f >= 0 && f < d.Fin;
    const float v = feats[((size_t)tl.b * d.T + min(max(t, 0), d.T - 1)) * d.Fin + min(max(f, 0), d.Fin - 1)];
    win[k] = ok ? v : 0.f;
  }
  __syncthreads();
  return tl;
}

// x[dt*3+df] of output pixel (row wave w, column f1); requires pf1 <= 1 (3x3, stride 2)
__device__ __forceinline__ void window9_lds(const float* win, const Tile1& tl, const Dims& d, int w, int f1,
                                            float (&x)[9]) {
#pragma unroll
  for (int dt = 0; dt < 3; ++dt)
#pragma unroll
    for (int df = 0; df < 3; ++df) x[dt * 3 + df] = win[(2 * w + dt) * tl.fpad + 2 * f1 - d.pf1 + df + 1];
}

// Partials slab[block][c] = (n, mean, M2).
__global__ __launch_bounds__(256) void conv1_fwd_kernel(
    const float* __restrict__ feats, const int* __restrict__ inp_len, Dims d, const float* __restrict__ ka,
    const float* __restrict__ ba, const float* __restrict__ kb, const float* __restrict__ bb, int training,
    float drop_p, unsigned long long seed, const unsigned long long* __restrict__ seed_src, float* __restrict__ y1, unsigned char* __restrict__ sel1,
    float* __restrict__ part, int nconv, const float* __restrict__ pk_a, const float* __restrict__ pk_b,
    _Float16* __restrict__ wp2, float* __restrict__ wsc, float* __restrict__ ymax) {
  // blocks past nconv pack the stage-2 split weights (one launch fewer per forward)
  if ((int)blockIdx.x >= nconv) {
    const int idx = (blockIdx.x - nconv) * blockDim.x + threadIdx.x;
    if (idx < kPackW2Threads) pack_w2_f16_body(idx, pk_a, pk_b, wp2, wsc);
    return;
  }
  seed = srf_step_seed(seed, seed_src);
  extern __shared__ __attribute__((aligned(16))) float win[];
  __shared__ float sh[3][kRows1][C];
  const int c = threadIdx.x & (C - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float wa[9], wb[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    wa[k] = ka[k * C + c];  // kernel [3][3][1][C]
    wb[k] = kb[k * C + c];
  }
  const float bia = ba[c], bib = bb[c];
  const float keep_scale = 1.f / (1.f - drop_p);
  const bool drop = training && drop_p > 0.f;
  const Tile1 tl = stage_rows1(feats, d, win);
  const int t1 = tl.t1_0 + w;
  // statistics as sums shifted by the channel biases (no per-element division)
  float n = 0.f, s1 = 0.f, s2 = 0.f, ym = 0.f;
  const float K = 0.5f * (bia + bib);
  if (t1 < d.T1) {
    const bool live = t1 < ceil_div_len(inp_len[tl.b], 2);
    const int pbase = (tl.b * d.T1 + t1) * d.F1;
#pragma unroll 2
    for (int f1 = 0; f1 < d.F1; ++f1) {
      float x[9];
      window9_lds(win, tl, d, w, f1, x);
      float a = bia, bv = bib;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        a += x[k] * wa[k];
        bv += x[k] * wb[k];
      }
      const int o = (pbase + f1) * C + c;
      if (drop) {
        bool ka, kb;
        srf_keep2(seed, kStreamConv0a, o, drop_p, ka, kb);
        a *= ka ? keep_scale : 0.f;
        bv *= kb ? keep_scale : 0.f;
      }
      const bool sl = a >= bv;  // TF Maximum gradient: ties go to the first operand
      const float y = live ? (sl ? a : bv) : 0.f;
      y1[o] = y;
      sel1[o] = sl ? 1 : 0;
      ym = fmaxf(ym, fabsf(y));
      n += 1.f;
      s1 += y - K;
      s2 += (y - K) * (y - K);
    }
  }
  float mean = n > 0.f ? K + s1 / n : 0.f;
  float m2 = n > 0.f ? fmaxf(s2 - s1 * s1 / n, 0.f) : 0.f;
  sh[0][w][c] = n; sh[1][w][c] = mean; sh[2][w][c] = m2;
  // max |y1| of the block (the stage-2 split exponent, bn_finalize_kernel)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ym = fmaxf(ym, __shfl_xor(ym, o, 64));
  __shared__ float smax[kRows1];
  if (c == 0) smax[w] = ym;
  __syncthreads();
  if (w == 0) {
    if (c == 0) {
      float m = smax[0];
      for (int r = 1; r < kRows1; ++r) m = fmaxf(m, smax[r]);
      ymax[blockIdx.x] = m;
    }
    for (int r = 1; r < kRows1; ++r) chan_merge(n, mean, m2, sh[0][r][c], sh[1][r][c], sh[2][r][c]);
    part[((size_t)blockIdx.x * 3 + 0) * C + c] = n;
    part[((size_t)blockIdx.x * 3 + 1) * C + c] = mean;
    part[((size_t)blockIdx.x * 3 + 2) * C + c] = m2;
  }
}

// Merge groups of Welford partials: block k merges parts [k*per, (k+1)*per) of
// every channel into out[k] (the first stage of the BN finalize).
__global__ __launch_bounds__(256) void bn_merge_kernel(const float* __restrict__ part, int nparts, int per,
                                                       float* __restrict__ out) {
  __shared__ float sh[3][4][C];
  const int c = threadIdx.x & (C - 1), r = threadIdx.x >> 6;
  const int k0 = blockIdx.x * per, k1 = min(nparts, k0 + per);
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int k = k0 + r; k < k1; k += 4)
    chan_merge(n, mu, m2, part[((size_t)k * 3 + 0) * C + c], part[((size_t)k * 3 + 1) * C + c],
               part[((size_t)k * 3 + 2) * C + c]);
  sh[0][r][c] = n; sh[1][r][c] = mu; sh[2][r][c] = m2;
  __syncthreads();
  if (r != 0) return;
  for (int q = 1; q < 4; ++q) chan_merge(n, mu, m2, sh[0][q][c], sh[1][q][c], sh[2][q][c]);
  out[((size_t)blockIdx.x * 3 + 0) * C + c] = n;
  out[((size_t)blockIdx.x * 3 + 1) * C + c] = mu;
  out[((size_t)blockIdx.x * 3 + 2) * C + c] = m2;
}

// ---------------------------------------------------------------- BN finalize
// stats[0][c] = mean, stats[1][c] = rstd, stats[2][c] = scale, stats[3][c] = shift.
// With ymax (the conv1 block maxima of |y|): stats[4][0] = 2^b, stats[4][1] = 2^-b, the
// split-fp16 exponent of the BN output, from the bound |scale_c y + shift_c| <=
// max|scale| max|y| + max|shift| (conv2_fwd32_kernel).
// 1024 threads = 16 partial streams x 64 channels, Chan-merged through LDS.
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float* __restrict__ part, int nparts,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           float* __restrict__ mmean, float* __restrict__ mvar,
                                                           int training, float* __restrict__ stats,
                                                           const float* __restrict__ ymax, int nymax) {
  __shared__ float sh[3][16][C];
  __shared__ float ysh[16], ab[2][C];
  const int c = threadIdx.x & (C - 1), r = threadIdx.x >> 6;
  if (ymax != nullptr) {
    float m = 0.f;
    for (int k = threadIdx.x; k < nymax; k += 1024) m = fmaxf(m, ymax[k]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (c == 0) ysh[r] = m;
  }
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (training)
#pragma unroll 8
    for (int k = r; k < nparts; k += 16)
      chan_merge(n, mu, m2, part[((size_t)k * 3 + 0) * C + c], part[((size_t)k * 3 + 1) * C + c],
                 part[((size_t)k * 3 + 2) * C + c]);
  sh[0][r][c] = n; sh[1][r][c] = mu; sh[2][r][c] = m2;
  __syncthreads();
  // wave 0 (r == 0) finalises the 64 channels; every wave then meets the one
  // barrier below (taken by all or none: ymax is a kernel argument)
  if (r == 0) {
    float mean, var;
    if (training) {
      for (int q = 1; q < 16; ++q) chan_merge(n, mu, m2, sh[0][q][c], sh[1][q][c], sh[2][q][c]);
      mean = mu;
      var = m2 / n;
      // moving averages; the fused NHWC kernel feeds the Bessel-corrected variance
      mmean[c] = mmean[c] * kBnMomentum + mean * (1.f - kBnMomentum);
      mvar[c] = mvar[c] * kBnMomentum + (n > 1.f ? var * n / (n - 1.f) : var) * (1.f - kBnMomentum);
    } else {
      mean = mmean[c];
      var = mvar[c];
    }
    const float rstd = 1.f / sqrtf(var + kBnEps);
    const float scale = gamma[c] * rstd;
    const float shift = beta[c] - mean * scale;
    stats[0 * C + c] = mean;
    stats[1 * C + c] = rstd;
    stats[2 * C + c] = scale;
    stats[3 * C + c] = shift;
    ab[0][c] = fabsf(scale);
    ab[1][c] = fabsf(shift);
  }
  if (ymax == nullptr) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    float y = ysh[0], sa = 0.f, sb = 0.f;
    for (int q = 1; q < 16; ++q) y = fmaxf(y, ysh[q]);
    for (int q = 0; q < C; ++q) {
      sa = fmaxf(sa, ab[0][q]);
      sb = fmaxf(sb, ab[1][q]);
    }
    const int e = srf_split_exp(sa * y + sb);
    stats[4 * C + 0] = srf_exp2i(e);
    stats[4 * C + 1] = srf_exp2i(-e);
  }
}

// ---------------------------------------------------------------- conv2 (split-fp16 MFMA)
// The same implicit GEMM on v_mfma_f32_32x32x16_f16 with fp32-accurate 2-term fp16
// splits of power-of-two scaled operands (as the routing pose, route_fwd32.hip:
// a1 b1 + a1 b2 + a2 b1, dropped a2 b2 <= 2^-22 |ab|): A = 2^b BN1(y1) (one exponent
// from bn_finalize_kernel's bound), B = 2^a_n k (one exponent per output column),
// undone per column in the epilogue; 16/3 of the fp32-MFMA rate.  Workgroup = 2 waves = 64
// output pixels x 128 outputs; a wave owns 32 pixels x all 128 outputs (conv a
// channels 0-31 / 32-63, conv b channels 0-31 / 32-63: the maxout pairs share a
// lane).  Per k-block (one tap, 16 input channels) the A fragments are gathered
// straight into registers (BN1 + mask1 + split on the VALU, one k-block ahead) and
// the B fragments (packed, pre-split weights, shared by both waves) are staged in
// LDS, double-buffered, one k-block ahead.  The epilogue fuses bias, dropout, maxout,
// mask and the BN2 Welford partials.
typedef __bf16 cbf8 __attribute__((ext_vector_type(8)));
typedef float cf16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ cf16 mfma32bf(const cbf8& a, const cbf8& b, const cf16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
typedef _Float16 ch8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ cf16 mfma32h(const ch8& a, const ch8& b, const cf16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void split8v(const float (&v)[8], cbf8& p1, cbf8& p2, cbf8& p3) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const __bf16 a1 = (__bf16)v[k];
    const float r = v[k] - (float)a1;
    const __bf16 a2 = (__bf16)r;
    p1[k] = a1;
    p2[k] = a2;
    p3[k] = (__bf16)(r - (float)a2);
  }
}

// Packed split-fp16 weights wp2[plane][tap][n][cin] (n = ab*C + cout) of 2^a_n k (one
// exponent per output column n, uniform over the GEMM's K = taps x cin), and
// wsc[n] = 2^-a_n for the epilogue.  One wave per n, a lane per cin (9 taps each).
__device__ __forceinline__ void pack_w2_f16_body(int idx, const float* __restrict__ ka, const float* __restrict__ kb,
                                                 _Float16* __restrict__ wp2, float* __restrict__ wsc) {
  const int n = idx >> 6, cin = idx & 63;
  const float* k = n < C ? ka : kb;
  const int co = n % C;
  float v[9], m = 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    v[tap] = k[((size_t)tap * C + cin) * C + co];
    m = fmaxf(m, fabsf(v[tap]));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int e = srf_split_exp(m);
  const float sc = srf_exp2i(e);
  const size_t plane = (size_t)9 * 2 * C * C;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    _Float16 h1, h2;
    srf_split2h(v[tap] * sc, h1, h2);
    const size_t o = ((size_t)tap * 2 * C + n) * C + cin;
    wp2[o] = h1;
    wp2[plane + o] = h2;
  }
  if (cin == 0) wsc[n] = srf_exp2i(-e);
}

constexpr int kC2BStride = 24;   // bf16 per output row of an LDS B k-block (16 + 8: conflict-free b128 reads)
constexpr int kC2Waves = 4;      // 32 pixels each: 128 pixels per workgroup
constexpr int kC2Px = 32 * kC2Waves;
constexpr int kC2BLoads = 2 * 2 * C * 2 / (64 * kC2Waves);   // 16-byte B loads per thread per k-block (2 planes)

__global__ __launch_bounds__(64 * kC2Waves) __attribute__((amdgpu_waves_per_eu(2))) void conv2_fwd32_kernel(
    const float* __restrict__ y1, const float* __restrict__ stats1, const int* __restrict__ inp_len, Dims d,
    const _Float16* __restrict__ wp2, const float* __restrict__ wsc, const float* __restrict__ ba,
    const float* __restrict__ bb, int training, float drop_p, unsigned long long seed,
    const unsigned long long* __restrict__ seed_src, float* __restrict__ y2, unsigned char* __restrict__ sel2,
    float* __restrict__ part) {
  seed = srf_step_seed(seed, seed_src);
  __shared__ __attribute__((aligned(16))) _Float16 Bs[2][2][2 * C * kC2BStride];
  __shared__ __attribute__((aligned(16))) float ss[2][C];
  __shared__ float red[3][kC2Waves][2 * 32];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int P2 = d.B * d.T2 * d.F2;
  const int p0 = blockIdx.x * kC2Px;
  const size_t plane = (size_t)9 * 2 * C * C;
  // BN1 scale / shift times the split exponent 2^b (exact): the A operand is 2^b BN1(y1)
  if (tid < 2 * C) ss[tid >> 6][tid & 63] = stats1[(2 + (tid >> 6)) * C + (tid & 63)] * stats1[4 * C];

  // A row of this lane: pixel p0 + 32 wv + r
  const int pa = p0 + 32 * wv + r;
  const bool alive = pa < P2;
  const int pc = min(pa, P2 - 1);
  const int af2 = pc % d.F2, at2 = (pc / d.F2) % d.T2, ab = pc / (d.F2 * d.T2);
  const int alen1 = ceil_div_len(inp_len[ab], 2);

  // k-block kk = tap * 4 + kb: input channels [16 kb, 16 kb + 16)
  auto load_b = [&](int kk, ch8 (&bv)[kC2BLoads]) {
    const int tap = kk >> 2, kb = kk & 3;
#pragma unroll
    for (int q = 0; q < kC2BLoads; ++q) {
      const int idx = q * 64 * kC2Waves + tid;
      const int pl = idx >> 8, rem = idx & 255, n = rem >> 1, half = rem & 1;
      bv[q] = *reinterpret_cast<const ch8*>(wp2 + pl * plane + ((size_t)tap * 2 * C + n) * C + 16 * kb + 8 * half);
    }
  };
  auto store_b = [&](int buf, const ch8 (&bv)[kC2BLoads]) {
#pragma unroll
    for (int q = 0; q < kC2BLoads; ++q) {
      const int idx = q * 64 * kC2Waves + tid;
      const int pl = idx >> 8, rem = idx & 255, n = rem >> 1, half = rem & 1;
      *reinterpret_cast<ch8*>(&Bs[buf][pl][n * kC2BStride + 8 * half]) = bv[q];
    }
  };
  auto load_a = [&](int kk, f4 (&av)[2], bool& ok) {
    const int tap = kk >> 2, kb = kk & 3;
    const int dt = tap / 3, df = tap - dt * 3;
    const int t1 = 2 * at2 - d.pt2 + dt, f1 = 2 * af2 - d.pf2 + df;
    ok = alive && t1 >= 0 && t1 < d.T1 && f1 >= 0 && f1 < d.F1 && t1 < alen1;
    const int t1c = min(max(t1, 0), d.T1 - 1), f1c = min(max(f1, 0), d.F1 - 1);
    const float* src = y1 + (((size_t)ab * d.T1 + t1c) * d.F1 + f1c) * C + 16 * kb + 8 * h;
    av[0] = *reinterpret_cast<const f4*>(src);
    av[1] = *reinterpret_cast<const f4*>(src + 4);
  };

  cf16 acc[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = cf16{};
  // one k-block: A split from registers, B from LDS buffer buf, 12 MFMAs
  auto compute = [&](int kk, int buf, const f4 (&av)[2], bool aok) {
    ch8 a1, a2;
    {
      const int c0 = 16 * (kk & 3) + 8 * h;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float x = q < 4 ? av[0][q] : av[1][q - 4];
        _Float16 h1, h2;
        srf_split2h(aok ? x * ss[0][c0 + q] + ss[1][c0 + q] : 0.f, h1, h2);
        a1[q] = h1;
        a2[q] = h2;
      }
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int nrow = (nt >> 1) * C + 32 * (nt & 1) + r;   // nt: 0/1 conv a, 2/3 conv b
      const ch8 b1 = *reinterpret_cast<const ch8*>(&Bs[buf][0][nrow * kC2BStride + 8 * h]);
      const ch8 b2 = *reinterpret_cast<const ch8*>(&Bs[buf][1][nrow * kC2BStride + 8 * h]);
      cf16 c = acc[nt];
      c = mfma32h(a2, b1, c);
      c = mfma32h(a1, b2, c);
      c = mfma32h(a1, b1, c);
      acc[nt] = c;
    }
  };
  // software pipeline, two k-blocks ahead: at k-block kk the registers hold the
  // operands of kk + 1 (stored to LDS at the end of kk) and receive those of kk + 2
  ch8 bvA[kC2BLoads], bvB[kC2BLoads];
  f4 avA[2], avB[2], avC[2];
  bool okA, okB, okC;
  load_b(0, bvA);
  load_a(0, avA, okA);
  load_b(1, bvB);
  load_a(1, avB, okB);
  store_b(0, bvA);
  __syncthreads();
  // kk even: A-set = kk, B-set = kk + 1; loads of kk + 2 go to the A registers
  for (int kk = 0; kk < 36; kk += 2) {
    // even step kk
    {
      const f4 a0[2] = {avA[0], avA[1]};
      const bool ok0 = okA;
      if (kk + 2 < 36) {
        load_b(kk + 2, bvA);
        load_a(kk + 2, avA, okA);
      }
      compute(kk, 0, a0, ok0);
      store_b(1, bvB);
      __syncthreads();
    }
    // odd step kk + 1
    {
      const f4 a1v[2] = {avB[0], avB[1]};
      const bool ok1 = okB;
      if (kk + 3 < 36) {
        load_b(kk + 3, bvB);
        load_a(kk + 3, avB, okB);
      }
      compute(kk + 1, 1, a1v, ok1);
      if (kk + 2 < 36) store_b(0, bvA);
      __syncthreads();
    }
  }
  (void)avC;
  (void)okC;

  // epilogue: lane column r = channel (32 g + r), rows = pixels 8q + 4h + v of the wave
  const float keep_scale = 1.f / (1.f - drop_p);
  const float inv_b = stats1[4 * C + 1];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int c = 32 * g + r;
    const float bia = ba[c], bib = bb[c];
    const float sca = wsc[c] * inv_b, scb = wsc[C + c] * inv_b;   // 2^-(a_n + b), exact
    float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int p = p0 + 32 * wv + 8 * q + 4 * h + v;
        if (p >= P2) continue;
        const int t2 = (p / d.F2) % d.T2, b = p / (d.F2 * d.T2);
        const size_t o = (size_t)p * C + c;
        float a = acc[g][4 * q + v] * sca + bia, bvv = acc[2 + g][4 * q + v] * scb + bib;
        if (training && drop_p > 0.f) {
          bool ka, kb;
          srf_keep2(seed, kStreamConv1a, o, drop_p, ka, kb);
          a *= ka ? keep_scale : 0.f;
          bvv *= kb ? keep_scale : 0.f;
        }
        const bool sel = a >= bvv;
        float y = sel ? a : bvv;
        if (t2 >= ceil_div_len(inp_len[b], 4)) y = 0.f;
        y2[o] = y;
        sel2[o] = sel ? 1 : 0;
        n += 1.f;
        const float delta = y - mean;
        mean += delta / n;
        m2 += delta * (y - mean);
      }
    // combine the two lane halves (same channel), then the waves through LDS
    {
      float nb, mb, qb, x;
      xpair32(n, x, nb);
      nb = h ? x : nb;
      xpair32(mean, x, mb);
      mb = h ? x : mb;
      xpair32(m2, x, qb);
      qb = h ? x : qb;
      if (h == 0) chan_merge(n, mean, m2, nb, mb, qb);
    }
    if (h == 0) {
      red[0][wv][g * 32 + r] = n;
      red[1][wv][g * 32 + r] = mean;
      red[2][wv][g * 32 + r] = m2;
    }
  }
  __syncthreads();
  if (tid < 2 * 32) {
    const int gc = tid;   // channel 0..63 (g * 32 + r)
    float n = red[0][0][gc], mean = red[1][0][gc], m2 = red[2][0][gc];
#pragma unroll
    for (int w = 1; w < kC2Waves; ++w) chan_merge(n, mean, m2, red[0][w][gc], red[1][w][gc], red[2][w][gc]);
    part[((size_t)blockIdx.x * 3 + 0) * C + gc] = n;
    part[((size_t)blockIdx.x * 3 + 1) * C + gc] = mean;
    part[((size_t)blockIdx.x * 3 + 2) * C + gc] = m2;
  }
}

// out = mask2(BN2(y2)), the CapsulationLayer output.
__global__ void bn_apply_kernel(const float* __restrict__ y, const float* __restrict__ stats,
                                const int* __restrict__ inp_len, int B, int Tk, int Fk, int div,
                                float* __restrict__ out) {
  const int n4 = B * Tk * Fk * C / 4;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += gridDim.x * blockDim.x) {
    const int c4 = (q * 4) % C;
    const int p = q * 4 / C;
    const int t = (p / Fk) % Tk;
    const int b = p / (Fk * Tk);
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (t < ceil_div_len(inp_len[b], div)) {
      const f4 x = reinterpret_cast<const f4*>(y)[q];
      v = x * *reinterpret_cast<const f4*>(stats + 2 * C + c4) + *reinterpret_cast<const f4*>(stats + 3 * C + c4);
    }
    reinterpret_cast<f4*>(out)[q] = v;
  }
}

// ================================================================ backward
// Gradient of the CapsulationLayer output g_out (of mask2(BN2(y2))).
//
// BN backward (training statistics): with dy = mask * g and xh = (y - mean) * rstd,
//   g_y = mask_pre * gamma * rstd * (dy - sum(dy)/N - xh * sum(dy*xh)/N)
// (mask_pre = the mask applied before BN; it equals the post-BN mask here).

// Per-channel partial sums (sum dy, sum dy*xh) over a stream of positions.  A lane
// owns 4 channels of one pixel (16 lanes per pixel, 16-byte loads, 4 pixels per wave
// per load); a wave takes kBnPx consecutive pixels per sweep, all loads issued first.
constexpr int kBnPx = 16;
__device__ __forceinline__ f4 wave_sum_px(f4 v) {   // sum over the 4 pixel groups of a wave
#pragma unroll
  for (int o = 16; o <= 32; o <<= 1) {
    v.x += __shfl_xor(v.x, o, 64); v.y += __shfl_xor(v.y, o, 64);
    v.z += __shfl_xor(v.z, o, 64); v.w += __shfl_xor(v.w, o, 64);
  }
  return v;
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                            const float* __restrict__ stats,
                                                            const int* __restrict__ inp_len, int B, int Tk, int Fk,
                                                            int div, float* __restrict__ part) {
  __shared__ f4 sh[2][4][C / 4];
  const int lane = threadIdx.x & 63, q = lane & 15, pg = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const f4 mean = reinterpret_cast<const f4*>(stats)[q], rstd = reinterpret_cast<const f4*>(stats + C)[q];
  const int P = B * Tk * Fk;
  f4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  for (int p0 = (blockIdx.x * 4 + wave) * kBnPx; p0 < P; p0 += gridDim.x * 4 * kBnPx) {
    constexpr int U = kBnPx / 4;
    f4 dy[U], yv[U];
    float m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pu = p0 + 4 * u + pg;
      const int p = min(pu, P - 1);
      const int t = (p / Fk) % Tk;
      const int b = p / (Fk * Tk);
      m[u] = (pu < P && t < ceil_div_len(inp_len[b], div)) ? 1.f : 0.f;
      dy[u] = reinterpret_cast<const f4*>(g)[(size_t)p * (C / 4) + q];
      yv[u] = reinterpret_cast<const f4*>(y)[(size_t)p * (C / 4) + q];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4 d = dy[u] * m[u];
      s0 += d;
      s1 += d * (yv[u] - mean) * rstd;
    }
  }
  s0 = wave_sum_px(s0);
  s1 = wave_sum_px(s1);
  if (pg == 0) { sh[0][wave][q] = s0; sh[1][wave][q] = s1; }
  __syncthreads();
  if (threadIdx.x < 2 * (C / 4)) {
    const int k = threadIdx.x / (C / 4), qq = threadIdx.x % (C / 4);
    const f4 v = sh[k][0][qq] + sh[k][1][qq] + sh[k][2][qq] + sh[k][3][qq];
    reinterpret_cast<f4*>(part + ((size_t)blockIdx.x * 2 + k) * C)[qq] = v;
  }
}

__device__ __forceinline__ float bn_bwd_elem(float gin, float y, float mask, float mean, float rstd, float gamma,
                                             float sdy_n, float sdyxh_n) {
  const float dy = mask * gin;
  const float xh = (y - mean) * rstd;
  return mask * gamma * rstd * (dy - sdy_n - xh * sdyxh_n);
}

// BN2 backward + maxout/dropout backward: g_ab[p][n] (n < C: conv a, else conv b);
// bias-gradient partials per block.
__global__ __launch_bounds__(256) void conv2_bwd_prep_kernel(
    const float* __restrict__ g_out, const float* __restrict__ y2, const unsigned char* __restrict__ sel2,
    const float* __restrict__ stats2, const float* __restrict__ gamma2, const float* __restrict__ bnsum2,
    const int* __restrict__ inp_len, Dims d, float drop_p, unsigned long long seed, const unsigned long long* __restrict__ seed_src, float* __restrict__ g_ab,
    float* __restrict__ part, int nprep, const float* __restrict__ pk_a, const float* __restrict__ pk_b,
    __bf16* __restrict__ wq3, _Float16* __restrict__ wq2h, float* __restrict__ wdsc, float* __restrict__ gmax) {
  // blocks past nprep pack the transposed split weights of the data gradient
  // (split-fp16 planes + per-cin exponents when wq2h != nullptr, else split-bf16)
  if ((int)blockIdx.x >= nprep) {
    const int idx = (blockIdx.x - nprep) * blockDim.x + threadIdx.x;
    if (wq2h != nullptr) {
      if (idx < kPackW2tF16Threads) pack_w2t_f16_body(idx, pk_a, pk_b, wq2h, wdsc);
    } else if (idx < kPackW2tThreads) {
      pack_w2t_split_body(idx, pk_a, pk_b, wq3);
    }
    return;
  }
  seed = srf_step_seed(seed, seed_src);
  // as bn_bwd_reduce_kernel: 4 channels of one pixel per lane, kBnPx pixels per wave sweep
  __shared__ f4 sh[2][4][C / 4];
  __shared__ float smax[4];
  const int lane = threadIdx.x & 63, q = lane & 15, pg = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P = d.B * d.T2 * d.F2;
  const f4 mean = reinterpret_cast<const f4*>(stats2)[q], rstd = reinterpret_cast<const f4*>(stats2 + C)[q];
  const f4 gam = {gamma2[4 * q], gamma2[4 * q + 1], gamma2[4 * q + 2], gamma2[4 * q + 3]};   // a parameter view
  const f4 sdy_n = reinterpret_cast<const f4*>(bnsum2)[q] / (float)P;
  const f4 sdyxh_n = reinterpret_cast<const f4*>(bnsum2 + C)[q] / (float)P;
  const float keep_scale = 1.f / (1.f - drop_p);
  f4 ga_s = {0.f, 0.f, 0.f, 0.f}, gb_s = ga_s;
  float gm = 0.f;
  for (int p0 = (blockIdx.x * 4 + wave) * kBnPx; p0 < P; p0 += nprep * 4 * kBnPx) {
    constexpr int U = kBnPx / 4;
    f4 gv[U], yv[U];
    unsigned sv[U];
    float m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pu = p0 + 4 * u + pg;
      const int p = min(pu, P - 1);
      const int t = (p / d.F2) % d.T2;
      const int b = p / (d.F2 * d.T2);
      m[u] = (pu < P && t < ceil_div_len(inp_len[b], 4)) ? 1.f : 0.f;
      gv[u] = reinterpret_cast<const f4*>(g_out)[(size_t)p * (C / 4) + q];
      yv[u] = reinterpret_cast<const f4*>(y2)[(size_t)p * (C / 4) + q];
      sv[u] = reinterpret_cast<const unsigned*>(sel2)[(size_t)p * (C / 4) + q];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int pu = p0 + 4 * u + pg;
      if (pu >= P) continue;
      const size_t o0 = (size_t)pu * C + 4 * q;
      f4 ga, gb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float gy = bn_bwd_elem(gv[u][e], yv[u][e], m[u], mean[e], rstd[e], gam[e], sdy_n[e], sdyxh_n[e]);
        const bool sel = ((sv[u] >> (8 * e)) & 0xffu) != 0;
        float a = sel ? gy : 0.f, bb = sel ? 0.f : gy;
        if (drop_p > 0.f) {
          bool ka, kb;
          srf_keep2(seed, kStreamConv1a, o0 + e, drop_p, ka, kb);
          a *= ka ? keep_scale : 0.f;
          bb *= kb ? keep_scale : 0.f;
        }
        ga[e] = a;
        gb[e] = bb;
        gm = fmaxf(gm, fmaxf(fabsf(a), fabsf(bb)));
      }
      reinterpret_cast<f4*>(g_ab + (size_t)pu * 2 * C)[q] = ga;
      reinterpret_cast<f4*>(g_ab + (size_t)pu * 2 * C + C)[q] = gb;
      ga_s += ga;
      gb_s += gb;
    }
  }
  ga_s = wave_sum_px(ga_s);
  gb_s = wave_sum_px(gb_s);
  if (pg == 0) { sh[0][wave][q] = ga_s; sh[1][wave][q] = gb_s; }
  // block max |g_ab| (the data gradient's split exponent, conv2_dgrad32_kernel)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) gm = fmaxf(gm, __shfl_xor(gm, o, 64));
  if (lane == 0) smax[wave] = gm;
  __syncthreads();
  if (threadIdx.x < 2 * (C / 4)) {
    const int k = threadIdx.x / (C / 4), qq = threadIdx.x % (C / 4);
    const f4 v = sh[k][0][qq] + sh[k][1][qq] + sh[k][2][qq] + sh[k][3][qq];
    reinterpret_cast<f4*>(part + (size_t)blockIdx.x * 2 * C + k * C)[qq] = v;
  }
  if (threadIdx.x == 0 && gmax != nullptr) gmax[blockIdx.x] = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
}

// ---------------------------------------------------------------- dgrad (split-bf16 MFMA)
// The data gradient on v_mfma_f32_32x32x16_bf16 with 3-term splits, structured as
// conv2_fwd32_kernel: all four stride-parity classes in one launch (block ranges
// cls.boff), a workgroup = 4 waves x 32 input pixels of one class, a wave owns its
// 32 pixels x all 64 cin (two N-tiles).  K = taps of the class x 128 (n) in
// k-blocks of 16; the A fragments (g_ab rows, split on the VALU) are gathered into
// registers two k-blocks ahead, the packed pre-split B (wq3[plane][tap][cin][n]) is
// staged in LDS, double-buffered.
struct DgCls {
  int boff[5];   // first block of parity class (qt, qf) = (c >> 1, c & 1); boff[4] = grid
};

// wq3[plane][tap][cin][n] = split(k_{a|b}[tap][cin][n % C]), one thread per 8 n.
__device__ __forceinline__ void pack_w2t_split_body(int idx, const float* __restrict__ ka,
                                                    const float* __restrict__ kb, __bf16* __restrict__ wq3) {
  // idx = (tap, cin, n/8)
  const int n8 = idx % (2 * C / 8), cin = (idx / (2 * C / 8)) % C, tap = idx / (C * (2 * C / 8));
  const int n = 8 * n8;
  const float* k = (n < C ? ka : kb) + ((size_t)tap * C + cin) * C + (n % C);
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = k[q];
  cbf8 p1, p2, p3;
  split8v(v, p1, p2, p3);
  const size_t plane = (size_t)9 * C * 2 * C;
  const size_t o = ((size_t)tap * C + cin) * 2 * C + n;
  *reinterpret_cast<cbf8*>(wq3 + o) = p1;
  *reinterpret_cast<cbf8*>(wq3 + plane + o) = p2;
  *reinterpret_cast<cbf8*>(wq3 + 2 * plane + o) = p3;
}

// wq2h[plane][tap][cin][n] = 2-term fp16 split of 2^e_cin k_{a|b}[tap][cin][n % C] (one
// exponent per data-gradient output column cin, uniform over K = taps x n), and
// wdsc[cin] = 2^-e_cin.  One wave per cin; lane l holds n = 2l, 2l+1 over the 9 taps.
__device__ __forceinline__ void pack_w2t_f16_body(int idx, const float* __restrict__ ka, const float* __restrict__ kb,
                                                  _Float16* __restrict__ wq2h, float* __restrict__ wdsc) {
  const int cin = idx >> 6, l = idx & 63;
  float v[9][2], m = 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int n = 2 * l + u;
      v[tap][u] = (n < C ? ka : kb)[((size_t)tap * C + cin) * C + (n % C)];
      m = fmaxf(m, fabsf(v[tap][u]));
    }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int e = srf_split_exp(m);
  const float sc = srf_exp2i(e);
  const size_t plane = (size_t)9 * C * 2 * C;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    _Float16 h1[2], h2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) srf_split2h(v[tap][u] * sc, h1[u], h2[u]);
    const size_t o = ((size_t)tap * C + cin) * 2 * C + 2 * l;
    wq2h[o] = h1[0];
    wq2h[o + 1] = h1[1];
    wq2h[plane + o] = h2[0];
    wq2h[plane + o + 1] = h2[1];
  }
  if (l == 0) wdsc[cin] = srf_exp2i(-e);
}

constexpr int kD2Waves = 4;
constexpr int kD2Px = 32 * kD2Waves;

// H = true: 2-term fp16 splits of power-of-two scaled operands (A = 2^ea g_ab with ea
// from conv2_bwd_prep's block maxima, reduced by every workgroup; B = 2^e_cin k from
// pack_w2t_f16_body), three f16 MFMAs per k-block tile instead of six bf16 ones;
// the epilogue multiplies column cin by 2^-ea wdsc[cin].
// split exponent of g_ab (max|g_ab| < 2^14 after scaling) from conv2_bwd_prep's block
// maxima; every thread of the block calls it (one barrier)
__device__ __forceinline__ int gab_exp(const float* __restrict__ gmax, int n) {
  __shared__ float wmx[16];
  const int tid = threadIdx.x, nw = (blockDim.x + 63) >> 6;
  float m = 0.f;
  for (int k = tid; k < n; k += blockDim.x) m = fmaxf(m, gmax[k]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((tid & 63) == 0) wmx[tid >> 6] = m;
  __syncthreads();
  for (int k = 0; k < nw; ++k) m = fmaxf(m, wmx[k]);
  return srf_split_exp(m);
}

template <bool H>
__global__ __launch_bounds__(64 * kD2Waves) __attribute__((amdgpu_waves_per_eu(2))) void conv2_dgrad32_kernel(
    const float* __restrict__ g_ab, const void* __restrict__ wqv, Dims d, DgCls cls, float* __restrict__ g_x1,
    const float* __restrict__ gmax, int ngmax, const float* __restrict__ wdsc) {
  using BT = std::conditional_t<H, _Float16, __bf16>;
  using V8 = std::conditional_t<H, ch8, cbf8>;
  constexpr int NPL = H ? 2 : 3;
  constexpr int BCH = NPL * C * 2;   // 16-byte B chunks per k-block (planes x cin x halves)
  const BT* __restrict__ wq3 = static_cast<const BT*>(wqv);
  __shared__ __attribute__((aligned(16))) BT Bs[2][NPL][C * kC2BStride];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int bid = blockIdx.x;
  const int c = (bid >= cls.boff[1]) + (bid >= cls.boff[2]) + (bid >= cls.boff[3]);
  const int qt = c >> 1, qf = c & 1;
  const int nkt = (d.T1 - qt + 1) / 2, nkf = (d.F1 - qf + 1) / 2;
  const int Pc = d.B * nkt * nkf;
  const int q0 = (bid - cls.boff[c]) * kD2Px;
  const int dt0 = (qt + d.pt2) & 1, df0 = (qf + d.pf2) & 1;
  const int ntf = (3 - df0 + 1) / 2, ntt = (3 - dt0 + 1) / 2;
  const int nkb = ntt * ntf * 8;
  const size_t plane = (size_t)9 * C * 2 * C;
  float sa = 1.f, inv_sa = 1.f;
  if constexpr (H) {   // split exponent of g_ab: max over conv2_bwd_prep's block maxima
    const int ea = gab_exp(gmax, ngmax);
    sa = srf_exp2i(ea);
    inv_sa = srf_exp2i(-ea);
  }

  // A row of this lane: class pixel q0 + 32 wv + r
  const int pa = q0 + 32 * wv + r;
  const bool alive = pa < Pc;
  const int pcl = min(pa, Pc - 1);
  const int akf = pcl % nkf, akt = (pcl / nkf) % nkt, ab = pcl / (nkf * nkt);
  const int at1 = qt + 2 * akt, af1 = qf + 2 * akf;
  auto tap_of = [&](int k) { return (dt0 + 2 * (k / ntf)) * 3 + df0 + 2 * (k % ntf); };

  constexpr int NBL = (BCH + 64 * kD2Waves - 1) / (64 * kD2Waves);
  auto load_b = [&](int kk, V8 (&bv)[NBL]) {
    const int tap = tap_of(kk >> 3), kb = kk & 7;
#pragma unroll
    for (int q = 0; q < NBL; ++q) {
      const int idx = min(q * 64 * kD2Waves + tid, BCH - 1);
      const int pl = idx / (2 * C), rem = idx % (2 * C), cin = rem >> 1, half = rem & 1;
      bv[q] = *reinterpret_cast<const V8*>(wq3 + pl * plane + ((size_t)tap * C + cin) * 2 * C + 16 * kb + 8 * half);
    }
  };
  auto store_b = [&](int buf, const V8 (&bv)[NBL]) {
#pragma unroll
    for (int q = 0; q < NBL; ++q) {
      const int idx = q * 64 * kD2Waves + tid;
      if (idx < BCH) {
        const int pl = idx / (2 * C), rem = idx % (2 * C), cin = rem >> 1, half = rem & 1;
        *reinterpret_cast<V8*>(&Bs[buf][pl][cin * kC2BStride + 8 * half]) = bv[q];
      }
    }
  };
  auto load_a = [&](int kk, f4 (&av)[2], bool& ok) {
    const int tap = tap_of(kk >> 3), kb = kk & 7;
    const int dt = tap / 3, df = tap - dt * 3;
    const int t2 = (at1 + d.pt2 - dt) >> 1, f2 = (af1 + d.pf2 - df) >> 1;   // even by the class parity
    ok = alive && t2 >= 0 && t2 < d.T2 && f2 >= 0 && f2 < d.F2;
    const int t2c = min(max(t2, 0), d.T2 - 1), f2c = min(max(f2, 0), d.F2 - 1);
    const float* src = g_ab + (((size_t)ab * d.T2 + t2c) * d.F2 + f2c) * 2 * C + 16 * kb + 8 * h;
    av[0] = *reinterpret_cast<const f4*>(src);
    av[1] = *reinterpret_cast<const f4*>(src + 4);
  };

  cf16 acc[2];
  acc[0] = cf16{};
  acc[1] = cf16{};
  auto compute = [&](int buf, const f4 (&av)[2], bool aok) {
    if constexpr (H) {
      ch8 a1, a2;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = aok ? (q < 4 ? av[0][q] : av[1][q - 4]) : 0.f;
        _Float16 h1, h2;
        srf_split2h(v * sa, h1, h2);
        a1[q] = h1;
        a2[q] = h2;
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int nrow = 32 * nt + r;
        const ch8 b1 = *reinterpret_cast<const ch8*>(&Bs[buf][0][nrow * kC2BStride + 8 * h]);
        const ch8 b2 = *reinterpret_cast<const ch8*>(&Bs[buf][1][nrow * kC2BStride + 8 * h]);
        cf16 cc = acc[nt];
        cc = mfma32h(a2, b1, cc);   // small terms first
        cc = mfma32h(a1, b2, cc);
        cc = mfma32h(a1, b1, cc);
        acc[nt] = cc;
      }
      return;
    } else {
    cbf8 a1, a2, a3;
    {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = aok ? (q < 4 ? av[0][q] : av[1][q - 4]) : 0.f;
      split8v(v, a1, a2, a3);
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int nrow = 32 * nt + r;
      const cbf8 b1 = *reinterpret_cast<const cbf8*>(&Bs[buf][0][nrow * kC2BStride + 8 * h]);
      const cbf8 b2 = *reinterpret_cast<const cbf8*>(&Bs[buf][1][nrow * kC2BStride + 8 * h]);
      const cbf8 b3 = *reinterpret_cast<const cbf8*>(&Bs[buf][2][nrow * kC2BStride + 8 * h]);
      cf16 cc = acc[nt];
      cc = mfma32bf(a3, b1, cc);
      cc = mfma32bf(a1, b3, cc);
      cc = mfma32bf(a2, b2, cc);
      cc = mfma32bf(a2, b1, cc);
      cc = mfma32bf(a1, b2, cc);
      cc = mfma32bf(a1, b1, cc);
      acc[nt] = cc;
    }
    }
  };
  // two k-blocks ahead, as conv2_fwd32_kernel (nkb is a multiple of 8)
  V8 bvA[NBL], bvB[NBL];
  f4 avA[2], avB[2];
  bool okA, okB;
  load_b(0, bvA);
  load_a(0, avA, okA);
  load_b(1, bvB);
  load_a(1, avB, okB);
  store_b(0, bvA);
  __syncthreads();
  for (int kk = 0; kk < nkb; kk += 2) {
    {
      const f4 a0[2] = {avA[0], avA[1]};
      const bool ok0 = okA;
      if (kk + 2 < nkb) {
        load_b(kk + 2, bvA);
        load_a(kk + 2, avA, okA);
      }
      compute(0, a0, ok0);
      store_b(1, bvB);
      __syncthreads();
    }
    {
      const f4 a1v[2] = {avB[0], avB[1]};
      const bool ok1 = okB;
      if (kk + 3 < nkb) {
        load_b(kk + 3, bvB);
        load_a(kk + 3, avB, okB);
      }
      compute(1, a1v, ok1);
      if (kk + 2 < nkb) store_b(0, bvA);
      __syncthreads();
    }
  }
  // epilogue: lane column r = cin (32 nt + r), rows = pixels 8q + 4h + v of the wave
  float osc[2] = {1.f, 1.f};
  if constexpr (H) {
    osc[0] = inv_sa * wdsc[r];
    osc[1] = inv_sa * wdsc[32 + r];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int p = q0 + 32 * wv + 8 * q + 4 * h + v;
      if (p >= Pc) continue;
      const int kf = p % nkf, kt = (p / nkf) % nkt, b = p / (nkf * nkt);
      float* dst = g_x1 + (((size_t)b * d.T1 + qt + 2 * kt) * d.F1 + qf + 2 * kf) * C + r;
      dst[0] = H ? acc[0][4 * q + v] * osc[0] : acc[0][4 * q + v];
      dst[32] = H ? acc[1][4 * q + v] * osc[1] : acc[1][4 * q + v];
    }
}

// Weight gradient of stage 2 for one tap and one pixel split:
// part[s][tap][cin][n] = sum_{p in split} xbn1(p, tap)[cin] * g_ab[p][n].
// K = pixels in chunks of kWgChunk.
constexpr int kWgChunk = 32;

struct WgDiv {
  FastDiv f2, t2;
};

// ---------------------------------------------------------------- wgrad (split-bf16 MFMA)
// g_ab [P2][n] -> pixel-minor split planes gsT3[plane][n][P2p] (zero past P2), the B
// operand image of conv2_wgrad32_kernel: 64 pixels per workgroup through LDS.
constexpr int kTpPx = 64;
// H: two fp16 planes of 2^ea g_ab (ea as conv2_dgrad32_kernel) instead of three bf16
template <bool H>
__global__ __launch_bounds__(256) void gab_split_t_kernel(const float* __restrict__ g_ab, int P2, int P2p,
                                                          void* __restrict__ gsTv, const float* __restrict__ gmax,
                                                          int ngmax) {
  __shared__ float tile[kTpPx][2 * C + 1];
  const int tid = threadIdx.x;
  const int p0 = blockIdx.x * kTpPx;
  float sa = 1.f;
  if constexpr (H) sa = srf_exp2i(gab_exp(gmax, ngmax));
  for (int k = tid; k < kTpPx * (2 * C / 4); k += 256) {
    const int px = k / (2 * C / 4), q = k % (2 * C / 4);
    const int p = p0 + px;
    const f4 v = p < P2 ? *reinterpret_cast<const f4*>(g_ab + (size_t)p * 2 * C + 4 * q) : f4{0.f, 0.f, 0.f, 0.f};
    tile[px][4 * q] = v.x;
    tile[px][4 * q + 1] = v.y;
    tile[px][4 * q + 2] = v.z;
    tile[px][4 * q + 3] = v.w;
  }
  __syncthreads();
  const size_t plane = (size_t)2 * C * P2p;
  for (int task = tid; task < 2 * C * (kTpPx / 8); task += 256) {
    const int o = task & 7, n = task >> 3;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = tile[8 * o + k][n];
    if constexpr (H) {
      ch8 p1, p2;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        _Float16 h1, h2;
        srf_split2h(v[k] * sa, h1, h2);
        p1[k] = h1;
        p2[k] = h2;
      }
      _Float16* dst = static_cast<_Float16*>(gsTv) + (size_t)n * P2p + p0 + 8 * o;
      *reinterpret_cast<ch8*>(dst) = p1;
      *reinterpret_cast<ch8*>(dst + plane) = p2;
    } else {
      cbf8 p1, p2, p3;
      split8v(v, p1, p2, p3);
      __bf16* dst = static_cast<__bf16*>(gsTv) + (size_t)n * P2p + p0 + 8 * o;
      *reinterpret_cast<cbf8*>(dst) = p1;
      *reinterpret_cast<cbf8*>(dst + plane) = p2;
      *reinterpret_cast<cbf8*>(dst + 2 * plane) = p3;
    }
  }
}

// Weight gradient on v_mfma_f32_32x32x16_bf16 with 3-term splits: per (tap, pixel
// split) part[s][tap][cin][n] = sum_p x(p, tap)[cin] g_ab[p][n], M = cin (two
// tiles), N = n (wave w owns n in [32w, 32w+32)), K = pixels in chunks of 32.
// The A image (BN1 + mask1 applied, split) is staged by the workgroup in LDS as
// natural [plane][pixel][cin] rows (one pixel x 8 channels per thread: two float4
// loads, one index decode) and read back transposed into the k = pixel operand with
// ds_read_b64_tr_b16; double-buffered.  Each wave loads its B fragments (8 pixels of
// one n, per plane) straight from gsT3, one chunk ahead.
constexpr int kW2Chunk = 32;
constexpr int kW2AStride = 96;   // bf16 per pixel row of the A image (64 cin + 32: conflict-free tr reads)

typedef short ws4 __attribute__((ext_vector_type(4)));

template <typename BT>
__device__ __forceinline__ ws4 lds_tr16(const BT* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) ws4*)(reinterpret_cast<uintptr_t>(p)));
}

// H = true: split-fp16 operands (A = 2^b BN1(y1) with bn_finalize's exponent, B = the
// 2^ea g_ab planes of gab_split_t_kernel<true>), three f16 MFMAs per tile instead of
// six bf16; the partial sums leave unscaled by 2^-(b + ea).
template <bool H>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void conv2_wgrad32_kernel(
    const float* __restrict__ y1, const float* __restrict__ stats1, const int* __restrict__ inp_len,
    const void* __restrict__ gsTv, int P2p, Dims d, WgDiv dv, int nsplit, int split_len, float* __restrict__ part,
    const float* __restrict__ gmax, int ngmax) {
  using BT = std::conditional_t<H, _Float16, __bf16>;
  using V8 = std::conditional_t<H, ch8, cbf8>;
  constexpr int NPL = H ? 2 : 3;
  const BT* __restrict__ gsT3 = static_cast<const BT*>(gsTv);
  __shared__ __attribute__((aligned(16))) BT As[2][NPL][kW2Chunk * kW2AStride];
  float out_sc = 1.f;
  if constexpr (H) out_sc = stats1[4 * C + 1] * srf_exp2i(-gab_exp(gmax, ngmax));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  // XCD-aware order (nsplit % 8 == 0): the nine taps of one pixel split run back to
  // back on one XCD (blocks b, b + 8, ... share an XCD), so its L2 serves the split's
  // B slab and x rows to all nine
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int tap = loc % 9, sp = xcd + 8 * (loc / 9);
  const int dt = tap / 3, df = tap - dt * 3;
  const int P2 = d.B * d.T2 * d.F2;
  const int pbeg = sp * split_len, pend = min(P2, pbeg + split_len);
  // staging task: pixel px of the chunk, channels 8 oc .. 8 oc + 7
  const int px = tid >> 3, oc = tid & 7;
  float scale[8], shift[8];
  const float bsc = H ? stats1[4 * C] : 1.f;   // 2^b (exact): the H operand is 2^b BN1(y1)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    scale[k] = stats1[2 * C + 8 * oc + k] * bsc;
    shift[k] = stats1[3 * C + 8 * oc + k] * bsc;
  }
  f4 xv[2];
  bool xok = false;
  auto gather = [&](int pc0) {
    const int p = pc0 + px;
    const unsigned pcl = (unsigned)min(p, P2 - 1);
    const unsigned r1 = fdiv(pcl, dv.f2);
    const int f2 = (int)(pcl - r1 * d.F2);
    const unsigned bq = fdiv(r1, dv.t2);
    const int t2 = (int)(r1 - bq * d.T2), b = (int)bq;
    const int t1 = 2 * t2 - d.pt2 + dt, f1 = 2 * f2 - d.pf2 + df;
    xok = p < pend && t1 >= 0 && t1 < d.T1 && f1 >= 0 && f1 < d.F1 && t1 < ceil_div_len(inp_len[b], 2);
    const int t1c = min(max(t1, 0), d.T1 - 1), f1c = min(max(f1, 0), d.F1 - 1);
    const float* src = y1 + (((size_t)b * d.T1 + t1c) * d.F1 + f1c) * C + 8 * oc;
    xv[0] = *reinterpret_cast<const f4*>(src);
    xv[1] = *reinterpret_cast<const f4*>(src + 4);
  };
  auto put = [&](int buf) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = xok ? (k < 4 ? xv[0][k] : xv[1][k - 4]) * scale[k] + shift[k] : 0.f;
    const int o = px * kW2AStride + 8 * oc;
    if constexpr (H) {
      ch8 p1, p2;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        _Float16 h1, h2;
        srf_split2h(v[k], h1, h2);
        p1[k] = h1;
        p2[k] = h2;
      }
      *reinterpret_cast<ch8*>(&As[buf][0][o]) = p1;
      *reinterpret_cast<ch8*>(&As[buf][1][o]) = p2;
    } else {
      cbf8 p1, p2, p3;
      split8v(v, p1, p2, p3);
      *reinterpret_cast<cbf8*>(&As[buf][0][o]) = p1;
      *reinterpret_cast<cbf8*>(&As[buf][1][o]) = p2;
      *reinterpret_cast<cbf8*>(&As[buf][2][o]) = p3;
    }
  };
  // transposed A read: lane 16 g + 4 q + p reads pixel row 8 (g >> 1) + q (+ 4) of the
  // k-block, cin 16 (g & 1) + 4 p .. + 3 of the M-tile; it receives cin 16 (g & 1) + (lane & 15)
  // at pixels 8 (g >> 1) + 0..7 = the 32x32x16 A fragment (row = l & 31, k = 8 (l >> 5) + j)
  const int gg = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int a_off = (8 * (gg >> 1) + qq) * kW2AStride + 16 * (gg & 1) + 4 * pp;
  auto read_a = [&](const BT* img, int kb, int mt) {
    const BT* base = img + a_off + 16 * kb * kW2AStride + 32 * mt;
    const ws4 lo = lds_tr16(base), hi = lds_tr16(base + 4 * kW2AStride);
    return __builtin_bit_cast(V8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  // B fragments of this wave: n = 32 wv + r, pixels 16 kb + 8 h .. + 7 of the chunk
  const size_t bplane = (size_t)2 * C * P2p;
  const BT* brow = gsT3 + (size_t)(32 * wv + r) * P2p + 8 * h;
  V8 bc[2][NPL], bn[2][NPL];
  auto load_bf = [&](int pc0, V8 (&bf)[2][NPL]) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) bf[kb][pl] = *reinterpret_cast<const V8*>(brow + pl * bplane + pc0 + 16 * kb);
  };

  cf16 acc[2];
  acc[0] = cf16{};
  acc[1] = cf16{};
  const int nch = (pend - pbeg + kW2Chunk - 1) / kW2Chunk;
  if (nch > 0) {
    gather(pbeg);
    load_bf(pbeg, bc);
    put(0);
  }
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const bool more = ch + 1 < nch;
    const int buf = ch & 1;
    if (more) {
      gather(pbeg + (ch + 1) * kW2Chunk);
      load_bf(pbeg + (ch + 1) * kW2Chunk, bn);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        if constexpr (H) {
          const ch8 a1 = read_a(As[buf][0], kb, mt);
          const ch8 a2 = read_a(As[buf][1], kb, mt);
          cf16 cc = acc[mt];
          cc = mfma32h(a2, bc[kb][0], cc);   // small terms first
          cc = mfma32h(a1, bc[kb][1], cc);
          cc = mfma32h(a1, bc[kb][0], cc);
          acc[mt] = cc;
        } else {
          const cbf8 a1 = read_a(As[buf][0], kb, mt);
          const cbf8 a2 = read_a(As[buf][1], kb, mt);
          const cbf8 a3 = read_a(As[buf][2], kb, mt);
          cf16 cc = acc[mt];
          cc = mfma32bf(a3, bc[kb][0], cc);
          cc = mfma32bf(a1, bc[kb][2], cc);
          cc = mfma32bf(a2, bc[kb][1], cc);
          cc = mfma32bf(a2, bc[kb][0], cc);
          cc = mfma32bf(a1, bc[kb][1], cc);
          cc = mfma32bf(a1, bc[kb][0], cc);
          acc[mt] = cc;
        }
      }
    if (more) {
      put(buf ^ 1);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) bc[kb][pl] = bn[kb][pl];
    }
    __syncthreads();
  }
  // C layout: col = n (32 wv + r), rows = cin 32 mt + 8 q + 4 h + v
  float* dst = part + ((size_t)sp * 9 + tap) * C * 2 * C + 32 * wv + r;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v) dst[(size_t)(32 * mt + 8 * q + 4 * h + v) * 2 * C] = acc[mt][4 * q + v] * out_sc;
}

// Sum the wgrad splits and unpack n -> (conv a|b, cout): gka/gkb [tap][cin][cout].
__global__ void conv2_wgrad_reduce_kernel(const float* __restrict__ part, int nsplit, float* __restrict__ gka,
                                          float* __restrict__ gkb) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 9 * C * 2 * C) return;
  float s = 0.f;
#pragma unroll 8
  for (int k = 0; k < nsplit; ++k) s += part[(size_t)k * 9 * C * 2 * C + idx];
  const int n = idx % (2 * C);
  const int tc = idx / (2 * C);   // tap*C + cin
  if (n < C)
    gka[(size_t)tc * C + n] = s;
  else
    gkb[(size_t)tc * C + n - C] = s;
}

// BN1 backward + maxout/dropout backward + stage-1 weight/bias gradient partials.
// part[block][j][c], j = 0..8 conv a taps, 9..17 conv b taps, 18 bias a, 19 bias b.
__global__ __launch_bounds__(256) void conv1_bwd_kernel(
    const float* __restrict__ feats, const int* __restrict__ inp_len, Dims d, const float* __restrict__ g_x1,
    const float* __restrict__ y1, const unsigned char* __restrict__ sel1, const float* __restrict__ stats1,
    const float* __restrict__ gamma1, const float* __restrict__ bnsum1, float drop_p, unsigned long long seed, const unsigned long long* __restrict__ seed_src,
    float* __restrict__ part) {
  seed = srf_step_seed(seed, seed_src);
  extern __shared__ __attribute__((aligned(16))) float win[];
  __shared__ float sh[kRows1][20][C];
  const int c = threadIdx.x & (C - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P = d.B * d.T1 * d.F1;
  const float mean = stats1[c], rstd = stats1[C + c], gam = gamma1[c];
  const float sdy_n = bnsum1[c] / (float)P, sdyxh_n = bnsum1[C + c] / (float)P;
  const float keep_scale = 1.f / (1.f - drop_p);
  float acc[20];
#pragma unroll
  for (int j = 0; j < 20; ++j) acc[j] = 0.f;
  const Tile1 tl = stage_rows1(feats, d, win);
  const int t1 = tl.t1_0 + w;
  if (t1 < d.T1) {
    const float mask = t1 < ceil_div_len(inp_len[tl.b], 2) ? 1.f : 0.f;
    const int pbase = (tl.b * d.T1 + t1) * d.F1;
    // columns in batches of 8: the batch's loads are all in flight before the first use
    constexpr int FB = 8;
    for (int f0 = 0; f0 < d.F1; f0 += FB) {
      float gxv[FB], yv[FB];
      unsigned char sv[FB];
#pragma unroll
      for (int u = 0; u < FB; ++u) {
        const int o = (pbase + min(f0 + u, d.F1 - 1)) * C + c;
        gxv[u] = g_x1[o];
        yv[u] = y1[o];
        sv[u] = sel1[o];
      }
#pragma unroll
      for (int u = 0; u < FB; ++u) {
        const int f1 = f0 + u;
        if (f1 >= d.F1) break;
        const int o = (pbase + f1) * C + c;
        const float gy = bn_bwd_elem(gxv[u], yv[u], mask, mean, rstd, gam, sdy_n, sdyxh_n);
        const bool sl = sv[u] != 0;
        float ga = sl ? gy : 0.f, gb = sl ? 0.f : gy;
        if (drop_p > 0.f) {
          bool ka, kb;
          srf_keep2(seed, kStreamConv0a, o, drop_p, ka, kb);
          ga *= ka ? keep_scale : 0.f;
          gb *= kb ? keep_scale : 0.f;
        }
        float x[9];
        window9_lds(win, tl, d, w, f1, x);
        acc[18] += ga;
        acc[19] += gb;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          acc[k] += x[k] * ga;
          acc[9 + k] += x[k] * gb;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 20; ++j) sh[w][j][c] = acc[j];
  __syncthreads();
  for (int j = w; j < 20; j += kRows1) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < kRows1; ++r) v += sh[r][j][c];
    part[((size_t)blockIdx.x * 20 + j) * C + c] = v;
  }
}

// ---------------------------------------------------------------- host
// conv1 workgroups: kRows1 output rows of one utterance each
inline int conv1_blocks(const Dims& d) { return d.B * ((d.T1 + kRows1 - 1) / kRows1); }
inline size_t conv1_lds(const Dims& d) { return (size_t)(2 * kRows1 + 1) * (d.Fin + 2) * sizeof(float); }

struct FwdSaved {
  float *y1, *y2, *stats1, *stats2;
  unsigned char *sel1, *sel2;
  size_t bytes;
};

FwdSaved saved_layout(const Dims& d, void* base) {
  const size_t P1 = (size_t)d.B * d.T1 * d.F1, P2 = (size_t)d.B * d.T2 * d.F2;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += srf::align_up(bytes, 256);
    return o;
  };
  const size_t oy1 = take(P1 * C * 4), oy2 = take(P2 * C * 4), os1 = take(5 * C * 4), os2 = take(5 * C * 4),
               osel1 = take(P1 * C), osel2 = take(P2 * C);
  char* b = static_cast<char*>(base);
  FwdSaved s;
  s.y1 = (float*)(b + oy1);
  s.y2 = (float*)(b + oy2);
  s.stats1 = (float*)(b + os1);
  s.stats2 = (float*)(b + os2);
  s.sel1 = (unsigned char*)(b + osel1);
  s.sel2 = (unsigned char*)(b + osel2);
  s.bytes = off;
  return s;
}

constexpr int kBnMerge = 32;   // first-stage groups of the BN finalize

// Two-stage finalize: kBnMerge groups of partials, then one block over the groups.
int bn_finalize(const float* part, int nparts, float* merged, const float* gamma, const float* beta, float* mmean,
                float* mvar, int training, float* stats, hipStream_t st, const float* ymax = nullptr,
                int nymax = 0) {
  const int per = (nparts + kBnMerge - 1) / kBnMerge;
  hipLaunchKernelGGL(bn_merge_kernel, dim3(kBnMerge), dim3(256), 0, st, part, nparts, per, merged);
  SRF_LAUNCH_CHECK("bn_merge");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(1), dim3(1024), 0, st, merged, kBnMerge, gamma, beta, mmean, mvar,
                     training, stats, ymax, nymax);
  SRF_LAUNCH_CHECK("bn_finalize");
  return SRF_OK;
}

struct FwdWs {
  float *part1, *part2, *wp, *merged;
  _Float16* wp2;   // split-fp16 packed stage-2 weights [2][tap][n][cin]
  float* wsc;      // their per-column exponents 2^-a_n [2C]
  float* ymax;     // conv1 block maxima of |y1|
  size_t bytes;
};

FwdWs fwd_ws_layout(const Dims& d, void* base) {
  const size_t P2 = (size_t)d.B * d.T2 * d.F2;
  const size_t nb2 = (P2 + 63) / 64;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += srf::align_up(bytes, 256);
    return o;
  };
  const size_t op1 = take((size_t)conv1_blocks(d) * 3 * C * 4), op2 = take(nb2 * 3 * C * 4),
               owp = take((size_t)9 * 2 * C * C * 4), omg = take((size_t)kBnMerge * 3 * C * 4),
               owp2 = take((size_t)2 * 9 * 2 * C * C * 2), owsc = take((size_t)2 * C * 4),
               oym = take((size_t)conv1_blocks(d) * 4);
  char* b = static_cast<char*>(base);
  FwdWs w;
  w.wp2 = (_Float16*)(b + owp2);
  w.wsc = (float*)(b + owsc);
  w.ymax = (float*)(b + oym);
  w.merged = (float*)(b + omg);
  w.part1 = (float*)(b + op1);
  w.part2 = (float*)(b + op2);
  w.wp = (float*)(b + owp);
  w.bytes = off;
  return w;
}

int check_dims(int B, int T, int Fin, int nfilt) {
  SRF_REQUIRE(B > 0 && T > 0 && Fin > 0, "bad CNN-FE shape B=%d T=%d F=%d", B, T, Fin);
  SRF_REQUIRE(nfilt == C, "model-conv-filter-num must be %d (got %d)", C, nfilt);
  return SRF_OK;
}

}  // namespace

extern "C" {

int srf_cnnfe_out_dims(int T, int feat_dim, int* T2, int* F2) {
  SRF_REQUIRE(T > 0 && feat_dim > 0 && T2 && F2, "bad arguments");
  Dims d = make_dims(1, T, feat_dim);
  *T2 = d.T2;
  *F2 = d.F2;
  return SRF_OK;
}

size_t srf_cnnfe_saved_bytes(int B, int T, int feat_dim, int nfilt) {
  (void)nfilt;
  return saved_layout(make_dims(B, T, feat_dim), nullptr).bytes;
}

size_t srf_cnnfe_fwd_workspace(int B, int T, int feat_dim, int nfilt) {
  (void)nfilt;
  return fwd_ws_layout(make_dims(B, T, feat_dim), nullptr).bytes;
}

int srf_cnnfe_fwd(const float* feats, const int* inp_len, int B, int T, int feat_dim, int nfilt,
                  const float* k0a, const float* b0a, const float* k0b, const float* b0b, const float* gamma0,
                  const float* beta0, const float* k1a, const float* b1a, const float* k1b, const float* b1b,
                  const float* gamma1, const float* beta1, float* mmean0, float* mvar0, float* mmean1, float* mvar1,
                  int training, float drop_p, unsigned long long seed, float* out, void* saved, size_t saved_bytes,
                  void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_dims(B, T, feat_dim, nfilt);
  if (rc) return rc;
  SRF_REQUIRE(feats && inp_len && k0a && b0a && k0b && b0b && gamma0 && beta0 && k1a && b1a && k1b && b1b &&
                  gamma1 && beta1 && mmean0 && mvar0 && mmean1 && mvar1 && out && saved && workspace,
              "null pointer argument");
  SRF_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "dropout rate %f out of [0,1)", drop_p);
  const Dims d = make_dims(B, T, feat_dim);
  FwdSaved sv = saved_layout(d, saved);
  FwdWs w = fwd_ws_layout(d, workspace);
  if (saved_bytes < sv.bytes || workspace_bytes < w.bytes) {
    srf::set_error("CNN-FE buffers too small (saved %zu < %zu or workspace %zu < %zu)", saved_bytes, sv.bytes,
                   workspace_bytes, w.bytes);
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t P2 = (size_t)d.B * d.T2 * d.F2;
  const int nb2 = (int)((P2 + 63) / 64);
  int nparts2 = nb2;
  const int npack = (kPackW2Threads + 64 * kRows1 - 1) / (64 * kRows1);
  hipLaunchKernelGGL(conv1_fwd_kernel, dim3(conv1_blocks(d) + npack), dim3(64 * kRows1), conv1_lds(d), st, feats,
                     inp_len, d, k0a, b0a, k0b, b0b, training, drop_p, seed, srf::seed_source(), sv.y1, sv.sel1,
                     w.part1, conv1_blocks(d), k1a, k1b, w.wp2, w.wsc, w.ymax);
  SRF_LAUNCH_CHECK("conv1_fwd");
  if ((rc = bn_finalize(w.part1, conv1_blocks(d), w.merged, gamma0, beta0, mmean0, mvar0, training, sv.stats1, st,
                        w.ymax, conv1_blocks(d))))
    return rc;
  SRF_LAUNCH_CHECK("bn_finalize(1)");
  {   // split weights packed by the conv1 launch
    const int nb32 = (int)((P2 + kC2Px - 1) / kC2Px);
    hipLaunchKernelGGL(conv2_fwd32_kernel, dim3(nb32), dim3(64 * kC2Waves), 0, st, sv.y1, sv.stats1, inp_len, d,
                       w.wp2, w.wsc, b1a, b1b, training, drop_p, seed, srf::seed_source(), sv.y2, sv.sel2,
                       w.part2);
    SRF_LAUNCH_CHECK("conv2_fwd32");
    nparts2 = nb32;
  }
  if ((rc = bn_finalize(w.part2, nparts2, w.merged, gamma1, beta1, mmean1, mvar1, training, sv.stats2, st)))
    return rc;
  SRF_LAUNCH_CHECK("bn_finalize(2)");
  hipLaunchKernelGGL(bn_apply_kernel, dim3(1024), dim3(256), 0, st, sv.y2, sv.stats2, inp_len, d.B, d.T2, d.F2, 4,
                     out);
  SRF_LAUNCH_CHECK("bn_apply");
  return SRF_OK;
}

}  // extern "C"

namespace {
struct BwdWs2 {
  float *bnpart, *bnsum2, *bnsum1, *g_ab, *biaspart, *g_x1, *wq, *wpart, *c1part, *c1sum, *scratch;
  __bf16* gsT3;   // split-bf16 g_ab planes, pixel-minor (conv2_wgrad32_kernel)
  float* gmax;    // block maxima of |g_ab| (conv2_bwd_prep_kernel)
  float* wdsc;    // 2^-e_cin of the split-fp16 transposed weights
  int P2p;
  size_t bytes;
};

constexpr int kBnBlocks = 1024;
constexpr int kWgrad32SplitsMax = 128;
// pixel splits of conv2_wgrad32_kernel (a multiple of 8)
constexpr int kWgrad32Splits = 56;

BwdWs2 bwd_ws_layout(const Dims& d, void* base) {
  const size_t P1 = (size_t)d.B * d.T1 * d.F1, P2 = (size_t)d.B * d.T2 * d.F2;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += srf::align_up(bytes, 256);
    return o;
  };
  const size_t obp = take((size_t)kBnBlocks * 2 * C * 4), os2 = take(2 * C * 4), os1 = take(2 * C * 4),
               oab = take(P2 * 2 * C * 4), obias = take((size_t)kBnBlocks * 2 * C * 4), ogx = take(P1 * C * 4),
               owq = take((size_t)9 * 2 * C * C * 4), owp = take((size_t)kWgrad32SplitsMax * 9 * C * 2 * C * 4),
               oc1 = take((size_t)conv1_blocks(d) * 20 * C * 4), oc1s = take(20 * C * 4),
               oscr = take(srf::colsum_scratch_floats(std::max(conv1_blocks(d), kBnBlocks), 20 * C) * 4);
  const int P2p = (int)((P2 + kTpPx - 1) / kTpPx * kTpPx);
  const size_t ogs3 = take((size_t)3 * 2 * C * P2p * 2);
  const size_t ogm = take((size_t)kBnBlocks * 4), ods = take((size_t)C * 4);
  char* b = static_cast<char*>(base);
  BwdWs2 w;
  w.bnpart = (float*)(b + obp);
  w.bnsum2 = (float*)(b + os2);
  w.bnsum1 = (float*)(b + os1);
  w.g_ab = (float*)(b + oab);
  w.biaspart = (float*)(b + obias);
  w.g_x1 = (float*)(b + ogx);
  w.wq = (float*)(b + owq);
  w.wpart = (float*)(b + owp);
  w.c1part = (float*)(b + oc1);
  w.c1sum = (float*)(b + oc1s);
  w.scratch = (float*)(b + oscr);
  w.gsT3 = (__bf16*)(b + ogs3);
  w.gmax = (float*)(b + ogm);
  w.wdsc = (float*)(b + ods);
  w.P2p = P2p;
  w.bytes = off;
  return w;
}

}  // namespace

extern "C" {

size_t srf_cnnfe_bwd_workspace(int B, int T, int feat_dim, int nfilt) {
  (void)nfilt;
  return bwd_ws_layout(make_dims(B, T, feat_dim), nullptr).bytes;
}

int srf_cnnfe_bwd(const float* feats, const int* inp_len, int B, int T, int feat_dim, int nfilt, const float* gamma0,
                  const float* k1a, const float* k1b, const float* gamma1, float drop_p, unsigned long long seed,
                  const void* saved, const float* g_out, float* g_k0a, float* g_b0a, float* g_k0b, float* g_b0b,
                  float* g_gamma0, float* g_beta0, float* g_k1a, float* g_b1a, float* g_k1b, float* g_b1b,
                  float* g_gamma1, float* g_beta1, void* workspace, size_t workspace_bytes, void* stream) {
  return srf_cnnfe_bwd_parts(SRF_CNNFE_BWD_ALL, feats, inp_len, B, T, feat_dim, nfilt, gamma0, k1a, k1b, gamma1, drop_p,
                             seed, saved, g_out, g_k0a, g_b0a, g_k0b, g_b0b, g_gamma0, g_beta0, g_k1a, g_b1a, g_k1b,
                             g_b1b, g_gamma1, g_beta1, workspace, workspace_bytes, stream);
}

int srf_cnnfe_bwd_parts(int parts, const float* feats, const int* inp_len, int B, int T, int feat_dim, int nfilt,
                        const float* gamma0, const float* k1a, const float* k1b, const float* gamma1, float drop_p,
                        unsigned long long seed, const void* saved, const float* g_out, float* g_k0a, float* g_b0a,
                        float* g_k0b, float* g_b0b, float* g_gamma0, float* g_beta0, float* g_k1a, float* g_b1a,
                        float* g_k1b, float* g_b1b, float* g_gamma1, float* g_beta1, void* workspace,
                        size_t workspace_bytes, void* stream) {
  SRF_REQUIRE(parts > 0 && (parts & ~SRF_CNNFE_BWD_ALL) == 0, "CNN-FE backward: bad parts mask %d", parts);
  int rc = check_dims(B, T, feat_dim, nfilt);
  if (rc) return rc;
  SRF_REQUIRE(feats && inp_len && gamma0 && k1a && k1b && gamma1 && saved && g_out && g_k0a && g_b0a && g_k0b &&
                  g_b0b && g_gamma0 && g_beta0 && g_k1a && g_b1a && g_k1b && g_b1b && g_gamma1 && g_beta1 &&
                  workspace,
              "null pointer argument");
  SRF_REQUIRE(((uintptr_t)g_out & 15) == 0 && ((uintptr_t)saved & 255) == 0 && ((uintptr_t)workspace & 255) == 0,
              "CNN-FE backward: g_out must be 16-byte and saved / workspace 256-byte aligned");
  const Dims d = make_dims(B, T, feat_dim);
  FwdSaved sv = saved_layout(d, const_cast<void*>(saved));
  BwdWs2 w = bwd_ws_layout(d, workspace);
  if (workspace_bytes < w.bytes) {
    srf::set_error("CNN-FE backward workspace too small: %zu < %zu", workspace_bytes, w.bytes);
    return SRF_EWORKSPACE;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int P2 = d.B * d.T2 * d.F2;
  __bf16* wq3 = reinterpret_cast<__bf16*>(w.wq);
  _Float16* wq2h = reinterpret_cast<_Float16*>(w.wq);
  if (parts & SRF_CNNFE_BWD_PREP) {
  // BN2: sums -> d(beta2) = sum dy, d(gamma2) = sum dy*xh
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(kBnBlocks), dim3(256), 0, st, g_out, sv.y2, sv.stats2, inp_len, d.B,
                     d.T2, d.F2, 4, w.bnpart);
  SRF_LAUNCH_CHECK("bn_bwd_reduce(2)");
  if ((rc = srf::colsum(w.bnpart, kBnBlocks, 2 * C, w.bnsum2, w.scratch, st, srf::ColSplit{{g_beta1, g_gamma1, nullptr, nullptr}, {C, C, 0, 0}})))
    return rc;
  const int npack = (kPackW2tF16Threads + 255) / 256;
  hipLaunchKernelGGL(conv2_bwd_prep_kernel, dim3(kBnBlocks + npack), dim3(256), 0, st, g_out, sv.y2, sv.sel2,
                     sv.stats2, gamma1, w.bnsum2, inp_len, d, drop_p, seed, srf::seed_source(), w.g_ab, w.biaspart,
                     kBnBlocks, k1a, k1b, wq3, wq2h, w.wdsc, w.gmax);
  SRF_LAUNCH_CHECK("conv2_bwd_prep");
  if ((rc = srf::colsum(w.biaspart, kBnBlocks, 2 * C, nullptr, w.scratch, st, srf::ColSplit{{g_b1a, g_b1b, nullptr, nullptr}, {C, C, 0, 0}})))
    return rc;
  }
  // stage-2 data gradient (4 stride-parity classes, split transposed weights packed by
  // the bwd_prep launch) and weight gradient, both on split-fp16 operands
  if (parts & SRF_CNNFE_BWD_DATA) {
    DgCls cls{};
    for (int c = 0; c < 4; ++c) {
      const int qt = c >> 1, qf = c & 1;
      const int Pc = d.B * ((d.T1 - qt + 1) / 2) * ((d.F1 - qf + 1) / 2);
      cls.boff[c + 1] = cls.boff[c] + (Pc + kD2Px - 1) / kD2Px;
    }
    hipLaunchKernelGGL(conv2_dgrad32_kernel<true>, dim3(cls.boff[4]), dim3(64 * kD2Waves), 0, st, w.g_ab,
                       (const void*)wq2h, d, cls, w.g_x1, (const float*)w.gmax, kBnBlocks, (const float*)w.wdsc);
    SRF_LAUNCH_CHECK("conv2_dgrad32");
  }
  const WgDiv dv{make_fastdiv(d.F2), make_fastdiv(d.T2)};
  const int nsplit = kWgrad32Splits;
  if (parts & SRF_CNNFE_BWD_WGRAD) {
    static_assert(kW2Chunk == kWgChunk, "wgrad splits are whole chunks");
    const int split_len = ((P2 + nsplit - 1) / nsplit + kWgChunk - 1) / kWgChunk * kWgChunk;
    hipLaunchKernelGGL(gab_split_t_kernel<true>, dim3(w.P2p / kTpPx), dim3(256), 0, st, w.g_ab, P2, w.P2p,
                       (void*)w.gsT3, (const float*)w.gmax, kBnBlocks);
    SRF_LAUNCH_CHECK("gab_split_t");
    hipLaunchKernelGGL(conv2_wgrad32_kernel<true>, dim3(9 * nsplit), dim3(256), 0, st, sv.y1, sv.stats1, inp_len,
                       (const void*)w.gsT3, w.P2p, d, dv, nsplit, split_len, w.wpart, (const float*)w.gmax,
                       kBnBlocks);
    SRF_LAUNCH_CHECK("conv2_wgrad32");
    hipLaunchKernelGGL(conv2_wgrad_reduce_kernel, dim3((9 * C * 2 * C + 255) / 256), dim3(256), 0, st, w.wpart,
                       nsplit, g_k1a, g_k1b);
    SRF_LAUNCH_CHECK("conv2_wgrad_reduce");
  }
  if (!(parts & SRF_CNNFE_BWD_DATA)) return SRF_OK;
  // BN1 backward sums, then stage-1 gradients
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(kBnBlocks), dim3(256), 0, st, w.g_x1, sv.y1, sv.stats1, inp_len, d.B,
                     d.T1, d.F1, 2, w.bnpart);
  SRF_LAUNCH_CHECK("bn_bwd_reduce(1)");
  if ((rc = srf::colsum(w.bnpart, kBnBlocks, 2 * C, w.bnsum1, w.scratch, st, srf::ColSplit{{g_beta0, g_gamma0, nullptr, nullptr}, {C, C, 0, 0}})))
    return rc;
  hipLaunchKernelGGL(conv1_bwd_kernel, dim3(conv1_blocks(d)), dim3(64 * kRows1), conv1_lds(d), st, feats, inp_len, d, w.g_x1, sv.y1,
                     sv.sel1, sv.stats1, gamma0, w.bnsum1, drop_p, seed, srf::seed_source(), w.c1part);
  SRF_LAUNCH_CHECK("conv1_bwd");
  // columns j*C + c: conv a taps, conv b taps, bias a, bias b -> straight into the gradients
  if ((rc = srf::colsum(w.c1part, conv1_blocks(d), 20 * C, nullptr, w.scratch, st,
                        srf::ColSplit{{g_k0a, g_k0b, g_b0a, g_b0b, nullptr, nullptr}, {9 * C, 9 * C, C, C, 0, 0}})))
    return rc;
  return SRF_OK;
}

}  // extern "C"
