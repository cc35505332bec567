// DR routing forward pass on 32x32 tiles with fp32-accurate split-fp16 MFMA, gfx950.
//
// Replaces, like route_dr.hip's route_pass_kernel, the forward routing iteration of
// sequence_router_naive.py:171-185 / _loop_body :199-206 (pose :154-159 recomputed
// per pass, window :150-151).  This variant is the forward pass for din in {8, 16, 32}
// and dout in {8, 16, 32} (din <= dout) with J*dout <= 1024 (BASELINE C1, C2 and the
// C3/C4 DR layers); other shapes keep route_pass_kernel.
//
// Pose product.  u = W x + b is formed on v_mfma_f32_32x32x16_f16 from 2-term fp16
// splits of power-of-two scaled operands: W' = 2^aw W and x' = 2^bx x with
// max|W'|, max|x'| < 2^14 (absmax_kernel + prep32_kernel, one global exponent per
// operand and forward), a' = a1 + a2 (a1 = f16(a'), a2 = f16(a' - a1)), keeping
//     W'x' ~ W1x1 + W1x2 + W2x1                          (dropped W2x2 <= 2^-22 |W'x'|)
// and the bias 2^(aw+bx) b through one bf16 MFMA (3-term bf16 split, exact to 2^-24)
// against a ones column, all in one fp32 accumulator.  f16 x f16 products are exact
// in fp32, so u' = 2^(aw+bx) u carries ~2^-22 relative error per product, the level
// of an fp32 FMA chain over din terms (tests/test_route_dr_gpu.py holds it to the same
// tolerances); consumers multiply by the exact inverse scale 2^-(aw+bx) (logits,
// final partial sums).  Four MFMAs per tile and 4 bytes of W per element (the
// split-bf16 3-term form of round 2 needed seven and 6 bytes).
//
// Tiles.  A workgroup owns 32 frames x all J*dout rows (32-row tiles, TW per wave)
// and an i-chunk of input capsules.  Lane l holds frame (l & 31) and, per tile,
// the 16 rows 8q + 4h + (0..3) (q = 0..3, h = l >> 5) of the MFMA's C/D map.  A
// lane therefore holds a whole 4- or 8-row piece of each output capsule, so the
// agreement logit of a capsule needs ONE cross-half exchange: v_permlane32_swap
// reduce-scatters two capsules' partial dots at once and leaves each lane half
// the logit of one of them.  Softmax over j: per-lane stats -> lane-half combine
// -> per-wave stats through LDS (one barrier per input capsule).  Vc (the
// agreement vector, naive:205 by linearity) lives in each wave's private LDS slab
// in fragment order (conflict-free ds_read_b128).
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <type_traits>

#include "srf_common.h"
#include "route_fwd32.h"

// Timing builds of the pipelined passes (wrong results, never shipped; scripts/build_ab.sh
// + scripts/gpu_ab_route.sh): bit 1 = x of the chunk's first capsule, 2 = its W and bias,
// 4 = no per-capsule barrier, 8 = no x reloads, 16 = no W reloads.
// Schedule choices of the passes, fixed by measurement (rounds 2-4): the next capsule's
// operands load between the MFMA steps of this capsule, each register group as soon as
// its last reader has issued (pose_prog; issuing them all after the MFMAs measured ~4 %
// slower in the graphed step); din 8 / 16 run the pose tile-major with the agreement dots
// of tile t - 1 beside tile t's MFMAs (din 32: pose_prog measured faster); the second
// half of a din <= 16 workgroup's waves runs at s_setprio 1 (~3 % on the backward pass).

// SRF_DR_IL (A/B builds only): 1 = the din-32 pipelined passes run the previous capsule's
// finish between the pose MFMAs (pose_prog32i); 0 = after them (pose_prog).
#ifndef SRF_DR_IL
#define SRF_DR_IL 1
#endif

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32(const bf8& a, const bf8& b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16v mfma32h(const h8& a, const h8& b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float exp2i(int e) { return srf_exp2i(e); }
__device__ __forceinline__ int split_exp(float m) { return srf_split_exp(m); }

// ------------------------------------------------------------------ splits
// a -> (a1, a2, a3), each round-to-nearest bf16 (the bias operand).
__device__ __forceinline__ void split3(float a, __bf16& a1, __bf16& a2, __bf16& a3) {
  a1 = (__bf16)a;
  const float r = a - (float)a1;
  a2 = (__bf16)r;
  a3 = (__bf16)(r - (float)a2);
}

__device__ __forceinline__ void split2h(float a, _Float16& a1, _Float16& a2) { srf_split2h(a, a1, a2); }

// 8 consecutive floats, scaled by s -> their two fp16 planes (16 bytes each)
__device__ __forceinline__ void split8h(const float* __restrict__ src, bool ok, float s, _Float16* d1,
                                        _Float16* d2) {
  f4 lo = {0.f, 0.f, 0.f, 0.f}, hi = lo;
  if (ok) {
    lo = *reinterpret_cast<const f4*>(src);
    hi = *reinterpret_cast<const f4*>(src + 4);
  }
  const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  h8 p1, p2;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    _Float16 a1, a2;
    split2h(v[k] * s, a1, a2);
    p1[k] = a1;
    p2[k] = a2;
  }
  *reinterpret_cast<h8*>(d1) = p1;
  *reinterpret_cast<h8*>(d2) = p2;
}

// Block maxima of |W| (blockIdx.y = 0) and |emb| (blockIdx.y = 1) -> part[y][blockIdx.x]
// (kAbsBlocks per operand); prep32_kernel reduces them to the split exponents.
constexpr int kAbsBlocks = 128;
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ a, size_t na,
                                                     const float* __restrict__ b, size_t nb, float* part) {
  const float* p = blockIdx.y ? b : a;
  const size_t n = blockIdx.y ? nb : na;
  float m = 0.f;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    const size_t n4 = n / 4;
    for (; i < n4; i += stride) {
      const f4 v = reinterpret_cast<const f4*>(p)[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    i = n4 * 4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  }
  for (; i < n; i += stride) m = fmaxf(m, fabsf(p[i]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.y * kAbsBlocks + blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// One launch prepares every operand of a forward (thread ranges in this order):
//   W [in_n][JD][din]   -> Ws [2][in_n][JDp][din] fp16 planes of 2^aw W (rows past JD = 0), 8 per thread;
//   bias [in_n][JD]     -> bs [in_n][JDp][4] = bf16 (b1, b2, b3, 0) of 2^(aw+bx) bias;
//   bsum[c][row]        =  sum of bias[i][row] over the capsules of i-chunk c (iteration-0 pass);
//   emb [F][N][din]     -> xs [2][plane] fp16 of 2^bx x, plane = [N][F][din] capsule-major + 16 zeros;
//   block 0 also writes the header hdr = {2^-(aw+bx), aw, bx} read by every pass.
//   (training forwards also write the fp32 operands of the backward passes:)
//   W                   -> WT [in_n][JD/16][4][din][4] (A of the gx contraction in fragment order:
//                          row quad g of 16-row tile t, input element e, rows 16t+4g..+3), 4 per thread;
//   window(emb)         -> xT [in_n][din][Fp] (A of the gW contraction, zero past F / the utterance).
struct PrepArgs {
  const float *W, *bias, *emb;
  _Float16 *Ws, *xs;
  __bf16* bs;
  float *bsum, *WT, *xT;
  const float* part;   // absmax_kernel block maxima
  float* hdr;
  int in_n, JD, JDp, din, n_chunks, chunk_len, F, N, T, lpad, Fp;
  int wt16;            // WT holds route_gux16_kernel's split-fp16 A planes instead of fp32
  int xt16;            // xT holds route_gw16s_kernel's blocked split-fp16 B planes instead of fp32
  size_t xplane;
  size_t n_a, n_b, n_c, n_d, n_e;   // thread counts of the first five ranges
  size_t n_f, xt_block0;             // xT: 64-frame tiles, one block each from block xt_block0 on
};

constexpr int kXtTile = 64;   // frames per xT tile of prep32_kernel

__global__ __launch_bounds__(256) void prep32_kernel(PrepArgs P) {
  if (P.n_f && blockIdx.x >= P.xt_block0) {
    // xT[i][e][f] (capsule i = w*N + n of frame f is emb[f + w - lpad][n] inside the
    // utterance, 0 past F): the tile's 64 window rows are read along e (coalesced),
    // transposed through LDS and written as din runs of 64 consecutive frames.
    // xt16 (din 32, route_gw16s_kernel): instead fp16 hi / lo planes of 2^bx x in
    // 16-frame blocks, xT16[i][f / 16][hi | lo][e][16 frames] (1 KiB per plane and
    // block: the B operand of one K step, read as 16 bytes per lane)
    __shared__ float tile[kXtTile][32 + 1];
    __shared__ int sbx;
    const int ntile = (P.Fp + kXtTile - 1) / kXtTile;
    const int blk = blockIdx.x - (int)P.xt_block0;
    const int i = blk / ntile, f0 = (blk - i * ntile) * kXtTile;
    const int w = i / P.N, n = i - w * P.N;
    if (P.xt16 && threadIdx.x < 64) {
      float m = 0.f;
      for (int k = threadIdx.x; k < kAbsBlocks; k += 64) m = fmaxf(m, P.part[kAbsBlocks + k]);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      if (threadIdx.x == 0) sbx = split_exp(m);
    }
    for (int k = threadIdx.x; k < kXtTile * P.din; k += blockDim.x) {
      const int fl = k / P.din, e = k - fl * P.din;
      const int f = f0 + fl;
      float v = 0.f;
      if (f < P.F) {
        const int b = f / P.T, t = f - b * P.T;
        const int ts = t + w - P.lpad;
        if (ts >= 0 && ts < P.T) v = P.emb[((size_t)(b * P.T + ts) * P.N + n) * P.din + e];
      }
      tile[fl][e] = v;
    }
    __syncthreads();
    if (P.xt16) {
      // item = (16-frame block kb of the tile, e, 8-frame half hf): 8 frames -> 16 bytes per plane
      const float sc = exp2i(sbx);
      _Float16* x16 = reinterpret_cast<_Float16*>(P.xT);
      for (int k = threadIdx.x; k < (kXtTile / 16) * 32 * 2; k += blockDim.x) {
        const int hf = k & 1, e = (k >> 1) & 31, kb = k >> 6;
        const int fb = f0 + kb * 16;
        if (fb >= P.Fp) continue;
        h8 p1, p2;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          _Float16 a1, a2;
          split2h(tile[kb * 16 + hf * 8 + q][e] * sc, a1, a2);
          p1[q] = a1;
          p2[q] = a2;
        }
        const size_t base = (((size_t)i * (P.Fp / 16) + fb / 16) * 2 * 32 + e) * 16 + hf * 8;
        *reinterpret_cast<h8*>(x16 + base) = p1;
        *reinterpret_cast<h8*>(x16 + base + 32 * 16) = p2;
      }
      return;
    }
    for (int k = threadIdx.x; k < kXtTile * P.din; k += blockDim.x) {
      const int e = k / kXtTile, fl = k - e * kXtTile;
      const int f = f0 + fl;
      if (f < P.Fp) P.xT[((size_t)i * P.din + e) * P.Fp + f] = tile[fl][e];
    }
    return;
  }
  // split exponents from the block maxima (every block with split work reduces the
  // same 2 x kAbsBlocks values; the block-uniform test keeps the barrier uniform)
  __shared__ int sexp[2];
  const size_t b0 = (size_t)blockIdx.x * blockDim.x, b1 = b0 + blockDim.x;
  const size_t ec = P.n_a + P.n_b, sd = ec + P.n_c, ed = sd + P.n_d;
  const bool split_work = b0 < ec || (b1 > sd && b0 < ed) || (P.wt16 && b1 > ed && b0 < ed + P.n_e);
  if (split_work && threadIdx.x < 128) {
    const int y = threadIdx.x >> 6, l = threadIdx.x & 63;
    float m = 0.f;
    for (int k = l; k < kAbsBlocks; k += 64) m = fmaxf(m, P.part[y * kAbsBlocks + k]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (l == 0) sexp[y] = split_exp(m);
  }
  if (split_work) __syncthreads();
  const int aw = split_work ? sexp[0] : 0, bx = split_work ? sexp[1] : 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    P.hdr[0] = exp2i(-(aw + bx));
    P.hdr[1] = (float)aw;
    P.hdr[2] = (float)bx;
  }
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < P.n_a) {
    const size_t e0 = idx * 8;
    const int e = e0 % P.din;
    const size_t rr = e0 / P.din;
    const int row = rr % P.JDp;
    const size_t i = rr / P.JDp;
    const size_t nw = (size_t)P.in_n * P.JDp * P.din;
    split8h(P.W + (i * P.JD + min(row, P.JD - 1)) * P.din + e, row < P.JD, exp2i(aw), P.Ws + e0, P.Ws + nw + e0);
    return;
  }
  idx -= P.n_a;
  if (idx < P.n_b) {
    const int row = idx % P.JDp;
    const size_t i = idx / P.JDp;
    const float b = row < P.JD ? P.bias[i * P.JD + row] * exp2i(aw + bx) : 0.f;
    __bf16 b1, b2, b3;
    split3(b, b1, b2, b3);
    bf4 v = {b1, b2, b3, (__bf16)0.f};
    *reinterpret_cast<bf4*>(P.bs + idx * 4) = v;
    return;
  }
  idx -= P.n_b;
  if (idx < P.n_c) {
    const int c = idx / P.JD, row = idx - (size_t)c * P.JD;
    const int i0 = c * P.chunk_len, i1 = min(P.in_n, i0 + P.chunk_len);
    float acc = 0.f;
    // loads in batches of 8 (one round trip each), summed in capsule order
    for (int i = i0; i < i1; i += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = i + k < i1 ? P.bias[(size_t)(i + k) * P.JD + row] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
    P.bsum[idx] = acc;
    return;
  }
  idx -= P.n_c;
  if (idx < P.n_d) {
    const size_t e0 = idx * 8;
    const size_t n_data = (size_t)P.F * P.N * P.din;
    const int e = e0 % P.din;
    const size_t rr = e0 / P.din;
    const int f = rr % P.F;
    const int n = rr / P.F;
    const bool ok = e0 < n_data;
    split8h(P.emb + ((size_t)(ok ? f : 0) * P.N + (ok ? n : 0)) * P.din + (ok ? e : 0), ok, exp2i(bx), P.xs + e0,
            P.xs + P.xplane + e0);
    return;
  }
  idx -= P.n_d;
  if (P.wt16 && idx < P.n_e) {
    // split-fp16 A planes of route_gux16_kernel (din 32): [i][t][h][e][8] hi, then lo,
    // = 2^aw W[i][16t + 8h + 0..7][e] (0 past JD); one 16-byte run per plane
    const int e = idx % P.din;
    const size_t r1 = idx / P.din;
    const int h = r1 % 2;
    const size_t r2 = r1 / 2;
    const int nt16 = (P.JD + 15) / 16;
    const int t = r2 % nt16;
    const size_t i = r2 / nt16;
    const int row = t * 16 + 8 * h;
    const float* w = P.W + (i * P.JD + min(row, P.JD - 1)) * P.din + e;
    const float s = exp2i(aw);
    h8 p1, p2;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      _Float16 a1, a2;
      split2h(row + k < P.JD ? w[(size_t)k * P.din] * s : 0.f, a1, a2);
      p1[k] = a1;
      p2[k] = a2;
    }
    _Float16* d = reinterpret_cast<_Float16*>(P.WT);
    *reinterpret_cast<h8*>(d + idx * 8) = p1;
    *reinterpret_cast<h8*>(d + P.n_e * 8 + idx * 8) = p2;
    return;
  }
  if (idx < P.n_e) {   // WT[i][t][g][e][0..3] = W[i][16t + 4g + 0..3][e] (0 past JD)
    const int e = idx % P.din;
    const size_t r1 = idx / P.din;
    const int g = r1 % 4;
    const size_t r2 = r1 / 4;
    const int nt16 = (P.JD + 15) / 16;
    const int t = r2 % nt16;
    const size_t i = r2 / nt16;
    const int row = t * 16 + 4 * g;
    const float* w = P.W + (i * P.JD + min(row, P.JD - 1)) * P.din + e;
    f4 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = row + q < P.JD ? w[(size_t)q * P.din] : 0.f;
    *reinterpret_cast<f4*>(P.WT + idx * 4) = v;
    return;
  }

}

// ------------------------------------------------------------------ fragments
// Per input capsule: A fragments (W splits) per tile, the bias fragment per tile,
// B fragments (x splits) shared by the tiles.
//   DIN 16: one MFMA covers din; A_p = W plane p (k = 8h + j), B_q = x plane q:
//           W2x1, W1x2, W1x1.
//   DIN  8: K = 16 packs two planes: A = [W1 | W2], B1 = [x1 | x1], B2 = [x2 | 0]
//           (lane half h holds k = 8h..8h+7): A B2 = W1x2, A B1 = W1x1 + W2x1.
// Bias: A = bf16 (b1, b2, b3, 0, 0, 0, 0, 0) of the row, B = ones at k = 0..2 of
// lane half 0 and zero elsewhere, so only (b1 + b2 + b3) reaches the accumulator.
// All operands come through buffer loads: one descriptor per array, the per-lane
// byte offset in voffset (fixed per tile), the per-capsule / per-plane offset in
// soffset.  Invalid window frames read the zero row at the end of each x plane.
constexpr int kTW = srf::kFwd32TW;       // 32-row tiles per wave (din 8, 16; din 32: Fwd32Plan::TW)
constexpr int kMaxNW = 32 / kTW;         // J*dout <= 1024
constexpr int kWavesPerEU = 8 / kTW;

template <int DIN>
struct SplitFrags {
  static constexpr int NA = DIN / 8;              // A fragments per tile (W planes x k-halves)
  static constexpr int NB = DIN == 32 ? 4 : 2;    // B fragments per frame tile
};

template <int DIN, int TW>
struct Frags32 {
  h8 a[TW][SplitFrags<DIN>::NA];
  bf8 bias[TW];
  h8 b[SplitFrags<DIN>::NB];
};

struct Rsrc3 {
  __amdgpu_buffer_rsrc_t w, b, x;
};

__device__ __forceinline__ h8 hload(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// raw buffer store of one float; a voffset past the buffer drops it (no branch, so the
// compiler's vmcnt bookkeeping stays exact)
constexpr uint32_t kNoStore = 0x80000000u;
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t rs, float v, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, voff, soff, 0);
}

// Window source of capsule i = w*N + n for this lane (naive:150-151): frame
// t + w - lpad of the same utterance, i.e. row f + w - lpad of capsule n's plane,
// or the zero row when it falls outside [0, T).
template <int DIN>
__device__ __forceinline__ uint32_t x_voff(int i, int N, int lpad, int T, int F, int f, int ft, bool fvalid, int h,
                                           uint32_t zero_off) {
  const int w = i / N, n = i - w * N;
  const int ts = ft + w - lpad;
  const bool ok = fvalid && ts >= 0 && ts < T;
  const uint32_t o = (uint32_t)(((n * F + f + w - lpad) * DIN) * 2 + (DIN >= 16 ? 16 * h : 0));
  return ok ? o : zero_off;
}

// the x fragments of one capsule (DIN 8: [x1 | x1] and [x2 | 0]; DIN 32: x1, x2 of
// k-half 0, then of k-half 1 at +32 bytes; the zero row is 32 halves long for DIN 32)
template <int DIN>
__device__ __forceinline__ void fetch_x(const Rsrc3& rs, uint32_t xvo, int h, uint32_t xplane_b, uint32_t zero_off,
                                        h8 (&b)[SplitFrags<DIN>::NB]) {
  if constexpr (DIN == 32) {
    b[0] = hload(rs.x, xvo, 0);
    b[1] = hload(rs.x, xvo, xplane_b);
    b[2] = hload(rs.x, xvo, 32);
    b[3] = hload(rs.x, xvo, xplane_b + 32);
  } else if constexpr (DIN == 16) {
    b[0] = hload(rs.x, xvo, 0);
    b[1] = hload(rs.x, xvo, xplane_b);
  } else {
    b[0] = hload(rs.x, xvo, 0);
    b[1] = hload(rs.x, h ? zero_off : xvo, h ? 0u : xplane_b);
  }
}

template <int DIN>
__device__ __forceinline__ void fetch_w(const Rsrc3& rs, uint32_t vo, int h, uint32_t wplane_b, uint32_t wcap_b,
                                        h8 (&a)[SplitFrags<DIN>::NA]) {
  if constexpr (DIN == 32) {   // (W1, W2) of k-half 0, then of k-half 1 (+32 bytes)
    a[0] = hload(rs.w, vo, wcap_b);
    a[1] = hload(rs.w, vo, wcap_b + wplane_b);
    a[2] = hload(rs.w, vo, wcap_b + 32);
    a[3] = hload(rs.w, vo, wcap_b + wplane_b + 32);
  } else if constexpr (DIN == 16) {
    a[0] = hload(rs.w, vo, wcap_b);
    a[1] = hload(rs.w, vo, wcap_b + wplane_b);
  } else {
    a[0] = hload(rs.w, vo + (h ? wplane_b : 0), wcap_b);   // [W1 | W2]: lane half 1 reads plane 2
  }
}

template <int DIN, int TW, bool BIAS>
__device__ __forceinline__ void fetch32(const Rsrc3& rs, uint32_t wvo, uint32_t bvo, uint32_t xvo, int h,
                                        uint32_t wplane_b, uint32_t xplane_b, uint32_t zero_off, uint32_t wcap_b,
                                        uint32_t bcap_b, Frags32<DIN, TW>& fr) {
  constexpr uint32_t TSTEP = 32 * DIN * 2;   // bytes between row tiles
  fetch_x<DIN>(rs, xvo, h, xplane_b, zero_off, fr.b);
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    fetch_w<DIN>(rs, wvo + t * TSTEP, h, wplane_b, wcap_b, fr.a[t]);
    if constexpr (BIAS) {
      // (b1, b2, b3, 0) of the row; the upper half of the fragment stays zero
      const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rs.b, bvo + t * 32 * 8, bcap_b, 0);
      fr.bias[t] = __builtin_bit_cast(bf8, (unsigned __attribute__((ext_vector_type(4)))){v2[0], v2[1], 0u, 0u});
    }
  }
}

template <int DIN>
__device__ __forceinline__ f16v pose_chain(const h8 (&a)[SplitFrags<DIN>::NA], const h8 (&b)[SplitFrags<DIN>::NB],
                                           f16v acc) {
  if constexpr (DIN == 32) {   // small terms first, both k-halves
    acc = mfma32h(a[1], b[0], acc);   // W2 x1
    acc = mfma32h(a[3], b[2], acc);
    acc = mfma32h(a[0], b[1], acc);   // W1 x2
    acc = mfma32h(a[2], b[3], acc);
    acc = mfma32h(a[0], b[0], acc);   // W1 x1
    acc = mfma32h(a[2], b[2], acc);
  } else if constexpr (DIN == 16) {   // small terms first
    acc = mfma32h(a[1], b[0], acc);   // W2 x1
    acc = mfma32h(a[0], b[1], acc);   // W1 x2
    acc = mfma32h(a[0], b[0], acc);   // W1 x1
  } else {
    acc = mfma32h(a[0], b[1], acc);   // W1 x2
    acc = mfma32h(a[0], b[0], acc);   // W1 x1 + W2 x1
  }
  return acc;
}

// The pose tiles of one capsule (as pose_chain, bias first) with the next capsule's
// operands loaded into each register group right after its last reader is issued.
// XL (din 32): the next capsule's x fragments come from the workgroup's LDS copy xl
// (kXlPiece bytes per fragment, this lane's 16 bytes at xl + q * kXlPiece for b[q],
// staged by x_dma) instead of one global load per wave.
constexpr int kXlPiece = 1024;
// LDS read of the shared x fragments as inline asm: a plain read of the buffer the DMA
// (global_load_lds) fills would make the compiler wait for every DMA in flight (vmcnt(0))
// before it, draining the operand prefetch; pose_prog waits for these reads (lgkmcnt)
// itself, before the MFMAs that consume them.
__device__ __forceinline__ h8 xl_read(const char* p) {
  h8 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"((uint32_t)reinterpret_cast<uintptr_t>(p)));
  return r;
}
// XJ (with XL, din 32): x just in time -- this capsule's fragments are read from xl at
// the start and not prefetched for the next capsule, so they hold no registers between
// poses (the four-row-tile passes have none to spare).
template <int DIN, int TW, bool XL = false, bool XJ = false>
__device__ __forceinline__ void pose_prog(Frags32<DIN, TW>& fr, const bf8& ones, f16v (&u)[TW],
                                          const Rsrc3& rs, uint32_t wvo, uint32_t bvo, uint32_t xvo, int h,
                                          uint32_t wplane_b, uint32_t xplane_b, uint32_t zero_off, uint32_t wcap_b,
                                          uint32_t bcap_b, const char* xl = nullptr) {
  constexpr uint32_t TSTEP = 32 * DIN * 2;
  static_assert(!XJ || (XL && DIN == 32), "XJ: the shared x fragments of din 32");
  if constexpr (XJ) {
#pragma unroll
    for (int q = 0; q < 4; ++q) fr.b[q] = xl_read(xl + q * kXlPiece);
  } else if constexpr (XL) {   // the x fragments the previous call read from LDS (xl_read) have arrived
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fr.b[0]), "+v"(fr.b[1]), "+v"(fr.b[2]), "+v"(fr.b[3]));
  }
#pragma unroll
  for (int t = 0; t < TW; ++t) u[t] = mfma32(fr.bias[t], ones, f16v{});
  __builtin_amdgcn_sched_barrier(0);
  {
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rs.b, bvo + t * 32 * 8, bcap_b, 0);
      fr.bias[t] = __builtin_bit_cast(bf8, (unsigned __attribute__((ext_vector_type(4)))){v2[0], v2[1], 0u, 0u});
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (XJ)   // this capsule's x fragments (read above, behind the bias MFMAs)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fr.b[0]), "+v"(fr.b[1]), "+v"(fr.b[2]), "+v"(fr.b[3]));
  if constexpr (DIN == 32) {
#pragma unroll
    for (int t = 0; t < TW; ++t) {   // W2 x1, both k-halves
      u[t] = mfma32h(fr.a[t][1], fr.b[0], u[t]);
      u[t] = mfma32h(fr.a[t][3], fr.b[2], u[t]);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      fr.a[t][1] = hload(rs.w, wvo + t * TSTEP, wcap_b + wplane_b);
      fr.a[t][3] = hload(rs.w, wvo + t * TSTEP, wcap_b + wplane_b + 32);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TW; ++t) {   // W1 x2
      u[t] = mfma32h(fr.a[t][0], fr.b[1], u[t]);
      u[t] = mfma32h(fr.a[t][2], fr.b[3], u[t]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (XJ) {
    } else if constexpr (XL) {
      fr.b[1] = xl_read(xl + 1 * kXlPiece);
      fr.b[3] = xl_read(xl + 3 * kXlPiece);
    } else {
      fr.b[1] = hload(rs.x, xvo, xplane_b);
      fr.b[3] = hload(rs.x, xvo, xplane_b + 32);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TW; ++t) {   // W1 x1
      u[t] = mfma32h(fr.a[t][0], fr.b[0], u[t]);
      u[t] = mfma32h(fr.a[t][2], fr.b[2], u[t]);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      fr.a[t][0] = hload(rs.w, wvo + t * TSTEP, wcap_b);
      fr.a[t][2] = hload(rs.w, wvo + t * TSTEP, wcap_b + 32);
    }
    if constexpr (XJ) {
    } else if constexpr (XL) {
      fr.b[0] = xl_read(xl);
      fr.b[2] = xl_read(xl + 2 * kXlPiece);
    } else {
      fr.b[0] = hload(rs.x, xvo, 0);
      fr.b[2] = hload(rs.x, xvo, 32);
    }
    __builtin_amdgcn_sched_barrier(0);
    return;
  } else if constexpr (DIN == 16) {
#pragma unroll
    for (int t = 0; t < TW; ++t) u[t] = mfma32h(fr.a[t][1], fr.b[0], u[t]);   // W2 x1
    __builtin_amdgcn_sched_barrier(0);
    {
#pragma unroll
      for (int t = 0; t < TW; ++t) fr.a[t][1] = hload(rs.w, wvo + t * TSTEP, wcap_b + wplane_b);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TW; ++t) u[t] = mfma32h(fr.a[t][0], fr.b[1], u[t]);   // W1 x2
    __builtin_amdgcn_sched_barrier(0);
    fr.b[1] = hload(rs.x, xvo, xplane_b);
    __builtin_amdgcn_sched_barrier(0);
  } else {
#pragma unroll
    for (int t = 0; t < TW; ++t) u[t] = mfma32h(fr.a[t][0], fr.b[1], u[t]);   // W1 x2
    __builtin_amdgcn_sched_barrier(0);
    fr.b[1] = hload(rs.x, h ? zero_off : xvo, h ? 0u : xplane_b);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int t = 0; t < TW; ++t) u[t] = mfma32h(fr.a[t][0], fr.b[0], u[t]);   // W1 x1 (+ W2 x1 for DIN 8)
  __builtin_amdgcn_sched_barrier(0);
  {
#pragma unroll
    for (int t = 0; t < TW; ++t) fr.a[t][0] = hload(rs.w, wvo + t * TSTEP + (DIN == 8 && h ? wplane_b : 0), wcap_b);
    fr.b[0] = hload(rs.x, xvo, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// Scheduling hint for the region just written: K MFMAs, each followed by up to V VALU
// instructions of the region (igrouplp sched_group_barrier: MFMA = 0x008, VALU = 0x002).
template <int K, int V>
__device__ __forceinline__ void mfma_valu_hint() {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
  }
}

// The pose tiles of one capsule (din 32, shared x fragments in LDS) like pose_prog<32, TW,
// true>, with the previous capsule's VALU finish placed between the MFMAs: fill(S) for
// stage S = 0 (before the MFMAs: issue the LDS reads the finish needs), 1, 2, 3 (after the
// W2x1 / W1x2 / W1x1 MFMA groups, issued between them).  A wave issues in order: the
// finish then runs in the MFMA gaps (an MFMA holds vector issue for 8 of its 32 cycles)
// instead of after all of them, and the next MFMA issues as soon as the pipe frees.
template <int TW, int V1, int V2, int V3, class Fill>
__device__ __forceinline__ void pose_prog32i(Frags32<32, TW>& fr, const bf8& ones, f16v (&u)[TW], const Rsrc3& rs,
                                             uint32_t wvo, uint32_t bvo, uint32_t wplane_b, uint32_t wcap_b,
                                             uint32_t bcap_b, const char* xl, Fill&& fill) {
  constexpr uint32_t TSTEP = 32 * 32 * 2;
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fr.b[0]), "+v"(fr.b[1]), "+v"(fr.b[2]), "+v"(fr.b[3]));
  fill(std::integral_constant<int, 0>{});
#pragma unroll
  for (int t = 0; t < TW; ++t) u[t] = mfma32(fr.bias[t], ones, f16v{});
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rs.b, bvo + t * 32 * 8, bcap_b, 0);
    fr.bias[t] = __builtin_bit_cast(bf8, (unsigned __attribute__((ext_vector_type(4)))){v2[0], v2[1], 0u, 0u});
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < TW; ++t) {   // W2 x1, both k-halves
    u[t] = mfma32h(fr.a[t][1], fr.b[0], u[t]);
    u[t] = mfma32h(fr.a[t][3], fr.b[2], u[t]);
  }
  fill(std::integral_constant<int, 1>{});
  mfma_valu_hint<2 * TW, V1>();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    fr.a[t][1] = hload(rs.w, wvo + t * TSTEP, wcap_b + wplane_b);
    fr.a[t][3] = hload(rs.w, wvo + t * TSTEP, wcap_b + wplane_b + 32);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < TW; ++t) {   // W1 x2
    u[t] = mfma32h(fr.a[t][0], fr.b[1], u[t]);
    u[t] = mfma32h(fr.a[t][2], fr.b[3], u[t]);
  }
  fill(std::integral_constant<int, 2>{});
  mfma_valu_hint<2 * TW, V2>();
  __builtin_amdgcn_sched_barrier(0);
  fr.b[1] = xl_read(xl + 1 * kXlPiece);
  fr.b[3] = xl_read(xl + 3 * kXlPiece);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < TW; ++t) {   // W1 x1
    u[t] = mfma32h(fr.a[t][0], fr.b[0], u[t]);
    u[t] = mfma32h(fr.a[t][2], fr.b[2], u[t]);
  }
  fill(std::integral_constant<int, 3>{});
  mfma_valu_hint<2 * TW, V3>();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    fr.a[t][0] = hload(rs.w, wvo + t * TSTEP, wcap_b);
    fr.a[t][2] = hload(rs.w, wvo + t * TSTEP, wcap_b + 32);
  }
  fr.b[0] = xl_read(xl);
  fr.b[2] = xl_read(xl + 2 * kXlPiece);
  __builtin_amdgcn_sched_barrier(0);
}

// ones column of the bias MFMA: k = 0, 1, 2 of lane half 0
__device__ __forceinline__ bf8 ones_frag(int h) {
  const __bf16 o = (__bf16)(h == 0 ? 1.f : 0.f), z = (__bf16)0.f;
  bf8 v = {o, o, o, z, z, z, z, z};
  return v;
}

// capsule partial k of a wave's tile t / register v (rows 8(v>>2) + 4h + (v&3))
template <int DOUT>
__device__ __forceinline__ constexpr int kpart(int t, int v) {
  return DOUT == 8 ? 4 * t + (v >> 2) : DOUT == 16 ? 2 * t + (v >> 3) : t;
}

struct Args32 {
  const void *Ws, *bs, *xs;
  const float* hdr;   // {2^-(aw+bx), aw, bx} of the operand planes (prep32_kernel)
  size_t ws_bytes, bs_bytes, xs_bytes;
  uint32_t wplane_b, xplane_b, zero_off;
  int F, T, N, lpad, in_n, J, JDp, n_chunks, chunk_len, mask_first, n_tgroups;
  const float* vc;
  const float* bsum;
  float* slab;
  // forward passes r >= 1: when cst != nullptr, the couplings c^r [in_n][JP][Fs]
  // and logZ^r [in_n][Fs] (frame-minor: coalesced for every reader) are stored for
  // the backward (route_bwd32_kernel reads them instead of recomputing the logits)
  float* cst;
  float* lzst;
  int JP, Fs;
};



// ------------------------------------------------------------------ kernels
// Iteration-0 pass (naive:172-181: logits 0 + mask, so c is uniform):
// s = c0 (sum_i W_i x_i + sum_i b_i).  A pure GEMM: each wave owns
// (kFFB x 32 frames, kFTW row tiles, i-chunk) and accumulates the pose sum in its MFMA
// accumulators; the chunk's bias sum is added at the end.  Operands are double
// buffered: capsule k+1's loads are issued before capsule k's MFMAs, into the
// registers capsule k-1 used, so no load waits on a queued MFMA's operand read.
constexpr int kFTW = 2;   // row tiles per wave
constexpr int kFFB = 2;   // frame tiles per wave

template <int DIN>
struct FirstFrags {
  h8 a[kFTW][SplitFrags<DIN>::NA];
  h8 b[kFFB][SplitFrags<DIN>::NB];
};

template <int DIN, int DOUT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void route_fwd32_first_kernel(Args32 A) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  // XCD-aware order: the dispatcher deals workgroups round-robin over the 8 XCDs, so
  // XCD x receives blocks x, x+8, ...; remap them to one contiguous range of tasks,
  // ordered (i-chunk, frame pair, row group).  An XCD then works through one or two
  // i-chunks (their W slice stays in its L2) and reads each frame pair's x slice once,
  // where the row-group-fastest order had every XCD read all of x.
  int blk = blockIdx.x;
  {
    const int nb = gridDim.x, q = nb >> 3, rem = nb & 7, x = blk & 7, idx = blk >> 3;
    blk = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + idx;
  }
  const int task = blk * 4 + (threadIdx.x >> 6);
  const int nfp = (A.F + 32 * kFFB - 1) / (32 * kFFB);
  const int tg = task % A.n_tgroups;
  const int rest = task / A.n_tgroups;
  const int fp = rest % nfp, chunk = rest / nfp;
  if (chunk >= A.n_chunks) return;
  const int tbase = tg * kFTW;
  const int JD = A.J * DOUT;
  const Rsrc3 rs{make_rsrc(A.Ws, A.ws_bytes), make_rsrc(A.bs, A.bs_bytes), make_rsrc(A.xs, A.xs_bytes)};
  int f[kFFB], ftt[kFFB];
  bool fv[kFFB];
#pragma unroll
  for (int b = 0; b < kFFB; ++b) {
    f[b] = (fp * kFFB + b) * 32 + r;
    const int fc = min(f[b], A.F - 1);
    ftt[b] = fc - (fc / A.T) * A.T;
    fv[b] = f[b] < A.F;
  }
  const uint32_t wvo = (uint32_t)(((tbase * 32 + r) * DIN + (DIN >= 16 ? 8 * h : 0)) * 2);
  const int i0 = chunk * A.chunk_len, i1 = min(A.in_n, i0 + A.chunk_len);
  const uint32_t capb = (uint32_t)A.JDp * DIN * 2;
  constexpr uint32_t TSTEP = 32 * DIN * 2;
  f16v acc[kFTW][kFFB];
#pragma unroll
  for (int t = 0; t < kFTW; ++t)
#pragma unroll
    for (int b = 0; b < kFFB; ++b) acc[t][b] = f16v{};
  auto fetch = [&](int i, FirstFrags<DIN>& fr) {
#pragma unroll
    for (int b = 0; b < kFFB; ++b)
      fetch_x<DIN>(rs, x_voff<DIN>(i, A.N, A.lpad, A.T, A.F, f[b], ftt[b], fv[b], h, A.zero_off), h, A.xplane_b,
                   A.zero_off, fr.b[b]);
#pragma unroll
    for (int t = 0; t < kFTW; ++t) fetch_w<DIN>(rs, wvo + t * TSTEP, h, A.wplane_b, (uint32_t)i * capb, fr.a[t]);
  };
  auto mfmas = [&](const FirstFrags<DIN>& fr) {
#pragma unroll
    for (int t = 0; t < kFTW; ++t)
#pragma unroll
      for (int b = 0; b < kFFB; ++b) acc[t][b] = pose_chain<DIN>(fr.a[t], fr.b[b], acc[t][b]);
  };
  if (i0 < i1) {
    FirstFrags<DIN> f0, f1;
    fetch(i0, f0);
    int i = i0;
    for (; i + 1 < i1; i += 2) {
      fetch(i + 1, f1);
      mfmas(f0);
      if (i + 2 < i1) fetch(i + 2, f0);
      mfmas(f1);
    }
    if (i < i1) mfmas(f0);
  }
  const int Jeff = A.J - (A.mask_first ? 1 : 0);
  const float inv = A.hdr[0];
#pragma unroll
  for (int t = 0; t < kFTW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      const int j = row / DOUT;
      const float c0 = (j < A.J && !(A.mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
      if (row < JD) {
        const f4 bsv = *reinterpret_cast<const f4*>(A.bsum + (size_t)chunk * JD + row);
#pragma unroll
        for (int b = 0; b < kFFB; ++b) {
          if (!fv[b]) continue;
          f4 v = {acc[t][b][4 * q], acc[t][b][4 * q + 1], acc[t][b][4 * q + 2], acc[t][b][4 * q + 3]};
          *reinterpret_cast<f4*>(A.slab + ((size_t)chunk * A.F + f[b]) * JD + row) = (v * inv + bsv) * c0;
        }
      }
    }
}

// Iteration-0 pass over ALL input capsules, din = dout = 32 (the C3/C4 DR layers):
// s^0 = c0 (sum_i W_i x_i + sum_i b_i) and its squash in the epilogue, so this pass
// writes s^0 and Vc^1 = v^0 itself: no i-chunk slabs, no finish launch.
// Workgroup = 128 rows x 64 frames, 4 waves (2 row halves x 2 frame tiles; a wave
// owns 2 row tiles x 1 frame tile).  The split-fp16 operands of one capsule (W: 128
// rows, x: 64 frames, hi and lo planes, 64 B per row and plane) are staged global ->
// LDS by global_load_lds (16 B per lane, no registers, no ds_write) into two buffers,
// one capsule ahead.  LDS image per plane: [rows][4 slots of 16 B], chunk c of row r
// in slot 4r + (c ^ ((r >> 2) & 3)): the fragment reads (ds_read_b128, rows 0-31 of a
// tile, one chunk) then hit 16 distinct slots per lane group; the DMA writes slots
// lane-linearly, so each lane fetches the chunk its slot holds.  XCD-aware block
// order: the row tiles of a frame tile run on one XCD (x read once per XCD).
constexpr int kFfBM = 128;
constexpr int kFfA = 2 * kFfBM * 64;   // A bytes per stage (two planes)
// frames per workgroup BN (32-frame tiles; 2 row halves x BN / 32 frame tiles of waves):
// a stage holds A (16 KiB) and B (BN x 128 B); two stages
template <int BN>
constexpr int ff_stage() { return kFfA + 2 * BN * 64; }


__device__ __forceinline__ uint32_t ff_slot(int r, int c) { return (uint32_t)(4 * r + (c ^ ((r >> 2) & 3))); }

__device__ __forceinline__ void glds16(const void* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// One capsule's x fragments (din 32: hi / lo plane x two k-halves, 16 bytes per lane
// each) global -> LDS for all the workgroup's waves, which share them: wave w DMAs
// fragment q = w & 3 (plane q & 1, k-half q >> 1) of the 64 lanes' frames into
// dst + q * kXlPiece (lane-linear; waves w and w + 4 write the same bytes).  Every wave
// issues it (no branch: the compiler keeps counting the loads in flight exactly) and
// waits for it (xl_wait) before the barrier that publishes it.
// The DMA is inline asm: issued through the builtin, the compiler stops counting the
// loads in flight across it and waits for all of them at the next operand use.  Its own
// waits stay correct, only conservative, with one more load in flight than it knows of.
// The source as a wave-uniform base (SGPRs) + the lane's 32-bit offset: no 64-bit
// per-lane address is held across the capsule loop.
__device__ __forceinline__ void x_dma(const char* xs, uint32_t xplane_b, uint32_t xvo, int wv, char* dst) {
  const int q = __builtin_amdgcn_readfirstlane(wv) & 3;
  const char* base = xs + (q & 1) * xplane_b + (q >> 1) * 32;
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(dst + q * kXlPiece));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(m0), "v"(xvo), "s"(base)
               : "memory", "m0");
}
// The lane id, re-derived where it is used (asm: not hoisted): a per-lane offset held
// across a capsule loop at 256 registers is spilled, and its reload's vmcnt(0) drains
// the operand prefetch.
__device__ __forceinline__ int lane_asm() {
  int lid;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
  return lid;
}
// K: the vector-memory instructions the wave issues after the DMA (they may stay in
// flight); each kernel's count is checked against its ISA (scripts/dbg/check_xl_wait.py)
template <int K = 0>
__device__ __forceinline__ void xl_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K) : "memory");
}

// CPS capsules per stage buffer (one barrier per stage: CPS = 2 halves the barriers and
// lets capsule 1's fragment reads ride under capsule 0's MFMAs; two buffers of two
// capsules fill the 160 KiB of LDS at BN = 192)
template <int BN, int CPS = 1>
__global__ __launch_bounds__(64 * 2 * (BN / 32)) void route_fwd32_first_full_kernel(
    Args32 A, float* __restrict__ s_out, float* __restrict__ vc_out, float* __restrict__ v_out) {
  constexpr int NWF = BN / 32, NWV = 2 * NWF;         // frame tiles, waves
  constexpr int NPA = kFfA / 1024, NPB = 2 * BN * 64 / 1024, NP = NPA + NPB;   // 1 KiB DMA pieces
  constexpr int NPW = (NP + NWV - 1) / NWV;           // pieces per wave (the last ones may idle)
  constexpr int BPP = BN / 16;                        // B pieces per plane
  constexpr int kCap = ff_stage<BN>();                // LDS bytes of one capsule
  constexpr int kStage = CPS * kCap;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int n_rt = A.JDp / kFfBM;
  int blk = blockIdx.x;
  {
    const int nb = gridDim.x, q = nb >> 3, rem = nb & 7, x = blk & 7, idx = blk >> 3;
    blk = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + idx;
  }
  const int rt = blk % n_rt, ft = blk / n_rt;
  const int row0 = rt * kFfBM, f0 = ft * BN;
  const int wr = wv / NWF, wc = wv - wr * NWF;   // row half, frame tile of this wave
  const char* Wb = static_cast<const char*>(A.Ws);
  const char* Xb = static_cast<const char*>(A.xs);
  const size_t capb = (size_t)A.JDp * 64;   // bytes of one capsule's W rows per plane
  // DMA roles: wave wv fills pieces wv, wv + NWV, ... (1 KiB each, 16 B per lane): A piece
  // q < NPA: plane q / 8, slots (q % 8) * 64 + lane -> row slot >> 2; B piece q - NPA: plane
  // (q - NPA) / BPP, slots ((q - NPA) % BPP) * 64 + lane -> frame slot >> 2
  uint32_t src_o[NPW];
  const char* src_b[NPW];
  bool is_b[NPW], live[NPW];
  int bf_[NPW], btt[NPW];
  bool bok[NPW];
#pragma unroll
  for (int k = 0; k < NPW; ++k) {
    const int q = wv + k * NWV;
    live[k] = q < NP;
    is_b[k] = q >= NPA;
    if (!is_b[k]) {
      const int slot = (q & 7) * 64 + lane, r = slot >> 2, c = (slot & 3) ^ ((r >> 2) & 3);
      src_b[k] = Wb + (size_t)(q >> 3) * A.wplane_b;
      src_o[k] = (uint32_t)((row0 + r) * 64 + c * 16);
      bf_[k] = 0, btt[k] = 0, bok[k] = false;
    } else {
      const int qb = q - NPA;
      const int slot = (qb % BPP) * 64 + lane, r = slot >> 2, c = (slot & 3) ^ ((r >> 2) & 3);
      src_b[k] = Xb + (size_t)(qb / BPP) * A.xplane_b;
      src_o[k] = (uint32_t)(c * 16);
      bf_[k] = f0 + r;
      bok[k] = bf_[k] < A.F;
      const int fc = min(bf_[k], A.F - 1);
      btt[k] = fc - (fc / A.T) * A.T;
    }
  }
  auto stage = [&](int i0, int buf) {
#pragma unroll
    for (int c = 0; c < CPS; ++c) {
      // a slot past the last capsule re-DMAs its W and the zero x row: its MFMAs then add
      // exact zeros
      const int i = min(i0 + c, A.in_n - 1);
      char* dst = smem + buf * kStage + c * kCap;
#pragma unroll
      for (int k = 0; k < NPW; ++k) {
        if (!live[k]) continue;   // uniform per wave
        const int q = wv + k * NWV;
        if (!is_b[k])
          glds16(src_b[k] + (size_t)i * capb + src_o[k], dst + q * 1024);
        else
          glds16(src_b[k] +
                     x_voff<32>(i, A.N, A.lpad, A.T, A.F, bf_[k], btt[k], bok[k] && i0 + c < A.in_n, 0,
                                A.zero_off) +
                     src_o[k],
                 dst + q * 1024);
      }
    }
  };
  // fragment reads: A rows wr*64 + t*32 + r32, B frames wc*32 + r32, chunk 2s + h
  auto afrag = [&](const char* base, int t, int plane, int sstep) -> h8 {
    const int r = wr * 64 + t * 32 + r32;
    return *reinterpret_cast<const h8*>(base + plane * (kFfBM * 64) + ff_slot(r, 2 * sstep + h) * 16);
  };
  auto bfrag = [&](const char* base, int plane, int sstep) -> h8 {
    const int r = wc * 32 + r32;
    return *reinterpret_cast<const h8*>(base + kFfA + plane * (BN * 64) + ff_slot(r, 2 * sstep + h) * 16);
  };
  f16v acc[2] = {f16v{}, f16v{}};
  const int n_in = A.in_n;
  stage(0, 0);
  for (int i = 0, buf = 0; i < n_in; i += CPS, buf ^= 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of stage i has landed
    __syncthreads();                                    // ... and every wave's; buf ^ 1 no longer read
    if (i + CPS < n_in) stage(i + CPS, buf ^ 1);
    // capsule 1's twelve fragment reads ride in the gaps of capsule 0's twelve MFMAs (one
    // ds_read_b128 per gap is free of LDS-array stalls, MI355X_MICROARCH §LDS), so only
    // the stage's first reads wait in the open
    auto frags = [&](const char* base, h8 (&b)[4], h8 (&a)[2][4]) {
#pragma unroll
      for (int s = 0; s < 4; ++s) b[s] = bfrag(base, s & 1, s >> 1);   // x hi / lo, k-step s / 2
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) a[t][s] = afrag(base, t, s & 1, s >> 1);   // W hi / lo
    };
    // pose_chain<32>'s six steps, the two row tiles alternating (no back-to-back MFMAs on
    // one accumulator)
    auto pose2 = [&](const h8 (&a)[2][4], const h8 (&b)[4]) {
      constexpr int ka[6] = {1, 3, 0, 2, 0, 2}, kb[6] = {0, 2, 1, 3, 0, 2};
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mfma32h(a[t][ka[k]], b[kb[k]], acc[t]);
    };
    const char* base0 = smem + buf * kStage;
    h8 b0[4], a0[2][4];
    frags(base0, b0, a0);
    if constexpr (CPS == 2) {   // no tail branch: a slot past the last capsule holds x = 0
      h8 b1[4], a1[2][4];
      __builtin_amdgcn_sched_barrier(0);
      frags(base0 + kCap, b1, a1);
      pose2(a0, b0);
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one LDS read
      }
      __builtin_amdgcn_sched_barrier(0);
      pose2(a1, b1);
    } else {
      pose2(a0, b0);
    }
  }
  // epilogue: s = c0 (2^-(aw+bx) acc + sum_i b_i), v = squash over the capsule's 32 rows
  // (16 in this lane, 16 in lane ^ 32), Vc^1 = v
  const int f = f0 + wc * 32 + r32;
  const bool fv = f < A.F;
  const int JD = A.J * 32;
  const int Jeff = A.J - (A.mask_first ? 1 : 0);
  const float inv = A.hdr[0];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int rbase = row0 + wr * 64 + t * 32;   // one output capsule j = rbase / 32
    const int j = rbase / 32;
    const float c0 = (j < A.J && !(A.mask_first && j == 0)) ? 1.f / (float)Jeff : 0.f;
    f4 sv[4];
    float n2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = rbase + 8 * q + 4 * h;
      f4 bs = {0.f, 0.f, 0.f, 0.f};
      if (row < JD)
        for (int ch = 0; ch < A.n_chunks; ++ch) bs += *reinterpret_cast<const f4*>(A.bsum + (size_t)ch * JD + row);
      const f4 u = {acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
      sv[q] = (u * inv + bs) * c0;
      n2 += (sv[q].x * sv[q].x + sv[q].y * sv[q].y) + (sv[q].z * sv[q].z + sv[q].w * sv[q].w);
    }
    n2 = xor32_sum(n2);
    const float fac = n2 / (1.f + n2) / sqrtf(n2 + 1e-7f);   // squash (naive:247-252)
    if (fv && rbase < JD) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const size_t o = (size_t)f * JD + rbase + 8 * q + 4 * h;
        *reinterpret_cast<f4*>(s_out + o) = sv[q];
        const f4 v = sv[q] * fac;
        *reinterpret_cast<f4*>(vc_out + o) = v;
        if (v_out) *reinterpret_cast<f4*>(v_out + o) = v;
      }
    }
  }
}

// Routing pass r >= 1.  grid: n_ftiles * n_chunks (chunk = blockIdx % n_chunks);
// block: NW waves of kTW row tiles.  LDS: NW * kTW * 4 KiB of Vc fragments, then
// 2 x NW x 32 float2 of per-wave softmax stats.
template <int DIN, int DOUT, int NW, int TW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(kWavesPerEU))) void route_fwd32_kernel(Args32 A) {
  constexpr int CP = TW * 32 / DOUT;   // capsule partials per lane
  constexpr int OWN = CP / 2;          // capsules whose logit this lane owns
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int JD = A.J * DOUT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);   // wave index in an SGPR (stats slots)
  const int r = lane & 31, h = lane >> 5;
  const int bid = blockIdx.x;
  const int ft = bid / A.n_chunks, chunk = bid - ft * A.n_chunks;
  const int f = ft * 32 + r;
  const int fc = min(f, A.F - 1);
  const int fb = fc / A.T, ftt = fc - fb * A.T;
  const bool fvalid = f < A.F;
  const int i0 = chunk * A.chunk_len, i1 = min(A.in_n, i0 + A.chunk_len);
  const int tbase = __builtin_amdgcn_readfirstlane(wv * TW);
  const int j0 = tbase * 32 / DOUT;
  const Rsrc3 rs{make_rsrc(A.Ws, A.ws_bytes), make_rsrc(A.bs, A.bs_bytes), make_rsrc(A.xs, A.xs_bytes)};
  if (DIN <= 16 && NW > 1 && wv >= NW / 2) __builtin_amdgcn_s_setprio(1);   // din 32: measured faster without
  const uint32_t wvo = (uint32_t)(((tbase * 32 + r) * DIN + (DIN >= 16 ? 8 * h : 0)) * 2);
  const uint32_t bvo = (uint32_t)((tbase * 32 + r) * 8);
  const __amdgpu_buffer_rsrc_t crs = make_rsrc(A.cst, A.cst ? (size_t)A.in_n * A.JP * A.Fs * 4 : 0);
  const __amdgpu_buffer_rsrc_t lzs = make_rsrc(A.lzst, A.cst ? (size_t)A.in_n * A.Fs * 4 : 0);

  f4* vcl = reinterpret_cast<f4*>(lds) + (size_t)wv * TW * 4 * 64;
  float2* st = reinterpret_cast<float2*>(lds + (size_t)NW * TW * 4 * 64 * 4);
  // din 32: each capsule's x fragments DMA'd once per workgroup into LDS (x_dma, two
  // buffers) and read just in time by the pose (pose_prog XJ): no per-wave x loads, and
  // no x registers held between poses (a separate LDS object: no aliasing with the stats)
  constexpr bool XJ = DIN == 32 && NW > 1;
  __shared__ __attribute__((aligned(16))) char xls[XJ ? 2 * 4 * kXlPiece : 16];
  const char* xs_b = static_cast<const char*>(A.xs);
  auto xsrc = [&](int c) { return x_voff<DIN>(min(c, i1 - 1), A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off); };
  auto xbuf = [&](int c) { return xls + (c & 1) * 4 * kXlPiece; };
  // Vc rows of this wave's tiles -> private LDS in fragment order
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (fvalid && row < JD) v = *reinterpret_cast<const f4*>(A.vc + (size_t)f * JD + row);
      vcl[(t * 4 + q) * 64 + lane] = v;
    }
  // owned-capsule masks: 0 or -inf added to the logit
  float mk[OWN];
#pragma unroll
  for (int a = 0; a < OWN; ++a) {
    const int j = j0 + 2 * a + h;
    mk[a] = (j < A.J && !(A.mask_first && j == 0)) ? 0.f : -INFINITY;
  }
  const bf8 ones = ones_frag(h);
  const float inv = A.hdr[0];   // 2^-(aw+bx): the pose tiles hold 2^(aw+bx) u
  f16v acc[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) acc[t] = f16v{};
  int par = 0;
  if (i0 < i1) {
    Frags32<DIN, TW> fr;
    fetch32<DIN, TW, true>(rs, wvo, bvo, x_voff<DIN>(i0, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                           A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)i0 * A.JDp * DIN * 2, (uint32_t)i0 * A.JDp * 8,
                           fr);
    if constexpr (XJ) {   // x of capsules i0, i0 + 1 before the first pose
      x_dma(xs_b, A.xplane_b, xsrc(i0), wv, xbuf(i0));
      x_dma(xs_b, A.xplane_b, xsrc(i0 + 1), wv, xbuf(i0 + 1));
      xl_wait();
      __syncthreads();
    }
    for (int i = i0; i < i1; ++i) {
      f16v u[TW];
      // partial agreement dots <u_ij, Vc_j> over this lane's rows (packed FMA pairs)
      f2 P2[CP];
#pragma unroll
      for (int k = 0; k < CP; ++k) P2[k] = f2{0.f, 0.f};
      if constexpr (DIN <= 16) {   // tile-major pose; din 32: pose_prog measured faster (C4 A/B)
      {
        constexpr uint32_t TSTEP = 32 * DIN * 2;
        const int in = min(i + 1, i1 - 1);
        const uint32_t wcap = (uint32_t)in * A.JDp * DIN * 2, bcap = (uint32_t)in * A.JDp * 8;
        const uint32_t xvn = x_voff<DIN>(in, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off);
        f4 vv[4];
        auto dots = [&](int t) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int k = kpart<DOUT>(t, 4 * q);
            P2[k] += f2{u[t][4 * q], u[t][4 * q + 1]} * f2{vv[q].x, vv[q].y};
            P2[k] += f2{u[t][4 * q + 2], u[t][4 * q + 3]} * f2{vv[q].z, vv[q].w};
          }
        };
#pragma unroll
        for (int t = 0; t < TW; ++t) {
          if (t > 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) vv[q] = vcl[((t - 1) * 4 + q) * 64 + lane];
          }
          __builtin_amdgcn_sched_barrier(0);
          u[t] = pose_chain<DIN>(fr.a[t], fr.b, mfma32(fr.bias[t], ones, f16v{}));
          __builtin_amdgcn_sched_barrier(0);
          fetch_w<DIN>(rs, wvo + t * TSTEP, h, A.wplane_b, wcap, fr.a[t]);
          {
            const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rs.b, bvo + t * 32 * 8, bcap, 0);
            fr.bias[t] = __builtin_bit_cast(bf8, (unsigned __attribute__((ext_vector_type(4)))){v2[0], v2[1], 0u, 0u});
          }
          if (t == TW - 1) fetch_x<DIN>(rs, xvn, h, A.xplane_b, A.zero_off, fr.b);
          __builtin_amdgcn_sched_barrier(0);
          if (t > 0) dots(t - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) vv[q] = vcl[((TW - 1) * 4 + q) * 64 + lane];
        dots(TW - 1);
      }
      } else {
      const int in = min(i + 1, i1 - 1);
      pose_prog<DIN, TW, XJ, XJ>(fr, ones, u, rs, wvo, bvo,
                                 x_voff<DIN>(in, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                                 A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)in * A.JDp * DIN * 2,
                                 (uint32_t)in * A.JDp * 8, xbuf(i) + lane * 16);
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 vv = vcl[(t * 4 + q) * 64 + lane];
          const int k = kpart<DOUT>(t, 4 * q);
          P2[k] += f2{u[t][4 * q], u[t][4 * q + 1]} * f2{vv.x, vv.y};
          P2[k] += f2{u[t][4 * q + 2], u[t][4 * q + 3]} * f2{vv.z, vv.w};
        }
      }
      // reduce-scatter over lane halves: half h owns capsule partial 2a + h
      float L[OWN], e[OWN];
      float m = -1e30f;
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        const float pa = P2[2 * a].x + P2[2 * a].y, pb = P2[2 * a + 1].x + P2[2 * a + 1].y;
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(pa), __float_as_uint(pb), false, false);
        L[a] = (__uint_as_float(sw[0]) + __uint_as_float(sw[1])) * inv + mk[a];
        m = fmaxf(m, L[a]);
      }
      float z = 0.f;
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        e[a] = __expf(L[a] - m);
        z += e[a];
      }
      // combine the two lane halves (same order on both: bit-identical)
      float M, Z;
      {
        float m0, m1, z0, z1;
        xpair32(m, m0, m1);
        xpair32(z, z0, z1);
        M = fmaxf(m0, m1);
        Z = z0 * __expf(m0 - M) + z1 * __expf(m1 - M);
      }
      if constexpr (NW > 1) {
        // per-wave stats of the 32 frames -> LDS; half h combines waves [h*NW/2, (h+1)*NW/2)
        // the stats slot addresses re-derived from the lane id here (asm: not hoisted): held
        // across the capsule loop they were spilled, and a spill reload's vmcnt(0) drains
        // the next capsule's operand prefetch
        int lid;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
        const int sr = lid & 31, sh = lid >> 5;
        float2* slot = st + par * NW * 32;
        if (sh == 0) slot[wvu * 32 + sr] = make_float2(M, Z);
        // x of capsule i + 1 (DMA'd after the last barrier) lands before this one; the next
        // capsule's W / bias loads (5 per tile) and the last capsule's coupling / logZ
        // stores issued since may stay in flight (scripts/dbg/check_xl_wait4.py)
        if constexpr (XJ) xl_wait<5 * TW + OWN + 1>();
        __syncthreads();
        // every wave's pose read x of capsule i: its buffer takes capsule i + 2's (unconditional:
        // past the chunk it reloads the last capsule into a buffer no pose reads any more)
        if constexpr (XJ) x_dma(xs_b, A.xplane_b, xsrc(i + 2), wv, xbuf(i + 2));
        constexpr int HW = NW / 2;
        float2 sv[HW];
#pragma unroll
        for (int w = 0; w < HW; ++w) sv[w] = slot[(sh * HW + w) * 32 + sr];
        float mh = sv[0].x;
#pragma unroll
        for (int w = 1; w < HW; ++w) mh = fmaxf(mh, sv[w].x);
        float zh = 0.f;
#pragma unroll
        for (int w = 0; w < HW; ++w) zh += sv[w].y * __expf(sv[w].x - mh);
        float m0, m1, z0, z1;
        xpair32(mh, m0, m1);
        xpair32(zh, z0, z1);
        const float MM = fmaxf(m0, m1);
        Z = z0 * __expf(m0 - MM) + z1 * __expf(m1 - MM);
        M = MM;
        par ^= 1;
      }
      // next capsule's operands: issued once every MFMA result has been consumed
      // (the dots), so no load waits on a queued MFMA's operand read
      __builtin_amdgcn_sched_barrier(0);
      // c = exp(L - M) / Z = e * exp(m - M) / Z; then all-gather over the halves
      const float sc = __expf(m - M) * __builtin_amdgcn_rcpf(Z);   // Z >= 1: 1-ulp v_rcp
      {
        // lane half h owns capsules j0 + 2a + h after the logit reduce-scatter; frames
        // past F (up to the 32-frame stride) store 0, which the gW pass relies on.
        // Branch-free buffer stores (no storage: zero-record descriptors drop them).
#pragma unroll
        for (int a = 0; a < OWN; ++a)
          bstore(crs, fvalid ? e[a] * sc : 0.f, (uint32_t)((j0 + h + 2 * a) * A.Fs + f) * 4u,
                 (uint32_t)i * A.JP * A.Fs * 4u);
        bstore(lzs, M + __builtin_amdgcn_logf(Z) * 0.69314718f, (h == 0 && wv == 0 && fvalid) ? (uint32_t)f * 4u : kNoStore,
               (uint32_t)i * A.Fs * 4u);
      }
      float c[CP];
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        float c0, c1;
        xpair32(e[a] * sc, c0, c1);
        c[2 * a] = c0;
        c[2 * a + 1] = c1;
      }
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int v = 0; v < 16; v += 2) {
          const float cv = c[kpart<DOUT>(t, v)];
          f2 a2 = {acc[t][v], acc[t][v + 1]};
          a2 += f2{cv, cv} * f2{u[t][v], u[t][v + 1]};
          acc[t][v] = a2.x;
          acc[t][v + 1] = a2.y;
        }
    }
  }
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      if (fvalid && row < JD) {
        f4 v = {acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
        *reinterpret_cast<f4*>(A.slab + ((size_t)chunk * A.F + f) * JD + row) = v * inv;
      }
    }
}


// Routing pass r >= 1, software-pipelined over the input capsules: while the matrix
// cores form capsule i + 1's pose tiles (pose_prog, which also streams in capsule
// i + 2's operands), the VALU finishes capsule i -- the cross-wave softmax statistics
// behind last iteration's barrier, the coupling stores and s += c u -- so the one
// barrier per capsule no longer leaves the matrix pipe idle while the waves meet.
// Same tiles, LDS and results as route_fwd32_kernel (one more u set in registers).
template <int DIN, int DOUT, int NW, int TW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(kWavesPerEU))) void route_fwd32p_kernel(Args32 A) {
  constexpr int CP = TW * 32 / DOUT;   // capsule partials per lane
  constexpr int OWN = CP / 2;          // capsules whose logit this lane owns
  static_assert(NW > 1, "the pipelined pass exchanges softmax stats between waves");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int JD = A.J * DOUT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int bid = blockIdx.x;
  const int ft = bid / A.n_chunks, chunk = bid - ft * A.n_chunks;
  const int f = ft * 32 + r;
  const int fc = min(f, A.F - 1);
  const int fb = fc / A.T, ftt = fc - fb * A.T;
  const bool fvalid = f < A.F;
  const int i0 = chunk * A.chunk_len, i1 = min(A.in_n, i0 + A.chunk_len);
  const int tbase = __builtin_amdgcn_readfirstlane(wv * TW);
  const int j0 = tbase * 32 / DOUT;
  const Rsrc3 rs{make_rsrc(A.Ws, A.ws_bytes), make_rsrc(A.bs, A.bs_bytes), make_rsrc(A.xs, A.xs_bytes)};
  const uint32_t wvo = (uint32_t)(((tbase * 32 + r) * DIN + (DIN >= 16 ? 8 * h : 0)) * 2);
  const uint32_t bvo = (uint32_t)((tbase * 32 + r) * 8);
  const __amdgpu_buffer_rsrc_t crs = make_rsrc(A.cst, A.cst ? (size_t)A.in_n * A.JP * A.Fs * 4 : 0);
  const __amdgpu_buffer_rsrc_t lzs = make_rsrc(A.lzst, A.cst ? (size_t)A.in_n * A.Fs * 4 : 0);
  // this lane's Vc fragments in registers (no LDS reads per capsule); LDS: the softmax
  // stats, then (din 32) two buffers of the shared x fragments (x_dma)
  float2* st = reinterpret_cast<float2*>(lds);
  constexpr bool XL = DIN == 32;
  f4 vcr[TW][4];
  // a separate LDS object: the compiler then sees no DMA aliasing the stats
  __shared__ __attribute__((aligned(16))) char xls[XL ? 2 * 4 * kXlPiece : 16];
  char* xb = xls;
  const char* xs_b = static_cast<const char*>(A.xs);
  auto xsrc = [&](int c) { return x_voff<DIN>(min(c, i1 - 1), A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off); };
  auto xbuf = [&](int c) { return xb + (c & 1) * 4 * kXlPiece; };
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (fvalid && row < JD) v = *reinterpret_cast<const f4*>(A.vc + (size_t)f * JD + row);
      vcr[t][q] = v;
    }
  float mk[OWN];
#pragma unroll
  for (int a = 0; a < OWN; ++a) {
    const int j = j0 + 2 * a + h;
    mk[a] = (j < A.J && !(A.mask_first && j == 0)) ? 0.f : -INFINITY;
  }
  const bf8 ones = ones_frag(h);
  const float inv = A.hdr[0];   // 2^-(aw+bx): the pose tiles hold 2^(aw+bx) u
  f16v acc[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) acc[t] = f16v{};
  if (i0 < i1) {
    Frags32<DIN, TW> fr;
    fetch32<DIN, TW, true>(rs, wvo, bvo, x_voff<DIN>(i0, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                           A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)i0 * A.JDp * DIN * 2, (uint32_t)i0 * A.JDp * 8,
                           fr);
    f16v uc[TW], un[TW];
    float e[OWN], m;   // the pending capsule's exponentials and lane max
    if constexpr (XL) {   // x of capsules i0 + 1, i0 + 2 into LDS before the first pose
      x_dma(xs_b, A.xplane_b, xsrc(i0 + 1), wv, xbuf(i0 + 1));
      x_dma(xs_b, A.xplane_b, xsrc(i0 + 2), wv, xbuf(i0 + 2));
      xl_wait();
      __syncthreads();
    }
    // the logits of one capsule's tiles -> e, m; the wave's (max, sum) -> LDS slot
    auto logits = [&](const f16v (&u)[TW], int slot_par) {
      f2 P2[CP];
#pragma unroll
      for (int k = 0; k < CP; ++k) P2[k] = f2{0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 vv = vcr[t][q];
          const int k = kpart<DOUT>(t, 4 * q);
          P2[k] += f2{u[t][4 * q], u[t][4 * q + 1]} * f2{vv.x, vv.y};
          P2[k] += f2{u[t][4 * q + 2], u[t][4 * q + 3]} * f2{vv.z, vv.w};
        }
      float L[OWN];
      m = -1e30f;
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        const float pa = P2[2 * a].x + P2[2 * a].y, pb = P2[2 * a + 1].x + P2[2 * a + 1].y;
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(pa), __float_as_uint(pb), false, false);
        L[a] = (__uint_as_float(sw[0]) + __uint_as_float(sw[1])) * inv + mk[a];
        m = fmaxf(m, L[a]);
      }
      float z = 0.f;
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        e[a] = __expf(L[a] - m);
        z += e[a];
      }
      float m0, m1, z0, z1;
      xpair32(m, m0, m1);
      xpair32(z, z0, z1);
      const float M = fmaxf(m0, m1);
      const float Z = z0 * __expf(m0 - M) + z1 * __expf(m1 - M);
      if (h == 0) st[(slot_par * NW + wv) * 32 + r] = make_float2(M, Z);
    };
    int par = 0;
    pose_prog<DIN, TW, XL>(fr, ones, uc, rs, wvo, bvo,
                           x_voff<DIN>(min(i0 + 1, i1 - 1), A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                           A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)min(i0 + 1, i1 - 1) * A.JDp * DIN * 2,
                           (uint32_t)min(i0 + 1, i1 - 1) * A.JDp * 8, xbuf(i0 + 1) + lane * 16);
    logits(uc, par);
    __syncthreads();
    // one capsule: i + 1's tiles into unext while capsule i (in ucur) is finished; the loop
    // runs two steps with the roles swapped, so no register copy moves u between them
    // IL: capsule i's finish between capsule i + 1's pose MFMAs (pose_prog32i)
    auto step_il = [&](int i, f16v (&ucur)[TW], f16v (&unext)[TW]) __attribute__((always_inline)) {
      if constexpr (DIN == 32) {
      const bool more = i + 1 < i1;
      x_dma(xs_b, A.xplane_b, xsrc(i + 3), wv, xbuf(i + 3));   // into the buffer capsule i + 1's x left
      constexpr int HW = NW / 2;
      float2 sv[HW];
      float M, Z, sc;
      float c[CP];
      // s += c u over tiles [t0, t1), scalar FMAs (a packed FMA costs more beside MFMAs),
      // each result pinned here so that no IR pass sinks it out of its MFMA region
      auto cfma = [&](int t0, int t1) __attribute__((always_inline)) {
#pragma unroll
        for (int t = t0; t < t1; ++t) {
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[t][v] = fmaf(c[kpart<DOUT>(t, v)], ucur[t][v], acc[t][v]);
          asm volatile("" : "+v"(acc[t]));
        }
      };
      auto fill = [&](auto stage) __attribute__((always_inline)) {
        constexpr int S = decltype(stage)::value;
        if constexpr (S == 0) {   // capsule i's softmax stats of the 4 waves of this lane half
          const float2* slot = st + par * NW * 32;
#pragma unroll
          for (int w = 0; w < HW; ++w) sv[w] = slot[(h * HW + w) * 32 + r];
        } else if constexpr (S == 1) {
          float mh = sv[0].x;
#pragma unroll
          for (int w = 1; w < HW; ++w) mh = fmaxf(mh, sv[w].x);
          float zh = 0.f;
#pragma unroll
          for (int w = 0; w < HW; ++w) zh += sv[w].y * __expf(sv[w].x - mh);
          float m0, m1, z0, z1;
          xpair32(mh, m0, m1);
          xpair32(zh, z0, z1);
          M = fmaxf(m0, m1);
          Z = z0 * __expf(m0 - M) + z1 * __expf(m1 - M);
          sc = __expf(m - M) * __builtin_amdgcn_rcpf(Z);   // Z >= 1: 1-ulp v_rcp
        } else if constexpr (S == 2) {
#pragma unroll
          for (int a = 0; a < OWN; ++a)
            bstore(crs, fvalid ? e[a] * sc : 0.f, (uint32_t)((j0 + h + 2 * a) * A.Fs + f) * 4u,
                   (uint32_t)i * A.JP * A.Fs * 4u);
          bstore(lzs, M + __builtin_amdgcn_logf(Z) * 0.69314718f,
                 (h == 0 && wv == 0 && fvalid) ? (uint32_t)f * 4u : kNoStore, (uint32_t)i * A.Fs * 4u);
#pragma unroll
          for (int a = 0; a < OWN; ++a) {
            float c0, c1;
            xpair32(e[a] * sc, c0, c1);
            c[2 * a] = c0;
            c[2 * a + 1] = c1;
          }
          cfma(0, TW / 2);
        } else {
          cfma(TW / 2, TW);
        }
      };
      {   // capsule i + 1's tiles on the matrix cores, capsule i finished in their gaps; after
          // the chunk's last capsule the pose runs anyway (on its own operands, unused): one
          // copy of the finish, not a second one outside the MFMA regions
        const int in = min(i + 2, i1 - 1);
        pose_prog32i<TW, 6, 6, 5>(fr, ones, unext, rs, wvo, bvo, A.wplane_b, (uint32_t)in * A.JDp * DIN * 2,
                                  (uint32_t)in * A.JDp * 8, xbuf(i + 2) + lane * 16, fill);
      }
      if (more) {
        par ^= 1;
        logits(unext, par);
        xl_wait<5 * TW + OWN + 1>();   // capsule i + 3's x has landed before the barrier
        __syncthreads();
      }
      }
    };
    auto step = [&](int i, f16v (&ucur)[TW], f16v (&unext)[TW]) __attribute__((always_inline)) {
      const bool more = i + 1 < i1;
      if constexpr (XL)   // x of capsule i + 3 into the buffer capsule i + 1's x left
        x_dma(xs_b, A.xplane_b, xsrc(i + 3), wv, xbuf(i + 3));
      if (more) {   // capsule i + 1's tiles on the matrix cores (operands of i + 2 streamed in)
        const int in = min(i + 2, i1 - 1);
        pose_prog<DIN, TW, XL>(fr, ones, unext, rs, wvo, bvo,
                               x_voff<DIN>(in, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h, A.wplane_b,
                               A.xplane_b, A.zero_off, (uint32_t)in * A.JDp * DIN * 2, (uint32_t)in * A.JDp * 8,
                               xbuf(i + 2) + lane * 16);
      }
      // finish capsule i: softmax over all waves' rows, couplings, s += c u
      float M, Z;
      {
        constexpr int HW = NW / 2;
        const float2* slot = st + par * NW * 32;
        float2 sv[HW];
#pragma unroll
        for (int w = 0; w < HW; ++w) sv[w] = slot[(h * HW + w) * 32 + r];
        float mh = sv[0].x;
#pragma unroll
        for (int w = 1; w < HW; ++w) mh = fmaxf(mh, sv[w].x);
        float zh = 0.f;
#pragma unroll
        for (int w = 0; w < HW; ++w) zh += sv[w].y * __expf(sv[w].x - mh);
        float m0, m1, z0, z1;
        xpair32(mh, m0, m1);
        xpair32(zh, z0, z1);
        M = fmaxf(m0, m1);
        Z = z0 * __expf(m0 - M) + z1 * __expf(m1 - M);
      }
      const float sc = __expf(m - M) * __builtin_amdgcn_rcpf(Z);   // Z >= 1: 1-ulp v_rcp
#pragma unroll
      for (int a = 0; a < OWN; ++a)
        bstore(crs, fvalid ? e[a] * sc : 0.f, (uint32_t)((j0 + h + 2 * a) * A.Fs + f) * 4u,
               (uint32_t)i * A.JP * A.Fs * 4u);
      bstore(lzs, M + __builtin_amdgcn_logf(Z) * 0.69314718f, (h == 0 && wv == 0 && fvalid) ? (uint32_t)f * 4u : kNoStore,
             (uint32_t)i * A.Fs * 4u);
      float c[CP];
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        float c0, c1;
        xpair32(e[a] * sc, c0, c1);
        c[2 * a] = c0;
        c[2 * a + 1] = c1;
      }
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int v = 0; v < 16; v += 2) {
          const float cv = c[kpart<DOUT>(t, v)];
          f2 a2 = {acc[t][v], acc[t][v + 1]};
          a2 += f2{cv, cv} * f2{ucur[t][v], ucur[t][v + 1]};
          acc[t][v] = a2.x;
          acc[t][v + 1] = a2.y;
        }
      if (more) {   // capsule i + 1's logits and stats, then the one barrier
        par ^= 1;
        logits(unext, par);
        if constexpr (XL) xl_wait<5 * TW + OWN + 1>();   // capsule i + 3's x has landed before the barrier
        __syncthreads();
      }
    };
    if constexpr (XL && SRF_DR_IL) {
      for (int i = i0; i < i1; i += 2) {
        step_il(i, uc, un);
        if (i + 1 < i1) step_il(i + 1, un, uc);
      }
    } else {
      for (int i = i0; i < i1; i += 2) {
        step(i, uc, un);
        if (i + 1 < i1) step(i + 1, un, uc);
      }
    }
    if constexpr (XL) xl_wait();   // no DMA into LDS outlives the workgroup
  }
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      if (fvalid && row < JD) {
        f4 v = {acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
        *reinterpret_cast<f4*>(A.slab + ((size_t)chunk * A.F + f) * JD + row) = v * inv;
      }
    }
}

// ------------------------------------------------------------------ backward pass
// Backward routing pass r >= 1 (the adjoint of _loop_body, naive:199-206), on the
// forward's tiles and split-bf16 pose.  The couplings c^r come from the forward
// (Args32::cst), so no logit is recomputed:
//   q_ij = <gs_j, u_ij>,  sigma_i = sum_j c_ij q_ij,  gL_ij = c_ij (q_ij - sigma_i),
//   gVc_j (partial over the i-chunk) = sum_i gL_ij u_ij      -> slab
//   stats[f][i] = (logZ_i, sigma_i)                            (for the gu pass)
// gs^r rows live in each wave's private LDS slab in fragment order (as Vc in the
// forward); sigma needs one cross-wave sum per input capsule (one barrier).
struct Bwd32Args {
  const float* cst;   // c^r [in_n][JP][Fs]
  const float* lz;    // logZ^r [in_n][Fs]
  const float* gs;    // gs^r [F][JD]
  float* stats;       // [F][in_n][2]
  float* glst;        // gL^r [in_n][JP][Fs] (laid out as c^r), for the gu pass
};

// the owned couplings j0 + 2a + h of one capsule i (p points at capsule j0 + h, frame f)
template <int OWN>
__device__ __forceinline__ void load_c(const float* __restrict__ p, size_t fs, float (&c)[OWN]) {
#pragma unroll
  for (int a = 0; a < OWN; ++a) c[a] = p[2 * a * fs];
}

template <int DIN, int DOUT, int NW, int TW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(kWavesPerEU))) void route_bwd32_kernel(
    Args32 A, Bwd32Args Bk) {
  constexpr int CP = TW * 32 / DOUT;
  constexpr int OWN = CP / 2;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int JD = A.J * DOUT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);   // wave index in an SGPR (stats slots)
  const int r = lane & 31, h = lane >> 5;
  const int bid = blockIdx.x;
  const int ft = bid / A.n_chunks, chunk = bid - ft * A.n_chunks;
  const int f = ft * 32 + r;
  const int fc = min(f, A.F - 1);
  const int fb = fc / A.T, ftt = fc - fb * A.T;
  const bool fvalid = f < A.F;
  const int i0 = chunk * A.chunk_len, i1 = min(A.in_n, i0 + A.chunk_len);
  const int tbase = __builtin_amdgcn_readfirstlane(wv * TW);
  const int j0 = tbase * 32 / DOUT;
  const Rsrc3 rs{make_rsrc(A.Ws, A.ws_bytes), make_rsrc(A.bs, A.bs_bytes), make_rsrc(A.xs, A.xs_bytes)};
  if (DIN <= 16 && NW > 1 && wv >= NW / 2) __builtin_amdgcn_s_setprio(1);   // din 32: measured faster without
  const uint32_t wvo = (uint32_t)(((tbase * 32 + r) * DIN + (DIN >= 16 ? 8 * h : 0)) * 2);
  const uint32_t bvo = (uint32_t)((tbase * 32 + r) * 8);
  // logZ^r through a buffer descriptor: a 32-bit lane offset instead of a 64-bit
  // pointer held across the capsule loop (which spilled, its reload's vmcnt(0) draining
  // the operand prefetch)
  const __amdgpu_buffer_rsrc_t lzr = make_rsrc(Bk.lz, (size_t)A.in_n * A.Fs * 4);

  f4* gsl = reinterpret_cast<f4*>(lds) + (size_t)wv * TW * 4 * 64;
  float* st = lds + (size_t)NW * TW * 4 * 64 * 4;
  // din 32: shared x fragments read just in time, as route_fwd32_kernel
  constexpr bool XJ = DIN == 32 && NW > 1;
  __shared__ __attribute__((aligned(16))) char xls[XJ ? 2 * 4 * kXlPiece : 16];
  const char* xs_b = static_cast<const char*>(A.xs);
  auto xsrc = [&](int c) { return x_voff<DIN>(min(c, i1 - 1), A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off); };
  auto xbuf = [&](int c) { return xls + (c & 1) * 4 * kXlPiece; };
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (fvalid && row < JD) v = *reinterpret_cast<const f4*>(Bk.gs + (size_t)f * JD + row);
      gsl[(t * 4 + q) * 64 + lane] = v;
    }
  const bf8 ones = ones_frag(h);
  const float inv = A.hdr[0];   // 2^-(aw+bx): the pose tiles hold 2^(aw+bx) u
  f16v acc[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) acc[t] = f16v{};
  const float* crow = Bk.cst + (size_t)(j0 + h) * A.Fs + fc;
  const __amdgpu_buffer_rsrc_t sts = make_rsrc(Bk.stats, (size_t)A.F * A.in_n * 8);
  const size_t cstep = (size_t)A.JP * A.Fs;   // next capsule i
  int par = 0;
  if (i0 < i1) {
    Frags32<DIN, TW> fr;
    fetch32<DIN, TW, true>(rs, wvo, bvo, x_voff<DIN>(i0, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                           A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)i0 * A.JDp * DIN * 2, (uint32_t)i0 * A.JDp * 8,
                           fr);
    if constexpr (XJ) {   // x of capsules i0, i0 + 1 before the first pose
      x_dma(xs_b, A.xplane_b, xsrc(i0), wv, xbuf(i0));
      x_dma(xs_b, A.xplane_b, xsrc(i0 + 1), wv, xbuf(i0 + 1));
      xl_wait();
      __syncthreads();
    }
    for (int i = i0; i < i1; ++i) {
      f16v u[TW];
      // partial dots <u_ij, gs_j> over this lane's rows
      f2 P2[CP];
#pragma unroll
      for (int k = 0; k < CP; ++k) P2[k] = f2{0.f, 0.f};
      float cc[OWN];
      if constexpr (DIN <= 16) {   // tile-major pose; din 32: pose_prog measured faster (C4 A/B)
      // this capsule's couplings, then the tile-major pose with the dots of tile t - 1
      // behind tile t's MFMAs (as route_fwd32_kernel)
      load_c<OWN>(crow + (size_t)i * cstep, A.Fs, cc);
      {
        constexpr uint32_t TSTEP = 32 * DIN * 2;
        const int in = min(i + 1, i1 - 1);
        const uint32_t wcap = (uint32_t)in * A.JDp * DIN * 2, bcap = (uint32_t)in * A.JDp * 8;
        const uint32_t xvn = x_voff<DIN>(in, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off);
        f4 gq[4];
        auto dots = [&](int t) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int k = kpart<DOUT>(t, 4 * q);
            P2[k] += f2{u[t][4 * q], u[t][4 * q + 1]} * f2{gq[q].x, gq[q].y};
            P2[k] += f2{u[t][4 * q + 2], u[t][4 * q + 3]} * f2{gq[q].z, gq[q].w};
          }
        };
#pragma unroll
        for (int t = 0; t < TW; ++t) {
          if (t > 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) gq[q] = gsl[((t - 1) * 4 + q) * 64 + lane];
          }
          __builtin_amdgcn_sched_barrier(0);
          u[t] = pose_chain<DIN>(fr.a[t], fr.b, mfma32(fr.bias[t], ones, f16v{}));
          __builtin_amdgcn_sched_barrier(0);
          fetch_w<DIN>(rs, wvo + t * TSTEP, h, A.wplane_b, wcap, fr.a[t]);
          {
            const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rs.b, bvo + t * 32 * 8, bcap, 0);
            fr.bias[t] = __builtin_bit_cast(bf8, (unsigned __attribute__((ext_vector_type(4)))){v2[0], v2[1], 0u, 0u});
          }
          if (t == TW - 1) fetch_x<DIN>(rs, xvn, h, A.xplane_b, A.zero_off, fr.b);
          __builtin_amdgcn_sched_barrier(0);
          if (t > 0) dots(t - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) gq[q] = gsl[((TW - 1) * 4 + q) * 64 + lane];
        dots(TW - 1);
      }
      } else {
      const int in = min(i + 1, i1 - 1);
      pose_prog<DIN, TW, XJ, XJ>(fr, ones, u, rs, wvo, bvo,
                                 x_voff<DIN>(in, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                                 A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)in * A.JDp * DIN * 2,
                                 (uint32_t)in * A.JDp * 8, xbuf(i) + lane_asm() * 16);
      // this capsule's couplings: the pose MFMAs in flight hide their latency (no
      // registers held across capsules)
      load_c<OWN>(crow + (size_t)i * cstep, A.Fs, cc);
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 gv = gsl[(t * 4 + q) * 64 + lane];
          const int k = kpart<DOUT>(t, 4 * q);
          P2[k] += f2{u[t][4 * q], u[t][4 * q + 1]} * f2{gv.x, gv.y};
          P2[k] += f2{u[t][4 * q + 2], u[t][4 * q + 3]} * f2{gv.z, gv.w};
        }
      }
      float Q[OWN];
      float sp = 0.f;
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        const float pa = P2[2 * a].x + P2[2 * a].y, pb = P2[2 * a + 1].x + P2[2 * a + 1].y;
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(pa), __float_as_uint(pb), false, false);
        Q[a] = (__uint_as_float(sw[0]) + __uint_as_float(sw[1])) * inv;
        sp += cc[a] * Q[a];
      }
      float S;
      {
        float s0, s1;
        xpair32(sp, s0, s1);
        S = s0 + s1;
      }
      if constexpr (NW > 1) {
        int lid;   // the slot addresses from the lane id, as route_fwd32_kernel
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
        const int sr = lid & 31, shf = lid >> 5;
        float* slot = st + par * NW * 32;
        if (shf == 0) slot[wvu * 32 + sr] = S;
        if constexpr (XJ) xl_wait();   // x of capsule i + 1 lands before the barrier that publishes it
        __syncthreads();
        if constexpr (XJ) x_dma(xs_b, A.xplane_b, xsrc(i + 2), wv, xbuf(i + 2));   // into capsule i's buffer
        constexpr int HW = NW / 2;
        float sh = 0.f;
#pragma unroll
        for (int w = 0; w < HW; ++w) sh += slot[(shf * HW + w) * 32 + sr];
        float s0, s1;
        xpair32(sh, s0, s1);
        S = s0 + s1;
        par ^= 1;
      }
      // logZ of capsule i before the next capsule's operand loads: waiting for it at its
      // store then leaves those (younger) loads in flight
      const float lzv =
          __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lzr, (uint32_t)fc * 4u, (uint32_t)i * A.Fs * 4u, 0));
      __builtin_amdgcn_sched_barrier(0);
      {
        // (logZ, sigma) of frame f, capsule i: branch-free (wave 0, half 0, valid frames)
        __builtin_amdgcn_raw_buffer_store_b64(
            (unsigned __attribute__((ext_vector_type(2)))){__float_as_uint(lzv), __float_as_uint(S)}, sts,
            (wv == 0 && h == 0 && fvalid) ? (uint32_t)(f * A.in_n) * 8u : kNoStore, (uint32_t)i * 8u, 0);
      }
      // gL of the owned capsules (stored for the gu pass), then all-gather over the lane halves
      float gown[OWN];
#pragma unroll
      for (int a = 0; a < OWN; ++a) gown[a] = cc[a] * (Q[a] - S);
      {
        float* dst = Bk.glst + ((size_t)i * A.JP + j0 + h) * A.Fs + f;   // 0 past F, as the couplings
#pragma unroll
        for (int a = 0; a < OWN; ++a) dst[(size_t)2 * a * A.Fs] = fvalid ? gown[a] : 0.f;
      }
      float g[CP];
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        float g0, g1;
        xpair32(gown[a], g0, g1);
        g[2 * a] = g0;
        g[2 * a + 1] = g1;
      }
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int v = 0; v < 16; v += 2) {
          const float gv = g[kpart<DOUT>(t, v)];
          f2 a2 = {acc[t][v], acc[t][v + 1]};
          a2 += f2{gv, gv} * f2{u[t][v], u[t][v + 1]};
          acc[t][v] = a2.x;
          acc[t][v + 1] = a2.y;
        }
    }
  }
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      if (fvalid && row < JD) {
        f4 v = {acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
        *reinterpret_cast<f4*>(A.slab + ((size_t)chunk * A.F + f) * JD + row) = v * inv;
      }
    }
}


// Backward pass r >= 1, software-pipelined as route_fwd32p_kernel: capsule i + 1's
// pose tiles run on the matrix cores while the VALU finishes capsule i (sigma over all
// waves from behind last iteration's barrier, the stats / gL stores, gVc += gL u).
template <int DIN, int DOUT, int NW, int TW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(kWavesPerEU))) void route_bwd32p_kernel(
    Args32 A, Bwd32Args Bk) {
  constexpr int CP = TW * 32 / DOUT;
  constexpr int OWN = CP / 2;
  static_assert(NW > 1, "the pipelined pass exchanges sigma partials between waves");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int JD = A.J * DOUT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int bid = blockIdx.x;
  const int ft = bid / A.n_chunks, chunk = bid - ft * A.n_chunks;
  const int f = ft * 32 + r;
  const int fc = min(f, A.F - 1);
  const int fb = fc / A.T, ftt = fc - fb * A.T;
  const bool fvalid = f < A.F;
  const int i0 = chunk * A.chunk_len, i1 = min(A.in_n, i0 + A.chunk_len);
  const int tbase = __builtin_amdgcn_readfirstlane(wv * TW);
  const int j0 = tbase * 32 / DOUT;
  const Rsrc3 rs{make_rsrc(A.Ws, A.ws_bytes), make_rsrc(A.bs, A.bs_bytes), make_rsrc(A.xs, A.xs_bytes)};
  const uint32_t wvo = (uint32_t)(((tbase * 32 + r) * DIN + (DIN >= 16 ? 8 * h : 0)) * 2);
  const uint32_t bvo = (uint32_t)((tbase * 32 + r) * 8);
  f4* gsl = reinterpret_cast<f4*>(lds) + (size_t)wv * TW * 4 * 64;
  float* st = lds + (size_t)NW * TW * 4 * 64 * 4;
  // din 32: two buffers of the shared x fragments (x_dma) after the sigma partials
  constexpr bool XL = DIN == 32;
  // a separate LDS object: the compiler then sees no DMA aliasing the gs / sigma LDS
  __shared__ __attribute__((aligned(16))) char xls[XL ? 2 * 4 * kXlPiece : 16];
  char* xb = xls;
  const char* xs_b = static_cast<const char*>(A.xs);
  auto xsrc = [&](int c) { return x_voff<DIN>(min(c, i1 - 1), A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off); };
  auto xbuf = [&](int c) { return xb + (c & 1) * 4 * kXlPiece; };
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (fvalid && row < JD) v = *reinterpret_cast<const f4*>(Bk.gs + (size_t)f * JD + row);
      gsl[(t * 4 + q) * 64 + lane] = v;
    }
  const bf8 ones = ones_frag(h);
  const float inv = A.hdr[0];
  f16v acc[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) acc[t] = f16v{};
  const float* crow = Bk.cst + (size_t)(j0 + h) * A.Fs + fc;
  const __amdgpu_buffer_rsrc_t sts = make_rsrc(Bk.stats, (size_t)A.F * A.in_n * 8);
  const size_t cstep = (size_t)A.JP * A.Fs;
  if (i0 < i1) {
    Frags32<DIN, TW> fr;
    fetch32<DIN, TW, true>(rs, wvo, bvo, x_voff<DIN>(i0, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                           A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)i0 * A.JDp * DIN * 2, (uint32_t)i0 * A.JDp * 8,
                           fr);
    f16v uc[TW], un[TW];
    float cc[OWN], cn[OWN], Q[OWN];   // couplings of the pending / next capsule; the pending capsule's q
    // q = <gs_j, u_ij> of the owned capsules, the wave's sigma partial -> LDS slot
    auto dots = [&](const f16v (&u)[TW], const float (&c)[OWN], int slot_par) {
      f2 P2[CP];
#pragma unroll
      for (int k = 0; k < CP; ++k) P2[k] = f2{0.f, 0.f};
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 gv = gsl[(t * 4 + q) * 64 + lane];
          const int k = kpart<DOUT>(t, 4 * q);
          P2[k] += f2{u[t][4 * q], u[t][4 * q + 1]} * f2{gv.x, gv.y};
          P2[k] += f2{u[t][4 * q + 2], u[t][4 * q + 3]} * f2{gv.z, gv.w};
        }
      float sp = 0.f;
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        const float pa = P2[2 * a].x + P2[2 * a].y, pb = P2[2 * a + 1].x + P2[2 * a + 1].y;
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(pa), __float_as_uint(pb), false, false);
        Q[a] = (__uint_as_float(sw[0]) + __uint_as_float(sw[1])) * inv;
        sp += c[a] * Q[a];
      }
      float s0, s1;
      xpair32(sp, s0, s1);
      if (h == 0) st[(slot_par * NW + wv) * 32 + r] = s0 + s1;
    };
    int par = 0;
    if constexpr (XL) {   // x of capsules i0 + 1, i0 + 2 into LDS before the first pose
      x_dma(xs_b, A.xplane_b, xsrc(i0 + 1), wv, xbuf(i0 + 1));
      x_dma(xs_b, A.xplane_b, xsrc(i0 + 2), wv, xbuf(i0 + 2));
      xl_wait();
      __syncthreads();
    }
    load_c<OWN>(crow + (size_t)i0 * cstep, A.Fs, cc);
    pose_prog<DIN, TW, XL>(fr, ones, uc, rs, wvo, bvo,
                           x_voff<DIN>(min(i0 + 1, i1 - 1), A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h,
                           A.wplane_b, A.xplane_b, A.zero_off, (uint32_t)min(i0 + 1, i1 - 1) * A.JDp * DIN * 2,
                           (uint32_t)min(i0 + 1, i1 - 1) * A.JDp * 8, xbuf(i0 + 1) + lane * 16);
    dots(uc, cc, par);
    __syncthreads();
    // one capsule, as route_fwd32p_kernel's step: two steps per loop turn with the roles of
    // (uc, cc) and (un, cn) swapped, so no copies
    // IL: capsule i's finish between capsule i + 1's pose MFMAs (pose_prog32i)
    auto step_il = [&](int i, f16v (&ucur)[TW], f16v (&unext)[TW], float (&ccur)[OWN], float (&cnext)[OWN])
        __attribute__((always_inline)) {
      if constexpr (DIN == 32) {
      const bool more = i + 1 < i1;
      x_dma(xs_b, A.xplane_b, xsrc(i + 3), wv, xbuf(i + 3));   // into the buffer capsule i + 1's x left
      const float lzv = Bk.lz[(size_t)i * A.Fs + fc];
      load_c<OWN>(crow + (size_t)min(i + 1, i1 - 1) * cstep, A.Fs, cnext);
      constexpr int HW = NW / 2;
      float sv[HW];
      float g[CP];
      auto gfma = [&](int t0, int t1) __attribute__((always_inline)) {
#pragma unroll
        for (int t = t0; t < t1; ++t) {
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[t][v] = fmaf(g[kpart<DOUT>(t, v)], ucur[t][v], acc[t][v]);
          asm volatile("" : "+v"(acc[t]));   // keeps the FMAs in their MFMA region
        }
      };
      auto fill = [&](auto stage) __attribute__((always_inline)) {
        constexpr int S = decltype(stage)::value;
        if constexpr (S == 0) {   // capsule i's sigma partials of the 4 waves of this lane half
          const float* slot = st + par * NW * 32;
#pragma unroll
          for (int w = 0; w < HW; ++w) sv[w] = slot[(h * HW + w) * 32 + r];
        } else if constexpr (S == 1) {
          float sh = 0.f;
#pragma unroll
          for (int w = 0; w < HW; ++w) sh += sv[w];
          float s0, s1;
          xpair32(sh, s0, s1);
          const float Sg = s0 + s1;
          __builtin_amdgcn_raw_buffer_store_b64(
              (unsigned __attribute__((ext_vector_type(2)))){__float_as_uint(lzv), __float_as_uint(Sg)}, sts,
              (wv == 0 && h == 0 && fvalid) ? (uint32_t)(f * A.in_n) * 8u : kNoStore, (uint32_t)i * 8u, 0);
          float gown[OWN];
#pragma unroll
          for (int a = 0; a < OWN; ++a) gown[a] = ccur[a] * (Q[a] - Sg);
          float* dst = Bk.glst + ((size_t)i * A.JP + j0 + h) * A.Fs + f;
#pragma unroll
          for (int a = 0; a < OWN; ++a) dst[(size_t)2 * a * A.Fs] = fvalid ? gown[a] : 0.f;
#pragma unroll
          for (int a = 0; a < OWN; ++a) {
            float g0, g1;
            xpair32(gown[a], g0, g1);
            g[2 * a] = g0;
            g[2 * a + 1] = g1;
          }
        } else if constexpr (S == 2) {
          gfma(0, TW / 2);
        } else {
          gfma(TW / 2, TW);
        }
      };
      {   // the next capsules' loads and pose run unconditionally (the chunk's last capsule
          // re-reads itself, its pose unused), as in step
        const int in = min(i + 2, i1 - 1);
        pose_prog32i<TW, 4, 6, 6>(fr, ones, unext, rs, wvo, bvo, A.wplane_b, (uint32_t)in * A.JDp * DIN * 2,
                                  (uint32_t)in * A.JDp * 8, xbuf(i + 2) + lane * 16, fill);
      }
      if (more) {
        par ^= 1;
        dots(unext, cnext, par);
        xl_wait<1 + OWN + 5 * TW + 1 + OWN>();   // capsule i + 3's x has landed
        __syncthreads();
      }
      }
    };
    auto step = [&](int i, f16v (&ucur)[TW], f16v (&unext)[TW], float (&ccur)[OWN], float (&cnext)[OWN])
        __attribute__((always_inline)) {
      const bool more = i + 1 < i1;
      if constexpr (XL)   // x of capsule i + 3 into the buffer capsule i + 1's x left
        x_dma(xs_b, A.xplane_b, xsrc(i + 3), wv, xbuf(i + 3));
      // logZ of capsule i before the next capsule's loads: waiting for it at its store
      // then leaves those (younger) loads in flight
      const float lzv = Bk.lz[(size_t)i * A.Fs + fc];
      // the next capsules' loads and pose run unconditionally (the chunk's last capsule
      // re-reads itself, its pose unused): with a branch around them the compiler cannot
      // count the loads in flight and waits for all of them at the stores below
      {
        load_c<OWN>(crow + (size_t)min(i + 1, i1 - 1) * cstep, A.Fs, cnext);
        const int in = min(i + 2, i1 - 1);
        pose_prog<DIN, TW, XL>(fr, ones, unext, rs, wvo, bvo,
                               x_voff<DIN>(in, A.N, A.lpad, A.T, A.F, f, ftt, fvalid, h, A.zero_off), h, A.wplane_b,
                               A.xplane_b, A.zero_off, (uint32_t)in * A.JDp * DIN * 2, (uint32_t)in * A.JDp * 8,
                               xbuf(i + 2) + lane * 16);
      }
      // finish capsule i: sigma over all waves, stats, gL, gVc += gL u
      float S;
      {
        constexpr int HW = NW / 2;
        const float* slot = st + par * NW * 32;
        float sh = 0.f;
#pragma unroll
        for (int w = 0; w < HW; ++w) sh += slot[(h * HW + w) * 32 + r];
        float s0, s1;
        xpair32(sh, s0, s1);
        S = s0 + s1;
      }
      __builtin_amdgcn_raw_buffer_store_b64(
          (unsigned __attribute__((ext_vector_type(2)))){__float_as_uint(lzv), __float_as_uint(S)}, sts,
          (wv == 0 && h == 0 && fvalid) ? (uint32_t)(f * A.in_n) * 8u : kNoStore, (uint32_t)i * 8u, 0);
      float gown[OWN];
#pragma unroll
      for (int a = 0; a < OWN; ++a) gown[a] = ccur[a] * (Q[a] - S);
      {
        float* dst = Bk.glst + ((size_t)i * A.JP + j0 + h) * A.Fs + f;
#pragma unroll
        for (int a = 0; a < OWN; ++a) dst[(size_t)2 * a * A.Fs] = fvalid ? gown[a] : 0.f;
      }
      float g[CP];
#pragma unroll
      for (int a = 0; a < OWN; ++a) {
        float g0, g1;
        xpair32(gown[a], g0, g1);
        g[2 * a] = g0;
        g[2 * a + 1] = g1;
      }
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int v = 0; v < 16; v += 2) {
          const float gv = g[kpart<DOUT>(t, v)];
          f2 a2 = {acc[t][v], acc[t][v + 1]};
          a2 += f2{gv, gv} * f2{ucur[t][v], ucur[t][v + 1]};
          acc[t][v] = a2.x;
          acc[t][v + 1] = a2.y;
        }
      if (more) {
        par ^= 1;
        dots(unext, cnext, par);
        if constexpr (XL) xl_wait<1 + OWN + 5 * TW + 1 + OWN>();   // capsule i + 3's x has landed
        __syncthreads();
      }
    };
    if constexpr (XL && SRF_DR_IL) {
      for (int i = i0; i < i1; i += 2) {
        step_il(i, uc, un, cc, cn);
        if (i + 1 < i1) step_il(i + 1, un, uc, cn, cc);
      }
    } else {
      for (int i = i0; i < i1; i += 2) {
        step(i, uc, un, cc, cn);
        if (i + 1 < i1) step(i + 1, un, uc, cn, cc);
      }
    }
    if constexpr (XL) xl_wait();   // no DMA into LDS outlives the workgroup
  }
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (tbase + t) * 32 + 8 * q + 4 * h;
      if (fvalid && row < JD) {
        f4 v = {acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
        *reinterpret_cast<f4*>(A.slab + ((size_t)chunk * A.F + f) * JD + row) = v * inv;
      }
    }
}

}  // namespace

namespace srf {

bool fwd32_supported(int din, int dout, int J) {
  return (din == 8 || din == 16 || din == 32) && (dout == 8 || dout == 16 || dout == 32) && din <= dout &&
         J * dout <= 32 * kTW * kMaxNW && (J * dout) % 8 == 0;
}

// Row tiles per wave: kTW, except (a) din 32 with J*dout <= 512, where the six-MFMA
// pose keeps 2 tiles per wave (4 measured the same at C4), and (b) small din <= 16
// layers (J*dout <= 128, C2 layers 1-2), which run 2 tiles on each of two waves
// instead of 4 on one: twice the waves on the one-wave-per-SIMD grid, the softmax
// across the pair through LDS (C2 step -0.5 to -1 %)
static int plan_tw(int din, int JD) {
  if (din <= 16) return JD <= 128 ? 2 : kTW;
  return (din == 32 && JD <= 32 * 2 * kMaxNW) ? 2 : kTW;
}

Fwd32Plan fwd32_plan(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int n_chunks) {
  Fwd32Plan p;
  const int in_n = N * (lpad + rpad + 1);
  const int JD = J * dout;
  const int NT = (JD + 31) / 32;
  p.TW = plan_tw(din, JD);
  p.NW = 1;
  while (p.NW * p.TW < NT) p.NW *= 2;
  p.JDp = p.NW * p.TW * 32;
  p.xpad = din == 32 ? 32 : 16;
  const int F = B * T;
  const int n_ftiles = (F + 31) / 32;
  // NW > 1: as many workgroups per CU as the waves (2 per SIMD) and the LDS (Vc
  // slabs) allow; single-wave workgroups: up to 4 per CU.
  const int per_cu = std::max(1, std::min(8 / p.NW, (int)(160 * 1024 / fwd32_lds(p))));
  const int slots = p.NW > 1 ? 256 * per_cu : 1024;
  int best = 1;
  double best_cost = 1e30;
  const int forced = n_chunks;
  for (int c = 1; c <= std::min(in_n, 96); ++c) {
    const int rounds = (n_ftiles * c + slots - 1) / slots;
    const int len = (in_n + c - 1) / c;
    double cost = (double)rounds * (len + 3) * (1.0 + 0.002 * c);
    if (forced > 0) cost = (c == std::min(forced, in_n)) ? 0.0 : 1.0;
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  p.n_chunks = best;
  p.chunk_len = (in_n + best - 1) / best;
  p.n_ftiles = n_ftiles;
  p.xplane = (size_t)F * N * din + p.xpad;
  p.ws_w = srf::align_up((size_t)2 * in_n * p.JDp * din * 2, 256);
  p.ws_b = srf::align_up((size_t)in_n * p.JDp * 4 * 2, 256);
  p.ws_x = srf::align_up((size_t)2 * p.xplane * 2, 256);
  p.ws_h = (size_t)(2 * kAbsBlocks + 64) * 4;   // header + absmax block maxima
  p.ws_bsum = srf::align_up((size_t)best * JD * 4, 256);
  p.ws_slab = srf::align_up((size_t)best * F * JD * 4, 256);
  return p;
}

const float* fwd32_hdr(const Fwd32Plan& p, const void* planes) {
  return reinterpret_cast<const float*>(static_cast<const char*>(planes) + p.ws_w + p.ws_b + p.ws_x);
}
size_t fwd32_planes_bytes(const Fwd32Plan& p) { return p.ws_w + p.ws_b + p.ws_x + p.ws_h; }
size_t fwd32_scratch_bytes(const Fwd32Plan& p) { return p.ws_bsum + p.ws_slab; }
size_t fwd32_workspace(const Fwd32Plan& p) { return fwd32_planes_bytes(p) + fwd32_scratch_bytes(p); }
float* fwd32_slab(const Fwd32Plan& p, void* scratch) {
  return reinterpret_cast<float*>(static_cast<char*>(scratch) + p.ws_bsum);
}

size_t fwd32_lds(const Fwd32Plan& p) {
  // Vc / gs fragment slabs and softmax statistics (the pipelined din-32 passes add their
  // two shared x buffers, 8 KiB, as a static LDS object)
  return (size_t)p.NW * p.TW * 4 * 64 * 16 + (p.NW > 1 ? (size_t)2 * 32 * p.NW * 8 : 0);
}

int fwd32_prepare(const Fwd32Plan& p, const float* emb, const float* W, const float* bias, int B, int T, int N,
                  int din, int lpad, int rpad, int J, int dout, void* planes, void* scratch, float* WT, float* xT,
                  hipStream_t st, bool wt16, bool xt16) {
  char* base = static_cast<char*>(planes);
  float* hdr = reinterpret_cast<float*>(base + p.ws_w + p.ws_b + p.ws_x);
  const int in_n = N * (lpad + rpad + 1);
  hipLaunchKernelGGL(absmax_kernel, dim3(kAbsBlocks, 2), dim3(256), 0, st, W, (size_t)in_n * J * dout * din, emb,
                     (size_t)B * T * N * din, hdr + 64);
  SRF_LAUNCH_CHECK("absmax");
  PrepArgs P;
  P.W = W;
  P.bias = bias;
  P.emb = emb;
  P.Ws = reinterpret_cast<_Float16*>(base);
  P.bs = reinterpret_cast<__bf16*>(base + p.ws_w);
  P.xs = reinterpret_cast<_Float16*>(base + p.ws_w + p.ws_b);
  P.part = hdr + 64;
  P.hdr = hdr;
  P.bsum = reinterpret_cast<float*>(scratch);
  P.WT = WT;
  P.xT = xT;
  P.T = T;
  P.lpad = lpad;
  P.Fp = (B * T + 15) / 16 * 16;
  P.in_n = N * (lpad + rpad + 1);
  P.JD = J * dout;
  P.JDp = p.JDp;
  P.din = din;
  P.n_chunks = p.n_chunks;
  P.chunk_len = p.chunk_len;
  P.F = B * T;
  P.N = N;
  P.xplane = p.xplane;
  P.n_a = (size_t)P.in_n * p.JDp * din / 8;
  P.n_b = (size_t)P.in_n * p.JDp;
  P.n_c = (size_t)p.n_chunks * P.JD;
  P.n_d = p.xplane / 8;
  SRF_REQUIRE(!wt16 || din == 32, "prep32: split W^T planes need din 32, got %d", din);
  P.wt16 = wt16 ? 1 : 0;
  SRF_REQUIRE(!xt16 || din == 32, "prep32: split x^T planes need din 32, got %d", din);
  P.xt16 = xt16 ? 1 : 0;
  P.n_e = WT ? (size_t)P.in_n * ((P.JD + 15) / 16) * (wt16 ? 2 : 4) * din : 0;
  SRF_REQUIRE(din <= 32, "prep32: xT tile holds din <= 32, got %d", din);
  P.n_f = xT ? (size_t)P.in_n * ((P.Fp + kXtTile - 1) / kXtTile) : 0;   // xT tiles (one block each)
  P.xt_block0 = (P.n_a + P.n_b + P.n_c + P.n_d + P.n_e + 255) / 256;
  hipLaunchKernelGGL(prep32_kernel, dim3(P.xt_block0 + P.n_f), dim3(256), 0, st, P);
  SRF_LAUNCH_CHECK("prep32");
  return SRF_OK;
}

template <int DIN, int DOUT, int NW, int TW = kTW>
static int launch_rpass(const Fwd32Plan& p, const Args32& a, hipStream_t st) {
  const size_t lds = fwd32_lds(p);
  // the pipelined pass holds a second u set: TW = 4 would spill
  auto kern = (NW > 1 && TW <= 2) ? route_fwd32p_kernel<DIN, DOUT, (NW > 1 ? NW : 2), (TW <= 2 ? TW : 2)>
                                                    : route_fwd32_kernel<DIN, DOUT, NW, TW>;
  if (lds > 64 * 1024)
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(p.n_ftiles * p.n_chunks), dim3(64 * NW), lds, st, a);
  SRF_LAUNCH_CHECK("route_fwd32");
  return SRF_OK;
}

template <int DIN, int DOUT>
static int launch_pass32_t(const Fwd32Plan& p, bool first, const Args32& a, hipStream_t st) {
  if (first) {
    Args32 b = a;
    b.n_tgroups = p.JDp / (32 * kFTW);
    const int tasks = (p.n_ftiles + kFFB - 1) / kFFB * b.n_tgroups * p.n_chunks;
    hipLaunchKernelGGL((route_fwd32_first_kernel<DIN, DOUT>), dim3((tasks + 3) / 4), dim3(256), 0, st, b);
    SRF_LAUNCH_CHECK("route_fwd32_first");
    return SRF_OK;
  }
  if constexpr (DIN <= 16) {
    if (p.TW == 2) return p.NW == 1 ? launch_rpass<DIN, DOUT, 1, 2>(p, a, st) : launch_rpass<DIN, DOUT, 2, 2>(p, a, st);
  }
  if constexpr (DIN == 32) {
    if (p.TW == 2) {
      switch (p.NW) {
        case 1: return launch_rpass<DIN, DOUT, 1, 2>(p, a, st);
        case 2: return launch_rpass<DIN, DOUT, 2, 2>(p, a, st);
        case 4: return launch_rpass<DIN, DOUT, 4, 2>(p, a, st);
        default: return launch_rpass<DIN, DOUT, 8, 2>(p, a, st);
      }
    }
  }
  switch (p.NW) {
    case 1: return launch_rpass<DIN, DOUT, 1>(p, a, st);
    case 2: return launch_rpass<DIN, DOUT, 2>(p, a, st);
    case 4: return launch_rpass<DIN, DOUT, 4>(p, a, st);
    case 8: return launch_rpass<DIN, DOUT, 8>(p, a, st);
    default: return launch_rpass<DIN, DOUT, kMaxNW>(p, a, st);
  }
}

static Args32 make_args32(const Fwd32Plan& p, const void* planes, void* scratch, int B, int T, int N, int din,
                          int lpad, int rpad, int J, int dout, int mask_first) {
  const int in_n = N * (lpad + rpad + 1);
  const char* base = static_cast<const char*>(planes);
  Args32 a{};
  a.Ws = base;
  a.bs = base + p.ws_w;
  a.xs = base + p.ws_w + p.ws_b;
  a.hdr = reinterpret_cast<const float*>(base + p.ws_w + p.ws_b + p.ws_x);
  a.ws_bytes = p.ws_w;
  a.bs_bytes = (size_t)in_n * p.JDp * 8;
  a.xs_bytes = 2 * p.xplane * 2;
  a.wplane_b = (uint32_t)((size_t)in_n * p.JDp * din * 2);
  a.xplane_b = (uint32_t)(p.xplane * 2);
  a.zero_off = (uint32_t)((p.xplane - p.xpad) * 2);
  a.F = B * T;
  a.T = T;
  a.N = N;
  a.lpad = lpad;
  a.in_n = in_n;
  a.J = J;
  a.JDp = p.JDp;
  a.n_chunks = p.n_chunks;
  a.chunk_len = p.chunk_len;
  a.mask_first = mask_first;
  a.n_tgroups = p.NW;
  a.vc = nullptr;
  a.bsum = reinterpret_cast<const float*>(scratch);
  a.slab = fwd32_slab(p, scratch);
  a.cst = nullptr;
  a.lzst = nullptr;
  a.JP = p.JDp / dout;
  a.Fs = fwd32_frame_stride(B * T);
  return a;
}

Fwd32Cpl fwd32_cpl_layout(const Fwd32Plan& p, int F, int in_n, int din, int dout, int J, int iters) {
  Fwd32Cpl c{};
  const size_t blk = (size_t)fwd32_frame_stride(F) * in_n;
  const int R1 = std::max(iters - 1, 0);
  c.c = 0;
  c.lz = (size_t)R1 * blk * (p.JDp / dout);
  size_t off = c.lz + (size_t)R1 * blk;
  off = (off + 63) / 64 * 64;   // 256-byte aligned regions
  c.planes = off;
  off += (fwd32_planes_bytes(p) + 255) / 256 * 64;
  c.WT = off;
  off += ((size_t)in_n * din * ((J * dout + 15) / 16 * 16) + 63) / 64 * 64;
  c.xT = off;
  off += ((size_t)in_n * din * ((F + 15) / 16 * 16) + 63) / 64 * 64;
  c.total = off;
  return c;
}

// Iteration-0 pass with its finish fused (route_fwd32_first_full_kernel): din = dout = 32.
bool fwd32_first_full_supported(const Fwd32Plan& p, int din, int dout) {
  return din == 32 && dout == 32 && p.JDp % kFfBM == 0;
}

// Frames per workgroup of the iteration-0 GEMM: the widest tile (fewest operand bytes
// staged per MFMA) that still gives every CU a workgroup -- one 128-row x BN-frame
// workgroup per CU moves 16 KiB + BN x 128 B per capsule through LDS where BN = 64
// workgroups three to a CU moved 72 KiB.  SRF_FF_BN (A/B builds) forces one.
#ifndef SRF_FF_BN
#define SRF_FF_BN 0
#endif
static int ff_frames(int n_rt, int F) {
  if (SRF_FF_BN) return SRF_FF_BN;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  for (int bn : {192, 128, 96})
    if ((long)n_rt * ((F + bn - 1) / bn) >= cus * 9 / 10) return bn;
  return 64;
}

int fwd32_first_full(const Fwd32Plan& p, const void* planes, void* scratch, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int mask_first, float* s_out, float* vc_out, float* v_out,
                     hipStream_t st) {
  SRF_REQUIRE(fwd32_first_full_supported(p, din, dout), "fwd32_first_full: din %d dout %d JDp %d", din, dout, p.JDp);
  SRF_REQUIRE(2 * p.xplane * 2 < (1ull << 31) && p.ws_w < (1ull << 31), "fwd32: operand planes exceed 2 GiB");
  const Args32 a = make_args32(p, planes, scratch, B, T, N, din, lpad, rpad, J, dout, mask_first);
  const int bn = ff_frames(p.JDp / kFfBM, B * T);
  const int nb = (p.JDp / kFfBM) * ((B * T + bn - 1) / bn);
#define SRF_FF_LAUNCH(BN)                                                                                          \
  if (bn == BN) {                                                                                                 \
    constexpr int CPS_ = BN >= 96 ? 2 : 1;                                                                        \
    const size_t lds = 2 * CPS_ * (size_t)ff_stage<BN>();                                                        \
    if (lds > 64 * 1024)                                                                                          \
      SRF_HIP_TRY(hipFuncSetAttribute((const void*)route_fwd32_first_full_kernel<BN, CPS_>,                       \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                      \
    hipLaunchKernelGGL((route_fwd32_first_full_kernel<BN, CPS_>), dim3(nb), dim3(64 * 2 * (BN / 32)), lds, st, a, \
                       s_out, vc_out, v_out);                                                                     \
  }
  SRF_FF_LAUNCH(64)
  SRF_FF_LAUNCH(96)
  SRF_FF_LAUNCH(128)
  SRF_FF_LAUNCH(192)
#undef SRF_FF_LAUNCH
  SRF_LAUNCH_CHECK("route_fwd32_first_full");
  return SRF_OK;
}

int fwd32_pass(const Fwd32Plan& p, bool first, const void* planes, void* scratch, int B, int T,
               int N, int din, int lpad, int rpad, int J, int dout, int mask_first, const float* vc, float* cst,
               float* lzst, hipStream_t st) {
  Args32 a = make_args32(p, planes, scratch, B, T, N, din, lpad, rpad, J, dout, mask_first);
  a.vc = vc;
  a.cst = first ? nullptr : cst;
  a.lzst = first ? nullptr : lzst;
  SRF_REQUIRE(2 * p.xplane * 2 < (1ull << 31) && p.ws_w < (1ull << 31), "fwd32: operand planes exceed 2 GiB");
#define SRF_P32(DI, DO) \
  if (din == DI && dout == DO) return launch_pass32_t<DI, DO>(p, first, a, st);
  SRF_P32(8, 8)
  SRF_P32(8, 16)
  SRF_P32(8, 32)
  SRF_P32(16, 16)
  SRF_P32(16, 32)
  SRF_P32(32, 32)
#undef SRF_P32
  srf::set_error("fwd32: unsupported din %d dout %d", din, dout);
  return SRF_EUNSUPPORTED;
}

template <int DIN, int DOUT, int NW, int TW = kTW>
static int launch_bpass(const Fwd32Plan& p, const Args32& a, const Bwd32Args& b, hipStream_t st) {
  const size_t lds = fwd32_lds(p);
  auto kern = (NW > 1 && TW <= 2) ? route_bwd32p_kernel<DIN, DOUT, (NW > 1 ? NW : 2), (TW <= 2 ? TW : 2)>
                                                    : route_bwd32_kernel<DIN, DOUT, NW, TW>;
  if (lds > 64 * 1024)
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(p.n_ftiles * p.n_chunks), dim3(64 * NW), lds, st, a, b);
  SRF_LAUNCH_CHECK("route_bwd32");
  return SRF_OK;
}

template <int DIN, int DOUT>
static int launch_bpass_t(const Fwd32Plan& p, const Args32& a, const Bwd32Args& b, hipStream_t st) {
  if constexpr (DIN <= 16) {
    if (p.TW == 2)
      return p.NW == 1 ? launch_bpass<DIN, DOUT, 1, 2>(p, a, b, st) : launch_bpass<DIN, DOUT, 2, 2>(p, a, b, st);
  }
  if constexpr (DIN == 32) {
    if (p.TW == 2) {
      switch (p.NW) {
        case 1: return launch_bpass<DIN, DOUT, 1, 2>(p, a, b, st);
        case 2: return launch_bpass<DIN, DOUT, 2, 2>(p, a, b, st);
        case 4: return launch_bpass<DIN, DOUT, 4, 2>(p, a, b, st);
        default: return launch_bpass<DIN, DOUT, 8, 2>(p, a, b, st);
      }
    }
  }
  switch (p.NW) {
    case 1: return launch_bpass<DIN, DOUT, 1>(p, a, b, st);
    case 2: return launch_bpass<DIN, DOUT, 2>(p, a, b, st);
    case 4: return launch_bpass<DIN, DOUT, 4>(p, a, b, st);
    case 8: return launch_bpass<DIN, DOUT, 8>(p, a, b, st);
    default: return launch_bpass<DIN, DOUT, kMaxNW>(p, a, b, st);
  }
}

int bwd32_pass(const Fwd32Plan& p, const void* planes, void* scratch, int B, int T, int N, int din, int lpad,
               int rpad, int J, int dout, const float* cst, const float* lz, const float* gs, float* stats,
               float* glst, hipStream_t st) {
  Args32 a = make_args32(p, planes, scratch, B, T, N, din, lpad, rpad, J, dout, 0);
  Bwd32Args b{cst, lz, gs, stats, glst};
#define SRF_B32(DI, DO) \
  if (din == DI && dout == DO) return launch_bpass_t<DI, DO>(p, a, b, st);
  SRF_B32(8, 8)
  SRF_B32(8, 16)
  SRF_B32(8, 32)
  SRF_B32(16, 16)
  SRF_B32(16, 32)
  SRF_B32(32, 32)
#undef SRF_B32
  srf::set_error("bwd32: unsupported din %d dout %d", din, dout);
  return SRF_EUNSUPPORTED;
}

}  // namespace srf
