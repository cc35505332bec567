// CTC loss and gradient, replacing tf.nn.ctc_loss as called at trainer_sr.py:64-66
// (dense labels, batch-major logits, blank_index = C-1, logit_length =
// ceil(len/4)) and its autodiff.  One workgroup per utterance and direction (the
// recursion itself runs in one wave, states in registers):
//   lp      = log_softmax(logits[b, t, :])                 t < T_b
//   alpha/beta recursions in log space over the extended label l' (|l'| = 2L+1)
//   nll_b   = -log sum_s alpha_{T_b-1}(s) (last two states)
//   grad    = scale * (softmax - exp(LSE_{s: l'_s=c}(alpha+beta) - lp + nll))
// Both alpha_t(s) and beta_t(s) include the emission at t.  An infeasible
// utterance (T_b too short for its labels) yields nll = +inf and a zero gradient.
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "srf_common.h"
#include "../../include/srf.h"

namespace {

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + __logf(__expf(a - m) + __expf(b - m));
}

// Branch-free log(e^a + e^b) for the serial recursions: with m = max(a, b) taken as
// 0 when both are -inf, e^(a-m) + e^(b-m) is 0 there and v_log_f32 returns -inf; the
// sum lies in [1, 2] otherwise, so the raw exp2/log2 instructions need no range fix-up.
__device__ __forceinline__ float lse2f(float a, float b) {
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  const float m = fmaxf(a, b);
  const float ms = m == -INFINITY ? 0.f : m;
  const float z = __builtin_amdgcn_exp2f((a - ms) * kLog2e) + __builtin_amdgcn_exp2f((b - ms) * kLog2e);
  return ms + __builtin_amdgcn_logf(z) * kLn2;
}

// log(e^a + e^b + e^c) in one step (one max3, three exp, one log; the sum lies in
// [1, 3], or is 0 when all three are -inf), so a recursion step has one
// log-sum-exp on its serial chain instead of two nested ones.
__device__ __forceinline__ float lse3(float a, float b, float c) {
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  const float m = fmaxf(fmaxf(a, b), c);
  const float ms = m == -INFINITY ? 0.f : m;
  const float z = __builtin_amdgcn_exp2f((a - ms) * kLog2e) + __builtin_amdgcn_exp2f((b - ms) * kLog2e) +
                  __builtin_amdgcn_exp2f((c - ms) * kLog2e);
  return ms + __builtin_amdgcn_logf(z) * kLn2;
}

// Wave-resident recursions (KM > 0, S <= 64*KM): wave 0 holds states
// s = lane + 64k in registers; the s-1 / s-2 (alpha) or s+1 / s+2 (beta)
// neighbours come from DPP whole-wave shifts (wave_shr:1 / wave_shl:1, a VALU
// move instead of an LDS-crossbar shuffle on the serial path), the lanes at a
// 64-state boundary taking the neighbouring group's values (v_readlane), so a
// time step needs no barrier.
__device__ __forceinline__ float dpp_wave_shr1(float old, float src) {   // lane l <- src[l-1], lane 0 <- old
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_wave_shl1(float old, float src) {   // lane l <- src[l+1], lane 63 <- old
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), 0x130, 0xF, 0xF, false));
}
__device__ __forceinline__ float read_lane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// The emission row of step t + 1 is read while step t's log-sum-exps run.
template <int KM>
__device__ __forceinline__ float alpha_wave(const int* __restrict__ ext, const float* __restrict__ lp, int C, int S,
                                            int Tb, int Smax, int blank, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const auto ors = __builtin_amdgcn_make_buffer_rsrc(out, 0, Tb * Smax * 4, 0x00020000);
  float a[KM], em[KM];
  int e[KM];
  bool sk[KM], live[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int s = lane + 64 * k;
    live[k] = s < S;
    e[k] = live[k] ? ext[s] : blank;
    sk[k] = live[k] && s >= 2 && ext[s] != blank && ext[s] != ext[s - 2];
    a[k] = -INFINITY;
    em[k] = Tb > 0 ? lp[e[k]] : 0.f;
  }
  for (int t = 0; t < Tb; ++t) {
    float emn[KM];
    const int tn = min(t + 1, Tb - 1);
#pragma unroll
    for (int k = 0; k < KM; ++k) emn[k] = lp[(size_t)tn * C + e[k]];
    float na[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int s = lane + 64 * k;
      float v;
      if (t == 0) {
        v = s < 2 ? 0.f : -INFINITY;
      } else {
        const float l63 = k > 0 ? read_lane(a[k - 1], 63) : -INFINITY;
        const float l62 = k > 0 ? read_lane(a[k - 1], 62) : -INFINITY;
        const float p1 = dpp_wave_shr1(l63, a[k]);    // state s - 1
        const float p2 = dpp_wave_shr1(l62, p1);      // state s - 2
        v = lse3(a[k], p1, sk[k] ? p2 : -INFINITY);
      }
      v = live[k] ? v + em[k] : -INFINITY;            // -inf stays -inf
      na[k] = v;
      // no exec branch on the serial path: dead lanes store out of the buffer's range
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ors, live[k] ? (uint32_t)(t * Smax + s) * 4 : 0x80000000u,
                                            0, 0);
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      a[k] = na[k];
      em[k] = emn[k];
    }
  }
  // log-likelihood: the last two states at t = Tb-1
  float loc = -INFINITY;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int s = lane + 64 * k;
    if (Tb > 0 && (s == S - 1 || s == S - 2)) loc = lse2(loc, a[k]);
  }
  float m = loc;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (m == -INFINITY) return -INFINITY;
  const float z = wave_sum(loc == -INFINITY ? 0.f : __expf(loc - m));
  return m + __logf(z);
}

template <int KM>
__device__ __forceinline__ void beta_wave(const int* __restrict__ ext, const float* __restrict__ lp, int C, int S,
                                          int Tb, int Smax, int blank, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const auto ors = __builtin_amdgcn_make_buffer_rsrc(out, 0, Tb * Smax * 4, 0x00020000);
  float a[KM], em[KM];
  int e[KM];
  bool sk[KM], live[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    const int s = lane + 64 * k;
    live[k] = s < S;
    e[k] = live[k] ? ext[s] : blank;
    sk[k] = s + 2 < S && ext[s] != blank && ext[s] != ext[s + 2];
    a[k] = -INFINITY;
    em[k] = Tb > 0 ? lp[(size_t)(Tb - 1) * C + e[k]] : 0.f;
  }
  for (int t = Tb - 1; t >= 0; --t) {
    float emn[KM];
    const int tn = max(t - 1, 0);
#pragma unroll
    for (int k = 0; k < KM; ++k) emn[k] = lp[(size_t)tn * C + e[k]];
    float na[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int s = lane + 64 * k;
      float v;
      if (t == Tb - 1) {
        v = s >= S - 2 ? 0.f : -INFINITY;
      } else {
        const float h0 = k + 1 < KM ? read_lane(a[k + 1], 0) : -INFINITY;
        const float h1 = k + 1 < KM ? read_lane(a[k + 1], 1) : -INFINITY;
        const float q1 = dpp_wave_shl1(h0, a[k]);     // state s + 1
        const float q2 = dpp_wave_shl1(h1, q1);       // state s + 2
        v = lse3(a[k], q1, sk[k] ? q2 : -INFINITY);
      }
      v = live[k] ? v + em[k] : -INFINITY;
      na[k] = v;
      // no exec branch on the serial path: dead lanes store out of the buffer's range
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ors, live[k] ? (uint32_t)(t * Smax + s) * 4 : 0x80000000u,
                                            0, 0);
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      a[k] = na[k];
      em[k] = emn[k];
    }
  }
}

// Recursion kernel: grid (B, 2).  Block (b, 0) runs the alpha recursion and
// writes nll[b]; block (b, 1) runs beta.  Both recompute the log-softmax into
// LDS (LPLDS; else workspace) and stream their rows to workspace.
// Dynamic LDS: ext[Smax] (int) | row[2][Smax] | lp[T*C].
template <int KM, bool LPLDS>
__global__ __launch_bounds__(256) void ctc_recursion_kernel(const float* __restrict__ logits,
                                                            const int* __restrict__ labels,
                                                            const int* __restrict__ label_len,
                                                            const int* __restrict__ logit_len, int Tmax, int C,
                                                            int Lmax, int blank, int want_beta,
                                                            float* __restrict__ nll, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Smax = 2 * Lmax + 1;
  int* ext = reinterpret_cast<int*>(smem);
  float* row = smem + Smax;
  const int b = blockIdx.x;
  const bool is_beta = blockIdx.y == 1;
  if (is_beta && !want_beta) return;
  const int L = label_len[b];
  const int Tb = min(logit_len[b], Tmax);
  const int S = 2 * L + 1;
  float* gws = ws + (size_t)b * Tmax * (C + 2 * Smax);
  float* lpg = gws;                                       // [Tmax][C] (global copy, for the gradient)
  float* lp = LPLDS ? (row + 2 * Smax) : lpg;
  float* out = gws + (size_t)Tmax * C + (is_beta ? (size_t)Tmax * Smax : 0);
  const float* lg = logits + (size_t)b * Tmax * C;
  for (int s = threadIdx.x; s < S; s += blockDim.x) ext[s] = (s & 1) ? labels[(size_t)b * Lmax + (s >> 1)] : blank;
  if constexpr (LPLDS) {
    // rows staged into LDS (coalesced), then one thread per row: max, log-sum-exp,
    // normalise in place; the alpha block copies the rows out for the gradient kernel
    const int n = Tb * C;
    for (int i0 = threadIdx.x; i0 < n; i0 += 8 * 256) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = lg[min(i0 + u * 256, n - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + u * 256 < n) lp[i0 + u * 256] = v[u];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < Tb; t += blockDim.x) {
      float* r = lp + (size_t)t * C;
      float m = -INFINITY;
#pragma unroll 8
      for (int c = 0; c < C; ++c) m = r[c] > m ? r[c] : m;
      float z = 0.f;
#pragma unroll 8
      for (int c = 0; c < C; ++c) z += __expf(r[c] - m);
      const float lz = m + __logf(z);
#pragma unroll 8
      for (int c = 0; c < C; ++c) r[c] -= lz;
    }
    if (!is_beta) {
      __syncthreads();
      for (int i = threadIdx.x; i < Tb * C; i += blockDim.x) lpg[i] = lp[i];
    }
  } else {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
    for (int t = w; t < Tb; t += nw) {
      float m = -INFINITY;
      for (int c = l; c < C; c += 64) m = fmaxf(m, lg[(size_t)t * C + c]);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      float z = 0.f;
      for (int c = l; c < C; c += 64) z += __expf(lg[(size_t)t * C + c] - m);
      z = wave_sum(z);
      const float lz = m + __logf(z);
      for (int c = l; c < C; c += 64) lp[(size_t)t * C + c] = lg[(size_t)t * C + c] - lz;
    }
  }
  __syncthreads();
  if constexpr (KM > 0) {
    if (threadIdx.x >= 64) return;
    if (!is_beta) {
      const float ll = alpha_wave<KM>(ext, lp, C, S, Tb, Smax, blank, out);
      if (threadIdx.x == 0) nll[b] = -ll;
    } else {
      beta_wave<KM>(ext, lp, C, S, Tb, Smax, blank, out);
    }
    return;
  }
  if (!is_beta) {
    for (int t = 0; t < Tb; ++t) {
      const float* ap = row + ((t + 1) & 1) * Smax;
      float* an = row + (t & 1) * Smax;
      for (int s = threadIdx.x; s < S; s += blockDim.x) {
        float a;
        if (t == 0) {
          a = (s < 2) ? 0.f : -INFINITY;
        } else {
          a = ap[s];
          if (s >= 1) a = lse2(a, ap[s - 1]);
          if (s >= 2 && ext[s] != blank && ext[s] != ext[s - 2]) a = lse2(a, ap[s - 2]);
        }
        a = (a == -INFINITY) ? -INFINITY : a + lp[(size_t)t * C + ext[s]];
        an[s] = a;
        out[(size_t)t * Smax + s] = a;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      float ll = -INFINITY;
      if (Tb > 0) {
        const float* al = row + ((Tb - 1) & 1) * Smax;
        ll = al[S - 1];
        if (S >= 2) ll = lse2(ll, al[S - 2]);
      }
      nll[b] = -ll;
    }
  } else {
    for (int t = Tb - 1; t >= 0; --t) {
      const float* bp = row + ((t + 1) & 1) * Smax;
      float* bn = row + (t & 1) * Smax;
      for (int s = threadIdx.x; s < S; s += blockDim.x) {
        float a;
        if (t == Tb - 1) {
          a = (s >= S - 2) ? 0.f : -INFINITY;
        } else {
          a = bp[s];
          if (s + 1 < S) a = lse2(a, bp[s + 1]);
          if (s + 2 < S && ext[s] != blank && ext[s] != ext[s + 2]) a = lse2(a, bp[s + 2]);
        }
        a = (a == -INFINITY) ? -INFINITY : a + lp[(size_t)t * C + ext[s]];
        bn[s] = a;
        out[(size_t)t * Smax + s] = a;
      }
      __syncthreads();
    }
  }
}

// Gradient kernel: grid (B, ceil(Tmax/FR)), 256 threads = FR frames x 256/FR class
// lanes.  Per class the label positions are walked through a next-occurrence list
// (built in LDS, one thread per label position), over alpha + beta of the block's
// FR frames staged in LDS (STAGE), so a frame costs O(L + C) LDS reads, not
// O(C * L) loads.  FR (16 down to 1) is the largest whose staging fits
// kCtcGradLds; past that (very long label sequences) alpha + beta are read from
// the workspace directly (STAGE = false).
// Dynamic LDS: head[C] | next[Lmax] (int) | ab[FR][Smax] (STAGE only).
constexpr size_t kCtcGradLds = 64 * 1024;

template <bool STAGE>
__global__ __launch_bounds__(256) void ctc_grad_kernel(const int* __restrict__ labels,
                                                       const int* __restrict__ label_len,
                                                       const int* __restrict__ logit_len,
                                                       const float* __restrict__ nll, int Tmax, int C, int Lmax,
                                                       int blank, float scale, int FR, const float* __restrict__ ws,
                                                       float* __restrict__ grad) {
  extern __shared__ int lists[];
  int* head = lists;
  int* next = lists + C;
  const int Smax = 2 * Lmax + 1;
  float* ab = reinterpret_cast<float*>(lists + C + Lmax);
  const int b = blockIdx.x;
  const int L = label_len[b];
  const int Tb = min(logit_len[b], Tmax);
  const float ll = -nll[b];
  const bool feasible = ll > -INFINITY;
  const int* lab = labels + (size_t)b * Lmax;
  const int t0 = blockIdx.y * FR;
  const float* gws = ws + (size_t)b * Tmax * (C + 2 * Smax);
  const float* lp = gws;
  const float* alpha = gws + (size_t)Tmax * C;
  const float* beta = alpha + (size_t)Tmax * Smax;
  // first occurrence of each class and next occurrence of each label position
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    int h = -1;
    for (int k = L - 1; k >= 0; --k) h = lab[k] == c ? k : h;
    head[c] = h;
  }
  for (int k = threadIdx.x; k < L; k += blockDim.x) {
    const int c = lab[k];
    int nx = -1;
    for (int k2 = L - 1; k2 > k; --k2) nx = lab[k2] == c ? k2 : nx;
    next[k] = nx;
  }
  const int S = 2 * L + 1;
  const int nt = min(FR, Tb - t0);
  if constexpr (STAGE) {
    for (int i = threadIdx.x; i < FR * S; i += blockDim.x) {
      const int tt = i / S, sidx = i - tt * S;
      float v = -INFINITY;
      if (tt < nt) {
        const size_t o = (size_t)(t0 + tt) * Smax + sidx;
        v = alpha[o] + beta[o];
      }
      ab[tt * Smax + sidx] = v;
    }
  }
  __syncthreads();
  const int lanes = blockDim.x / FR;
  const int tt = threadIdx.x / lanes;
  const int t = t0 + tt;
  if (t >= Tmax) return;
  float* gb = grad + ((size_t)b * Tmax + t) * C;
  const float* abt = ab + tt * Smax;
  const float* at = alpha + (size_t)t * Smax;
  const float* bt = beta + (size_t)t * Smax;
  auto abv = [&](int sidx) { return STAGE ? abt[sidx] : at[sidx] + bt[sidx]; };
  for (int c = threadIdx.x % lanes; c < C; c += lanes) {
    float g = 0.f;
    if (t < Tb && feasible) {
      float acc = -INFINITY;
      if (c == blank) {
        for (int s2 = 0; s2 <= 2 * L; s2 += 2) acc = lse2f(acc, abv(s2));
      } else {
        for (int k = head[c]; k >= 0; k = next[k]) acc = lse2f(acc, abv(2 * k + 1));
      }
      const float l = lp[(size_t)t * C + c];
      g = (__expf(l) - (acc == -INFINITY ? 0.f : __expf(acc - l - ll))) * scale;
    }
    gb[c] = g;
  }
}

}  // namespace

extern "C" {

size_t srf_ctc_workspace(int B, int Tmax, int C, int Lmax) {
  return (size_t)B * Tmax * (C + 2 * (2 * Lmax + 1)) * sizeof(float);
}

int srf_ctc_loss(const float* logits, const int* labels, const int* label_len, const int* logit_len, int B, int Tmax,
                 int C, int Lmax, int blank, float grad_scale, float* nll, float* grad, void* workspace,
                 size_t workspace_bytes, void* stream) {
  SRF_REQUIRE(logits && labels && label_len && logit_len && nll && workspace, "null pointer argument");
  SRF_REQUIRE(B > 0 && Tmax > 0 && C > 1 && Lmax >= 0 && blank >= 0 && blank < C, "bad CTC shape");
  if (workspace_bytes < srf_ctc_workspace(B, Tmax, C, Lmax)) {
    srf::set_error("CTC workspace too small");
    return SRF_EWORKSPACE;
  }
  const size_t Smax = 2 * (size_t)Lmax + 1;
  size_t shmem = 3 * Smax * sizeof(float);
  const size_t lp_bytes = (size_t)Tmax * C * sizeof(float);
  const bool lp_in_lds = (shmem + lp_bytes) <= 96 * 1024;
  if (lp_in_lds) shmem += lp_bytes;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // wave-resident recursion for up to 512 extended-label states, else the block loop
  auto pick = [&](auto lds) {
    constexpr bool LDS = decltype(lds)::value;
    return Smax > 512 ? ctc_recursion_kernel<0, LDS>
           : Smax <= 128      ? ctc_recursion_kernel<2, LDS>
           : Smax <= 256      ? ctc_recursion_kernel<4, LDS>
                              : ctc_recursion_kernel<8, LDS>;
  };
  auto kern = lp_in_lds ? pick(std::true_type{}) : pick(std::false_type{});
  hipLaunchKernelGGL(kern, dim3(B, 2), dim3(256), shmem, st, logits, labels, label_len, logit_len, Tmax, C, Lmax,
                     blank, grad ? 1 : 0, nll, static_cast<float*>(workspace));
  SRF_LAUNCH_CHECK("ctc_recursion");
  if (grad) {
    const size_t lists = (size_t)(C + Lmax) * sizeof(int);
    SRF_REQUIRE(lists <= kCtcGradLds, "CTC: labels too long for the gradient kernel's LDS lists");
    int fr = 16;
    while (fr > 1 && lists + (size_t)fr * Smax * sizeof(float) > kCtcGradLds) fr >>= 1;
    const bool stage = lists + (size_t)fr * Smax * sizeof(float) <= kCtcGradLds;
    if (!stage) fr = 16;
    hipLaunchKernelGGL(stage ? ctc_grad_kernel<true> : ctc_grad_kernel<false>, dim3(B, (Tmax + fr - 1) / fr),
                       dim3(256), lists + (stage ? (size_t)fr * Smax * sizeof(float) : 0), st, labels, label_len,
                       logit_len, nll, Tmax, C, Lmax, blank, grad_scale, fr, static_cast<const float*>(workspace),
                       grad);
  }
  SRF_LAUNCH_CHECK("ctc");
  return SRF_OK;
}

}  // extern "C"
