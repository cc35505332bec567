// CTC loss and gradient, replacing tf.nn.ctc_loss as called at trainer_sr.py:64-66
// (dense labels, batch-major logits, blank_index = C-1, logit_length =
// ceil(len/4)) and its autodiff.  One workgroup per utterance:
//   lp      = log_softmax(logits[b, t, :])                 t < T_b
//   alpha/beta recursions in log space over the extended label l' (|l'| = 2L+1)
//   nll_b   = -log sum_s alpha_{T_b-1}(s) (last two states)
//   grad    = scale * (softmax - exp(LSE_{s: l'_s=c}(alpha+beta) - lp + nll))
// Both alpha_t(s) and beta_t(s) include the emission at t.  An infeasible
// utterance (T_b too short for its labels) yields nll = +inf and a zero gradient.
#include <cmath>

#include "srf_common.h"
#include "../../include/srf.h"

namespace {

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + __logf(__expf(a - m) + __expf(b - m));
}

__global__ __launch_bounds__(256) void ctc_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                                  const int* __restrict__ label_len,
                                                  const int* __restrict__ logit_len, int Tmax, int C, int Lmax,
                                                  int blank, float scale, float* __restrict__ nll,
                                                  float* __restrict__ grad, float* __restrict__ ws) {
  extern __shared__ int ext[];   // 2*Lmax+1
  const int b = blockIdx.x;
  const int L = label_len[b];
  const int Tb = min(logit_len[b], Tmax);
  const int S = 2 * L + 1;
  const int Smax = 2 * Lmax + 1;
  float* lp = ws + (size_t)b * Tmax * (C + 2 * Smax);
  float* alpha = lp + (size_t)Tmax * C;
  float* beta = alpha + (size_t)Tmax * Smax;
  const float* lg = logits + (size_t)b * Tmax * C;
  for (int s = threadIdx.x; s < S; s += blockDim.x) ext[s] = (s & 1) ? labels[(size_t)b * Lmax + (s >> 1)] : blank;
  // log-softmax, one thread per frame
  for (int t = threadIdx.x; t < Tb; t += blockDim.x) {
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, lg[(size_t)t * C + c]);
    float z = 0.f;
    for (int c = 0; c < C; ++c) z += __expf(lg[(size_t)t * C + c] - m);
    const float lz = m + __logf(z);
    for (int c = 0; c < C; ++c) lp[(size_t)t * C + c] = lg[(size_t)t * C + c] - lz;
  }
  __syncthreads();
  // alpha
  for (int t = 0; t < Tb; ++t) {
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      float a;
      if (t == 0) {
        a = (s < 2) ? 0.f : -INFINITY;
      } else {
        const float* ap = alpha + (size_t)(t - 1) * Smax;
        a = ap[s];
        if (s >= 1) a = lse2(a, ap[s - 1]);
        if (s >= 2 && ext[s] != blank && ext[s] != ext[s - 2]) a = lse2(a, ap[s - 2]);
      }
      alpha[(size_t)t * Smax + s] = (a == -INFINITY) ? -INFINITY : a + lp[(size_t)t * C + ext[s]];
    }
    __syncthreads();
  }
  // beta
  for (int t = Tb - 1; t >= 0; --t) {
    for (int s = threadIdx.x; s < S; s += blockDim.x) {
      float a;
      if (t == Tb - 1) {
        a = (s >= S - 2) ? 0.f : -INFINITY;
      } else {
        const float* bp = beta + (size_t)(t + 1) * Smax;
        a = bp[s];
        if (s + 1 < S) a = lse2(a, bp[s + 1]);
        if (s + 2 < S && ext[s] != blank && ext[s] != ext[s + 2]) a = lse2(a, bp[s + 2]);
      }
      beta[(size_t)t * Smax + s] = (a == -INFINITY) ? -INFINITY : a + lp[(size_t)t * C + ext[s]];
    }
    __syncthreads();
  }
  float ll = -INFINITY;
  if (Tb > 0) {
    ll = alpha[(size_t)(Tb - 1) * Smax + S - 1];
    if (S >= 2) ll = lse2(ll, alpha[(size_t)(Tb - 1) * Smax + S - 2]);
  }
  if (threadIdx.x == 0) nll[b] = -ll;
  if (!grad) return;
  float* gb = grad + (size_t)b * Tmax * C;
  const bool feasible = ll > -INFINITY;
  for (int idx = threadIdx.x; idx < Tmax * C; idx += blockDim.x) {
    const int t = idx / C, c = idx - t * C;
    float g = 0.f;
    if (t < Tb && feasible) {
      float acc = -INFINITY;
      for (int s = 0; s < S; ++s)
        if (ext[s] == c) acc = lse2(acc, alpha[(size_t)t * Smax + s] + beta[(size_t)t * Smax + s]);
      const float l = lp[(size_t)t * C + c];
      g = __expf(l) - (acc == -INFINITY ? 0.f : __expf(acc - l - ll));
      g *= scale;
    }
    gb[idx] = g;
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
  hipLaunchKernelGGL(ctc_kernel, dim3(B), dim3(256), (size_t)(2 * Lmax + 1) * sizeof(int),
                     static_cast<hipStream_t>(stream), logits, labels, label_len, logit_len, Tmax, C, Lmax, blank,
                     grad_scale, nll, grad, static_cast<float*>(workspace));
  SRF_LAUNCH_CHECK("ctc");
  return SRF_OK;
}

}  // extern "C"
