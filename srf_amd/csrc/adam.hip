// Fused Adam update over one flat fp32 parameter buffer (train_helper.py:60-70,
// Keras Adam semantics: epsilon is "epsilon hat", added after the bias-corrected
// sqrt).  alpha = lr * sqrt(1 - b2^t) / (1 - b1^t) is computed on the host.
#include "srf_common.h"
#include "../../include/srf.h"

namespace {
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, size_t n, float alpha, float b1, float b2, float eps,
                            const unsigned* __restrict__ fault) {
  // a grouped recurrence of this step (or an earlier one not yet checked) gave wrong
  // results: its gradient must not reach the parameters or the moments
  if (fault != nullptr && *fault != 0u) return;
  const size_t n4 = n / 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
    f4 gg = reinterpret_cast<const f4*>(g)[q];
    f4 mm = reinterpret_cast<f4*>(m)[q];
    f4 vv = reinterpret_cast<f4*>(v)[q];
    f4 pp = reinterpret_cast<f4*>(p)[q];
    mm = b1 * mm + (1.f - b1) * gg;
    vv = b2 * vv + (1.f - b2) * gg * gg;
#pragma unroll
    for (int k = 0; k < 4; ++k) pp[k] -= alpha * mm[k] / (sqrtf(vv[k]) + eps);
    reinterpret_cast<f4*>(m)[q] = mm;
    reinterpret_cast<f4*>(v)[q] = vv;
    reinterpret_cast<f4*>(p)[q] = pp;
  }
  // tail (n % 4) handled by the first threads
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t k = n4 * 4 + t;
  if (t < 4 && k < n) {
    const float gk = g[k];
    m[k] = b1 * m[k] + (1.f - b1) * gk;
    v[k] = b2 * v[k] + (1.f - b2) * gk * gk;
    p[k] -= alpha * m[k] / (sqrtf(v[k]) + eps);
  }
}
}  // namespace

extern "C" int srf_adam_step(float* params, const float* grads, float* m, float* v, size_t n, float alpha, float b1,
                             float b2, float eps, void* stream) {
  SRF_REQUIRE(params && grads && m && v, "null pointer argument");
  SRF_REQUIRE(((uintptr_t)params | (uintptr_t)grads | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
              "adam buffers must be 16-byte aligned");
  if (n == 0) return SRF_OK;
  size_t blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), params,
                     grads, m, v, n, alpha, b1, b2, eps, static_cast<const unsigned*>(srf::fault_flag()));
  SRF_LAUNCH_CHECK("adam");
  return SRF_OK;
}
