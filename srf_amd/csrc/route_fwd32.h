// Host interface of the 32x32-tile split-fp16 DR forward pass (route_fwd32.hip),
// used by route_dr.hip's srf_route_dr_fwd for the shapes it supports.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>

namespace srf {

// Row tiles (of 32 rows) per wave of route_fwd32 / route_bwd32 for din 8, 16.
constexpr int kFwd32TW = 4;
// Frame stride of the stored couplings (frame-minor layout, 32-frame aligned).
__host__ __device__ inline int fwd32_frame_stride(int F) { return (F + 31) / 32 * 32; }

struct Fwd32Plan {
  int NW;              // waves per workgroup
  int TW;              // 32-row tiles per wave (kFwd32TW; 2 for din 32 with J*dout <= 512)
  int JDp;             // J*dout padded to NW*TW*32 rows
  int xpad;            // zero halves after each x plane (the invalid-frame row)
  int n_chunks, chunk_len, n_ftiles;
  size_t xplane;       // elements per x plane (data + zero row)
  size_t ws_w, ws_b, ws_x, ws_h, ws_bsum, ws_slab;   // workspace regions (bytes)
};

bool fwd32_supported(int din, int dout, int J);
// n_chunks: the input-capsule chunks (workgroups per frame tile) of the routing passes,
// 0 = the cost model's choice (srf_route_dr_auto_chunks returns it)
Fwd32Plan fwd32_plan(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int n_chunks = 0);
// Operand planes (split W, bias, x and their scale header: written by fwd32_prepare,
// read by every pass)
// and per-pass scratch (i-chunk bias sums + partial slabs) may live apart: a
// training forward keeps its planes for the backward (coupling storage).
size_t fwd32_planes_bytes(const Fwd32Plan& p);
size_t fwd32_scratch_bytes(const Fwd32Plan& p);
size_t fwd32_workspace(const Fwd32Plan& p);   // planes + scratch
size_t fwd32_lds(const Fwd32Plan& p);
float* fwd32_slab(const Fwd32Plan& p, void* scratch);
// the planes' scale header {2^-(aw+bx), aw, bx} (written by fwd32_prepare)
const float* fwd32_hdr(const Fwd32Plan& p, const void* planes);
// split W / emb into scaled fp16 planes, bias into bf16 planes, and the i-chunk bias
// sums (two launches per forward: absmax, prep);
// WT / xT (nullable): also the fp32 W^T [in_n][din][JD] and window^T [in_n][din][Fp]
// operands of the backward gx / gW contractions; wt16 (din 32): WT instead holds the
// split-fp16 A planes of route_gux16_kernel (same bytes); xt16 (din 32): xT instead
// holds route_gw16s_kernel's blocked split-fp16 B planes [in_n][Fp/16][2][din][16]
// (same bytes)
int fwd32_prepare(const Fwd32Plan& p, const float* emb, const float* W, const float* bias, int B, int T, int N,
                  int din, int lpad, int rpad, int J, int dout, void* planes, void* scratch, float* WT, float* xT,
                  hipStream_t st, bool wt16 = false, bool xt16 = false);
// one routing pass: partial s over i-chunks into fwd32_slab(p, scratch); passes r >= 1
// also store the couplings c^r (cst) and logZ^r (lzst) when cst != nullptr.
int fwd32_pass(const Fwd32Plan& p, bool first, const void* planes, void* scratch, int B, int T,
               int N, int din, int lpad, int rpad, int J, int dout, int mask_first, const float* vc, float* cst,
               float* lzst, hipStream_t st);
// iteration 0 over all input capsules with the finish fused: writes s^0 (s_out),
// Vc^1 = v^0 (vc_out) and, for one-iteration layers, v (v_out); din = dout = 32
bool fwd32_first_full_supported(const Fwd32Plan& p, int din, int dout);
int fwd32_first_full(const Fwd32Plan& p, const void* planes, void* scratch, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int mask_first, float* s_out, float* vc_out, float* v_out,
                     hipStream_t st);
// Coupling storage of one training forward (float offsets): c^r [iters-1][in_n][JP][Fs],
// logZ^r [iters-1][in_n][Fs], the operand planes, WT, xT; JP = JDp / dout,
// Fs = fwd32_frame_stride(F).
struct Fwd32Cpl {
  size_t c, lz, planes, WT, xT, total;
};
Fwd32Cpl fwd32_cpl_layout(const Fwd32Plan& p, int F, int in_n, int din, int dout, int J, int iters);
// one backward routing pass r >= 1 from the stored couplings: partial gVc^r over
// i-chunks into fwd32_slab(p, scratch), the (logZ, sigma) stats and the logit
// gradients gL^r (glst, laid out as the couplings) of the gu pass
int bwd32_pass(const Fwd32Plan& p, const void* planes, void* scratch, int B, int T, int N, int din, int lpad,
               int rpad, int J, int dout, const float* cst, const float* lz, const float* gs, float* stats,
               float* glst, hipStream_t st);

}  // namespace srf
