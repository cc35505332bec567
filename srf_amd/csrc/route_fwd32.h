// Host interface of the 32x32-tile split-bf16 DR forward pass (route_fwd32.hip),
// used by route_dr.hip's srf_route_dr_fwd for the shapes it supports.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>

namespace srf {

struct Fwd32Plan {
  int NW;              // waves per workgroup (TW = 4 row tiles of 32 each)
  int JDp;             // J*dout padded to NW*4*32 rows
  int n_chunks, chunk_len, n_ftiles;
  size_t xplane;       // elements per x plane (data + zero row)
  size_t ws_w, ws_b, ws_x, ws_bsum, ws_slab;   // workspace regions (bytes)
};

bool fwd32_supported(int din, int dout, int J);
Fwd32Plan fwd32_plan(int B, int T, int N, int din, int lpad, int rpad, int J, int dout);
size_t fwd32_workspace(const Fwd32Plan& p);
size_t fwd32_lds(const Fwd32Plan& p);
float* fwd32_slab(const Fwd32Plan& p, void* ws);
// split W / bias / emb into bf16 planes and the i-chunk bias sums (once per forward)
int fwd32_prepare(const Fwd32Plan& p, const float* emb, const float* W, const float* bias, int B, int T, int N,
                  int din, int lpad, int rpad, int J, int dout, void* ws, hipStream_t st);
// one routing pass: partial s over i-chunks into fwd32_slab(p, ws)
int fwd32_pass(const Fwd32Plan& p, bool first, const void* ws, int B, int T, int N, int din, int lpad, int rpad,
               int J, int dout, int mask_first, const float* vc, hipStream_t st);

}  // namespace srf
