// Sequential dynamic routing (SDR) recurrence with register-resident frames, gfx950.
//
// Replaces the frame loop of sequence_router_naive.py:162-170 (tf.while_loop over
// T' with body_context :231-245 / pad_body_context :212-229), one utterance per
// workgroup.  route_sdr.hip forms u = W x + b for every frame on MFMA first; this
// file walks the frames (forward here, backward in route_sdr_seq_bwd.hip).
//
// Mapping (route_sdr_seq_dev.h).  A 1024-thread workgroup holds the frame's whole
// u_t [in_n][J][D] in registers.  J is padded to JP (a power of two); a capsule's
// D values are split over Q lanes of KD values, so one input capsule is a "row" of
// ROWL = JP*Q lanes and a wave holds SUB = 64/ROWL rows.  The G = 16*SUB row slots
// take input capsules i = g, g + G, ... (at most NIM per lane).  Per iteration:
//   logits  b_ij += <u_ij, w_j>: KD FMAs per lane + a butterfly over the Q lanes;
//   softmax over j: butterflies over the JP capsules of the row;
//   s_j = sum_i c_ij u_ij: in-lane over the lane's rows, a butterfly over the
//         wave's rows, then the 16 wave partials through LDS;
//   squash: thread e = j*D + d owns element e; the norm is a butterfly over D lanes.
// Butterflies stay on the VALU where they can (DPP quad_perm / row_ror, permlane
// swaps; ds_swizzle only for a lone xor 4).  Two barriers per iteration;
// the next frame's u is loaded while the last reduction and squash of the
// current frame run.  HBM traffic per frame: u_t once (in_n*J*D floats) + v_t.
#include <algorithm>
#include <cstdlib>

#include "route_sdr_seq.h"
#include "route_sdr_seq_dev.h"
#include "srf_group.h"

namespace {

using namespace srf_seq;

#if SRF_SEQ_STAMP
__device__ unsigned long long* g_stamps;   // diagnostic builds: phase cycle sums
#else
constexpr unsigned long long* g_stamps = nullptr;
#endif

// LDS: w [JP * D] (agreement input of the iteration: v_{t-1} at r = 0, then v^{r-1};
// the padded capsules' tail zero), part [16][JD].  GRP: X.G workgroups per utterance split its input capsules
// (srf_group.h); member 0 stores v and s^r, every member its own capsules' c^r.
// KS > 0: the lane's last KS rows of frame t + 1 come through LDS, staged by
// global_load_lds (no registers) while frame t computes -- one CU fetches its frame at
// about 10 B/cycle, so the burst of loads at the frame's end is most of the frame; the
// stage [KS][KD/4][16 waves][64 lanes][16 B] is written lane-linearly by each wave's DMA
// and read back by the same lanes (a wave's own vmcnt orders it).
__device__ __forceinline__ void glds16(const float* src, float* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

template <int D, int JP, int NIM, bool GRP, int KS = 0>
__global__ __launch_bounds__(kThreads) void sdr_seq_fwd_kernel(srf::SeqItems items, int T, int in_n, int J,
                                                               int iters, int mask_first, srf_grp::Grp X) {
  using C = Cfg<D, JP, NIM>;
  const srf::SeqItem& I = items.it[blockIdx.y];   // the frame range of this launch item
  const float* __restrict__ u = I.u;
  float* __restrict__ v_out = I.v;
  float* __restrict__ cs = I.cs;
  const srf::SeqRange rg = I.rg;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int JD = J * D;
  constexpr int JDp = JP * D;
  float* wl = lds;
  float* part = lds + JDp;
  float* stage = part + kWaves * JD;   // KS > 0
  const int tid = threadIdx.x;
  const int utt = GRP ? blockIdx.x / X.G : blockIdx.x;   // utterance
  const int gm = GRP ? blockIdx.x - utt * X.G : 0;       // member of its group
  const bool lead = gm == 0;
  const Lane L = lane_map<C>(in_n, J, mask_first, gm, GRP ? X.G : 1);
  const size_t ff = (size_t)in_n * JD;
  const float* ub = u + (size_t)utt * rg.tu_n * ff;   // frame t at ub + (t - tu0) * ff
  float* vo = v_out + (size_t)utt * T * JD;
  const bool owner_wave = (tid >> 6) * 64 < JD;   // waves holding elements e = tid < JD
  const bool ev = tid < JD;
  const size_t csr = (size_t)iters * (in_n * JP + JD);   // coupling record per frame (cs != nullptr)
  if (rg.t0 >= rg.t1) return;
  if (ev) wl[tid] = rg.t0 > 0 ? vo[(size_t)(rg.t0 - 1) * JD + tid] : 0.f;   // v_{t0-1} (v_{-1} = 0)
  zero_tail(wl, 1, JD, JDp);
  float ur[C::NIM][C::KD];
  constexpr int KF = C::NIM - KS;   // rows from global memory into registers
  constexpr int NC = C::KD / 4;
  const int lane = tid & 63, wv = tid >> 6;
  // DMA of the lane's rows KF.. of the frame at ut into the stage (absent rows read the
  // frame's first row and are zeroed when taken)
  auto stage_issue = [&](const float* ut) {
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int k = KF + kk;
      const bool ok = L.jv && k < L.NI;
      const float* src = ut + (ok ? (size_t)(L.g + k * C::G) * JD + L.eoff : 0);
#pragma unroll
      for (int c = 0; c < NC; ++c) glds16(src + 4 * c, stage + ((kk * NC + c) * kWaves + wv) * 256);
    }
  };
  auto stage_take = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA has landed
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int k = KF + kk;
      const bool ok = L.jv && k < L.NI;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const f4 x = *reinterpret_cast<const f4*>(stage + (((kk * NC + c) * kWaves + wv) * 64 + lane) * 4);
        ur[k][4 * c] = ok ? x.x : 0.f;
        ur[k][4 * c + 1] = ok ? x.y : 0.f;
        ur[k][4 * c + 2] = ok ? x.z : 0.f;
        ur[k][4 * c + 3] = ok ? x.w : 0.f;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read before the next DMA overwrites it
  };
  auto& urf = *reinterpret_cast<float(*)[KF > 0 ? KF : 1][C::KD]>(&ur[0][0]);
  // the iteration inlined twice (the last one unconditionally loading the next frame)
  // where the registers allow; frames of more than 48 registers (the J = 32 last layer,
  // at the 1024-thread limit of 128) keep one copy and branch around the loads
  constexpr bool UNC = KS > 0 || C::NIM * C::KD <= 48;
  // KS > 0: barriers without the vmcnt(0) of __syncthreads, so the next frames' loads and
  // DMA stay in flight across them; LDS ordering by lgkmcnt(0) (global stores of this
  // kernel are never read back by it)
  auto bar = [&]() {
    if constexpr (KS > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  load_frame<C>(ub + (size_t)(rg.t0 - rg.tu0) * ff, JD, L, ur);
  if constexpr (KS > 0) stage_issue(ub + (size_t)(min(rg.t0 + 1, rg.t1 - 1) - rg.tu0) * ff);
  __syncthreads();
  SEQ_STAMP_DECL
  for (int t = rg.t0; t < rg.t1; ++t) {
    float b[C::NIM], c[C::NIM];
#pragma unroll
    for (int k = 0; k < C::NIM; ++k) b[k] = 0.f;
    const int tn = min(t + 1, rg.t1 - 1);   // the next frame (the range's last reloads itself)
    // one routing iteration; the last one also loads frame tn into the registers u_t
    // leaves.  The loads are unconditional: a branch around them would merge the old and
    // new registers and wait for the loads right there, instead of at their first use
    // (iteration 0 of the next frame), past the barriers and the squash in between.
    auto iteration = [&](int r, bool last) __attribute__((always_inline)) {
      float w[C::KD];
      lds_slice<C::KD>(wl, L.eoff, w);
      logits_softmax<C>(ur, w, L, b, c);
      row_partial<C>(c, ur, L, JD, part);
      if (cs) store_ij<C>(c, L, cs + ((size_t)utt * T + t) * csr + (size_t)r * in_n * JP);
      if (last) {   // u_t is dead
        if constexpr (KS > 0) {
          stage_take();   // frame tn's staged rows (the wait covers only the DMA issued a frame ago)
          load_rows<C, KF>(ub + (size_t)(tn - rg.tu0) * ff, JD, L, urf);
          stage_issue(ub + (size_t)(min(tn + 1, rg.t1 - 1) - rg.tu0) * ff);
        } else {
          load_frame<C>(ub + (size_t)(tn - rg.tu0) * ff, JD, L, ur);
        }
      }
      SEQ_MARK(0);   // logits, softmax, row partials (+ next frame's loads issued)
      bar();
      if constexpr (GRP) srf_grp::allreduce<kWaves, kThreads>(part, JD, I.ws, X, utt, gm, (t - rg.t0) * iters + r, tid);
      SEQ_MARK(1);
      if (owner_wave) {
        const float s = ev ? (GRP ? part[tid] : sum_parts(part, JD, tid)) : 0.f;
        const float v = squash_elem<D>(s);
        if (ev) {
          wl[tid] = v;
          if (lead) {
            if (last) vo[(size_t)t * JD + tid] = v;
            if (cs) cs[((size_t)utt * T + t) * csr + (size_t)iters * in_n * JP + r * JD + tid] = s;
          }
        }
      }
      SEQ_MARK(2);   // wave sums + squash (owner waves)
      bar();
      SEQ_MARK(3);
    };
    if constexpr (UNC) {
      for (int r = 0; r + 1 < iters; ++r) iteration(r, false);
      iteration(iters - 1, true);
    } else {   // one copy of the iteration (registers): the next frame's loads under a branch
      for (int r = 0; r < iters; ++r) {
        float w[C::KD];
        lds_slice<C::KD>(wl, L.eoff, w);
        logits_softmax<C>(ur, w, L, b, c);
        row_partial<C>(c, ur, L, JD, part);
        if (cs) store_ij<C>(c, L, cs + ((size_t)utt * T + t) * csr + (size_t)r * in_n * JP);
        if (r == iters - 1 && t + 1 < rg.t1) load_frame<C>(ub + (size_t)(tn - rg.tu0) * ff, JD, L, ur);
        SEQ_MARK(0);
        bar();
        if constexpr (GRP)
          srf_grp::allreduce<kWaves, kThreads>(part, JD, I.ws, X, utt, gm, (t - rg.t0) * iters + r, tid);
        SEQ_MARK(1);
        if (owner_wave) {
          const float s = ev ? (GRP ? part[tid] : sum_parts(part, JD, tid)) : 0.f;
          const float v = squash_elem<D>(s);
          if (ev) {
            wl[tid] = v;
            if (lead) {
              if (r == iters - 1) vo[(size_t)t * JD + tid] = v;
              if (cs) cs[((size_t)utt * T + t) * csr + (size_t)iters * in_n * JP + r * JD + tid] = s;
            }
          }
        }
        SEQ_MARK(2);
        bar();
        SEQ_MARK(3);
      }
    }
  }
  SEQ_FLUSH(g_stamps);
  srf_grp::depart<GRP>(I.ws, X, utt, tid);
}

size_t fwd_lds(int J, int D) {
  return ((size_t)pow2_at_least(J) * D + (size_t)kWaves * J * D) * sizeof(float);
}

// rows per lane staged through LDS (sdr_seq_fwd_kernel KS): the C3 inner layers, three of
// five (96 KB beside w and the partials); the J = 32 last layer has no registers to spare
// for the second copy of the iteration that keeps the loads unconditional
constexpr int stage_rows(int D, int JP, int NIM) {
  return (D == 32 && NIM == 5 && JP == 16) ? 3 : 0;
}

template <int D, int JP, int NIM>
int launch_fwd(const srf::SeqItems& items, const srf_grp::Grp& X, int B, int T, int in_n, int J, int iters,
               int mask_first, hipStream_t st) {
  constexpr int KS = stage_rows(D, JP, NIM);
  if constexpr (KS > 0) {
    const size_t lds = fwd_lds(J, D) + (size_t)KS * kThreads * seq_kd(D, JP) * sizeof(float);
    if (X.G == 1 && lds <= 160 * 1024) {
      auto k = sdr_seq_fwd_kernel<D, JP, NIM, false, KS>;
      SRF_HIP_TRY(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(k, dim3(B, items.n), dim3(kThreads), lds, st, items, T, in_n, J, iters, mask_first, X);
      SRF_LAUNCH_CHECK("sdr_seq_fwd");
      return SRF_OK;
    }
  }
  const size_t lds = fwd_lds(J, D);
  auto k = X.G > 1 ? sdr_seq_fwd_kernel<D, JP, NIM, true> : sdr_seq_fwd_kernel<D, JP, NIM, false>;
  if (lds > 64 * 1024)
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k, dim3(B * X.G, items.n), dim3(kThreads), lds, st, items, T, in_n, J, iters, mask_first, X);
  SRF_LAUNCH_CHECK("sdr_seq_fwd");
  return SRF_OK;
}

template <int D, int JP>
int fwd_nim(int nim, const srf::SeqItems& items, const srf_grp::Grp& X, int B, int T, int in_n, int J, int iters,
            int mask_first, hipStream_t st) {
  if (nim == 2) return launch_fwd<D, JP, 2>(items, X, B, T, in_n, J, iters, mask_first, st);
  if constexpr (D == 32 && JP == 32)
    if (nim == 3) return launch_fwd<D, JP, 3>(items, X, B, T, in_n, J, iters, mask_first, st);
  if (nim == 5) return launch_fwd<D, JP, 5>(items, X, B, T, in_n, J, iters, mask_first, st);
  if constexpr (seq_kd(D, JP) <= 8)
    return launch_fwd<D, JP, 10>(items, X, B, T, in_n, J, iters, mask_first, st);
  srf::set_error("sdr_seq: no forward kernel for %d input capsules per lane", nim);
  return SRF_EUNSUPPORTED;
}

}  // namespace

#if SRF_SEQ_STAMP
extern "C" int srf_seq_fwd_stamp_buffer(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

namespace srf {

bool sdr_seq_plan(int in_n, int J, int dout, int iters, int* nim, int* rm, int group) {
  if (J < 2 || J > 64 || iters < 1 || iters > 5 || in_n < 1) return false;
  if (dout != 8 && dout != 16 && dout != 32) return false;
  const int JP = srf_seq::pow2_at_least(J);
  if (dout * JP > 1024) return false;
  const int KD = srf_seq::seq_kd(dout, JP);
  const int G = srf_seq::seq_slots(dout, JP);
  const int ng = std::max(1, group), blk = (in_n + ng - 1) / ng;   // a group member's block (lane_map)
  const int NI = (blk + G - 1) / G;
  // 3 rows per lane only for dout = JP = 32 (the C3 last layer split over two
  // workgroups: 48 registers of u instead of 80, no spills, every row resident backward)
  const int m = NI <= 2                                ? 2
                : (NI <= 3 && dout == 32 && JP == 32) ? 3
                : NI <= 5                              ? 5
                : (NI <= 10 && KD <= 8)                ? 10
                                                       : 0;
  if (m == 0) return false;
  const int r = iters <= 3 ? 3 : 5;
  if (r == 5 && m != 2) return false;   // five-iteration backward kept for small layers only
  if (nim) *nim = m;
  if (rm) *rm = r;
  return true;
}

bool sdr_seq_supported(int in_n, int J, int dout, int iters) {
  return sdr_seq_plan(in_n, J, dout, iters, nullptr, nullptr);
}

size_t sdr_seq_cs_floats(int in_n, int J, int dout, int iters) {
  if (!sdr_seq_supported(in_n, J, dout, iters)) return 0;
  return (size_t)iters * ((size_t)in_n * srf_seq::pow2_at_least(J) + (size_t)J * dout);
}

size_t sdr_seq_fact_floats(int in_n, int J, int dout, int iters) {
  if (!sdr_seq_supported(in_n, J, dout, iters)) return 0;
  return (size_t)iters * ((size_t)in_n * srf_seq::pow2_at_least(J) + 2 * (size_t)J * dout);
}

int sdr_seq_fwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                hipStream_t st) {
  int nim = 0, rm = 0;
  srf_grp::Grp X;
  if (int rc = srf_grp::setup(items, B, 0, X, st)) return rc;
  if (!sdr_seq_plan(in_n, J, dout, iters, nullptr, nullptr) || !sdr_seq_plan(in_n, J, dout, iters, &nim, &rm, X.G)) {
    srf::set_error("sdr_seq: unsupported shape in_n=%d J=%d dout=%d iters=%d", in_n, J, dout, iters);
    return SRF_EUNSUPPORTED;
  }
  const int JP = srf_seq::pow2_at_least(J);
#define SRF_SEQ_F(DD, PP) \
  if (dout == DD && JP == PP) return fwd_nim<DD, PP>(nim, items, X, B, T, in_n, J, iters, mask_first, st);
  SRF_SEQ_CASES(SRF_SEQ_F)
#undef SRF_SEQ_F
  srf::set_error("sdr_seq: unsupported shape J=%d dout=%d", J, dout);
  return SRF_EUNSUPPORTED;
}

}  // namespace srf
