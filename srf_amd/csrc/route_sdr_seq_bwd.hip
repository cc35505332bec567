// Backward of the SDR recurrence (route_sdr_seq.hip) with register-resident
// frames, gfx950: the autodiff of sequence_router_naive.py:162-170 / 212-245.
//
// One workgroup per utterance walks its frames in reverse.  Per frame it
// recomputes the R routing iterations from v_{t-1} (the forward's saved v), with
// Vc^r = v_{t-1} + sum_{k<r} v^k so that b^r = <u, Vc^r> (+ mask) by linearity of
// the b += <u, v> update, then runs the routing adjoint:
//   gs^r  = squash'(s^r)^T a^r,        a^{R-1} = g_v[t] + carry,
//   q_ij  = <u_ij, gs^r_j>,  sigma_i = sum_j c_ij q_ij,  gL_ij = c_ij (q_ij - sigma_i),
//   gVc^r = sum_i gL_ij u_ij,          a^{r-1} = sum_{r' >= r} gVc^{r'},
//   gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j,
//   carry (dL/dv_{t-1} for frame t-1) = sum_r gVc^r.
// u stays in registers (lane map of route_sdr_seq_dev.h); c^r and gL^r are per
// (lane, row) registers or LDS slabs; s^r, the running adjoints and the carry live in the
// registers of the thread that owns element e = j*D + d; Vc^r and gs^r go through
// LDS because every row reads them.
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

// c^r and gL^r of the lane's rows live in registers or, with CL (chosen when u
// already takes most of the lane's register budget and the slabs fit), in LDS
// [RM][in_n][JP] (written by the first lane of each capsule, read by all Q lanes).
constexpr bool cl_wanted(int nim, int kd) { return nim * kd >= 40; }

// LDS: w [JDp], Vc [RM][JDp], gs [RM][JDp], part [16][JD] (+ c, gL [RM][in_n][JP]);
// JDp = JP * D, the padded capsules' tails zero (lds_slice reads them unconditionally).
// CS: the forward stored each frame's couplings c^r and s^r (srf::sdr_seq_cs_floats
// per frame): the backward reads them instead of recomputing the R iterations, so
// only the adjoint runs per frame (and the logits no longer hold registers).
// With CS the lane keeps only its first KR rows of u in registers and re-reads the
// others from L2 where the adjoint uses them (once per iteration), and the gu pass
// runs over quarter slices of every row per LDS read of gs^r / Vc^r: the J = 32 last
// layer otherwise needs more than the 128 registers a 1024-thread workgroup allows.
// GRP (with CS): X.G workgroups per utterance split its input capsules (srf_group.h)
// and add their gVc^r partials inside the launch; member 0 writes the carry out.
// FACT (with CS): the frame's gu factors instead of gu (SeqItem::fact).
template <int D, int JP, int NIM, int RM, bool CL, bool CS, int KR = NIM, bool GRP = false, bool FACT = false>
__global__ __launch_bounds__(kThreads) void sdr_seq_bwd_kernel(srf::SeqItems items, int T, int in_n, int J,
                                                               int iters, int mask_first, srf_grp::Grp X) {
  using C = Cfg<D, JP, NIM>;
  const srf::SeqItem& I = items.it[blockIdx.y];   // the frame range of this launch item
  const float* __restrict__ u = I.u;
  const float* __restrict__ v_saved = I.v;
  const float* __restrict__ g_v = I.g_v;
  float* __restrict__ gu = I.gu;
  const float* __restrict__ cs = I.cs;
  const srf::SeqRange rg = I.rg;
  constexpr int RR = CL ? 1 : RM;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int JD = J * D;
  constexpr int JDa = JP * D;
  const int R = iters;
  float* wl = lds;
  float* vcl = wl + JDa;
  float* gsl = vcl + RM * JDa;
  float* part = gsl + RM * JDa;
  float* cl = part + kWaves * JD;          // [RM][in_n][JP] (CL only)
  float* gll = cl + RM * in_n * JP;        // [RM][in_n][JP] (CL only)
  const int tid = threadIdx.x;
  static_assert(CS || !GRP, "grouped backward reads the stored couplings");
  const int utt = GRP ? blockIdx.x / X.G : blockIdx.x;   // utterance
  const int gm = GRP ? blockIdx.x - utt * X.G : 0;       // member of its group
  const Lane L = lane_map<C>(in_n, J, mask_first, gm, GRP ? X.G : 1);
  const size_t ff = (size_t)in_n * JD;
  const size_t f0 = (size_t)utt * T;
  const float* ub = u + (size_t)utt * rg.tu_n * ff;    // frame t at ub + (t - tu0) * ff
  float* gub = gu + (size_t)utt * rg.tg_n * ff;        // frame t at gub + (t - tg0) * ff
  const bool owner_wave = (tid >> 6) * 64 < JD;
  const bool ev = tid < JD;
  if (rg.t0 >= rg.t1) return;
  float* carry_io = rg.carry ? rg.carry + (size_t)utt * JD : nullptr;
  // dL/dv_t carried back from frame t+1 (owner threads), from the later range
  float carry = (carry_io && ev) ? carry_io[tid] : 0.f;
  constexpr int KRES = CS ? KR : C::NIM;   // rows of u held in registers
  float ur[KRES][C::KD];
  float cr[RR][C::NIM], gl[RR][C::NIM];
  float sr[RM];        // s^r of the owned element
#pragma unroll
  for (int r = 0; r < RM; ++r) sr[r] = 0.f;
  if constexpr (!CS) load_rows<C, KRES>(ub + (size_t)(rg.t1 - 1 - rg.tu0) * ff, JD, L, ur);
  zero_tail(wl, 1 + 2 * RM, JD, JDa);   // w, Vc, gs are consecutive
  // ungrouped: barriers that wait on LDS only (no global data is exchanged inside the
  // kernel).  With CS the frame's rows of u are loaded right after its couplings are
  // requested, unconditionally, and stay in flight through the s^r / Vc^r phase and its
  // barriers to their first use in the adjoint (the group exchange drains all memory
  // operations anyway)
  auto bar = [&]() {
    if constexpr (!GRP) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  SEQ_STAMP_DECL
  for (int t = rg.t1 - 1; t >= rg.t0; --t) {
    const size_t f = f0 + t;
    float a = 0.f;
    if (ev) {
      const float vp = t > 0 ? v_saved[(f - 1) * JD + tid] : 0.f;
      wl[tid] = vp;
      vcl[tid] = vp;                       // Vc^0 = v_{t-1}
      a = g_v[f * JD + tid] + carry;       // dL/dv^{R-1}
      carry = 0.f;
    }
    if constexpr (CS) {
      // ---- the forward's c^r, s^r of this frame; Vc^{r+1} = Vc^r + squash(s^r)
      const int P = in_n * JP;
      const float* rec = cs + f * (size_t)R * (P + JD);
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        if (r < R) {
          if constexpr (CL) {
            for (int idx = tid; idx < P; idx += kThreads) cl[r * P + idx] = rec[r * P + idx];
          } else {
            load_ij<C>(rec + r * P, L, cr[r]);
          }
        }
      }
      // s^r of the owned element before the rows of u: waiting for them then leaves
      // the (younger) row loads in flight
#pragma unroll
      for (int r = 0; r < RM; ++r) sr[r] = (r < R && ev) ? rec[(size_t)R * P + r * JD + tid] : 0.f;
      load_rows<C, KRES>(ub + (size_t)(t - rg.tu0) * ff, JD, L, ur);
      bar();   // Vc^0 (above) before the owner threads extend it
      SEQ_MARK(0);       // v_{t-1}, g_v, c^r loads (+ the previous frame's barrier)
      if (owner_wave) {
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          if (r < R) {
            const float s = sr[r];
            if (r + 1 < R) {
              const float v = squash_elem<D>(s);
              if (ev) vcl[(r + 1) * JDa + tid] = vcl[r * JDa + tid] + v;
            }
          }
        }
      }
      bar();
      SEQ_MARK(1);       // s^r loads, Vc^r
    } else {
    bar();
    // ---- recompute the frame's iterations: c^r, s^r, Vc^r
    float b[C::NIM];
#pragma unroll
    for (int k = 0; k < C::NIM; ++k) b[k] = 0.f;
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      if (r < R) {
        float w[C::KD], cc[C::NIM];
        lds_slice<C::KD>(wl, L.eoff, w);
        logits_softmax<C>(ur, w, L, b, cc);
        row_partial<C>(cc, ur, L, JD, part);
        if constexpr (CL) {
          store_ij<C>(cc, L, cl + r * in_n * JP);
        } else {
#pragma unroll
          for (int k = 0; k < C::NIM; ++k) cr[r][k] = cc[k];
        }
        bar();
        if (owner_wave) {
          const float s = ev ? sum_parts(part, JD, tid) : 0.f;
          sr[r] = s;
          const float v = squash_elem<D>(s);
          if (ev) {
            wl[tid] = v;
            if (r + 1 < R) vcl[(r + 1) * JDa + tid] = vcl[r * JDa + tid] + v;
          }
        }
        bar();
      }
    }
    }   // recompute
    // ---- adjoint, r = R-1 .. 0 (a = dL/dv^r)
    float grun = 0.f;
#pragma unroll
    for (int r = RM - 1; r >= 0; --r) {
      if (r < R) {
        if (owner_wave) {
          const float s = sr[r];
          const float n2 = group_sum<1, D>(s * s);
          const float sa = group_sum<1, D>(s * a);
          const float rs = __builtin_amdgcn_rsqf(n2 + kSquashEps);
          const float ip = __builtin_amdgcn_rcpf(1.f + n2);
          const float gfac = n2 * ip * rs;
          const float dg2 = 2.f * rs * ip * (ip - 0.5f * n2 * rs * rs) * sa;
          if (ev) gsl[r * JDa + tid] = gfac * a + dg2 * s;
        }
        bar();
        SEQ_MARK(2);     // squash adjoint

        float gsv[C::KD], cc[C::NIM], gg[C::NIM];
        lds_slice<C::KD>(gsl + r * JDa, L.eoff, gsv);
        if constexpr (CL) {
          load_ij<C>(cl + r * in_n * JP, L, cc);
        } else {
#pragma unroll
          for (int k = 0; k < C::NIM; ++k) cc[k] = cr[r][k];
        }
        if constexpr (CS) {
          // rows in registers (k < KR): q, sigma, gL first; then the rows re-read from L2
          // one at a time (q, sigma, gL and their gVc share); then the resident rows' share
          auto adjoint = [&](int k, const float (&urow)[C::KD]) {
            float p0 = 0.f, p1 = 0.f;
#pragma unroll
            for (int d = 0; d < C::KD; d += 2) {
              p0 += urow[d] * gsv[d];
              p1 += urow[d + 1] * gsv[d + 1];
            }
            const float q = group_sum<1, C::Q>(p0 + p1);
            const float sig = group_sum<C::Q, C::ROWL>(cc[k] * q);
            gg[k] = cc[k] * (q - sig);
          };
#pragma unroll
          for (int k = 0; k < C::NIM; ++k) {
            gg[k] = 0.f;
            if (k < KR && k < L.NI) adjoint(k, ur[k < KR ? k : 0]);
          }
          float sp[C::KD];
#pragma unroll
          for (int d = 0; d < C::KD; ++d) sp[d] = 0.f;
          const float* uf = ub + (size_t)(t - rg.tu0) * ff;
#pragma unroll
          for (int k = KR; k < C::NIM; ++k) {
            __builtin_amdgcn_sched_barrier(0);   // one re-read row in flight at a time
            if (k < L.NI) {
              float urow[C::KD];
              load_row<C>(uf, JD, L, k, urow);
              adjoint(k, urow);
#pragma unroll
              for (int d = 0; d < C::KD; ++d) sp[d] += gg[k] * urow[d];
            }
          }
#pragma unroll
          for (int k = 0; k < KR; ++k)
#pragma unroll
            for (int d = 0; d < C::KD; ++d) sp[d] += gg[k] * ur[k][d];
          partial_out<C>(sp, L, JD, part);
        } else {
#pragma unroll
        for (int k = 0; k < C::NIM; ++k) {
          gg[k] = 0.f;
          if (k < L.NI) {
            float p0 = 0.f, p1 = 0.f;
#pragma unroll
            for (int d = 0; d < C::KD; d += 2) {
              p0 += ur[k][d] * gsv[d];
              p1 += ur[k][d + 1] * gsv[d + 1];
            }
            const float q = group_sum<1, C::Q>(p0 + p1);
            const float sig = group_sum<C::Q, C::ROWL>(cc[k] * q);
            gg[k] = cc[k] * (q - sig);
          }
        }
        row_partial<C>(gg, ur, L, JD, part);
        }   // CS
        if constexpr (CL) {
          store_ij<C>(gg, L, gll + r * in_n * JP);
        } else {
#pragma unroll
          for (int k = 0; k < C::NIM; ++k) gl[r][k] = gg[k];
        }
        SEQ_MARK(3);     // q, sigma, gL, gVc partials (+ re-read rows)
        bar();
        if constexpr (GRP)
          srf_grp::allreduce<kWaves, kThreads>(part, JD, I.ws, X, utt, gm, (rg.t1 - 1 - t) * R + (R - 1 - r), tid);
        SEQ_MARK(4);
        if (ev) {
          const float g = GRP ? part[tid] : sum_parts(part, JD, tid);   // gVc^r_e
          carry += g;
          grun = (r == R - 1) ? g : grun + g;
          a = grun;
        }
        SEQ_MARK(5);
      }
    }
    // ---- gu (u is dead: its registers take the next frame's loads, issued right
    // after); without CS one input capsule of the lane at a time
    if constexpr (CS && FACT) {
      // the frame's gu factors instead of gu (SeqItem::fact): gL^r of the member's input
      // capsules, gs^r and Vc^r (member 0: the members hold the same sums); the
      // consumer forms gu with the forward's c^r
      const int P = in_n * JP;
      float* rec = gu + ((size_t)utt * rg.tg_n + (t - rg.tg0)) * ((size_t)R * (P + 2 * JD));
      if constexpr (CL) {
        const int ng = GRP ? X.G : 1, blk = (in_n + ng - 1) / ng, b0 = gm * blk;
        const int nl = max(0, min(in_n, b0 + blk) - b0) * JP;
        for (int idx = tid; idx < R * nl; idx += kThreads) {
          const int r = idx / nl, o = b0 * JP + idx - r * nl;
          rec[r * P + o] = gll[r * P + o];
        }
      } else {
#pragma unroll
        for (int r = 0; r < RM; ++r)
          if (r < R) store_ij<C>(gl[r], L, rec + r * P);
      }
      if (ev && gm == 0) {
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          if (r < R) {
            rec[R * P + r * JD + tid] = gsl[r * JDa + tid];
            rec[R * (P + JD) + r * JD + tid] = vcl[r * JDa + tid];
          }
        }
      }
    } else if constexpr (CS) {
      // four of the lane's KD values per pass, every row at once: one LDS read of each
      // gs^r / Vc^r quarter slice per pass serves all NIM rows
      constexpr int HD = 4;
#pragma unroll
      for (int d0 = 0; d0 < C::KD; d0 += HD) {
        float acc[C::NIM][HD];
#pragma unroll
        for (int k = 0; k < C::NIM; ++k)
#pragma unroll
          for (int d = 0; d < HD; ++d) acc[k][d] = 0.f;
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          if (r < R) {
            float gsv[HD], vcv[HD];
            lds_slice<HD>(gsl + r * JDa, L.eoff + d0, gsv);
            lds_slice<HD>(vcl + r * JDa, L.eoff + d0, vcv);
#pragma unroll
            for (int k = 0; k < C::NIM; ++k) {
              if (k < L.NI) {
                float ck, gk;
                if constexpr (CL) {
                  const int idx = (L.g + k * C::G) * JP + L.j;
                  ck = cl[r * in_n * JP + idx];
                  gk = gll[r * in_n * JP + idx];
                } else {
                  ck = cr[r][k];
                  gk = gl[r][k];
                }
#pragma unroll
                for (int d = 0; d < HD; ++d) acc[k][d] += ck * gsv[d] + gk * vcv[d];
              }
            }
          }
        }
#pragma unroll
        for (int k = 0; k < C::NIM; ++k) {
          if (k < L.NI && L.jv) {
            float* dst = gub + (size_t)(t - rg.tg0) * ff + (size_t)(L.g + k * C::G) * JD + L.eoff + d0;
            *reinterpret_cast<f4*>(dst) = f4{acc[k][0], acc[k][1], acc[k][2], acc[k][3]};
          }
        }
      }
    } else {
#pragma unroll
    for (int k = 0; k < C::NIM; ++k) {
      if (k < L.NI) {
        float acc[C::KD];
#pragma unroll
        for (int d = 0; d < C::KD; ++d) acc[d] = 0.f;
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          if (r < R) {
            float gsv[C::KD], vcv[C::KD];
            lds_slice<C::KD>(gsl + r * JDa, L.eoff, gsv);
            lds_slice<C::KD>(vcl + r * JDa, L.eoff, vcv);
            float ck, gk;
            if constexpr (CL) {
              const int idx = (L.g + k * C::G) * JP + L.j;
              ck = cl[r * in_n * JP + idx];
              gk = gll[r * in_n * JP + idx];
            } else {
              ck = cr[r][k];
              gk = gl[r][k];
            }
#pragma unroll
            for (int d = 0; d < C::KD; ++d) acc[d] += ck * gsv[d] + gk * vcv[d];
          }
        }
        if (L.jv) {
          float* dst = gub + (size_t)(t - rg.tg0) * ff + (size_t)(L.g + k * C::G) * JD + L.eoff;
#pragma unroll
          for (int c = 0; c < C::KD; c += 4) *reinterpret_cast<f4*>(dst + c) = f4{acc[c], acc[c + 1], acc[c + 2], acc[c + 3]};
        }
      }
    }
    }   // CS gu
    SEQ_MARK(6);       // gu
    if constexpr (!CS)   // unconditional (the range's first frame reloads itself): no register merge
      load_rows<C, KRES>(ub + (size_t)(max(t - 1, rg.t0) - rg.tu0) * ff, JD, L, ur);
    bar();   // the next frame overwrites w, Vc^0 and the c / gL slabs
    SEQ_MARK(7);
  }
  SEQ_FLUSH(g_stamps);
  if (carry_io && ev && gm == 0) carry_io[tid] = carry;   // dL/dv_{t0-1} for the earlier range
  srf_grp::depart<GRP>(I.ws, X, utt, tid);
}

size_t bwd_lds(int J, int D, int RM, int in_n, bool cl) {
  const size_t JP = (size_t)pow2_at_least(J);
  const size_t JDa = JP * D;
  return (JDa * (1 + 2 * (size_t)RM) + (size_t)kWaves * J * D + (cl ? 2 * (size_t)RM * in_n * JP : 0)) *
         sizeof(float);
}

template <int D, int JP, int NIM, int RM>
int launch_bwd(const srf::SeqItems& items, const srf_grp::Grp& X, bool cs, bool fact, int B, int T, int in_n, int J, int iters,
               int mask_first, hipStream_t st) {
  constexpr bool want = cl_wanted(NIM, seq_kd(D, JP));
  const bool cl = want && bwd_lds(J, D, RM, in_n, true) <= 160 * 1024;
  const size_t lds = bwd_lds(J, D, RM, in_n, cl);
  // with stored couplings: rows past KR re-read from L2 when u would take more than 48
  // of the 128 registers (the J = 32, dout = 32 last layer: 5 rows of 16 values)
  constexpr int KD = seq_kd(D, JP);
  constexpr int KR = NIM * KD > 48 ? 32 / KD : NIM;
  SRF_REQUIRE(cs || X.G == 1, "sdr_seq: a grouped backward needs the forward's stored couplings");
  SRF_REQUIRE(cs || !fact, "sdr_seq: gu factors need the forward's stored couplings");
  // factor instances for dout 32 only (their consumer, the din = dout = 32 gx / gW pass)
  constexpr bool FT = D == 32;
  SRF_REQUIRE(FT || !fact, "sdr_seq: gu factors for dout 32 only, got %d", D);
  auto k = X.G > 1 ? (fact ? (cl ? sdr_seq_bwd_kernel<D, JP, NIM, RM, want, true, KR, true, FT>
                                 : sdr_seq_bwd_kernel<D, JP, NIM, RM, false, true, KR, true, FT>)
                           : (cl ? sdr_seq_bwd_kernel<D, JP, NIM, RM, want, true, KR, true>
                                 : sdr_seq_bwd_kernel<D, JP, NIM, RM, false, true, KR, true>))
           : cs    ? (fact ? (cl ? sdr_seq_bwd_kernel<D, JP, NIM, RM, want, true, KR, false, FT>
                                 : sdr_seq_bwd_kernel<D, JP, NIM, RM, false, true, KR, false, FT>)
                           : (cl ? sdr_seq_bwd_kernel<D, JP, NIM, RM, want, true, KR>
                                 : sdr_seq_bwd_kernel<D, JP, NIM, RM, false, true, KR>))
                   : (cl ? sdr_seq_bwd_kernel<D, JP, NIM, RM, want, false>
                         : sdr_seq_bwd_kernel<D, JP, NIM, RM, false, false>);
  if (lds > 64 * 1024)
    SRF_HIP_TRY(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k, dim3(B * X.G, items.n), dim3(kThreads), lds, st, items, T, in_n, J, iters, mask_first, X);
  SRF_LAUNCH_CHECK("sdr_seq_bwd");
  return SRF_OK;
}

template <int D, int JP>
int bwd_nim(int nim, int rm, const srf::SeqItems& items, const srf_grp::Grp& X, bool cs, bool fact, int B, int T, int in_n,
            int J, int iters, int mask_first, hipStream_t st) {
  if (rm == 5) return launch_bwd<D, JP, 2, 5>(items, X, cs, fact, B, T, in_n, J, iters, mask_first, st);
  if (nim == 2) return launch_bwd<D, JP, 2, 3>(items, X, cs, fact, B, T, in_n, J, iters, mask_first, st);
  if constexpr (D == 32 && JP == 32)
    if (nim == 3) return launch_bwd<D, JP, 3, 3>(items, X, cs, fact, B, T, in_n, J, iters, mask_first, st);
  if (nim == 5) return launch_bwd<D, JP, 5, 3>(items, X, cs, fact, B, T, in_n, J, iters, mask_first, st);
  if constexpr (seq_kd(D, JP) <= 8)
    return launch_bwd<D, JP, 10, 3>(items, X, cs, fact, B, T, in_n, J, iters, mask_first, st);
  srf::set_error("sdr_seq: no backward kernel for %d input capsules per lane", nim);
  return SRF_EUNSUPPORTED;
}

}  // namespace

#if SRF_SEQ_STAMP
extern "C" int srf_seq_bwd_stamp_buffer(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#endif

namespace srf {

int sdr_seq_bwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                hipStream_t st) {
  // the items of one launch share the kernel: all with stored couplings or none
  const bool cs = items.n > 0 && items.it[0].cs != nullptr;
  const bool fact = items.n > 0 && items.it[0].fact;
  for (int k = 1; k < items.n; ++k) {
    SRF_REQUIRE((items.it[k].cs != nullptr) == cs, "sdr_seq: launch items mix stored and recomputed couplings");
    SRF_REQUIRE((items.it[k].fact != 0) == fact, "sdr_seq: launch items mix gu and gu factors");
  }
  int nim = 0, rm = 0;
  srf_grp::Grp X;
  if (int rc = srf_grp::setup(items, B, 0, X, st)) return rc;
  if (!sdr_seq_plan(in_n, J, dout, iters, nullptr, nullptr) || !sdr_seq_plan(in_n, J, dout, iters, &nim, &rm, X.G)) {
    srf::set_error("sdr_seq: unsupported shape in_n=%d J=%d dout=%d iters=%d", in_n, J, dout, iters);
    return SRF_EUNSUPPORTED;
  }
  const int JP = srf_seq::pow2_at_least(J);
#define SRF_SEQ_B(DD, PP)     \
  if (dout == DD && JP == PP) \
    return bwd_nim<DD, PP>(nim, rm, items, X, cs, fact, B, T, in_n, J, iters, mask_first, st);
  SRF_SEQ_CASES(SRF_SEQ_B)
#undef SRF_SEQ_B
  srf::set_error("sdr_seq: unsupported shape J=%d dout=%d", J, dout);
  return SRF_EUNSUPPORTED;
}

}  // namespace srf
