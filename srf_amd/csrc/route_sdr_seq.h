// Register-resident sequential routing kernels (route_sdr_seq*.hip): the
// per-utterance recurrence of SDR with the frame's u held in the registers of a
// 1024-thread workgroup.  Used by route_sdr.hip when the layer shape fits.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>

namespace srf {

// A range of frames of every utterance and the buffer views the recurrence kernels
// address (the chunked, layer-pipelined SDR stack runs a layer as several ranges):
//   frames t in [t0, t1) of each utterance are routed (backward: from t1-1 down);
//   u holds frames [tu0, tu0 + tu_n) of each utterance, laid out [B][tu_n][in_n][JD];
//   gu likewise holds frames [tg0, tg0 + tg_n);
//   v_out / v_saved / g_v are always whole [B][T][JD];
//   carry [B][JD] (backward): dL/dv_{t1-1} carried in from the later frames, and
//   dL/dv_{t0-1} carried out -- nullptr: start from 0 and drop it (whole-T calls).
// The forward starts from v_out[t0 - 1] (0 at t0 = 0).
struct SeqRange {
  int t0, t1, tu0, tu_n, tg0, tg_n;
  float* carry;
  static SeqRange whole(int T) { return SeqRange{0, T, 0, T, 0, T, nullptr}; }
};

// One recurrence launch runs up to kMaxItems frame ranges of layers with the same
// shape at once (grid.y = item): the layer-pipelined stack batches the ranges of one
// anti-diagonal of its wavefront into one launch instead of one stream per layer.
//   u: pose output view of the range; v: v_out (forward) / v_saved (backward);
//   g_v, gu: backward; cs: the range's layer couplings ([B][T][cs floats]);
//   ws: the stream backward's scratch (sdr_stream_workspace_floats).
constexpr int kMaxItems = 8;
struct SeqItem {
  const float* u;   // fp32, or bf16 (u_bf16: the streaming kernels only) behind the same pointer
  float* v;
  const float* g_v;
  float* gu;
  float* cs;
  float* ws;
  SeqRange rg;
  int u_bf16;
  int group;        // streaming kernels: workgroups per utterance (0, 1: one; route_sdr_stream.hip)
  int fact;         // register backward with cs: gu holds the per-frame gu factors (sdr_seq_fact_floats)
};
struct SeqItems {
  SeqItem it[kMaxItems];
  int n;
};

// True when sdr_seq_fwd/bwd handle (in_n, J, dout, iters): dout in {8,16,32},
// J <= 64 (padded to a power of two JP, dout*JP <= 1024), in_n within the
// per-lane register budget.
bool sdr_seq_supported(int in_n, int J, int dout, int iters);

// u [B*T][in_n][J*dout] (pose output) -> v_out [B*T][J*dout]; one workgroup per utterance.
// cs (optional, [B*T][sdr_seq_cs_floats]): the forward stores each frame's couplings
// c^r [iters][in_n][JP] and pre-squash s^r [iters][J*dout]; a backward given them
// skips recomputing the iterations.
size_t sdr_seq_cs_floats(int in_n, int J, int dout, int iters);
// gu factors of one frame (SeqItem::fact): gL^r [iters][in_n][JP], gs^r [iters][J*dout],
// Vc^r [iters][J*dout]; with the forward's c^r they give
// gu_ij = sum_r c^r_ij gs^r_j + gL^r_ij Vc^r_j (the consumer forms it).  The frame's record
// sits at gu + (b * tg_n + t - tg0) * sdr_seq_fact_floats.
size_t sdr_seq_fact_floats(int in_n, int J, int dout, int iters);
int sdr_seq_fwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                hipStream_t st);

// Reverse-time pass: recomputes each frame's iterations from v_saved (the
// forward's v_out), writes gu [B*T][in_n][J*dout] = dL/du.
int sdr_seq_bwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                hipStream_t st);

// Template choice for a shape: per-lane input-capsule count NIM in {2, 5, 10} and
// the iteration bound RM of the backward in {3, 5}, for `group` workgroups per
// utterance (SeqItem::group).  False when unsupported.
bool sdr_seq_plan(int in_n, int J, int dout, int iters, int* nim, int* rm, int group = 1);

// Streaming recurrence (route_sdr_stream.hip) for frames beyond the register budget
// (BASELINE C5): dout in {32, 64} with J*dout in {512, 1024, 2048} (dout 32: 512,
// 1024), in_n >= 8.  u_t is re-read from HBM once per iteration.  The forward
// stores per frame c^r [iters][in_n][J] and s^r [iters][J*dout]
// (sdr_stream_cs_floats, 256-B padded); the backward requires them and a scratch of
// sdr_stream_workspace_floats (gL^r of every utterance, and the exchange area of
// grouped launches: SeqItem::group > 1 workgroups per utterance).
bool sdr_stream_supported(int in_n, int J, int dout, int iters);
size_t sdr_stream_cs_floats(int in_n, int J, int dout, int iters);
size_t sdr_stream_workspace_floats(int B, int in_n, int J, int dout, int iters);
// the kernel's own scratch at the workspace start (the `pre` of srf_group.h)
size_t sdr_stream_pre_floats(int B, int in_n, int J, int iters);
int sdr_stream_fwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                   hipStream_t st);
int sdr_stream_bwd(const SeqItems& items, int B, int T, int in_n, int J, int dout, int iters, hipStream_t st);

}  // namespace srf
