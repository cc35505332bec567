// Register-resident sequential routing kernels (route_sdr_seq*.hip): the
// per-utterance recurrence of SDR with the frame's u held in the registers of a
// 1024-thread workgroup.  Used by route_sdr.hip when the layer shape fits.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>

namespace srf {

// True when sdr_seq_fwd/bwd handle (in_n, J, dout, iters): dout in {8,16,32},
// J <= 64 (padded to a power of two JP, dout*JP <= 1024), in_n within the
// per-lane register budget.  Disabled by SRF_SDR_SEQ=0 (A/B runs, legacy tests).
bool sdr_seq_supported(int in_n, int J, int dout, int iters);

// u [B*T][in_n][J*dout] (pose output) -> v_out [B*T][J*dout]; one workgroup per utterance.
int sdr_seq_fwd(const float* u, int B, int T, int in_n, int J, int dout, int iters, int mask_first, float* v_out,
                hipStream_t st);

// Reverse-time pass: recomputes each frame's iterations from v_saved (the
// forward's v_out), writes gu [B*T][in_n][J*dout] = dL/du.
int sdr_seq_bwd(const float* u, const float* v_saved, const float* g_v, int B, int T, int in_n, int J, int dout,
                int iters, int mask_first, float* gu, hipStream_t st);

// Template choice for a shape: per-lane input-capsule count NIM in {2, 5, 10} and
// the iteration bound RM of the backward in {3, 5}.  False when unsupported.
bool sdr_seq_plan(int in_n, int J, int dout, int iters, int* nim, int* rm);

}  // namespace srf
