/* srf.h -- C ABI of the MI355X-native Sequential Routing Framework hot path.
 *
 * Every entry point takes caller-owned device pointers (fp32 unless stated),
 * plain int shapes and a hipStream_t passed as void*.  Nothing allocates and
 * nothing synchronises: calls are stream-ordered and may be captured into a
 * hipGraph.  One piece of process-wide state exists, set only by the caller: the
 * dropout step counter of srf_set_seed_source (below); every other call depends
 * on its arguments alone.  Return value: 0 on success, < 0 on error
 * (SRF_EINVAL -1 bad argument, SRF_EHIP -2 HIP error, SRF_EUNSUPPORTED -3,
 * SRF_EWORKSPACE -4); srf_last_error() then holds a thread-local message.
 *
 * Layouts (HBM):
 *   emb   [B*T][N][din]          capsules of one routing layer's input frames
 *   W     [in_n][J][dout][din]   in_n = N*(lpad+1+rpad); the reference variable
 *                                W%d of shape (1,1,in_n,J,dout,din)
 *   bias  [in_n][J][dout]        the reference b%d of shape (1,1,in_n,J,dout,1)
 *   v     [B*T][J][dout]
 */
#ifndef SRF_H_
#define SRF_H_
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Library identity / diagnostics. */
int srf_version(void);
const char* srf_last_error(void);

/* ---- Dynamic routing layer: window + pose transform + DR ------------------
 * Replaces tfsr/model/sequence_router_naive.py:149-185 (ZeroPadding2D+concat
 * window :150-151, tile+matmul pose :154-159, tf.while_loop DR :171-185 with
 * _loop_body :199-206) and, for the backward, its TF autodiff.
 * mask_first = 1 for the last layer (the -1e9 logit mask on capsule 0,
 * naive:173-178).  n_chunks splits the input capsules over workgroups
 * (srf_route_dr_auto_chunks gives the tuned default).
 * saved: 2*iters*B*T*J*dout floats written by the forward and read by the
 * backward (s^r and the accumulated agreement vector after each iteration). */
int srf_route_dr_auto_chunks(int B, int T, int N, int din, int lpad, int rpad, int J, int dout);
size_t srf_route_dr_saved_floats(int B, int T, int J, int dout, int iters);
size_t srf_route_dr_fwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters,
                                  int n_chunks);
size_t srf_route_dr_bwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters,
                                  int n_chunks);
int srf_route_dr_fwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int iters, int mask_first, int n_chunks, float* v_out,
                     float* saved, void* workspace, size_t workspace_bytes, void* stream);
/* Coupling storage (the 32x32 split-fp16 path: din in {8, 16, 32} <= dout in {8, 16, 32},
 * J*dout <= 1024; 0 for other shapes or iters < 2): the couplings c^r and logZ^r
 * of the routing iterations r >= 1, written by srf_route_dr_fwd_ex when
 * couplings != NULL and read by srf_route_dr_bwd_ex / _bwd_data_ex, whose
 * backward routing passes then skip the logit and softmax recompute.  NULL
 * couplings: the plain entry points' behaviour (forward stores nothing, backward
 * recomputes).  Inference passes NULL. */
size_t srf_route_dr_coupling_floats(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters);
int srf_route_dr_fwd_ex(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                        int rpad, int J, int dout, int iters, int mask_first, int n_chunks, float* v_out,
                        float* saved, float* couplings, void* workspace, size_t workspace_bytes, void* stream);
int srf_route_dr_bwd_ex(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                        int rpad, int J, int dout, int iters, int mask_first, int n_chunks, const float* saved,
                        const float* couplings, const float* g_v, float* g_emb, float* g_W, float* g_bias,
                        void* workspace, size_t workspace_bytes, void* stream);
/* _bwd_weights of a backward whose _bwd_data_ex was given couplings: the same
 * saved and couplings buffers. */
int srf_route_dr_bwd_weights_ex(const float* emb, int B, int T, int N, int din, int lpad, int rpad, int J, int dout,
                                int iters, int mask_first, int n_chunks, const float* saved, const float* couplings,
                                float* g_W, float* g_bias, void* workspace, size_t workspace_bytes, void* stream);
int srf_route_dr_bwd_data_ex(const float* emb, const float* W, const float* bias, int B, int T, int N, int din,
                             int lpad, int rpad, int J, int dout, int iters, int mask_first, int n_chunks,
                             const float* saved, const float* couplings, const float* g_v, float* g_emb,
                             void* workspace, size_t workspace_bytes, void* stream);
/* Dropout step counter -- PROCESS-GLOBAL state: a device uint64 that every dropout
 * kernel launched afterwards, from any thread and for any model, mixes into its
 * seed (NULL restores the per-call seeds alone).  It lets a training step captured
 * into a hipGraph draw fresh masks on every replay: the step advances the counter
 * on the device.  Forward and backward of one step must see the same counter value
 * (the autograd backward runs on torch's device worker thread, hence process-wide,
 * not per thread).  One process drives one GPU, so the host keeps one counter per
 * process and never detaches it (srf_amd.trainer_sr.seed_counter). */
int srf_set_seed_source(const void* step_counter);
/* Fault word -- PROCESS-GLOBAL state like the step counter: a device uint32 that a
 * grouped SDR recurrence (srf_sdr_range.group > 1) sets to nonzero when a member gave
 * up waiting for the others (they were not resident together), i.e. when the launch's
 * results are wrong.  Kernels only set it; the caller reads and clears it at its next
 * synchronisation (srf_amd.ops.check_faults).  NULL: no reporting. */
int srf_set_fault_flag(void* flag);
/* Gradients are written (not accumulated): g_emb [B*T][N][din], g_W like W,
 * g_bias like bias. */
int srf_route_dr_bwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int iters, int mask_first, int n_chunks, const float* saved,
                     const float* g_v, float* g_emb, float* g_W, float* g_bias, void* workspace,
                     size_t workspace_bytes, void* stream);
/* The same backward in two stream-ordered parts.  _data writes g_emb and leaves the
 * gu blocks in the workspace; _weights (same workspace, same geometry) then writes
 * g_W and g_bias.  _weights depends on nothing else, so a caller may launch it on a
 * second stream that waits for _data, and join that stream before reading g_W /
 * g_bias or reusing the workspace: the weight contraction then overlaps the
 * backward of the layers below.  srf_route_dr_bwd = _data + _weights on one stream. */
int srf_route_dr_bwd_data(const float* emb, const float* W, const float* bias, int B, int T, int N, int din,
                          int lpad, int rpad, int J, int dout, int iters, int mask_first, int n_chunks,
                          const float* saved, const float* g_v, float* g_emb, void* workspace,
                          size_t workspace_bytes, void* stream);
int srf_route_dr_bwd_weights(const float* emb, int B, int T, int N, int din, int lpad, int rpad, int J, int dout,
                             int iters, int mask_first, int n_chunks, float* g_W, float* g_bias, void* workspace,
                             size_t workspace_bytes, void* stream);

/* ---- Sequential dynamic routing layer: window + pose transform + SDR -------
 * Replaces tfsr/model/sequence_router_naive.py:162-170 (tf.while_loop over the
 * frames) with body_context :231-245 and, for the last layer, pad_body_context
 * :212-229; and their TF autodiff.  Frames of an utterance are routed in order,
 * the previous frame's final v seeding the next frame's logits.  saved: the
 * per-frame v (srf_route_sdr_saved_floats), written by the forward, read by the
 * backward.  Returns SRF_EUNSUPPORTED when one frame's routing state exceeds a
 * CU's LDS. */
size_t srf_route_sdr_saved_floats(int B, int T, int J, int dout);
size_t srf_route_sdr_fwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout);
size_t srf_route_sdr_bwd_workspace(int B, int T, int N, int din, int lpad, int rpad, int J, int dout, int iters);
int srf_route_sdr_fwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                      int rpad, int J, int dout, int iters, int mask_first, float* v_out, float* saved,
                      void* workspace, size_t workspace_bytes, void* stream);
int srf_route_sdr_bwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                      int rpad, int J, int dout, int iters, int mask_first, const float* saved, const float* g_v,
                      float* g_emb, float* g_W, float* g_bias, void* workspace, size_t workspace_bytes,
                      void* stream);

/* ---- Batched frame ranges (the layer-pipelined SDR stack, ops.SdrStack): one launch
 * runs up to SRF_SDR_MAX_ITEMS frame ranges [t0, t1) of layers with the same shape
 * (one anti-diagonal of the stack's wavefront), instead of one HIP stream per layer.
 * Each entry point reads only its fields; the single-range functions below are the
 * n = 1 case.  Ranges with t0 == t1 are skipped (gW: one with accumulate == 0 still
 * zeroes its layer's gradient).  Replaces the per-layer loop of
 * sequence_router_naive.py:145-191 over the frames of :162-170. */
#define SRF_SDR_MAX_ITEMS 8
typedef struct {
  int t0, t1;                  /* frame range of every utterance */
  const float* emb;            /* layer input [B][T][N][din] (pose, gW) */
  const float* W;              /* pose: [in_n][J*dout][din] */
  const float* bias;           /* pose: [in_n][J*dout] */
  const float* WT;             /* gx: W^T [in_n][din][J*dout] */
  float* u;                    /* pose output / recurrence input, frames [v0, v0 + vn) */
  int v0, vn;
  float* v;                    /* recur_fwd: v_out; recur_bwd: the forward's v [B][T][J*dout] */
  float* couplings;            /* [B][T][srf_route_sdr_coupling_floats] or NULL */
  void* workspace;             /* srf_route_sdr_recur_workspace bytes, per range */
  size_t workspace_bytes;
  const float* g_v;            /* recur_bwd: dL/dv [B][T][J*dout] */
  float* carry;                /* recur_bwd: [B][J*dout] in / out */
  float* gu;                   /* recur_bwd output, gx / gW input: frames [g0, g0 + gn) */
  int g0, gn;
  float* g_emb;                /* gx: added into [B][T][N][din] */
  float* g_W;                  /* gW: [in_n][J*dout][din] */
  float* g_bias;               /* gW: [in_n][J*dout] */
  int accumulate;              /* gW: add to g_W / g_bias (else overwrite) */
  int u_bf16;                  /* u holds bf16 (written by pose_n mode 2; read by the streaming
                                  recurrence kernels only, i.e. srf_route_sdr_couplings_required) */
  int group;                   /* recur_fwd_n / recur_bwd_n on the streaming kernels: workgroups per
                                  utterance (0 or 1: one; at most 8, equal over a launch's ranges).
                                  A group splits the input capsules and adds its partial sums inside
                                  the launch, spin-waiting on its members: the launch's
                                  B * n * group workgroups must be resident together.  The library
                                  cannot see what else holds CUs: it refuses a launch above the
                                  device's CU count less 4, and the caller keeps other grouped
                                  launches, and kernels that occupy CUs for long (collectives),
                                  off the device meanwhile.  A member that waits too long stops
                                  and sets the fault word (srf_set_fault_flag): the results of
                                  that launch are then wrong.  The group's counters live in the
                                  workspace: it must be zero before the first grouped launch on
                                  it, and each grouped launch leaves its counters zero again
                                  (the timeout word excepted).  Other shapes ignore it. */
  int gu_factored;             /* recur_bwd_n on the register kernels with couplings (C3): gu holds
                                  each frame's gu factors (srf_route_sdr_fact_floats per frame)
                                  instead of gu; srf_route_sdr_gx_gw_fact_n reads them */
} srf_sdr_range;
/* pose_n fp8: 0 fp32 pose, 1 fp8 pose (fp32 u), 2 fp8 pose storing u in bf16 */
int srf_route_sdr_pose_n(const srf_sdr_range* ranges, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                         int dout, int fp8, void* stream);
int srf_route_sdr_recur_fwd_n(const srf_sdr_range* ranges, int n, int B, int T, int in_n, int J, int dout, int iters,
                              int mask_first, void* stream);
int srf_route_sdr_recur_bwd_n(const srf_sdr_range* ranges, int n, int B, int T, int in_n, int J, int dout, int iters,
                              int mask_first, void* stream);
int srf_route_sdr_gx_n(const srf_sdr_range* ranges, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                       int dout, void* stream);
int srf_route_sdr_gw_n(const srf_sdr_range* ranges, int n, int B, int T, int N, int din, int lpad, int rpad, int J,
                       int dout, void* stream);
/* gx_n and gw_n of the same ranges in one launch that reads gu once (din 32; other
 * shapes run the two entry points above).  Reads W (not WT) besides their fields. */
int srf_route_sdr_gx_gw_n(const srf_sdr_range* ranges, int n, int B, int T, int N, int din, int lpad, int rpad,
                          int J, int dout, void* stream);
/* The same from the recurrence's gu factors (ranges with gu_factored, whose recur_bwd_n
 * wrote srf_route_sdr_fact_floats per frame into gu): gu_ij = sum_r c^r_ij gs^r_j +
 * gL^r_ij Vc^r_j is formed inside the contraction with the forward's couplings, so gu
 * never crosses HBM.  din = dout = 32, J a multiple of 8, iters <= 3.  Reads couplings,
 * gu (the factors), W, emb; writes as gx_gw_n. */
int srf_route_sdr_gx_gw_fact_n(const srf_sdr_range* ranges, int n, int B, int T, int N, int din, int lpad, int rpad,
                               int J, int dout, int iters, void* stream);

/* ---- The SDR layer in frame ranges (the layer-pipelined SDR stack) ----------
 * srf_route_sdr_fwd/bwd split into calls over frames [t0, t1) of every utterance,
 * so a host can run an SDR stack as a wavefront over (layer, frame range): layer
 * l's range k needs only layer l-1's output up to frame t1 - 1 + rpad (the window,
 * naive:150-151), and, going backward, layer l+1's gx down to frame t0 - rpad.
 * Same arithmetic as the whole-layer calls (naive:162-170, 212-245 and autodiff).
 *   u / gu buffers hold frames [v0, v0 + vn) / [g0, g0 + gn) of each utterance,
 *   laid out [B][vn][in_n][J*dout] (v0 = 0, vn = T: the whole layer);
 *   v_out, v_saved, g_v are whole [B][T][J*dout];
 *   recur_fwd starts from v_out[t0 - 1] (0 at t0 = 0): earlier ranges first;
 *   recur_bwd walks t1-1 .. t0, carry [B][J*dout] holds dL/dv_{t1-1} on entry
 *   (zero it before the last range) and dL/dv_{t0-1} on return: later ranges first;
 *   gx adds W^T gu of the range's frames into g_emb through the window adjoint
 *   (zero g_emb first); gw writes (accumulate = 0) or adds the range's
 *   gW = sum_f gu x^T and g_bias = sum_f gu.
 * recur_workspace: state slices for shapes beyond the register / LDS budget (0 else). */
int srf_route_sdr_pose(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                       int rpad, int J, int dout, int t0, int t1, float* u, int v0, int vn, void* stream);
/* The same on fp8 (OCP e4m3) MFMA, opt-in (BASELINE C5 "fp8 pose-transform MFMA"): x
 * per frame and W per row scaled by powers of two into e4m3 range, fp32 accumulation,
 * fp32 bias.  Bound per element: |u - u_exact| <= 0.13 * sum_k |W_rk| |x_k| (+ fp32
 * rounding).  in_d 32 or 64. */
int srf_route_sdr_pose_fp8(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                           int rpad, int J, int dout, int t0, int t1, float* u, int v0, int vn, void* stream);
size_t srf_route_sdr_recur_workspace(int B, int in_n, int J, int dout, int iters);
/* The part of that workspace that must be zero before its first grouped launch (the
 * group counters and the timeout word, srf_sdr_range.group): *offset_bytes from the
 * workspace's start, the return value its length in bytes.  The rest (kernel scratch,
 * exchange area) needs no initialisation.  Shapes on the LDS / global-state kernels
 * return the whole workspace. */
size_t srf_route_sdr_recur_zero_range(int B, int in_n, int J, int dout, int iters, size_t* offset_bytes);
/* Coupling storage per frame (0 when the shape runs on the LDS / global-state
 * kernels): with couplings != NULL ([B][T][this many floats]) recur_fwd stores each
 * frame's couplings c^r and pre-squash s^r, and recur_bwd reads them instead of
 * recomputing the frame's iterations (NULL: recompute).  Shapes on the streaming
 * kernels (frames beyond the register budget, e.g. BASELINE C5) have no recompute
 * path: srf_route_sdr_couplings_required is 1 and recur_bwd needs them. */
size_t srf_route_sdr_coupling_floats(int in_n, int J, int dout, int iters);
int srf_route_sdr_couplings_required(int in_n, int J, int dout, int iters);
/* Floats of one frame's gu factors (srf_sdr_range.gu_factored): gL^r [iters][in_n][JP],
 * gs^r and Vc^r [iters][J*dout] each (JP = J rounded up to a power of two, at least 4);
 * 0 where the layer's backward cannot write them (no register kernel for the shape). */
size_t srf_route_sdr_fact_floats(int in_n, int J, int dout, int iters);
int srf_route_sdr_recur_fwd(const float* u, int v0, int vn, int B, int T, int in_n, int J, int dout, int iters,
                            int mask_first, int t0, int t1, float* v_out, float* couplings, void* workspace,
                            size_t workspace_bytes, void* stream);
int srf_route_sdr_recur_bwd(const float* u, int v0, int vn, const float* v_saved, const float* couplings,
                            const float* g_v, int B, int T, int in_n, int J, int dout, int iters, int mask_first,
                            int t0, int t1, float* carry, float* gu, int g0, int gn, void* workspace,
                            size_t workspace_bytes, void* stream);
/* W [in_n][J*dout][din] -> WT [in_n][din][J*dout] (the gx operand). */
int srf_route_sdr_transpose_w(const float* W, int in_n, int J, int dout, int din, float* WT, void* stream);
int srf_route_sdr_gx(const float* gu, int g0, int gn, const float* WT, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int t0, int t1, float* g_emb, void* stream);
int srf_route_sdr_gw(const float* gu, int g0, int gn, const float* emb, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int t0, int t1, int accumulate, float* g_W, float* g_bias,
                     void* stream);

/* ---- CNN front end (CapsulationLayer, tfsr/model/sequence_router.py:44-82) ---
 * feats [B][T][feat_dim] fp32 (already cropped to max(inp_len), trainer_sr.py:59-60),
 * inp_len [B] int32 (device).  Kernels [3][3][Cin][64] (kh, kw, cin, cout), as the
 * reference's Conv2D variables; biases/gamma/beta [64].  The two convolutions of
 * each stage are the reference's conv_layers[0][k] and conv_layers[1][k]
 * (sequence_router.py:76-77).  out = mask2(BN2(.)) [B][T2][F2][64] with
 * T2 = ceil(ceil(T/2)/2), F2 = ceil(ceil(feat_dim/2)/2) (srf_cnnfe_out_dims).
 * training = 1: batch statistics, moving statistics updated in place (momentum
 * 0.99), dropout drop_p on every conv output; training = 0: moving statistics,
 * no dropout.  Dropout masks are a pure function of (seed, element), so
 * srf_cnnfe_bwd regenerates them.  nfilt must be 64. */
int srf_cnnfe_out_dims(int T, int feat_dim, int* T2, int* F2);
size_t srf_cnnfe_saved_bytes(int B, int T, int feat_dim, int nfilt);
size_t srf_cnnfe_fwd_workspace(int B, int T, int feat_dim, int nfilt);
size_t srf_cnnfe_bwd_workspace(int B, int T, int feat_dim, int nfilt);
int srf_cnnfe_fwd(const float* feats, const int* inp_len, int B, int T, int feat_dim, int nfilt,
                  const float* k0a, const float* b0a, const float* k0b, const float* b0b, const float* gamma0,
                  const float* beta0, const float* k1a, const float* b1a, const float* k1b, const float* b1b,
                  const float* gamma1, const float* beta1, float* mmean0, float* mvar0, float* mmean1, float* mvar1,
                  int training, float drop_p, unsigned long long seed, float* out, void* saved, size_t saved_bytes,
                  void* workspace, size_t workspace_bytes, void* stream);
/* Gradients (written) of every CNN-FE parameter from g_out = dL/d out. */
int srf_cnnfe_bwd(const float* feats, const int* inp_len, int B, int T, int feat_dim, int nfilt, const float* gamma0,
                  const float* k1a, const float* k1b, const float* gamma1, float drop_p, unsigned long long seed,
                  const void* saved, const float* g_out, float* g_k0a, float* g_b0a, float* g_k0b, float* g_b0b,
                  float* g_gamma0, float* g_beta0, float* g_k1a, float* g_b1a, float* g_k1b, float* g_b1b,
                  float* g_gamma1, float* g_beta1, void* workspace, size_t workspace_bytes, void* stream);

/* The same backward in parts (bit mask), for a caller that runs the stage-2 weight
 * gradient on a second stream: PREP (BN2 sums, the stage-2 output gradient g_ab and
 * the bias gradients) first; then DATA (stage-2 data gradient, BN1, stage 1) and WGRAD
 * (stage-2 kernel gradients) both read what PREP wrote and nothing of each other, so
 * they may run concurrently after it.  One workspace for all parts.  ALL = the
 * sequential srf_cnnfe_bwd. */
#define SRF_CNNFE_BWD_PREP 1
#define SRF_CNNFE_BWD_DATA 2
#define SRF_CNNFE_BWD_WGRAD 4
#define SRF_CNNFE_BWD_ALL 7
int srf_cnnfe_bwd_parts(int parts, const float* feats, const int* inp_len, int B, int T, int feat_dim, int nfilt,
                        const float* gamma0, const float* k1a, const float* k1b, const float* gamma1, float drop_p,
                        unsigned long long seed, const void* saved, const float* g_out, float* g_k0a, float* g_b0a,
                        float* g_k0b, float* g_b0b, float* g_gamma0, float* g_beta0, float* g_k1a, float* g_b1a,
                        float* g_k1b, float* g_b1b, float* g_gamma1, float* g_beta1, void* workspace,
                        size_t workspace_bytes, void* stream);

/* ---- Primary capsules (sequence_router_naive.py:129-142) -------------------
 * X = CNN-FE output viewed as [B*T][K] (K = F2*64, index f*64 + c as the
 * reference's reshape, :131); Wp [K][PH], bp [PH]; encaps kernels [3][3][1][PD],
 * biases [PD]; LN gamma/beta [PH*PD].  z [B*T][PH][PD] =
 * drop_in(LN(squash_PD(mask(max(drop(encaps1(e)), drop(encaps2(e))))))).
 * p_caps is the hard-coded 0.2 of naive:82, p_in = --train-inp-dropout. */
size_t srf_primary_caps_saved_bytes(int B, int T, int PH, int PD);
size_t srf_primary_caps_bwd_workspace(int B, int T, int K, int PH, int PD);
int srf_primary_caps_fwd(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                         const float* bp, const float* K1, const float* b1, const float* K2, const float* b2,
                         const float* gamma, const float* beta, int training, float p_caps, float p_in,
                         unsigned long long seed, float* z, void* saved, size_t saved_bytes, void* stream);
int srf_primary_caps_bwd(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                         const float* K1, const float* K2, const float* gamma, const float* beta, int training,
                         float p_caps, float p_in, unsigned long long seed, const void* saved, const float* g_z,
                         float* g_X, float* g_Wp, float* g_bp, float* g_K1, float* g_b1, float* g_K2, float* g_b2,
                         float* g_gamma, float* g_beta, void* workspace, size_t workspace_bytes, void* stream);
/* The einsum variant (sequence_router_einsum.py:129-131): e = (X Wp + bp) * proj_scale
 * (+ get_pos_enc(T, PH), model_helper.py:30-58, when pos_enc != 0; PH even, >= 4)
 * before the encaps convs.  The plain entry points are proj_scale = 1, pos_enc = 0
 * (naive and lowmemory, naive:131-132 / lowmemory:133-135). */
int srf_primary_caps_fwd_ex(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                            const float* bp, const float* K1, const float* b1, const float* K2, const float* b2,
                            const float* gamma, const float* beta, int training, float p_caps, float p_in,
                            unsigned long long seed, float proj_scale, int pos_enc, float* z, void* saved,
                            size_t saved_bytes, void* stream);
int srf_primary_caps_bwd_ex(const float* X, const int* inp_len, int B, int T, int K, int PH, int PD, const float* Wp,
                            const float* K1, const float* K2, const float* gamma, const float* beta, int training,
                            float p_caps, float p_in, unsigned long long seed, float proj_scale, const void* saved,
                            const float* g_z, float* g_X, float* g_Wp, float* g_bp, float* g_K1, float* g_b1,
                            float* g_K2, float* g_b2, float* g_gamma, float* g_beta, void* workspace,
                            size_t workspace_bytes, void* stream);

/* ---- Per-layer LayerNorm + dropout and the output head (naive:187-193) -----
 * capsnorm: y = drop(LN(x)) per frame over n = J*D (ln_mid%d + dropout_mid_%d);
 * head: logits[F][J] = LN_out(length_D(drop(LN_mid(v)))), lens[F][J] saved.
 * stat [F][4] is written by the forward and read by the backward. */
size_t srf_capsnorm_bwd_workspace(int F, int n, int J);
int srf_capsnorm_fwd(const float* x, int F, int n, const float* gamma, const float* beta, int training, float p,
                     unsigned long long seed, int layer, float* y, float* stat, void* stream);
int srf_capsnorm_bwd(const float* x, int F, int n, const float* gamma, const float* beta, int training, float p,
                     unsigned long long seed, int layer, const float* stat, const float* g_y, float* g_x,
                     float* g_gamma, float* g_beta, void* workspace, size_t workspace_bytes, void* stream);
/* capsnorm over the rows (b, t), t in [t0, t1), of every utterance of a [B][T] batch
 * (same masks and arithmetic as the whole call).  The backward writes g_x rows and
 * gpart rows [B*T][2n] (per-row gamma / beta gradient terms); once every range is
 * done, srf_capsnorm_bwd_params sums gpart into g_gamma / g_beta. */
int srf_capsnorm_fwd_range(const float* x, int B, int T, int t0, int t1, int n, const float* gamma, const float* beta,
                           int training, float p, unsigned long long seed, int layer, float* y, float* stat,
                           void* stream);
int srf_capsnorm_bwd_range(const float* x, int B, int T, int t0, int t1, int n, const float* gamma, const float* beta,
                           int training, float p, unsigned long long seed, int layer, const float* stat,
                           const float* g_y, float* g_x, float* gpart, void* stream);
/* The ranges of up to SRF_CAPSNORM_MAX_ITEMS same-width layers (n = J*D) in one launch
 * (the layer-pipelined SDR stack's inner layers, one anti-diagonal at a time): the
 * *_range calls above for each entry, non-head (ln_mid%d + dropout_mid_%d of `layer`).
 * The forward reads x / gamma / beta, writes y / stat; the backward reads x / gamma /
 * beta / stat / g_y, writes g_x / gpart.  Empty ranges are skipped. */
#define SRF_CAPSNORM_MAX_ITEMS 8
typedef struct {
  int t0, t1, layer;
  const float* x;
  const float* gamma;
  const float* beta;
  float* y;
  float* stat;
  const float* g_y;
  float* g_x;
  float* gpart;
} srf_capsnorm_range;
int srf_capsnorm_fwd_range_n(const srf_capsnorm_range* ranges, int n_ranges, int B, int T, int n, int training,
                             float p, unsigned long long seed, void* stream);
int srf_capsnorm_bwd_range_n(const srf_capsnorm_range* ranges, int n_ranges, int B, int T, int n, int training,
                             float p, unsigned long long seed, void* stream);
size_t srf_capsnorm_params_workspace(int F, int n);
int srf_capsnorm_bwd_params(const float* gpart, int F, int n, float* g_gamma, float* g_beta, void* workspace,
                            size_t workspace_bytes, void* stream);
int srf_caps_head_fwd(const float* v, int F, int J, int D, const float* gamma_mid, const float* beta_mid,
                      const float* gamma_out, const float* beta_out, int training, float p, unsigned long long seed,
                      int layer, float* logits, float* stat, float* lens, void* stream);
/* length_eps of the output length: 1e-7 for naive / lowmemory (naive:256,
 * sequence_router.py:39), 1e-9 for einsum (sequence_router_einsum.py:238).  The
 * backward reads the saved lens, so it is the same for every variant. */
int srf_caps_head_fwd_ex(const float* v, int F, int J, int D, const float* gamma_mid, const float* beta_mid,
                         const float* gamma_out, const float* beta_out, int training, float p, unsigned long long seed,
                         int layer, float length_eps, float* logits, float* stat, float* lens, void* stream);
int srf_caps_head_bwd(const float* v, int F, int J, int D, const float* gamma_mid, const float* beta_mid,
                      const float* gamma_out, int training, float p, unsigned long long seed, int layer,
                      const float* stat, const float* lens, const float* g_logits, float* g_v, float* g_gamma_mid,
                      float* g_beta_mid, float* g_gamma_out, float* g_beta_out, void* workspace,
                      size_t workspace_bytes, void* stream);

/* ---- CTC (tf.nn.ctc_loss at trainer_sr.py:64-66) ---------------------------
 * logits [B][Tmax][C] batch-major, labels [B][Lmax] int32 (dense, padded),
 * label_len / logit_len [B] int32 (logit_len = ceil(inp_len/4)).  nll [B]; if
 * grad != NULL also d(grad_scale * nll_b)/d logits [B][Tmax][C] (zero past
 * logit_len; zero for an infeasible utterance, whose nll is +inf). */
size_t srf_ctc_workspace(int B, int Tmax, int C, int Lmax);
int srf_ctc_loss(const float* logits, const int* labels, const int* label_len, const int* logit_len, int B, int Tmax,
                 int C, int Lmax, int blank, float grad_scale, float* nll, float* grad, void* workspace,
                 size_t workspace_bytes, void* stream);

/* ---- Fused Adam over one flat parameter buffer ----------------------------
 * Replaces the Keras Adam apply of trainer_sr.py:71 / train_helper.py:60-70:
 * m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= alpha m / (sqrt(v) + eps),
 * alpha = lr(step) sqrt(1-b2^t)/(1-b1^t) computed by the caller.  All four
 * buffers 16-byte aligned, n floats each. */
int srf_adam_step(float* params, const float* grads, float* m, float* v, size_t n, float alpha, float b1,
                  float b2, float eps, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SRF_H_ */
