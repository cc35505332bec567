/* srf.h -- C ABI of the MI355X-native Sequential Routing Framework hot path.
 *
 * Every entry point takes caller-owned device pointers (fp32 unless stated),
 * plain int shapes and a hipStream_t passed as void*.  Nothing allocates, nothing
 * synchronises, no global mutable state: calls are stream-ordered and may be
 * captured into a hipGraph.  Return value: 0 on success, < 0 on error
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
/* Profiling hook (opt-in, this thread only): the next srf_route_dr_fwd call
 * records starts[r] / stops[r] (hipEvent_t) on its stream around the routing-pass
 * kernel of iteration r < n, then forgets the arrays. */
int srf_route_dr_set_timing_events(void* const* starts, void* const* stops, int n);
/* Gradients are written (not accumulated): g_emb [B*T][N][din], g_W like W,
 * g_bias like bias. */
int srf_route_dr_bwd(const float* emb, const float* W, const float* bias, int B, int T, int N, int din, int lpad,
                     int rpad, int J, int dout, int iters, int mask_first, int n_chunks, const float* saved,
                     const float* g_v, float* g_emb, float* g_W, float* g_bias, void* workspace,
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
