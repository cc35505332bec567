/* srf_prof.h -- diagnostics of libsrf.so, not part of the product ABI (srf.h).
 *
 * Used by bench.py to time the dominant kernel with HIP events on the stream it
 * is launched on (torch.cuda.Event sees only torch's current stream).
 */
#ifndef SRF_PROF_H_
#define SRF_PROF_H_

#ifdef __cplusplus
extern "C" {
#endif

/* Thread-local, opt-in: the next srf_route_dr_fwd / srf_route_dr_fwd_ex call on
 * this thread records starts[r] / stops[r] (hipEvent_t) on its stream around the
 * routing-pass kernel of iteration r < n, then forgets the arrays. */
int srf_route_dr_set_timing_events(void* const* starts, void* const* stops, int n);

#ifdef __cplusplus
}
#endif
#endif /* SRF_PROF_H_ */
