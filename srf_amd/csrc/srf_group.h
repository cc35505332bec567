// Workgroup groups for the SDR recurrences (route_sdr_stream.hip, route_sdr_seq*.hip):
// G > 1 workgroups per utterance split its input capsules and add their per-iteration
// partial sums (s^r in the forward, gVc^r in the backward) inside the launch.
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1
// table): every member stores its partial write-through (sc1, 16 B), each storing
// wave drains its stores, one lane per workgroup adds to the utterance's arrival
// counter (agent scope), one lane polls it with sc1 loads, and after a barrier every
// wave reads the G partials with sc1 loads only.  All members sum the partials in the
// same order, so they hold bit-identical sums and need no second exchange.  The
// partials are double-buffered by phase parity: a member writing phase k + 2 has seen
// every member arrive at phase k + 1, i.e. done reading phase k.
//
// Residency: the members spin-wait on each other, so all B * items * G workgroups of
// a launch must be resident together (one per CU for these kernels): the host checks
// B * items * G <= CUs, and the caller runs at most one grouped launch at a time.
// That is an assumption about the device, not something a launch can check: another
// stream's kernels (the stack's own inner layers, RCCL collectives overlapping a
// backward) hold CUs too, so the host check keeps kReserveCUs free and the callers
// size G for what else they run.  Each spin is therefore bounded: past kSpinMax polls a
// member sets the item's timeout word and the process's fault word (srf_set_fault_flag)
// and stops waiting -- its results are then wrong, never a hang -- and every later wait
// of the launch returns at once; the host reads the fault word at its next sync
// (srf_amd.ops.check_faults) and fails the step.
#pragma once
#include <algorithm>

#include "route_sdr_seq.h"
#include "srf_common.h"

namespace srf_grp {

constexpr int kMaxGroup = 8;
constexpr unsigned kSpinMax = 1u << 20;
constexpr int kReserveCUs = 4;   // CUs a grouped launch leaves to other streams

struct Grp {
  int G;                // workgroups per utterance (1: no exchange)
  int B;                // utterances of the launch
  unsigned xoff, coff;  // floats from the item's workspace to the exchange area / the counters
  unsigned* fault;      // the process's fault word (srf_set_fault_flag), or NULL
};

// Item workspace: `pre` floats of the kernel's own (the stream backward's gL scratch),
// then the arrival counters [B], the timeout word and the departure counters [B]
// (256-B padded), then the exchange area [2][B][kMaxGroup][JD].
__host__ __device__ inline size_t coff(size_t pre) { return (pre + 63) / 64 * 64; }
__host__ __device__ inline size_t xoff(size_t pre, int B) { return coff(pre) + ((size_t)2 * B + 1 + 63) / 64 * 64; }
__host__ __device__ inline size_t floats(size_t pre, int B, int JD) {
  return xoff(pre, B) + (size_t)2 * B * kMaxGroup * JD;
}
inline Grp make(int G, int B, size_t pre) {
  return Grp{G, B, (unsigned)xoff(pre, B), (unsigned)coff(pre), srf::fault_flag()};
}

typedef unsigned u4 __attribute__((ext_vector_type(4)));

// part [NW][JD] (LDS: this workgroup's NW wave partials) -> part[0 .. JD) = the sum
// over the whole group, for exchange phase `phase` (counted from 0 in the launch).
// Called by all NT threads between barriers; JD % 4 == 0, JD / 4 <= NT.
template <int NW, int NT>
__device__ __forceinline__ void allreduce(float* part, int JD, float* ws, const Grp& X, int b, int gm,
                                          unsigned phase, int tid) {
  const int NV = JD / 4;
  float* xch = ws + X.xoff;
  unsigned* cnt = reinterpret_cast<unsigned*>(ws + X.coff);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(xch, 0, (int)((size_t)2 * X.B * X.G * JD * 4), 0x00020000);
  const uint32_t slot = (uint32_t)((((phase & 1) * X.B + b) * X.G) * JD) * 4;
  if (tid < NV) {
    f4 mine = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w2 = 0; w2 < NW; ++w2) mine += *reinterpret_cast<const f4*>(part + w2 * JD + 4 * tid);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, mine), rs, slot + (uint32_t)(gm * JD + 4 * tid) * 4,
                                           0, 16);   // aux 16: sc1 (write-through)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its partial
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_fetch_add(cnt + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned want = (unsigned)X.G * (phase + 1);
    unsigned spins = 0;
    while (__hip_atomic_load(cnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      if (__hip_atomic_load(cnt + X.B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;   // gave up earlier
      __builtin_amdgcn_s_sleep(2);
      if (++spins > kSpinMax) {
        __hip_atomic_store(cnt + X.B, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (X.fault) __hip_atomic_store(X.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  if (tid < NV) {
    f4 s = {0.f, 0.f, 0.f, 0.f};
    for (int g2 = 0; g2 < X.G; ++g2)
      s += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, slot + (uint32_t)(g2 * JD + 4 * tid) * 4,
                                                                        0, 16));   // sc1 loads only
    *reinterpret_cast<f4*>(part + 4 * tid) = s;
  }
  __syncthreads();
}

// A grouped launch leaves its counters zero for the next launch on the same workspace
// (no memset per launch: on the last layer's stream that was a fill kernel per range on
// the critical chain).  Every member counts itself out after its last exchange; the
// last of an utterance's G members zeroes the utterance's arrival and departure
// counters -- by then none of them polls.  The timeout word stays set: the caller
// zeroes the counter area before the first grouped launch on a workspace.
template <bool GRP>
__device__ __forceinline__ void depart(float* ws, const Grp& X, int b, int tid) {
  if constexpr (GRP) {
    if (tid == 0) {
      unsigned* cnt = reinterpret_cast<unsigned*>(ws + X.coff);
      unsigned* dep = cnt + X.B + 1;
      const unsigned old = __hip_atomic_fetch_add(dep + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == (unsigned)X.G) {
        __hip_atomic_store(cnt + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dep + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// The launch's group size (its items agree; 1 when ungrouped) and exchange geometry
// (`pre` floats of the kernel's own at each item workspace's start).
inline int setup(const srf::SeqItems& items, int B, size_t pre, Grp& X, hipStream_t st) {
  const int G = std::max(1, items.it[0].group);
  for (int k = 1; k < items.n; ++k)
    SRF_REQUIRE(std::max(1, items.it[k].group) == G, "SDR recurrence: launch items differ in group size");
  SRF_REQUIRE(G <= kMaxGroup, "SDR recurrence: group %d above %d", G, kMaxGroup);
  X = make(G, B, pre);
  if (G == 1) return SRF_OK;
  int dev = 0, cus = 0;
  SRF_HIP_TRY(hipGetDevice(&dev));
  SRF_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  SRF_REQUIRE((long)B * items.n * G <= cus - kReserveCUs,
              "SDR recurrence: %d utterances x %d ranges x group %d workgroups exceed the %d CUs they may take (%d "
              "kept free)", B, items.n, G, cus - kReserveCUs, kReserveCUs);
  for (int k = 0; k < items.n; ++k)
    SRF_REQUIRE(items.it[k].ws, "SDR recurrence: a grouped launch needs the range workspace");
  (void)st;
  return SRF_OK;
}

}  // namespace srf_grp
