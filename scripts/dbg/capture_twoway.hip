// Minimal HIP reproducer for the stream-capture failure recorded in srf_amd/ops.py
// (SdrStack: "forking the same side streams from the caller's thread and from
// autograd's thread, or ordering two side streams both ways, crashes capture_end").
// Each case captures a small multi-stream DAG on origin stream O, instantiates and
// replays it, and checks every HIP status and the kernels' results.
//   hipcc --offload-arch=gfx950 -O2 -o capture_twoway capture_twoway.hip -lpthread
//   ./capture_twoway            (prints one line per case: status codes, result)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <thread>

#define CK(call)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) {                                                             \
      printf("  %s -> %d (%s)\n", #call, (int)e_, hipGetErrorString(e_));               \
      return (int)e_;                                                                   \
    }                                                                                   \
  } while (0)

__global__ void add_k(float* p, float v, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + v;
}

constexpr int kN = 1 << 16;

static void launch(float* p, float v, hipStream_t s) { hipLaunchKernelGGL(add_k, dim3(kN / 256), dim3(256), 0, s, p, v, kN); }

// case: 0 fork/join once, 1 two-way (A -> B, then B -> A), 2 fork twice, 3 fork from a second thread,
// 4 two-way with both edges on events recorded before either wait (A <-> B crossing),
// 5 the SdrStack pattern in global mode: fork/join A, B from the capturing thread, then
//   fork/join the SAME A, B again from a second thread (torch's autograd thread runs the
//   backward of a captured step), 6 as 5 with the second thread ordering A and B both ways
static int run_case(int c, float* buf, float* out) {
  hipStream_t O, A, B;
  CK(hipStreamCreateWithFlags(&O, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  hipEvent_t ev[8];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipMemsetAsync(buf, 0, 3 * kN * sizeof(float), O));
  CK(hipStreamSynchronize(O));
  float *a = buf, *b = buf + kN, *o = buf + 2 * kN;
  CK(hipStreamBeginCapture(O, c == 3 ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeGlobal));
  hipError_t terr = hipSuccess;
  auto other_thread = [&](bool twoway) {
    std::thread th([&] {
      auto ck = [&](hipError_t e) { if (e != hipSuccess && terr == hipSuccess) terr = e; };
      ck(hipEventRecord(ev[6], O));
      ck(hipStreamWaitEvent(A, ev[6], 0));
      ck(hipStreamWaitEvent(B, ev[6], 0));
      launch(a, 6.f, A);
      launch(b, 7.f, B);
      if (twoway) {
        ck(hipEventRecord(ev[2], A));
        ck(hipStreamWaitEvent(B, ev[2], 0));
        launch(b, 8.f, B);
        ck(hipEventRecord(ev[3], B));
        ck(hipStreamWaitEvent(A, ev[3], 0));
        launch(a, 9.f, A);
      }
      ck(hipEventRecord(ev[4], A));
      ck(hipEventRecord(ev[5], B));
      ck(hipStreamWaitEvent(O, ev[4], 0));
      ck(hipStreamWaitEvent(O, ev[5], 0));
    });
    th.join();
    if (terr != hipSuccess) printf("  second thread: %d (%s)\n", (int)terr, hipGetErrorString(terr));
    return (int)terr;
  };
  auto fork = [&](int e0) -> int {
    CK(hipEventRecord(ev[e0], O));
    CK(hipStreamWaitEvent(A, ev[e0], 0));
    CK(hipStreamWaitEvent(B, ev[e0], 0));
    return 0;
  };
  auto join = [&](int e0) -> int {
    CK(hipEventRecord(ev[e0], A));
    CK(hipEventRecord(ev[e0 + 1], B));
    CK(hipStreamWaitEvent(O, ev[e0], 0));
    CK(hipStreamWaitEvent(O, ev[e0 + 1], 0));
    return 0;
  };
  int rc = 0;
  launch(o, 1.f, O);
  if (c == 3) {
    // the side streams are forked and joined by a second host thread while O is captured
    CK(hipEventRecord(ev[0], O));
    std::thread t([&] {
      rc = hipStreamWaitEvent(A, ev[0], 0);
      if (!rc) launch(a, 2.f, A);
      if (!rc) rc = hipEventRecord(ev[1], A);
    });
    t.join();
    if (rc) {
      printf("  second thread: %d (%s)\n", rc, hipGetErrorString((hipError_t)rc));
      return rc;
    }
    CK(hipStreamWaitEvent(O, ev[1], 0));
  } else {
    if ((rc = fork(0))) return rc;
    launch(a, 2.f, A);
    launch(b, 3.f, B);
    if (c == 1) {   // A -> B, then B -> A
      CK(hipEventRecord(ev[2], A));
      CK(hipStreamWaitEvent(B, ev[2], 0));
      launch(b, 4.f, B);
      CK(hipEventRecord(ev[3], B));
      CK(hipStreamWaitEvent(A, ev[3], 0));
      launch(a, 5.f, A);
    } else if (c == 4) {   // both events recorded, then both waits
      CK(hipEventRecord(ev[2], A));
      CK(hipEventRecord(ev[3], B));
      CK(hipStreamWaitEvent(B, ev[2], 0));
      CK(hipStreamWaitEvent(A, ev[3], 0));
      launch(a, 5.f, A);
      launch(b, 4.f, B);
    }
    if ((rc = join(4))) return rc;
    if (c == 5 || c == 6) {   // the same side streams forked again, from another thread
      launch(o, 2.f, O);
      if ((rc = other_thread(c == 6))) return rc;
    }
    if (c == 2) {   // the same side streams forked again
      if ((rc = fork(6))) return rc;
      launch(a, 6.f, A);
      launch(b, 7.f, B);
      if ((rc = join(4))) return rc;
    }
  }
  launch(o, 1.f, O);
  hipGraph_t g;
  hipError_t e = hipStreamEndCapture(O, &g);
  printf("  end_capture -> %d (%s)\n", (int)e, hipGetErrorString(e));
  if (e != hipSuccess) return (int)e;
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, O));
  CK(hipStreamSynchronize(O));
  CK(hipMemcpy(out, buf, 3 * kN * sizeof(float), hipMemcpyDeviceToHost));
  printf("  nodes %zu  a %.4f  b %.4f  o %.4f\n", nn, out[0], out[kN], out[2 * kN]);
  CK(hipGraphExecDestroy(x));
  CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  float* buf;
  if (hipMalloc(&buf, 3 * kN * sizeof(float)) != hipSuccess) return 1;
  static float out[3 * kN];
  const char* names[] = {"fork_join",       "two_way",           "fork_twice",          "second_thread",
                         "two_way_crossed", "refork_other_thread", "refork_other_twoway"};
  int bad = 0;
  for (int c = 0; c < 7; ++c) {
    printf("case %s\n", names[c]);
    const int rc = run_case(c, buf, out);
    printf("case %s rc=%d\n", names[c], rc);
    bad += rc != 0;
    (void)hipGetLastError();
  }
  return bad ? 2 : 0;
}
