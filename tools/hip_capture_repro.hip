// Stream-capture corner cases of the HIP runtime, one per process (argv[1]), to find which
// pattern makes hipStreamEndCapture crash instead of returning an error (round-3 segfault
// in torch's capture_end with the KD step's forked streams).  Run under MALLOC_PERTURB_ so
// that a runtime use-after-free reads poisoned memory deterministically.
//   hipcc --offload-arch=gfx950 -O1 -g tools/hip_capture_repro.hip -o tools/hip_capture_repro
//   MALLOC_PERTURB_=165 tools/hip_capture_repro <case>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void bump(float* p) { p[threadIdx.x] += 1.f; }

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) printf("  %s -> %s\n", #x, hipGetErrorString(e_));           \
  } while (0)

static void fork_join(hipStream_t from, hipStream_t to) {  // torch's Stream.wait_stream
  hipEvent_t e;
  CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipEventRecord(e, from));
  CK(hipStreamWaitEvent(to, e, 0));
  CK(hipEventDestroy(e));
}

int main(int argc, char** argv) {
  const char* c = argc > 1 ? argv[1] : "torch_pattern";
  float* buf;
  CK(hipMalloc(&buf, 4096));
  hipStream_t A, B, C, D;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&D, hipStreamNonBlocking));
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  printf("case %s\n", c);
  fflush(stdout);
  CK(hipStreamBeginCapture(A, hipStreamCaptureModeGlobal));
  hipLaunchKernelGGL(bump, 1, 64, 0, A, buf);
  if (!strcmp(c, "torch_pattern")) {
    // many short-lived events forking / joining 3 side streams, as torch.wait_stream does
    for (int i = 0; i < 2000; ++i) {
      hipStream_t s = i % 3 == 0 ? B : (i % 3 == 1 ? C : D);
      fork_join(A, s);
      hipLaunchKernelGGL(bump, 1, 64, 0, s, buf + 64 * (i % 3 + 1));
      if (i % 5 == 4) fork_join(s, A);
    }
    fork_join(B, A); fork_join(C, A); fork_join(D, A);
  } else if (!strcmp(c, "event_two_streams")) {
    // one event recorded on B, then on C, destroyed during the capture
    fork_join(A, B); fork_join(A, C);
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipLaunchKernelGGL(bump, 1, 64, 0, B, buf + 64);
    CK(hipEventRecord(e, B));
    hipLaunchKernelGGL(bump, 1, 64, 0, C, buf + 128);
    CK(hipEventRecord(e, C));
    CK(hipStreamWaitEvent(A, e, 0));
    CK(hipEventDestroy(e));
    fork_join(B, A); fork_join(C, A);
  } else if (!strcmp(c, "unjoined")) {
    // a forked stream with work after its last join
    fork_join(A, B);
    hipLaunchKernelGGL(bump, 1, 64, 0, B, buf + 64);
  } else if (!strcmp(c, "side_forks_side")) {
    // B forked from A, C forked from B (not from A), C joined into A only via B
    fork_join(A, B);
    fork_join(B, C);
    hipLaunchKernelGGL(bump, 1, 64, 0, C, buf + 128);
    fork_join(C, B);
    fork_join(B, A);
  } else if (!strcmp(c, "side_forks_side_unjoined")) {
    // C forked from B, its last work never joined anywhere
    fork_join(A, B);
    fork_join(B, C);
    hipLaunchKernelGGL(bump, 1, 64, 0, C, buf + 128);
    fork_join(B, A);
  } else if (!strcmp(c, "event_outlives_capture")) {
    // an event recorded on a forked stream inside the capture, waited on after it
    fork_join(A, B);
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipLaunchKernelGGL(bump, 1, 64, 0, B, buf + 64);
    CK(hipEventRecord(e, B));
    fork_join(B, A);
    CK(hipStreamEndCapture(A, &g));
    printf("  end capture ok (graph %p)\n", (void*)g);
    CK(hipStreamWaitEvent(D, e, 0));
    CK(hipEventDestroy(e));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, A));
    CK(hipStreamSynchronize(A));
    printf("done\n");
    return 0;
  } else if (!strcmp(c, "external_event_destroyed") || !strcmp(c, "external_event_kept")) {
    // the capturing stream waits on an event recorded on a stream that is NOT part of the
    // capture (torch: cur.wait_stream(idle_side) inside a capture), then the event is
    // destroyed before the graph is instantiated (a Python temporary)
    hipLaunchKernelGGL(bump, 1, 64, 0, D, buf + 192);
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventRecord(e, D));
    CK(hipStreamWaitEvent(A, e, 0));
    hipLaunchKernelGGL(bump, 1, 64, 0, A, buf);
    if (!strcmp(c, "external_event_destroyed")) CK(hipEventDestroy(e));
  } else if (!strcmp(c, "stream_destroyed_in_capture")) {
    hipStream_t E;
    CK(hipStreamCreateWithFlags(&E, hipStreamNonBlocking));
    fork_join(A, E);
    hipLaunchKernelGGL(bump, 1, 64, 0, E, buf + 64);
    fork_join(E, A);
    CK(hipStreamDestroy(E));
  }
  CK(hipStreamEndCapture(A, &g));
  printf("  end capture returned (graph %p)\n", (void*)g);
  fflush(stdout);
  if (g) {
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    if (ge) {
      CK(hipGraphLaunch(ge, A));
      CK(hipStreamSynchronize(A));
    }
  }
  printf("done\n");
  return 0;
}
