// anyorder_probe.hip -- does a HIP event recorded after a call of vame's
// one-stream launch structure wait for EVERY kernel of the call?
//
// vame_engine.hip issues a call's first kernel with the AQL barrier bit (the
// long quadrant kernel) and the rest with hipExtAnyOrderLaunch (no barrier
// bit: the short 128-class kernels, the last one possibly finishing before
// the first).  Consumers that order on events -- torch wait_stream /
// record_stream, an event record followed by a copy on another stream --
// rely on the event's marker waiting for all preceding packets, not just for
// the last dispatch.  This probe reproduces the structure with a kernel that
// runs for a fixed time (a bounded spin on the 100 MHz real-time counter, one
// workgroup per CU, each writing a done flag at its end) followed by a tiny
// any-order kernel, then records an event (timing on / off), and checks
//   * the host's hipEventSynchronize returns only after the spin ended, and
//   * a copy of the done flags on a second stream made to wait on the event
//     sees every flag set.
// Prints one JSON line; exit 0 when every variant orders correctly.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                   \
      return 2;                                                                         \
    }                                                                                   \
  } while (0)

// Spin for `ticks` of the 100 MHz counter (bounded: at most max_iter polls),
// then one lane per workgroup stores its done flag (a vector store).
__global__ void spin(unsigned long long ticks, unsigned max_iter, int* done) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned it = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks && it < max_iter) {
    __builtin_amdgcn_s_sleep(2);
    it++;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    volatile int* d = done;
    d[blockIdx.x] = 1;
  }
}

__global__ void tiny(int* out) {
  if (threadIdx.x == 0) out[0] = 1;
}

int main() {
  const int nblk = 256;
  const double spin_ms = 60.0;
  int *done = nullptr, *aux = nullptr;
  CHECK(hipMalloc(&done, nblk * sizeof(int)));
  CHECK(hipMalloc(&aux, sizeof(int)));
  hipStream_t s, s2;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  int* hflags = nullptr;
  CHECK(hipHostMalloc(&hflags, nblk * sizeof(int)));
  bool all_ok = true;
  printf("{\"spin_ms\": %.1f, \"variants\": [", spin_ms);
  for (int v = 0; v < 2; v++) {  // event with timing (v = 0) / hipEventDisableTiming (v = 1)
    hipEvent_t e;
    CHECK(v ? hipEventCreateWithFlags(&e, hipEventDisableTiming) : hipEventCreate(&e));
    CHECK(hipMemsetAsync(done, 0, nblk * sizeof(int), s));
    CHECK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    // the call: a long first kernel (barrier bit), then a short any-order one
    hipExtLaunchKernelGGL(spin, dim3(nblk), dim3(64), 0, s, nullptr, nullptr, 0,
                          (unsigned long long)(spin_ms * 1e5), 1u << 26, done);
    CHECK(hipGetLastError());
    hipExtLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, nullptr, nullptr, hipExtAnyOrderLaunch, aux);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e, s));
    // a consumer on another stream, ordered on the event only
    CHECK(hipStreamWaitEvent(s2, e, 0));
    CHECK(hipMemcpyAsync(hflags, done, nblk * sizeof(int), hipMemcpyDeviceToHost, s2));
    CHECK(hipEventSynchronize(e));
    const double waited =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    CHECK(hipStreamSynchronize(s2));
    int seen = 0;
    for (int i = 0; i < nblk; i++) seen += hflags[i] != 0;
    CHECK(hipStreamSynchronize(s));
    const bool ok = seen == nblk && waited >= 0.9 * spin_ms;
    all_ok &= ok;
    printf("%s{\"event_timing\": %s, \"event_sync_ms\": %.2f, \"flags_seen_by_waiting_stream\": %d, "
           "\"of\": %d, \"ordered\": %s}",
           v ? ", " : "", v ? "false" : "true", waited, seen, nblk, ok ? "true" : "false");
    CHECK(hipEventDestroy(e));
  }
  printf("], \"all_ordered\": %s}\n", all_ok ? "true" : "false");
  CHECK(hipHostFree(hflags));
  CHECK(hipFree(done));
  CHECK(hipFree(aux));
  CHECK(hipStreamDestroy(s));
  CHECK(hipStreamDestroy(s2));
  return all_ok ? 0 : 1;
}
