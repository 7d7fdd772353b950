// Latency of a cross-stream dependency on MI355X: a chain of N tiny kernels
// alternating between two streams, each hop ordered by (a) an event record +
// hipStreamWaitEvent, or (b) hipStreamWriteValue32 + hipStreamWaitValue32 on a
// device word; against the same N kernels on one stream.
//   hipcc --offload-arch=gfx950 -O2 -o stream_hop stream_hop.hip && ./stream_hop
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void tiny(int* p) {
  if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  int* buf;
  CK(hipMalloc(&buf, 4096));
  CK(hipMemset(buf, 0, 4096));
  uint32_t* flag;
  if (hipExtMallocWithFlags((void**)&flag, 8, hipMallocSignalMemory) != hipSuccess) {
    (void)hipGetLastError();
    CK(hipMalloc((void**)&flag, 4096));
    printf("(flag in plain device memory)\n");
  }
  CK(hipMemset(flag, 0, 8));
  hipStream_t s[2];
  for (int i = 0; i < 2; i++) CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
  const int N = 200;
  hipEvent_t ev[2 * N];
  for (int i = 0; i < 2 * N; i++) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 3; rep++) {
      CK(hipDeviceSynchronize());
      CK(hipMemset(flag, 0, 8));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, s[0]));
      for (int i = 0; i < N; i++) {
        const int from = i & 1, to = from ^ 1;
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, mode == 0 ? s[0] : s[from], buf);
        if (mode == 1) {
          CK(hipEventRecord(ev[i], s[from]));
          CK(hipStreamWaitEvent(s[to], ev[i], 0));
        } else if (mode == 2) {
          CK(hipStreamWriteValue32(s[from], flag, (uint32_t)(i + 1), 0));
          CK(hipStreamWaitValue32(s[to], flag, (uint32_t)(i + 1), hipStreamWaitValueGte, 0xFFFFFFFFu));
        }
      }
      if (mode != 0) {  // end on stream 0
        CK(hipEventRecord(ev[N], s[1]));
        CK(hipStreamWaitEvent(s[0], ev[N], 0));
      }
      CK(hipEventRecord(b, s[0]));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const char* name[] = {"one stream", "event hops", "write/wait value hops"};
      printf("%-22s %d kernels: %.1f us per kernel\n", name[mode], N, ms * 1e3 / N);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
