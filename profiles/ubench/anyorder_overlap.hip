// Do kernels launched on ONE stream with hipExtAnyOrderLaunch run concurrently
// on MI355X?  Two / three kernels whose workgroups each wait ~T us (constant
// 100 MHz realtime counter, bounded loop), few enough to fit the GPU at once:
// the pair's wall time is ~T if they overlap, ~2T if the second waits for the
// first.  Compared with the same kernels on two streams.
//   hipcc --offload-arch=gfx950 -O2 -o anyorder_overlap anyorder_overlap.hip && ./anyorder_overlap
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(unsigned long long ticks, int* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int n = 0;
  for (int i = 0; i < (1 << 22); i++) {  // bounded: ends within ~0.2 s whatever the counter does
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    n++;
    __builtin_amdgcn_s_sleep(1);
  }
  if (threadIdx.x == 0 && n == -1) sink[blockIdx.x] = n;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  int* sink;
  CK(hipMalloc(&sink, 1 << 20));
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b, f, j1, j2;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
  const unsigned long long T = 5000;  // 50 us at 100 MHz
  const int grids[] = {1, 256};
  for (int g : grids) {
    for (int mode = 0; mode < 5; mode++) {
      const char* name[] = {"1 stream, default flags", "1 stream, any-order 2nd+3rd", "1 stream, any-order all",
                            "3 streams", "1 stream, single kernel"};
      float best = 1e9, sum = 0;
      const int reps = 20;
      for (int r = 0; r < reps + 2; r++) {
        CK(hipEventRecord(a, s0));
        if (mode <= 2) {
          for (int k = 0; k < 3; k++) {
            const int flags = (mode == 1 && k > 0) || mode == 2 ? hipExtAnyOrderLaunch : 0;
            hipExtLaunchKernelGGL(spin, dim3(g), dim3(64), 0, s0, nullptr, nullptr, flags, T, sink);
          }
        } else if (mode == 3) {
          CK(hipEventRecord(f, s0));
          CK(hipStreamWaitEvent(s1, f, 0));
          CK(hipStreamWaitEvent(s2, f, 0));
          hipLaunchKernelGGL(spin, dim3(g), dim3(64), 0, s0, T, sink);
          hipLaunchKernelGGL(spin, dim3(g), dim3(64), 0, s1, T, sink);
          hipLaunchKernelGGL(spin, dim3(g), dim3(64), 0, s2, T, sink);
          CK(hipEventRecord(j1, s1));
          CK(hipEventRecord(j2, s2));
          CK(hipStreamWaitEvent(s0, j1, 0));
          CK(hipStreamWaitEvent(s0, j2, 0));
        } else {
          hipLaunchKernelGGL(spin, dim3(g), dim3(64), 0, s0, T, sink);
        }
        CK(hipGetLastError());
        CK(hipEventRecord(b, s0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2) {
          sum += ms;
          if (ms < best) best = ms;
        }
      }
      printf("grid %3d  %-28s  3 x 50 us kernels: mean %.1f us, best %.1f us\n", g, name[mode], sum / reps * 1e3,
             best * 1e3);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
