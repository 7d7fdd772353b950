// prof_kat_hip.cpp -- TEST INFRASTRUCTURE ONLY.  Runs oracle/prof_kat.cl's
// code object (the reference's PROF functions, see that file) on the cases of
// an input file and writes the outputs.
//   usage: prof_kat_hip <prof_kat.co> <in.bin> <out.bin>
//   in.bin : int32 n, then n x 121 window samples, then n x 12 parameters
//   out.bin: n x 48 int32 (deltaHor[16], deltaVer[16], prediction[16])
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HCHECK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                           \
    }                                                                                    \
  } while (0)

struct __attribute__((packed)) Args {
  const void* win;
  const void* prm;
  void* out;
  int32_t n;
  int32_t pad;
};

int main(int argc, char** argv) {
  if (argc != 4) { fprintf(stderr, "usage: %s co in out\n", argv[0]); return 1; }
  FILE* f = fopen(argv[2], "rb");
  if (!f) { fprintf(stderr, "cannot read %s\n", argv[2]); return 1; }
  int32_t n = 0;
  if (fread(&n, 4, 1, f) != 1 || n <= 0 || n > (1 << 20)) { fprintf(stderr, "bad n\n"); return 1; }
  std::vector<int32_t> win((size_t)n * 121), prm((size_t)n * 12), out((size_t)n * 48);
  if (fread(win.data(), 4, win.size(), f) != win.size() ||
      fread(prm.data(), 4, prm.size(), f) != prm.size()) {
    fprintf(stderr, "short input\n");
    return 1;
  }
  fclose(f);
  hipModule_t mod;
  hipFunction_t fn;
  HCHECK(hipModuleLoad(&mod, argv[1]));
  HCHECK(hipModuleGetFunction(&fn, mod, "prof_kat"));
  void *dw, *dp, *dout;
  HCHECK(hipMalloc(&dw, win.size() * 4));
  HCHECK(hipMalloc(&dp, prm.size() * 4));
  HCHECK(hipMalloc(&dout, out.size() * 4));
  HCHECK(hipMemcpy(dw, win.data(), win.size() * 4, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(dp, prm.data(), prm.size() * 4, hipMemcpyHostToDevice));
  HCHECK(hipMemset(dout, 0, out.size() * 4));
  Args a{dw, dp, dout, n, 0};
  size_t asz = sizeof(a);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz,
                 HIP_LAUNCH_PARAM_END};
  HCHECK(hipModuleLaunchKernel(fn, (n + 63) / 64, 1, 1, 64, 1, 1, 0, 0, nullptr, cfg));
  HCHECK(hipDeviceSynchronize());
  HCHECK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
  FILE* g = fopen(argv[3], "wb");
  if (!g) { fprintf(stderr, "cannot write %s\n", argv[3]); return 1; }
  fwrite(out.data(), 4, out.size(), g);
  fclose(g);
  printf("prof_kat: %d cases\n", n);
  return 0;
}
