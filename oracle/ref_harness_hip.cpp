// ref_harness_hip.cpp -- same job as ref_harness.cpp (run the REFERENCE kernels,
// compiled offline from /root/reference/affine.cl, on one (POC, ref) pair), but
// loads the code object through the HIP module API instead of the OpenCL
// runtime.  TEST INFRASTRUCTURE ONLY.
//
// The explicit kernel arguments are packed by hand in the layout the code
// object's metadata declares for affine.cl:11 / :960 (14 args, 100 bytes); the
// HIP runtime appends the hidden arguments (block counts, group sizes, global
// offsets = 0, printf buffer) from the same metadata.  Buffers and launch
// geometry follow main.cpp:473-552 and :754-966.
//
// usage: ref_harness_hip <affine_2cp.co> <affine_3cp.co> <jobfile>   (see ref_harness.cpp)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#define HCHECK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, \
              __LINE__, #x);                                                            \
      exit(2);                                                                          \
    }                                                                                   \
  } while (0)

static std::vector<unsigned char> slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) { fprintf(stderr, "cannot read %s\n", p.c_str()); exit(2); }
  return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), {});
}

static int num_ctus(int W, int H) {  // constants.h:73-79
  if (W == 3840 && H == 2160) return 510;
  if (W == 1920 && H == 1080) return 135;
  if (W == 1280 && H == 720) return 60;
  if (W == 832 && H == 480) return 28;
  if (W == 416 && H == 240) return 8;
  return 0;
}

// explicit kernarg layout of affine_gradient_mult_sizes(_HA) (code-object metadata)
struct __attribute__((packed)) Args {
  void* ref;       // 0
  void* cur;       // 8
  int32_t W;       // 16
  int32_t H;       // 20
  float lambda;    // 24
  int32_t pad0;    // 28
  void* hgrad;     // 32
  void* vgrad;     // 40
  void* eq;        // 48
  void* cost;      // 56
  void* cpmvs;     // 64
  void* prev;      // 72
  void* debug;     // 80
  void* retcu;     // 88
  int32_t extra;   // 96
  int32_t pad1;    // 100
};
static_assert(sizeof(Args) == 104, "kernarg layout");

int main(int argc, char** argv) {
  if (argc != 4) { fprintf(stderr, "usage: %s co2 co3 jobfile\n", argv[0]); return 1; }
  hipModule_t mod[2];
  hipFunction_t fn[4];
  HCHECK(hipModuleLoad(&mod[0], argv[1]));
  HCHECK(hipModuleLoad(&mod[1], argv[2]));
  HCHECK(hipModuleGetFunction(&fn[0], mod[0], "affine_gradient_mult_sizes"));
  HCHECK(hipModuleGetFunction(&fn[1], mod[1], "affine_gradient_mult_sizes"));
  HCHECK(hipModuleGetFunction(&fn[2], mod[0], "affine_gradient_mult_sizes_HA"));
  HCHECK(hipModuleGetFunction(&fn[3], mod[1], "affine_gradient_mult_sizes_HA"));
  const char* tag[4] = {"FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP"};
  const char* maskenv = getenv("REF_PRED_MASK");
  const int mask = maskenv ? atoi(maskenv) : 15;
  hipEvent_t e0, e1;
  HCHECK(hipEventCreate(&e0));
  HCHECK(hipEventCreate(&e1));

  std::ifstream jf(argv[3]);
  std::string line;
  while (std::getline(jf, line)) {
    if (line.empty() || line[0] == '#') continue;
    std::istringstream ss(line);
    int W, H, extra;
    float lambda;
    std::string refp, curp, outp;
    ss >> W >> H >> lambda >> extra >> refp >> curp >> outp;
    int nCtus = num_ctus(W, H);
    if (!nCtus) { fprintf(stderr, "unsupported resolution %dx%d\n", W, H); return 4; }
    std::vector<unsigned char> refb = slurp(refp), curb = slurp(curp);
    size_t fsz = (size_t)W * H * 2;
    if (refb.size() != fsz || curb.size() != fsz) { fprintf(stderr, "bad frame size\n"); return 4; }
    const size_t MAX_nWGs = (size_t)nCtus * 24;  // main.cpp:474
    void *ref, *cur, *hg, *vg, *eq, *dbg, *rcu, *cost[4], *cp[4];
    HCHECK(hipMalloc(&ref, fsz));
    HCHECK(hipMalloc(&cur, fsz));
    HCHECK(hipMemcpy(ref, refb.data(), fsz, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(cur, curb.data(), fsz, hipMemcpyHostToDevice));
    HCHECK(hipMalloc(&hg, MAX_nWGs * 128 * 128 * 2));
    HCHECK(hipMalloc(&vg, MAX_nWGs * 128 * 128 * 2));
    HCHECK(hipMalloc(&eq, MAX_nWGs * 256 * 49 * 8));
    HCHECK(hipMalloc(&dbg, MAX_nWGs * 256 * 4 * 8));
    HCHECK(hipMalloc(&rcu, 128 * 128 * 2));
    for (int p = 0; p < 4; p++) {
      size_t T = p < 2 ? 201 : 284;
      HCHECK(hipMalloc(&cost[p], nCtus * T * 8));
      HCHECK(hipMalloc(&cp[p], nCtus * T * 28));
      HCHECK(hipMemset(cost[p], 0, nCtus * T * 8));
      HCHECK(hipMemset(cp[p], 0, nCtus * T * 28));
    }
    for (int p = 0; p < 4; p++) {
      if (!((mask >> p) & 1)) continue;
      Args a;
      memset(&a, 0, sizeof(a));
      a.ref = ref; a.cur = cur; a.W = W; a.H = H; a.lambda = lambda;
      a.hgrad = hg; a.vgrad = vg; a.eq = eq; a.cost = cost[p]; a.cpmvs = cp[p];
      a.prev = (p == 1) ? cp[0] : (p == 3) ? cp[2] : cp[p];  // 2-CP launches: unread (main.cpp:837)
      a.debug = dbg; a.retcu = rcu; a.extra = extra;
      size_t asz = sizeof(a);
      void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz,
                     HIP_LAUNCH_PARAM_END};
      unsigned nwg = (unsigned)nCtus * (p < 2 ? 12 : 24);
      HCHECK(hipEventRecord(e0, 0));
      HCHECK(hipModuleLaunchKernel(fn[p], nwg, 1, 1, 256, 1, 1, 0, 0, nullptr, cfg));
      HCHECK(hipEventRecord(e1, 0));
      HCHECK(hipDeviceSynchronize());
      float ms = 0;
      HCHECK(hipEventElapsedTime(&ms, e0, e1));
      size_t T = p < 2 ? 201 : 284, n = nCtus * T;
      std::vector<unsigned char> hc(n * 8), hp(n * 28);
      HCHECK(hipMemcpy(hc.data(), cost[p], n * 8, hipMemcpyDeviceToHost));
      HCHECK(hipMemcpy(hp.data(), cp[p], n * 28, hipMemcpyDeviceToHost));
      std::string fnm = outp + "_" + tag[p] + ".bin";
      FILE* f = fopen(fnm.c_str(), "wb");
      if (!f) { fprintf(stderr, "cannot write %s\n", fnm.c_str()); return 5; }
      fwrite(hc.data(), 1, hc.size(), f);
      fwrite(hp.data(), 1, hp.size(), f);
      fclose(f);
      printf("%s %dx%d %s kernel_ms=%.3f\n", outp.c_str(), W, H, tag[p], ms);
      fflush(stdout);
    }
    for (int p = 0; p < 4; p++) { hipFree(cost[p]); hipFree(cp[p]); }
    hipFree(ref); hipFree(cur); hipFree(hg); hipFree(vg); hipFree(eq); hipFree(dbg); hipFree(rcu);
  }
  return 0;
}
