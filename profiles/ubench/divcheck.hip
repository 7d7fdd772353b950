// Exhaustive-ish check of the solve's shared-reciprocal division
// (vame_kernel.h: recip_refined / div_shared / div_range) against the
// compiler's correctly rounded n / d, on MI355X.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o profiles/ubench/divcheck profiles/ubench/divcheck.hip
//   ./profiles/ubench/divcheck            -> mismatches in range / out of range
// Operands: random mantissas, exponents uniform in [-320, 320] (so both the
// fast range and the fallback are hit), random signs, plus integer-valued
// operands like the normal-equation entries (|x| < 2^53).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double recip_refined(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double t = fma(-d, r, 1.0);
  r = fma(r, t, r);
  t = fma(-d, r, 1.0);
  return fma(r, t, r);
}
__device__ __forceinline__ double div_shared(double n, double d, double r) {
  const double q0 = __dmul_rn(n, r);
  return fma(fma(-d, q0, n), r, q0);
}
__device__ __forceinline__ bool div_range(double x) {
  const unsigned e = ((unsigned)__double2hiint(x) >> 20) & 0x7FFu;
  return e - 723u <= 600u;
}
__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}
__device__ double make(uint64_t h, int kind) {
  if (kind == 0) {  // random double, exponent in [-320, 320]
    const uint64_t mant = h & 0xFFFFFFFFFFFFFull;
    const int e = (int)((h >> 52) % 641) - 320;
    const uint64_t sign = (h >> 63) << 63;
    return __longlong_as_double((long long)(sign | ((uint64_t)(e + 1023) << 52) | mant));
  }
  // integer-valued, up to 2^(h%53) in magnitude
  const int bits = (int)((h >> 56) % 53) + 1;
  const long long v = (long long)(h & ((1ull << bits) - 1));
  return (h >> 63) ? -(double)v : (double)v;
}
__global__ void check(uint64_t seed, unsigned long long* bad, unsigned long long* fast) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = 0; k < 64; k++) {
    const uint64_t h1 = mix(seed ^ (i * 64 + k) * 0x9E3779B97F4A7C15ull), h2 = mix(h1 + 0x1234567ull);
    const int kind = (int)(h1 & 1) ^ (int)(h2 & 1);
    const double n = make(h1, kind), d = make(h2, kind);
    const double ref = n / d;
    if (div_range(n) && div_range(d)) {
      const double q = div_shared(n, d, recip_refined(d));
      atomicAdd(fast, 1ull);
      if (__double_as_longlong(q) != __double_as_longlong(ref)) atomicAdd(bad, 1ull);
    }
  }
}
int main() {
  unsigned long long *bad, *fast;
  hipMalloc(&bad, 8);
  hipMalloc(&fast, 8);
  hipMemset(bad, 0, 8);
  hipMemset(fast, 0, 8);
  for (int s = 0; s < 16; s++) hipLaunchKernelGGL(check, dim3(65536), dim3(256), 0, 0, 0xC0FFEEull + s, bad, fast);
  unsigned long long hb = 0, hf = 0;
  hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&hf, fast, 8, hipMemcpyDeviceToHost);
  printf("divcheck: %llu fast-path divisions, %llu differ from n / d\n", hf, hb);
  return hb != 0;
}
