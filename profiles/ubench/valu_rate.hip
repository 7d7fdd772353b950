// VALU issue-rate microbenchmark (gfx950): cycles per wave-instruction per SIMD
// for the instruction classes the affine-ME kernel uses, at 1..4 waves/SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
template <int OP>
__global__ __launch_bounds__(1024) void k(unsigned long long* cyc, int iters, unsigned seed) {
  unsigned a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11,
           a6 = a0 * 13, a7 = a0 + 17, b = seed * 3 + 1;
  const unsigned long long mask = 0x5555555555555555ull ^ seed;
  const unsigned sel = 0x05040100u + seed;
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3, e = 1.0000001;
  unsigned long long q0 = a0, q1 = a1, q2 = a2, q3 = a3;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if (OP == 0) {  // v_add_u32
      REP8(asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 1) {  // v_dot2_i32_i16 (VOP3)
      REP8(asm volatile("v_dot2_i32_i16 %0, %0, %8, %0\n v_dot2_i32_i16 %1, %1, %8, %1\n v_dot2_i32_i16 %2, %2, %8, %2\n v_dot2_i32_i16 %3, %3, %8, %3\n v_dot2_i32_i16 %4, %4, %8, %4\n v_dot2_i32_i16 %5, %5, %8, %5\n v_dot2_i32_i16 %6, %6, %8, %6\n v_dot2_i32_i16 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 2) {  // v_pk_add_u16
      REP8(asm volatile("v_pk_add_u16 %0, %0, %8\n v_pk_add_u16 %1, %1, %8\n v_pk_add_u16 %2, %2, %8\n v_pk_add_u16 %3, %3, %8\n v_pk_add_u16 %4, %4, %8\n v_pk_add_u16 %5, %5, %8\n v_pk_add_u16 %6, %6, %8\n v_pk_add_u16 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 3) {  // v_fma_f64
      REP8(asm volatile("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(e));)
    } else if (OP == 4) {  // v_mad_i64_i32
      REP8(asm volatile("v_mad_i64_i32 %0, vcc, %4, %4, %0\n v_mad_i64_i32 %1, vcc, %4, %4, %1\n v_mad_i64_i32 %2, vcc, %4, %4, %2\n v_mad_i64_i32 %3, vcc, %4, %4, %3" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(b) : "vcc");)
    } else if (OP == 5) {  // v_rcp_f64
      REP8(asm volatile("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));)
    } else if (OP == 6) {  // v_add_u32_dpp row_shr:1
      REP8(asm volatile("v_add_u32_dpp %0, %8, %0 row_shr:1 bound_ctrl:0\n v_add_u32_dpp %1, %8, %1 row_shr:1 bound_ctrl:0\n v_add_u32_dpp %2, %8, %2 row_shr:1 bound_ctrl:0\n v_add_u32_dpp %3, %8, %3 row_shr:1 bound_ctrl:0\n v_add_u32_dpp %4, %8, %4 row_shr:1 bound_ctrl:0\n v_add_u32_dpp %5, %8, %5 row_shr:1 bound_ctrl:0\n v_add_u32_dpp %6, %8, %6 row_shr:1 bound_ctrl:0\n v_add_u32_dpp %7, %8, %7 row_shr:1 bound_ctrl:0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 7) {  // v_cndmask_b32
      REP8(asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 8) {  // v_mul_lo_u32
      REP8(asm volatile("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 9) {  // v_mul_f64
      REP8(asm volatile("v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(e));)
    } else if (OP == 10) {  // v_pk_mad_i16
      REP8(asm volatile("v_pk_mad_i16 %0, %0, %8, %0\n v_pk_mad_i16 %1, %1, %8, %1\n v_pk_mad_i16 %2, %2, %8, %2\n v_pk_mad_i16 %3, %3, %8, %3\n v_pk_mad_i16 %4, %4, %8, %4\n v_pk_mad_i16 %5, %5, %8, %5\n v_pk_mad_i16 %6, %6, %8, %6\n v_pk_mad_i16 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 11) {  // v_alignbit_b32
      REP8(asm volatile("v_alignbit_b32 %0, %0, %8, 16\n v_alignbit_b32 %1, %1, %8, 16\n v_alignbit_b32 %2, %2, %8, 16\n v_alignbit_b32 %3, %3, %8, 16\n v_alignbit_b32 %4, %4, %8, 16\n v_alignbit_b32 %5, %5, %8, 16\n v_alignbit_b32 %6, %6, %8, 16\n v_alignbit_b32 %7, %7, %8, 16" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 12) {  // v_cndmask_b32 e64 with an SGPR pair
      REP8(asm volatile("v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n v_cndmask_b32_e64 %2, %2, %8, %9\n v_cndmask_b32_e64 %3, %3, %8, %9\n v_cndmask_b32_e64 %4, %4, %8, %9\n v_cndmask_b32_e64 %5, %5, %8, %9\n v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "s"(mask));)
    } else if (OP == 13) {  // v_max_i32
      REP8(asm volatile("v_max_i32 %0, %0, %8\n v_max_i32 %1, %1, %8\n v_max_i32 %2, %2, %8\n v_max_i32 %3, %3, %8\n v_max_i32 %4, %4, %8\n v_max_i32 %5, %5, %8\n v_max_i32 %6, %6, %8\n v_max_i32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 14) {  // v_and_b32
      REP8(asm volatile("v_and_b32 %0, %0, %8\n v_and_b32 %1, %1, %8\n v_and_b32 %2, %2, %8\n v_and_b32 %3, %3, %8\n v_and_b32 %4, %4, %8\n v_and_b32 %5, %5, %8\n v_and_b32 %6, %6, %8\n v_and_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 15) {  // v_perm_b32
      REP8(asm volatile("v_perm_b32 %0, %0, %8, %9\n v_perm_b32 %1, %1, %8, %9\n v_perm_b32 %2, %2, %8, %9\n v_perm_b32 %3, %3, %8, %9\n v_perm_b32 %4, %4, %8, %9\n v_perm_b32 %5, %5, %8, %9\n v_perm_b32 %6, %6, %8, %9\n v_perm_b32 %7, %7, %8, %9" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(sel));)
    } else if (OP == 16) {  // v_med3_i32
      REP8(asm volatile("v_med3_i32 %0, %0, %8, %9\n v_med3_i32 %1, %1, %8, %9\n v_med3_i32 %2, %2, %8, %9\n v_med3_i32 %3, %3, %8, %9\n v_med3_i32 %4, %4, %8, %9\n v_med3_i32 %5, %5, %8, %9\n v_med3_i32 %6, %6, %8, %9\n v_med3_i32 %7, %7, %8, %9" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(sel));)
    } else if (OP == 17) {  // v_cndmask_b32 vcc, condition from v_cmp each 8
      REP8(asm volatile("v_cmp_gt_i32 vcc, %8, %0\n v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");)
    } else if (OP == 18) {  // v_permlane32_swap
      REP8(asm volatile("v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7\n v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if (OP == 19) {  // v_mul_u32_u24
      REP8(asm volatile("v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 20) {  // v_lshlrev_b32
      REP8(asm volatile("v_lshlrev_b32 %0, 1, %0\n v_lshlrev_b32 %1, 1, %1\n v_lshlrev_b32 %2, 1, %2\n v_lshlrev_b32 %3, 1, %3\n v_lshlrev_b32 %4, 1, %4\n v_lshlrev_b32 %5, 1, %5\n v_lshlrev_b32 %6, 1, %6\n v_lshlrev_b32 %7, 1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if (OP == 21) {  // v_dot2c_i32_i16 (VOP2, accumulate in place)
      REP8(asm volatile("v_dot2c_i32_i16 %0, %8, %0\n v_dot2c_i32_i16 %1, %8, %1\n v_dot2c_i32_i16 %2, %8, %2\n v_dot2c_i32_i16 %3, %8, %3\n v_dot2c_i32_i16 %4, %8, %4\n v_dot2c_i32_i16 %5, %8, %5\n v_dot2c_i32_i16 %6, %8, %6\n v_dot2c_i32_i16 %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 22) {  // v_cndmask_b32_e64 with vcc as the condition operand
      REP8(asm volatile("v_cndmask_b32_e64 %0, %0, %8, vcc\n v_cndmask_b32_e64 %1, %1, %8, vcc\n v_cndmask_b32_e64 %2, %2, %8, vcc\n v_cndmask_b32_e64 %3, %3, %8, vcc\n v_cndmask_b32_e64 %4, %4, %8, vcc\n v_cndmask_b32_e64 %5, %5, %8, vcc\n v_cndmask_b32_e64 %6, %6, %8, vcc\n v_cndmask_b32_e64 %7, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 23) {  // v_cmp_e64 -> sgpr pair, then 7 cndmask_e64 on it
      REP8(asm volatile("v_cmp_gt_i32_e64 s[40:41], %8, %0\n v_cndmask_b32_e64 %1, %1, %8, s[40:41]\n v_cndmask_b32_e64 %2, %2, %8, s[40:41]\n v_cndmask_b32_e64 %3, %3, %8, s[40:41]\n v_cndmask_b32_e64 %4, %4, %8, s[40:41]\n v_cndmask_b32_e64 %5, %5, %8, s[40:41]\n v_cndmask_b32_e64 %6, %6, %8, s[40:41]\n v_cndmask_b32_e64 %7, %7, %8, s[40:41]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "s40", "s41");)
    } else if (OP == 24) {  // v_cmp_e32 (writes vcc) only
      REP8(asm volatile("v_cmp_gt_i32 vcc, %8, %0\n v_cmp_gt_i32 vcc, %8, %1\n v_cmp_gt_i32 vcc, %8, %2\n v_cmp_gt_i32 vcc, %8, %3\n v_cmp_gt_i32 vcc, %8, %4\n v_cmp_gt_i32 vcc, %8, %5\n v_cmp_gt_i32 vcc, %8, %6\n v_cmp_gt_i32 vcc, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");)
    } else if (OP == 25) {  // v_cmp_e64 to distinct sgpr pairs
      REP8(asm volatile("v_cmp_gt_i32_e64 s[40:41], %8, %0\n v_cmp_gt_i32_e64 s[42:43], %8, %1\n v_cmp_gt_i32_e64 s[44:45], %8, %2\n v_cmp_gt_i32_e64 s[46:47], %8, %3\n v_cmp_gt_i32_e64 s[40:41], %8, %4\n v_cmp_gt_i32_e64 s[42:43], %8, %5\n v_cmp_gt_i32_e64 s[44:45], %8, %6\n v_cmp_gt_i32_e64 s[46:47], %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");)
    } else if (OP == 26) {  // v_sub_u32 + v_cndmask_b32_e32 mix (1:1)
      REP8(asm volatile("v_sub_u32 %0, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n v_sub_u32 %2, %2, %8\n v_cndmask_b32 %3, %3, %8, vcc\n v_sub_u32 %4, %4, %8\n v_cndmask_b32 %5, %5, %8, vcc\n v_sub_u32 %6, %6, %8\n v_cndmask_b32 %7, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 27) {  // pairs of v_cndmask_b32_e32 (vcc) + one v_add_u32_dpp, as in the reductions
      REP8(asm volatile("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_add_u32_dpp %2, %8, %2 row_shr:1 bound_ctrl:0\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_add_u32_dpp %5, %8, %5 row_shr:1 bound_ctrl:0\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
    } else if (OP == 28) {  // the same with v_cndmask_b32_e64 on an SGPR pair
      REP8(asm volatile("v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n v_add_u32_dpp %2, %8, %2 row_shr:1 bound_ctrl:0\n v_cndmask_b32_e64 %3, %3, %8, %9\n v_cndmask_b32_e64 %4, %4, %8, %9\n v_add_u32_dpp %5, %8, %5 row_shr:1 bound_ctrl:0\n v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "s"(mask));)
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  if (a0 == 12345 && a1 == a2 && d0 == 0.5 && q0 == 7) cyc[0] = a3 + a4 + a5 + a6 + a7 + (unsigned)d1 + (unsigned)q1 + d2 + d3 + q2 + q3;
}

template <int OP>
void run(const char* name, int instrPerIter) {
  const int iters = 2000;
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int threads = 256 * wps;  // 4 SIMDs x wps waves
    const int blocks = cus;         // one block per CU
    unsigned long long* d;
    hipMalloc(&d, sizeof(unsigned long long) * blocks * threads / 64);
    k<OP><<<blocks, threads>>>(d, 10, 1);
    hipDeviceSynchronize();
    k<OP><<<blocks, threads>>>(d, iters, 1);
    hipDeviceSynchronize();
    unsigned long long* h = new unsigned long long[blocks * threads / 64];
    hipMemcpy(h, d, sizeof(unsigned long long) * blocks * threads / 64, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks * threads / 64; i++) s += (double)h[i];
    s /= blocks * threads / 64;
    // wave cycles / (instructions of the wave) * waves per SIMD = SIMD cycles per instruction
    const double perWaveInstr = s / ((double)iters * instrPerIter);
    printf("%-18s waves/SIMD %d: %.2f cyc per wave-instr per wave, %.2f SIMD cyc per instr\n", name, wps,
           perWaveInstr, perWaveInstr / wps);
    delete[] h;
    hipFree(d);
  }
}

int main() {
  run<27>("2 cndmask_e32 + dpp", 64);
  run<28>("2 cndmask_e64 + dpp", 64);
  return 0;
  run<22>("v_cndmask_e64_vcc", 64);
  run<23>("cmp_e64+7cndmask_e64", 64);
  run<24>("v_cmp_e32_vcc", 64);
  run<25>("v_cmp_e64_sgpr", 64);
  run<26>("sub+cndmask_e32 1:1", 64);
  run<7>("v_cndmask_b32", 64);
  run<12>("v_cndmask_e64_sgpr", 64);
  run<17>("v_cndmask_vcc_cmp", 64);
  run<13>("v_max_i32", 64);
  run<14>("v_and_b32", 64);
  run<15>("v_perm_b32", 64);
  run<16>("v_med3_i32", 64);
  run<18>("v_permlane32_swap", 64);
  run<19>("v_mul_u32_u24", 64);
  run<20>("v_lshlrev_b32", 64);
  run<21>("v_dot2c_i32_i16", 64);
  return 0;
  run<0>("v_add_u32", 64);
  run<1>("v_dot2_i32_i16", 64);
  run<2>("v_pk_add_u16", 64);
  run<10>("v_pk_mad_i16", 64);
  run<6>("v_add_u32_dpp", 64);
  run<7>("v_cndmask_b32", 64);
  run<11>("v_alignbit_b32", 64);
  run<8>("v_mul_lo_u32", 64);
  run<4>("v_mad_i64_i32", 32);
  run<3>("v_fma_f64", 32);
  run<9>("v_mul_f64", 32);
  run<5>("v_rcp_f64", 32);
  return 0;
}
