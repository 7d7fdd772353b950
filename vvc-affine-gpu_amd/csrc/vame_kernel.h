// vame_kernel.h -- HIP/CDNA4 device code of the affine-ME hot path.
//
// One workgroup = one work item: a 64x64 quadrant of a CTU (kernel
// affine_me_quad, 256 threads) or, for the 128-wide/high aligned sizes, the
// whole 128x128 CTU (kernel affine_me_ctu, 1024 threads), for one reference frame, holding
// the candidate CUs of one or more CU-size groups.  The workgroup runs the
// complete gradient-based CPMV refinement of affine.cl:195-917 for all of them
// -- 2 control points, then 3 control points seeded from the 2-CP winner of
// the same CU (affine.cl:81-105) -- without leaving the CU:
//   * the reference region (+16 px margin, clamp-to-edge padded) is staged
//     once into LDS; every 9x9 filter window of every iteration is read from
//     there (windows leaving the tile fall back to clamped global loads);
//   * predictions live in a CU-compact LDS buffer; gradients are computed on
//     the fly from it (no global gradient / equation scratch);
//   * each CU's normal equations are reduced as exact integer sums (14 values
//     for 2 CP, 24 moments for 3 CP) with DPP segment reductions and solved by
//     one lane per CU with the reference's double-precision elimination,
//     operation for operation, in registers.
// Two scheduling modes per work item (chosen on the host, vame_engine.hip):
//   autonomous  every CU has <= 64 sub-blocks and is owned by ONE wave; each
//               wave iterates its CUs on its own (wave-local LDS ordering
//               only, no workgroup barrier inside the iteration loop);
//   cooperative larger CUs span several waves; one workgroup barrier per phase
//               and the partial sums meet in LDS int64 atomics.
// Per iteration and CU: predict (one lane per 4x4 sub-block: MV field, window,
// 6-tap H/V filter on v_dot2_i32_i16, SATD) -> cost (one lane per CU) ->
// gradient (Sobel on packed int16 sample pairs, CU-border replication,
// residual, five dot2 sums per sub-block) -> solve (one lane per CU).
// Bit-exactness notes (SURVEY.md §8a traps): integer math is exact and
// order-free; the only float work is floor(lambda*bits) (single precision)
// and the FP64 solve (compiled with -ffp-contract=off, explicit fma where the
// reference's FP_CONTRACT=ON fuses, affine.cl:851); (int)double follows
// v_cvt_i32_f64 (NaN -> 0, saturate) explicitly.
#pragma once
#include <hip/hip_runtime.h>

#include "vame_tables.h"

namespace vame {

constexpr int kMaxCu = 16;    // CU state slots per workgroup (LDS)
constexpr int kMaxTasks = 16;  // autonomous items: wave tasks (wave w runs tasks w, w + 4, ...)
constexpr int kTaskCu = 4;    // CUs per wave task (<= 64 sub-blocks, >= 16 each)
constexpr int kItemCu = kMaxTasks * kTaskCu;  // CU slots per work item
constexpr int kThreads = 256;  // quadrant workgroups
constexpr int kNumMom = 24;   // 3 CP: {1,u,v,uu,uv,vv} x {xx,xy,yy} + {1,u,v} x {xe,ye}
constexpr int kNumVal2 = 14;  // 2 CP: 10 distinct matrix entries + 4 right-hand sides

// device view of vame_cpmvs / typedef.h Cpmvs (28 bytes)
struct vame_cpmvs_dev {
  int32_t ncps, ltx, lty, rtx, rty, lbx, lby;
};

struct CuSlot {          // 8 bytes
  uint8_t x, y;          // CTU-relative position
  uint8_t lw : 4, lh : 4;  // log2 width / height
  uint8_t align : 1;     // 0 FULL, 1 HALF
  uint8_t taskCus : 5;   // a task's first slot: CUs in the task (0 elsewhere)
  uint16_t outOff : 9;   // RETURN_STRIDE[group] + cuIdx
  uint16_t taskLogL : 4;  // a task's first slot: log2 lanes per CU
  uint16_t pad;
};
static_assert(sizeof(CuSlot) == 8, "CuSlot packing");

// An item's CUs come in tasks of one CU size each, run over the item's one
// staged tile: a cooperative item's tasks one after another by the whole
// workgroup, an autonomous item's tasks by its waves (wave w: tasks w, w + 4).
// Task t holds CU slots t * kTaskCu .. (a single-task cooperative item: up to
// kMaxCu slots from 0).
struct Item {
  int16_t nCu;      // CU slots (host view; unused slots have lw 0)
  int16_t rx, ry;   // region origin (CTU-relative)
  int16_t coop;     // bit 0: cooperative (a task's CUs span waves); bit 1: autonomous waves claim tasks;
                    // bit 2: two stacked sub-blocks per lane (affine_me_quad's SBL2 items)
  int16_t nTasks;
  int16_t rw, rh;   // affine_me_half items: the region's extent (the CU's); 0 elsewhere
  int16_t pad;
  CuSlot cu[kItemCu];
};

// One (POC, refIdx) pair of a launch: the reference's kernel arguments for it
// (affine.cl:11 / :960: frames, lambda, result arrays per PRED).
struct PairArgs {
  const uint16_t* cur;
  const uint16_t* ref;
  int64_t* cost[4];           // [FULL_2CP, FULL_3CP, HALF_2CP, HALF_3CP]
  vame_cpmvs_dev* cpmv[4];
  float lambda;
  int32_t pad;
};
constexpr int kMaxPairs = 32;  // pairs per launch (kernel-argument table, 2.9 KB)

struct KParams {
  PairArgs pair[kMaxPairs];
  const vame_cpmvs_dev* prev[2];  // [align]: 3-CP seeds when the 2-CP pass is not run
  // kernels with two sub-blocks per lane (affine_me_ctu2 / _half2w / _half2h):
  // the five gradient sums of every sub-block at its CU's best 2-CP iteration
  // (3-CP seed reuse), per (pair, CTU, item): [nPairs * nCtus * nItems][5][NSB]
  // -- global, not LDS, so that two / four workgroups fit a CU
  int32_t* bestS;
  const Item* items;
  const int32_t* order;      // [nChunks][cpp]: CTU of each padded combination slot, -1 = padding
  int nItems, nCtus, nPairs;
  int groupPairs, groupPer;  // groups of the block order (see affine_me_body)
  int nChunks, cpp;          // CTU chunks per pair, padded combination slots per (pair, chunk)
  int W, H, ctusPerRow;
  int extra;
  int run2, run3;
};

// Instrumentation builds only (the product build sets neither):
// VAME_ABLATE (timing-only builds, results are wrong): bit 0 skip the solve,
// bit 1 skip the gradient math, bit 2 skip the reductions of the equations,
// bit 3 skip the prediction math, bit 4 skip the 128-class launch, bit 5 skip
// the quadrant launch, bit 8 (host) 128-class templates without the 128x64 /
// 64x128 items, bit 9 every 9x9 window read from the tile (no clamped-global path),
// bit 10 the same in the 3-CP pass only, bit 11 no seed-reuse sums stored by
// the two-sub-block kernels' 2-CP pass.
#ifndef VAME_ABLATE
#define VAME_ABLATE 0
#endif
// VAME_DUP (timing-only builds, results stay correct): run a phase twice to
// price it in throughput terms: bit 0 prediction, bit 1 gradient, bit 2
// equation reduction, bit 6 the tile staging round trip, bit 4 the solve (on the system itself, before the real
// one rebuilds it: no extra LDS); with bit 5 set, only in the 3-CP pass.  The
// rest of an iteration: bit 7 the CU's MV field (mv_field), bit 8 the extended
// prediction rows (DPP neighbour columns, edge-row publication and reads),
// bit 9 the SATD segment sum, bit 10 the cost / best step, bit 11 the CPMV
// update (scaleDeltaMvs, clamp, clip, rate bits, flag sums).
#ifndef VAME_DUP
#define VAME_DUP 0
#endif
// Wave priority (s_setprio) during the latency-bound solve: its dependent
// FP64 / LDS chain issues ahead of other waves' prediction work (~0.5 %;
// priority 1 / 3 and priority over the whole post-prediction part measured
// the same).
constexpr int kSolvePrio = 3;

// VAME_COUNT_PRED (instrumentation builds, libvame_count.so): every lane counts
// the sub-block predictions it runs (the exact early exit skips the rest of
// the algorithmic n_pred per sub-block); g_pred_count[kernel: quad, ctu], and
// [2 + 2 kernel + (3-CP pass)]: those whose 9x9 window left the staged tile
// (the clamped-global path); [12 + kernel]: 64 lane slots per wave that runs a
// prediction step, [14 + kernel] / [16 + kernel]: the same slots and the
// predictions run, of waves holding several CUs (autonomous, < 64 sub-blocks
// per CU) -- the lanes an iteration spends on settled CUs.
#ifndef VAME_COUNT_PRED
#define VAME_COUNT_PRED 0
#endif
#if VAME_COUNT_PRED
__device__ unsigned long long g_pred_count[20];
#define PC_DECL unsigned pc_n = 0, pc_w = 0, pc_mw = 0, pc_me = 0;
#define PC_ADD                                                           \
  {                                                                      \
    pc_n++;                                                              \
    const unsigned long long m_ = __builtin_amdgcn_ballot_w64(true);     \
    if (__lane_id() == __builtin_ctzll(m_)) {                            \
      pc_w += 64;                                                        \
      if (!coop && logS < 6) {                                           \
        pc_mw += 64;                                                     \
        pc_me += __popcll(m_);                                           \
      }                                                                  \
    }                                                                    \
  }
#define PC_FLUSH                                                                                \
  {                                                                                             \
    if (pc_n) atomicAdd(&g_pred_count[REGION == 128], (unsigned long long)pc_n);               \
    if (pc_w) atomicAdd(&g_pred_count[12 + (REGION == 128)], (unsigned long long)pc_w);        \
    if (pc_mw) atomicAdd(&g_pred_count[14 + (REGION == 128)], (unsigned long long)pc_mw);      \
    if (pc_me) atomicAdd(&g_pred_count[16 + (REGION == 128)], (unsigned long long)pc_me);      \
  }
#else
#define PC_DECL
#define PC_ADD
#define PC_FLUSH
#endif

// VAME_PHASE_TIMING (profiling-only builds, libvame_phase.so): every wave sums
// the shader clock spent per phase and adds it to g_phase_cycles at exit.
#ifndef VAME_PHASE_TIMING
#define VAME_PHASE_TIMING 0
#endif
enum { kPhStage, kPhPredict, kPhCost, kPhGradient, kPhSolve, kPhTail, kPhReduce, kNumPhases };
#if VAME_PHASE_TIMING
// [kernel: quad, ctu, half, ctu2, half2w, half2h, quad2][phase + kNumPhases for the
// 3-CP pass; then SIMD-slot use (2), workgroups, workgroup lifetimes]
// (kPhGradient: the gradient sums; kPhReduce: the equations' reduction and
// the barrier after it)
constexpr int kPhSlots = 2 * kNumPhases + 4;
__device__ unsigned long long g_phase_cycles[7][kPhSlots];
#define PH_DECL unsigned long long ph_acc[2 * kNumPhases] = {}; unsigned long long ph_t = __builtin_amdgcn_s_memtime(); const unsigned long long ph_t0 = ph_t;
#define PH_MARK(i) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ph_acc[(i) + ph_off] += t_ - ph_t; ph_t = t_; }
// plus SIMD-slot use: [12] = waves x block lifetime, [13] = sum of wave lifetimes
__shared__ unsigned long long s_ph_blk[3];  // min start, max end, sum of lifetimes
__shared__ int s_ph_done;
#define PH_FLUSH { \
  if (lane == 0) { \
    for (int i_ = 0; i_ < 2 * kNumPhases; i_++) atomicAdd(&g_phase_cycles[KIND][i_], ph_acc[i_]); \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
    atomicMax(&s_ph_blk[1], t1_); \
    atomicAdd(&s_ph_blk[2], t1_ - ph_t0); \
    const int nw_ = (int)(blockDim.x >> 6); \
    if (atomicAdd(&s_ph_done, 1) == nw_ - 1) { \
      atomicAdd(&g_phase_cycles[KIND][2 * kNumPhases], (unsigned long long)nw_ * (s_ph_blk[1] - s_ph_blk[0])); \
      atomicAdd(&g_phase_cycles[KIND][2 * kNumPhases + 1], s_ph_blk[2]); \
      atomicAdd(&g_phase_cycles[KIND][2 * kNumPhases + 2], 1ull); \
      atomicAdd(&g_phase_cycles[KIND][2 * kNumPhases + 3], s_ph_blk[1] - s_ph_blk[0]); \
    } \
  } }
#define PH_INIT { if (tid == 0) { s_ph_blk[0] = ~0ull; s_ph_blk[1] = 0; s_ph_blk[2] = 0; s_ph_done = 0; } }
#define PH_START { if (lane == 0) atomicMin(&s_ph_blk[0], ph_t0); }
#elif defined(VAME_ISA_MARKS)  // analysis builds: phase ends as comments in the ISA
#define PH_DECL
#define PH_MARK(i) asm volatile("; PHASE_END " #i);
#define PH_FLUSH
#define PH_INIT
#define PH_START
#else
#define PH_DECL
#define PH_MARK(i)
#define PH_FLUSH
#define PH_INIT
#define PH_START
#endif

// ------------------------------------------------------------------ helpers
typedef short short2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }
__device__ __forceinline__ int shl(int a, int s) { return (int)((unsigned)a << s); }
__device__ __forceinline__ short2v as_s2(unsigned v) { return __builtin_bit_cast(short2v, v); }
__device__ __forceinline__ unsigned as_u(short2v v) { return __builtin_bit_cast(unsigned, v); }
// v_dot2_i32_i16: a.lo*b.lo + a.hi*b.hi + acc (signed 16-bit halves, no clamp)
__device__ __forceinline__ int dot2(unsigned a, unsigned b, int acc) {
  return __builtin_amdgcn_sdot2(as_s2(a), as_s2(b), acc, false);
}
// low 16 bits of lo | low 16 bits of hi << 16
__device__ __forceinline__ unsigned pack16(int lo, int hi) {
  return __builtin_amdgcn_perm((unsigned)hi, (unsigned)lo, 0x05040100u);
}

// LDS ordering between the lanes of one wave (a wave's LDS ops execute in order)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void phase_sync(bool coop) {
  if (coop)
    __syncthreads();
  else
    wave_sync();
}

// aux_functions.cl:51-67 clipMv
__device__ __forceinline__ void clip_mv(int& x, int& y, int bx, int by, int W, int H) {
  x = clampi(x, shl(-128 - 8 - bx + 1, 4), shl(W + 8 - bx - 1, 4));
  y = clampi(y, shl(-128 - 8 - by + 1, 4), shl(H + 8 - by - 1, 4));
}

// aux_functions.cl:106-141 (bipred == 0)
__device__ __forceinline__ bool spread_over_limit(int a, int b, int c, int d, bool six) {
  const int s4 = 4 << 11;
  int w = (abs(4 * a + s4) >> 11) + 9, h = (abs(4 * b) >> 11) + 9;
  if (w * h > 165) return true;
  // 2 CP: (c, d) = (-b, a), so the second test's w and h are the first's h and
  // w -- the same product
  if (!six) return false;
  w = (abs(4 * c) >> 11) + 9;
  h = (abs(4 * d + s4) >> 11) + 9;
  return w * h > 165;
}

// aux_functions.cl:2057-2075 (1/16 -> 1/4 pel)
__device__ __forceinline__ int to_quarter(int v) { return v >= 0 ? (v + 1) >> 2 : (v + 2) >> 2; }

// aux_functions.cl:2117-2129
__device__ __forceinline__ int eg_bits(int value) {
  unsigned t = value <= 0 ? ((unsigned)(-value) << 1) + 1u : (unsigned)value << 1;
  int len = 1;
  while (t > 128u) {
    len += 14;
    t >>= 7;
  }
  return len + ((31 - __clz((int)t)) << 1);
}

// aux_functions.cl:2140-2189 with zero predictors (affine.cl:431-434)
__device__ __forceinline__ int affine_bits(const int* c, int ncp) {
  int ltx = to_quarter(c[0]), lty = to_quarter(c[1]);
  int b = eg_bits(ltx) + eg_bits(lty) + eg_bits(to_quarter(c[2]) - ltx) +
          eg_bits(to_quarter(c[3]) - lty);
  if (ncp == 3) b += eg_bits(to_quarter(c[4]) - ltx) + eg_bits(to_quarter(c[5]) - lty);
  return b;
}

// (int)double with the semantics the reference's kernels get from the GPU:
// truncation, NaN -> 0, out-of-range values saturate -- exactly what
// v_cvt_i32_f64 does, so it is issued directly (a C++ cast of an out-of-range
// value is undefined and would need explicit checks).
__device__ __forceinline__ int cvt_i32_f64(double d) {
  int r;
  asm("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(d));
  return r;
}

// aux_functions.cl:2194-2215
__device__ __forceinline__ int scale_delta(double d) {
  double s = d >= 0 ? 1.0 : -1.0;
  return shl(cvt_i32_f64(d * 4.0 + s * 0.5), 2);
}

// DPP lane shift with zero fill for lanes whose source is outside the pattern
// (bound_ctrl) or whose row is masked off (old = 0).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xF, true);
}

// ---------------------------------------------------------- filter tap pairs
// kLuma6 (constants.cl:40-58) re-packed for v_dot2_i32_i16.  A 4-wide output
// row reads 5 dwords D[0..4] of its window row (two samples each); output c
// applies set s' + (c & 1) to D[(c >> 1) .. (c >> 1) + 3], where s' is the
// parity of the window start inside the dword stream:
//   set 0: (f0,f1) (f2,f3) (f4,f5) (0,0)     set 1: (0,f0) (f1,f2) (f3,f4) (f5,0)
//   set 2: (0,0) (f0,f1) (f2,f3) (f4,f5)
// The vertical pass uses sets 0/1 on row pairs (t[2k], t[2k+1]) the same way.
struct CoefTab {
  uint32_t v[16][3][4];
};
constexpr uint32_t pk16c(int lo, int hi) {
  return (uint32_t)(uint16_t)(int16_t)lo | ((uint32_t)(uint16_t)(int16_t)hi << 16);
}
constexpr CoefTab make_coef_tab() {
  CoefTab t{};
  for (int f = 0; f < 16; f++) {
    const int8_t* c = kLuma6[f];
    const uint32_t s0[4] = {pk16c(c[0], c[1]), pk16c(c[2], c[3]), pk16c(c[4], c[5]), 0u};
    const uint32_t s1[4] = {pk16c(0, c[0]), pk16c(c[1], c[2]), pk16c(c[3], c[4]), pk16c(c[5], 0)};
    const uint32_t s2[4] = {0u, pk16c(c[0], c[1]), pk16c(c[2], c[3]), pk16c(c[4], c[5])};
    for (int k = 0; k < 4; k++) {
      t.v[f][0][k] = s0[k];
      t.v[f][1][k] = s1[k];
      t.v[f][2][k] = s2[k];
    }
  }
  return t;
}
static __constant__ CoefTab kCoefTab = make_coef_tab();  // one copy per translation unit

// ------------------------------------------------------------- motion field
struct MvField {
  int bx, by, hx, hy, vx, vy;
  bool spread;
};

// deriveMv{2,3}Cps_and_spread (aux_functions.cl:146-212), once per CU and iteration
__device__ __forceinline__ MvField mv_field(const int* cp, int ncp, int lw, int lh) {
  MvField f;
  f.hx = shl(cp[2] - cp[0], 7 - lw);
  f.hy = shl(cp[3] - cp[1], 7 - lw);
  if (ncp == 3) {
    f.vx = shl(cp[4] - cp[0], 7 - lh);
    f.vy = shl(cp[5] - cp[1], 7 - lh);
  } else {
    f.vx = -f.hy;
    f.vy = f.hx;
  }
  f.spread = spread_over_limit(f.hx, f.hy, f.vx, f.vy, ncp == 3);
  f.bx = shl(cp[0], 7);
  f.by = shl(cp[1], 7);
  return f;
}

struct Geo {       // a lane's CU
  int x, y;        // frame position
  int lw, lh, w, h;
};

// Hide a value's origin from the optimizer: per-lane geometry is loop-invariant
// for a whole work item, and hoisting every address derived from it out of the
// iteration loop would pin ~60 VGPRs; recomputing them per phase is a few adds.
__device__ __forceinline__ void opaque(int& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void opaque_geo(Geo& g, int& sx, int& sy) {
  opaque(g.x); opaque(g.y); opaque(sx); opaque(sy);
  opaque(g.lw); opaque(g.lh);
}


// Horizontal 6-tap pass of one window row (5 dwords = samples 0..9 of the row
// in dword order), offset -IF_INTERNAL_OFFS << 2 = -32768, shift 2
// (aux_functions.cl:1128-1161).  |t| < 2^14, so rows pack into int16 pairs.
__device__ __forceinline__ void hrow(const unsigned (&D)[5], const uint4& KA, const uint4& KB,
                                     int (&t)[4]) {
  t[0] = dot2(D[0], KA.x, dot2(D[1], KA.y, dot2(D[2], KA.z, dot2(D[3], KA.w, -32768)))) >> 2;
  t[1] = dot2(D[0], KB.x, dot2(D[1], KB.y, dot2(D[2], KB.z, dot2(D[3], KB.w, -32768)))) >> 2;
  t[2] = dot2(D[1], KA.x, dot2(D[2], KA.y, dot2(D[3], KA.z, dot2(D[4], KA.w, -32768)))) >> 2;
  t[3] = dot2(D[1], KB.x, dot2(D[2], KB.y, dot2(D[3], KB.z, dot2(D[4], KB.w, -32768)))) >> 2;
}
// The same row before the >> 2 (the shift happens while packing, pack_shr2),
// with the offsets re-based so that no accumulator needs a non-inline
// constant: the six taps of every phase sum to 64, so
//   sum_v f_v * ((S_v - 32768) >> 2) + 512 + (8192 << 6)
//     = sum_v f_v * ((S_v - 32768) >> 2 + 8192 + 8)
//     = sum_v f_v * ((S_v + 32) >> 2)
// (32768 is a multiple of 4, so the floor shifts by exactly 8192): the rows
// start from +32 and the vertical accumulators from 0.  (S_v + 32) >> 2 stays
// within [-5619, 22008], so the packed int16 pairs are exact.
// a.lo*b.lo + a.hi*b.hi + K for an inline constant K, as the VOP3 form (the
// compiler picks the accumulate-in-place v_dot2c form and a v_mov of K)
template <int K>
__device__ __forceinline__ int dot2k(unsigned a, unsigned b) {
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "i"(K));
  return r;
}
__device__ __forceinline__ void hrow_raw(const unsigned (&D)[5], const uint4& KA, const uint4& KB,
                                         int (&t)[4]) {
  t[0] = dot2(D[0], KA.x, dot2(D[1], KA.y, dot2(D[2], KA.z, dot2k<32>(D[3], KA.w))));
  t[1] = dot2(D[0], KB.x, dot2(D[1], KB.y, dot2(D[2], KB.z, dot2k<32>(D[3], KB.w))));
  t[2] = dot2(D[1], KA.x, dot2(D[2], KA.y, dot2(D[3], KA.z, dot2k<32>(D[4], KA.w))));
  t[3] = dot2(D[1], KB.x, dot2(D[2], KB.y, dot2(D[3], KB.z, dot2k<32>(D[4], KB.w))));
}
// (lo >> 2) | (hi >> 2) << 16 in two instructions: the second shift writes its
// low 16 bits straight into the upper half (SDWA dst_sel:WORD_1, preserve).
__device__ __forceinline__ unsigned pack_shr2(int lo, int hi) {
  unsigned d = (unsigned)(lo >> 2);
  asm("v_ashrrev_i32_sdwa %0, 2, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "
      "src1_sel:DWORD"
      : "+v"(d)
      : "v"(hi));
  return d;
}
// (lo >> 10) | (hi >> 10) << 16, the same way (arithmetic shifts).
__device__ __forceinline__ unsigned pack_sra10(int lo, int hi) {
  unsigned d = (unsigned)(lo >> 10);
  asm("v_ashrrev_i32_sdwa %0, 10, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "
      "src1_sel:DWORD"
      : "+v"(d)
      : "v"(hi));
  return d;
}
// Vertical pass, streamed: row pair k = (t[2k], t[2k+1]) (pair 4 = (t[8], 0))
// feeds output row r through tap-pair set G_{r&1}, entry k - (r >> 1)
// (aux_functions.cl:1182-1223); integer sums, so the order is free.
// t0/t1 are the raw horizontal sums (before >> 2).
__device__ __forceinline__ void vpair(int k, const int (&t0)[4], const int (&t1)[4],
                                      const uint4& G0, const uint4& G1, int (&acc)[4][4]) {
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const unsigned P = pack_shr2(t0[c], t1[c]);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = k - (r >> 1);
      if (m < 0 || m > 3 || ((r & 1) == 0 && m == 3)) continue;  // set 0 ends with (0,0)
      const uint4& G = (r & 1) ? G1 : G0;
      const unsigned g = m == 0 ? G.x : m == 1 ? G.y : m == 2 ? G.z : G.w;
      acc[r][c] = m == 0 ? dot2k<0>(P, g) : dot2(P, g, acc[r][c]);  // first tap pair starts the sum
    }
  }
}
// Window rows from the LDS tile, one row pair at a time (software-pipelining
// the reads one pair ahead held ~20 more VGPRs for no measurable gain: the
// other waves hide the LDS latency).
template <int PITCH_DW>
__device__ __forceinline__ void filter_rows(const unsigned* src, const uint4& KA, const uint4& KB,
                                            const uint4& G0, const uint4& G1, int (&acc)[4][4]) {
#pragma unroll
  for (int k = 0; k < 5; k++) {
    unsigned E[2][5];
#pragma unroll
    for (int h = 0; h < 2; h++)
      if (2 * k + h < 9) {  // row 9 does not exist
#pragma unroll
        for (int q = 0; q < 5; q++) E[h][q] = src[(2 * k + h) * PITCH_DW + q];
      }
    int t0[4], t1[4] = {0, 0, 0, 0};
    hrow_raw(E[0], KA, KB, t0);
    if (k < 4) hrow_raw(E[1], KA, KB, t1);
    vpair(k, t0, t1, G0, G1, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
}
// A wave some of whose windows leave the LDS tile: every lane runs the one
// filter_rows computation, its window rows from the tile (in-tile lanes, taps
// of their start parity) or from the frame (the others, re-aligned to an even
// start, parity-0 taps), so such a wave computes its predictions once instead
// of once per path.  The frame rows come in two batches (rows 0-3, rows 4-8,
// each batch's loads in flight together): 6 dwords per row from the uniform
// frame base, re-aligned by v_alignbit, or -- a window crossing the left /
// right frame edge -- per-sample clamped loads; rows clamp to the frame
// (clamp-to-edge, affine.cl:254-326).
// One window row from the frame, as 5 dwords of sample pairs from an even
// start: 6 dwords from the uniform frame base re-aligned by v_alignbit, or --
// a window crossing the left / right frame edge -- per-sample clamped loads.
__device__ __forceinline__ void frame_row(const uint16_t* __restrict__ ref, int wx, int y, int W,
                                          bool wide, unsigned (&D)[5]) {
  if (wide) {
    const char* base = reinterpret_cast<const char*>(ref);
    const unsigned a = (unsigned)wx * 2u, b = a & ~3u, sh = (a & 2u) << 3;  // sh: 0 or 16 bits
    const unsigned off = (unsigned)y * (unsigned)W * 2u + b;
    unsigned raw[6];
    // dword-aligned 16 + 8 byte loads (global_load_dwordx4 / x2 need only dword alignment)
    typedef unsigned u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
    typedef unsigned u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
    const u32x4a4 v4 = *reinterpret_cast<const u32x4a4*>(base + off);
    const u32x2a4 v2 = *reinterpret_cast<const u32x2a4*>(base + (off + 16u));
    raw[0] = v4.x; raw[1] = v4.y; raw[2] = v4.z; raw[3] = v4.w; raw[4] = v2.x; raw[5] = v2.y;
#pragma unroll
    for (int q = 0; q < 5; q++) D[q] = __builtin_amdgcn_alignbit(raw[q + 1], raw[q], sh);
  } else {
    const uint16_t* row = ref + (size_t)y * W;
#pragma unroll
    for (int q = 0; q < 5; q++)
      D[q] = (unsigned)row[clampi(wx + 2 * q, 0, W - 1)] | ((unsigned)row[clampi(wx + 2 * q + 1, 0, W - 1)] << 16);
  }
}
// A wave some of whose windows leave the LDS tile: every lane runs the one
// filter_rows computation, its window rows from the tile (in-tile lanes, taps
// of their start parity) or from the frame (the others: rows clamped to the
// frame, clamp-to-edge as affine.cl:254-326, re-aligned to an even start,
// parity-0 taps), one row pair per step -- so such a wave computes its
// predictions once, not once per path, and waits for 5 rounds of frame
// loads instead of 9.
template <int PITCH_DW>
__device__ __forceinline__ void filter_rows_mixed(const unsigned* src, bool inTile,
                                                  const uint16_t* __restrict__ ref, int wx, int wy, int W,
                                                  int H, const uint4& KA, const uint4& KB, const uint4& G0,
                                                  const uint4& G1, int (&acc)[4][4]) {
  const bool wide = wx >= 0 && wx + 12 <= W;
#pragma unroll
  for (int k = 0; k < 5; k++) {
    unsigned E[2][5];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int row = 2 * k + h;
      if (row < 9) {
        if (inTile) {
#pragma unroll
          for (int q = 0; q < 5; q++) E[h][q] = src[row * PITCH_DW + q];
        } else {
          frame_row(ref, wx, clampi(wy + row, 0, H - 1), W, wide, E[h]);
        }
      }
    }
    int t0[4], t1[4] = {0, 0, 0, 0};
    hrow_raw(E[0], KA, KB, t0);
    if (k < 4) hrow_raw(E[1], KA, KB, t1);
    vpair(k, t0, t1, G0, G1, acc);
    __builtin_amdgcn_sched_barrier(0);
  }
}
// Window leaves the LDS tile: clamp-to-edge loads from the frame
// (affine.cl:254-326), one row at a time (a rare path, kept register-lean:
// scalar vertical taps read from the LDS tap table).
// Vertical taps of window row i into the output rows it feeds.
__device__ __forceinline__ void vrow_acc(int i, const int (&t)[4], const unsigned* s_coef_dw, int fy,
                                         int (&acc)[4][4]) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int m = i - r;  // vertical tap of window row i for output row r
    if (m < 0 || m > 5) continue;
    const unsigned pr = s_coef_dw[fy * 12 + (m >> 1)];  // set 0: (f0,f1) (f2,f3) (f4,f5)
    const int cf = (int)(short)(m & 1 ? pr >> 16 : pr & 0xFFFF);
#pragma unroll
    for (int c = 0; c < 4; c++) acc[r][c] += t[c] * cf;
  }
}

// The window read from the frame (it left the staged tile): rows clamped to
// the frame.  A window whose samples wx .. wx + 11 lie inside its rows is
// read as 6 dwords per row from the uniform frame base (32-bit offsets), the
// loads of three rows in flight together, and re-aligned by v_alignbit; one
// that crosses the left / right frame edge takes the per-sample clamped loads.
// (The rows' latency dominates this path: 9 dependent round trips cost the
// 2160p configs 10-20 % of their time.)
__device__ __forceinline__ void filter_rows_global(const uint16_t* __restrict__ ref, int wx, int wy,
                                                   int W, int H, const uint4& KA, const uint4& KB,
                                                   const unsigned* s_coef_dw, int fy,
                                                   int (&acc)[4][4]) {
  if (wx >= 0 && wx + 12 <= W) {
    const char* base = reinterpret_cast<const char*>(ref);
    const unsigned a = (unsigned)wx * 2u, b = a & ~3u, sh = (a & 2u) << 3;  // sh: 0 or 16 bits
    constexpr int NB = 5;  // rows whose loads are in flight together
#pragma unroll 1
    for (int i0 = 0; i0 < 9; i0 += NB) {
      unsigned raw[NB][6];
#pragma unroll
      for (int j = 0; j < NB; j++) {
        if (i0 + j >= 9) break;
        const unsigned off = (unsigned)clampi(wy + i0 + j, 0, H - 1) * (unsigned)W * 2u + b;
#pragma unroll
        for (int k = 0; k < 6; k++) raw[j][k] = *reinterpret_cast<const unsigned*>(base + (off + 4u * k));
      }
#pragma unroll
      for (int j = 0; j < NB; j++) {
        if (i0 + j >= 9) break;
        unsigned D[5];
#pragma unroll
        for (int q = 0; q < 5; q++) D[q] = __builtin_amdgcn_alignbit(raw[j][q + 1], raw[j][q], sh);
        D[4] &= 0xFFFFu;  // sample wx + 9 meets a zero tap (as in the clamped path)
        int t[4];
        hrow(D, KA, KB, t);
        vrow_acc(i0 + j, t, s_coef_dw, fy, acc);
      }
    }
    return;
  }
#pragma unroll 1
  for (int i = 0; i < 9; i++) {
    const uint16_t* row = ref + (size_t)clampi(wy + i, 0, H - 1) * W;
    unsigned D[5];
#pragma unroll
    for (int q = 0; q < 5; q++) {
      const unsigned lo = row[clampi(wx + 2 * q, 0, W - 1)];
      const unsigned hi = q < 4 ? row[clampi(wx + 2 * q + 1, 0, W - 1)] : 0u;
      D[q] = lo | (hi << 16);
    }
    int t[4];
    hrow(D, KA, KB, t);
    vrow_acc(i, t, s_coef_dw, fy, acc);
  }
}

// xCalcHADs4x4 with the JVET_R0164 DC weighting (aux_functions.cl:1940-2043)
// on packed int16 pairs: the residual o - p is within +-1023, so every stage
// of the 4x4 Hadamard stays within +-16368 and the packed 16-bit adds are
// exact.  Rows are transformed first (elementwise on row vectors), then each
// row vector (c0,c1)(c2,c3); the outputs are the same 16 Walsh-Hadamard
// coefficients as the reference's butterfly (in another order -- the sum of
// magnitudes does not depend on it), the DC term being the first lane of row
// vector 0.  |.| sums run on v_dot2 against (1,1).
__device__ __forceinline__ int satd_4x4(const uint2 (&O)[4], const uint2 (&P)[4]) {
  short2v a[4][2];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    a[r][0] = as_s2(O[r].x) - as_s2(P[r].x);
    a[r][1] = as_s2(O[r].y) - as_s2(P[r].y);
  }
  short2v d[4][2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const short2v m0 = a[0][k] + a[3][k], m1 = a[1][k] + a[2][k];
    const short2v m2 = a[1][k] - a[2][k], m3 = a[0][k] - a[3][k];
    d[0][k] = m0 + m1;
    d[1][k] = m2 + m3;
    d[2][k] = m0 - m1;
    d[3][k] = m3 - m2;
  }
  const short2v pm = {1, -1}, z = {0, 0};
  int sum = 0, dc = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const short2v X = d[r][0], Ys = __builtin_shufflevector(d[r][1], d[r][1], 1, 0);
    const short2v mm = X + Ys, nn = X - Ys;  // (c0+c3, c1+c2), (c0-c3, c1-c2)
    // (u + v, u - v) of each pair, one v_pk_mad_i16 with op_sel
    const short2v e0 = __builtin_shufflevector(mm, mm, 1, 1) * pm + __builtin_shufflevector(mm, mm, 0, 0);
    const short2v e1 = __builtin_shufflevector(nn, nn, 1, 1) * pm + __builtin_shufflevector(nn, nn, 0, 0);
    const short2v a0 = __builtin_elementwise_max(e0, z - e0), a1 = __builtin_elementwise_max(e1, z - e1);
    if (r == 0) {
      dc = (unsigned short)a0[0];
      sum = dot2(as_u(a0), 0x00010000u, sum);
    } else {
      sum = dot2(as_u(a0), 0x00010001u, sum);
    }
    sum = dot2(as_u(a1), 0x00010001u, sum);
  }
  sum += dc >> 2;
  return (sum + 1) >> 1;
}

// PROF, the reference's hard-disabled refinement (enablePROF = 0 at
// affine.cl:168 / :1132), offered as an option (vame_set_prof).  Per sample,
// the MV offset from the sub-block centre (aux_functions.cl:218-404,
// get{Horizontal,Vertical}DeltasPROF{2,3}Cps), linear in (r, c) before its
// rounding: m(r, c) = 2 (h + v) - 2 (4h + 4v) + 4h c + 4v r, rounded by 8 bits
// (roundValue16) and clamped to +-31.  Recomputed per sample from six
// registers instead of holding 32 deltas.
__device__ __forceinline__ int prof_delta(int base, int q4h, int q4v, int r, int c) {
  const int m = base + q4h * c + q4v * r;
  return clampi((m + 128 - (m >= 0)) >> 8, -31, 31);
}
// PROF proper (aux_functions.cl:471-605) on the vertical pass taken as not
// the last one (shift 6, no offset, no clip: aux_functions.cl:1163-1174):
// the block padded to 6x6 with the reference samples around the integer
// position nearest the fractional MV (xFrac >> 3, yFrac >> 3), scaled to the
// internal precision, gradients of the >> 6 samples, dI = gx dH + gy dV
// clamped to [-8192, 8191], then (p + dI + 8 + 8192) >> 4 clipped to 10 bits.
// acc holds the vertical sums + 524800 (the re-based filter offsets);
// smp(row, col) reads the 9x9 filter window (origin two samples above-left
// of the integer-MV corner).
template <typename Smp>
__device__ __forceinline__ void prof_refine(const int (&acc)[4][4], const MvField& f, int fx, int fy,
                                            Smp smp, int (&pr)[4][4]) {
  const int xo = fx >> 3, yo = fy >> 3;
  int L[4], R[4], T[4], B[4];  // padding columns / rows, >> 6 of the scaled samples
#pragma unroll
  for (int k = 0; k < 4; k++) {
    L[k] = ((smp(yo + 2 + k, xo + 1) << 4) - 8192) >> 6;
    R[k] = ((smp(yo + 2 + k, xo + 6) << 4) - 8192) >> 6;
    T[k] = ((smp(yo + 1, xo + 2 + k) << 4) - 8192) >> 6;
    B[k] = ((smp(yo + 6, xo + 2 + k) << 4) - 8192) >> 6;
  }
  int p[4][4], q[4][4];
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int c = 0; c < 4; c++) {
      p[r][c] = (acc[r][c] - 524800) >> 6;
      q[r][c] = p[r][c] >> 6;
    }
  const int q4hx = shl(f.hx, 2), q4vx = shl(f.vx, 2), q4hy = shl(f.hy, 2), q4vy = shl(f.vy, 2);
  const int bh = shl(f.hx + f.vx, 1) - shl(q4hx + q4vx, 1);
  const int bv = shl(f.hy + f.vy, 1) - shl(q4hy + q4vy, 1);
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int gx = (c == 3 ? R[r] : q[r][c + 1]) - (c == 0 ? L[r] : q[r][c - 1]);
      const int gy = (r == 3 ? B[c] : q[r + 1][c]) - (r == 0 ? T[c] : q[r - 1][c]);
      const int di = clampi(gx * prof_delta(bh, q4hx, q4vx, r, c) + gy * prof_delta(bv, q4hy, q4vy, r, c),
                            -8192, 8191);
      pr[r][c] = clampi((p[r][c] + di + 8 + 8192) >> 4, 0, 1023);
    }
}

// One 4x4 sub-block: affine MV (affine.cl:215-252), 9x9 window with
// clamp-to-edge (affine.cl:254-326), separable 6-tap filter (aux_functions.cl
// :1096-1239, PROF off), SATD against the original (aux_functions.cl:1940-2043).
// The prediction stays in registers (P[r] = packed sample pairs of row r) for
// the gradient step, and so do the original samples (O[r]).
template <int TILE, int TP, bool PROF, bool FORCE_TILE = false, int NCP = 3>
__device__ __forceinline__ int predict_sb(const MvField& f, int sx, int sy, const Geo& g,
                                          const uint16_t* s_tile, int tx0, int ty0, int tmx, int tmy,
                                          const uint16_t* __restrict__ ref,
                                          const uint16_t* __restrict__ cur, int W, int H,
                                          const uint4* s_coef, uint2 (&P)[4], uint2 (&O)[4],
                                          bool& outside) {
  {  // 32-bit byte offsets from the uniform frame base (frames < 4 GiB): the
     // saddr form of global_load, no 64-bit address arithmetic per row
    const unsigned b0 = (unsigned)((g.y + sy) * W + g.x + sx) * 2u, bw = (unsigned)W * 2u;
    const char* base = reinterpret_cast<const char*>(cur);
#pragma unroll
    for (int r = 0; r < 4; r++) O[r] = *reinterpret_cast<const uint2*>(base + (b0 + (unsigned)r * bw));
  }
  const int px = f.spread ? (g.w >> 1) : sx + 2, py = f.spread ? (g.h >> 1) : sy + 2;
  // |h|, |v| < 2^22 (clamped CPMVs, << (7 - log2 size)), px, py <= 128: 24-bit products are exact
  int mx, my;
  if constexpr (NCP == 2) {  // (vx, vy) = (-hy, hx): no negated operand
    mx = f.bx + __mul24(f.hx, px) - __mul24(f.hy, py);
    my = f.by + __mul24(f.hy, px) + __mul24(f.hx, py);
  } else {
    mx = f.bx + __mul24(f.hx, px) + __mul24(f.vx, py);
    my = f.by + __mul24(f.hy, px) + __mul24(f.vy, py);
  }
  mx = (mx + 64 - (mx >= 0)) >> 7;  // roundMv (aux_functions.cl:38-47)
  my = (my + 64 - (my >= 0)) >> 7;
  // clipMv (aux_functions.cl:51-67) on the frame position of the MV's target,
  // 16 x the CU position + mv: its bounds [(-135 - x) << 4, (W + 7 - x) << 4]
  // shifted by x << 4 become the frame constants [-135 << 4, (W + 7) << 4]
  // (the shift is a multiple of 16: the fractional phase is unchanged)
  const int ax = clampi(mx + shl(g.x, 4), -135 * 16, (W + 7) * 16);
  const int ay = clampi(my + shl(g.y, 4), -135 * 16, (H + 7) * 16);
  const int fx = ax & 15, fy = ay & 15;
  const int wx = (ax >> 4) + sx - 2, wy = (ay >> 4) + sy - 2;  // window origin (frame)
  int tx = wx - tx0, ty = wy - ty0;
  if ((VAME_ABLATE & 512) || FORCE_TILE) {  // timing-only: every window read from the tile (wrong results)
    tx = clampi(tx, 0, tmx);
    ty = clampi(ty, 0, tmy);
  }
  // tmx / tmy: the largest window origin inside the staged tile (its extent - 9)
  const bool inTile = (unsigned)tx <= (unsigned)tmx && (unsigned)ty <= (unsigned)tmy;
  outside = !inTile;
#if VAME_COUNT_PRED
  {  // instrumentation: outside windows that a 4 / 8 / 16 px wider margin would hold
#pragma unroll
    for (int e = 0; e < 3; e++) {
      const int x = 4 << e;
      const bool in = (unsigned)(tx + x) <= (unsigned)(tmx + 2 * x) && (unsigned)(ty + x) <= (unsigned)(tmy + 2 * x);
      const unsigned long long m = __builtin_amdgcn_ballot_w64(!inTile && in);
      if (m && __lane_id() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
        atomicAdd(&g_pred_count[6 + 3 * (TILE > 100) + e], (unsigned long long)__popcll(m));
    }
  }
#endif
  if (!PROF && __builtin_amdgcn_ballot_w64(!(inTile && (fx | fy) == 0)) == 0) {
    // Every active lane has an integer MV inside the tile (e.g. every sub-block
    // of the first 2-CP prediction, from zero CPMVs): the phase-0 filter is the
    // identity -- (64 s - 32768) >> 2 = 16 s - 8192, then
    // (64 (16 s - 8192) + 512 + (8192 << 6)) >> 10 = s, within [0, 1023] (KAT-1)
    // -- so the prediction is the window's inner 4x4, copied from the tile.
    const int i0 = (ty + 2) * TP + tx + 2;  // the block's first sample in the tile
    const unsigned* s32 = reinterpret_cast<const unsigned*>(s_tile) + (i0 >> 1);
    const unsigned sh = (unsigned)(i0 & 1) << 4;  // 0 or 16: its half of the dword
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned d0 = s32[r * (TP / 2)], d1 = s32[r * (TP / 2) + 1], d2 = s32[r * (TP / 2) + 2];
      P[r].x = __builtin_amdgcn_alignbit(d1, d0, sh);
      P[r].y = __builtin_amdgcn_alignbit(d2, d1, sh);
    }
    return satd_4x4(O, P);
  }
  const int sp = inTile ? (tx & 1) : 0;
  const uint4 KA = s_coef[fx * 3 + sp], KB = s_coef[fx * 3 + sp + 1];
  const uint4 G0 = s_coef[fy * 3 + 0], G1 = s_coef[fy * 3 + 1];
  int acc[4][4];
  if (!PROF) {
    // offsets folded into the rows (hrow_raw); the first tap pair overwrites acc (vpair)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int c = 0; c < 4; c++) acc[r][c] = 0;
    const unsigned* src = reinterpret_cast<const unsigned*>(s_tile) + ((ty * TP + tx) >> 1);  // in-tile lanes
    if (__builtin_amdgcn_ballot_w64(!inTile) == 0)
      filter_rows<TP / 2>(src, KA, KB, G0, G1, acc);
    else  // a wave with windows outside the tile: one filter pass for every lane
      filter_rows_mixed<TP / 2>(src, inTile, ref, wx, wy, W, H, KA, KB, G0, G1, acc);
  } else if (inTile) {
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int c = 0; c < 4; c++) acc[r][c] = 0;  // offsets folded into the rows (hrow_raw);
                                                  // the first tap pair overwrites it (vpair)
    const unsigned* src = reinterpret_cast<const unsigned*>(s_tile) + ((ty * TP + tx) >> 1);
    filter_rows<TP / 2>(src, KA, KB, G0, G1, acc);
  } else {
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int c = 0; c < 4; c++) acc[r][c] = 524800;  // (1 << 9) + (8192 << 6)
    filter_rows_global(ref, wx, wy, W, H, KA, KB, reinterpret_cast<const unsigned*>(s_coef), fy,
                       acc);
  }
  int pr[4][4];
  if (PROF && !f.spread) {  // applyPROF = enablePROF && !isSpread (aux_functions.cl:1101)
    if (inTile) {
      const uint16_t* win = s_tile + ty * TP + tx;
      prof_refine(acc, f, fx, fy, [&](int r, int c) { return (int)win[r * TP + c]; }, pr);
    } else {
      prof_refine(acc, f, fx, fy,
                  [&](int r, int c) {
                    return (int)ref[(size_t)clampi(wy + r, 0, H - 1) * W + clampi(wx + c, 0, W - 1)];
                  },
                  pr);
    }
  } else {
    // clipPel on packed pairs: acc >> 10 lies well inside int16 (the taps'
    // absolute sums are below 2^7 per pass), so pack first, then clamp both
    // halves at once (4 instructions per pair instead of 5)
    const short2v lo = {0, 0}, hi = {1023, 1023};
#pragma unroll
    for (int r = 0; r < 4; r++) {
      P[r].x = as_u(__builtin_elementwise_min(
          __builtin_elementwise_max(as_s2(pack_sra10(acc[r][0], acc[r][1])), lo), hi));
      P[r].y = as_u(__builtin_elementwise_min(
          __builtin_elementwise_max(as_s2(pack_sra10(acc[r][2], acc[r][3])), lo), hi));
    }
    return satd_4x4(O, P);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    P[r].x = pack16(pr[r][0], pr[r][1]);
    P[r].y = pack16(pr[r][2], pr[r][3]);
  }
  return satd_4x4(O, P);
}

// Extended prediction row of a sub-block: columns -1..4 as the packed pairs
// (c-1,c0) (c0,c1) (c2,c3) (c3,c4); (c1,c2) is re-derived where needed.
// Column -1 comes from the left lane's column 3 and column 4 from the right
// lane's column 0 (DPP wave_shr:1 / wave_shl:1 -- lanes of a CU row are
// consecutive; at CU edges the values are never used, see grad_sb).
__device__ __forceinline__ uint4 ext_row(const uint2& p, unsigned left, unsigned right) {
  return make_uint4(__builtin_amdgcn_alignbit(p.x, left, 16), p.x, p.y,
                    __builtin_amdgcn_alignbit(right, p.y, 16));
}

// One 4x4 sub-block of the gradient step (affine.cl:477-708): 3x3 Sobel on the
// 6x6 prediction patch (own rows as extended rows X[1..4], the neighbours' edge
// rows X[0] above and X[5] below) with the CU-border replication of
// affine.cl:506-540 (rows first, then columns) -- so patch samples outside the
// CU are never used -- the residual orig - pred (affine.cl:547-579) and the five
// sums S = (gx.gx, gx.gy, gy.gy, gx.e, gy.e).  Samples are handled as packed
// int16 pairs: |g| <= 4092 and |e| <= 1023 fit, and v_dot2_i32_i16 sums stay
// below 2^28 (exact).
// 2 a + b on both int16 halves in one v_pk_mad_i16 (op_sel_hi:0 on the inline
// constant: its low half, 2, multiplies the high halves too)
__device__ __forceinline__ short2v twice_plus(short2v a, short2v b) {
  unsigned r;
  asm("v_pk_mad_i16 %0, %1, 2, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(as_u(a)), "v"(as_u(b)));
  return as_s2(r);
}
__device__ __forceinline__ void grad_sb(int sx, int sy, const Geo& g, const uint4 (&X)[6],
                                        const uint2 (&Orig)[4], int S[5]) {
  short2v O[6][3], E[6][2];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    O[i][0] = as_s2(X[i].x);                                      // (sx-1, sx)
    O[i][1] = as_s2(__builtin_amdgcn_alignbit(X[i].z, X[i].y, 16));  // (sx+1, sx+2)
    O[i][2] = as_s2(X[i].w);                                      // (sx+3, sx+4)
    E[i][0] = as_s2(X[i].y);                                      // (sx, sx+1)
    E[i][1] = as_s2(X[i].z);                                      // (sx+2, sx+3)
  }
  short2v gx[4][2], gy[4][2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    short2v Hd[6], Vs[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
      Hd[i] = O[i][k + 1] - O[i][k];                       // p(c+1) - p(c-1)
      Vs[i] = twice_plus(E[i][k], O[i][k] + O[i][k + 1]);  // p(c-1) + 2 p(c) + p(c+1)
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      gx[r][k] = twice_plus(Hd[r + 1], Hd[r] + Hd[r + 2]);
      gy[r][k] = Vs[r + 2] - Vs[r];
    }
  }
  if (sy == 0) {
#pragma unroll
    for (int k = 0; k < 2; k++) { gx[0][k] = gx[1][k]; gy[0][k] = gy[1][k]; }
  }
  if (sy + 4 == g.h) {
#pragma unroll
    for (int k = 0; k < 2; k++) { gx[3][k] = gx[2][k]; gy[3][k] = gy[2][k]; }
  }
  if (sx == 0) {  // column 0 <- column 1: low half <- high half of pair 0
#pragma unroll
    for (int r = 0; r < 4; r++) {
      gx[r][0] = as_s2(__builtin_amdgcn_perm(as_u(gx[r][0]), as_u(gx[r][0]), 0x03020302u));
      gy[r][0] = as_s2(__builtin_amdgcn_perm(as_u(gy[r][0]), as_u(gy[r][0]), 0x03020302u));
    }
  }
  if (sx + 4 == g.w) {  // column 3 <- column 2: high half <- low half of pair 1
#pragma unroll
    for (int r = 0; r < 4; r++) {
      gx[r][1] = as_s2(__builtin_amdgcn_perm(as_u(gx[r][1]), as_u(gx[r][1]), 0x01000100u));
      gy[r][1] = as_s2(__builtin_amdgcn_perm(as_u(gy[r][1]), as_u(gy[r][1]), 0x01000100u));
    }
  }
  int sxx = 0, sxy = 0, syy = 0, sxe = 0, sye = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint2 o = Orig[r];
    const unsigned e0 = as_u(as_s2(o.x) - E[r + 1][0]), e1 = as_u(as_s2(o.y) - E[r + 1][1]);
    const unsigned x0 = as_u(gx[r][0]), x1 = as_u(gx[r][1]);
    const unsigned y0 = as_u(gy[r][0]), y1 = as_u(gy[r][1]);
    sxx = dot2(x0, x0, dot2(x1, x1, sxx));
    sxy = dot2(x0, y0, dot2(x1, y1, sxy));
    syy = dot2(y0, y0, dot2(y1, y1, syy));
    sxe = dot2(x0, e0, dot2(x1, e1, sxe));
    sye = dot2(y0, e0, dot2(y1, e1, sye));
  }
  S[0] = sxx; S[1] = sxy; S[2] = syy; S[3] = sxe; S[4] = sye;
}

// VTM solveEqual (affine.cl:782-856), forward elimination shared by the lanes
// of a CU's segment (li = lane in the segment, Ls = segment size) on the CU's
// matrix M (row r = private_dEqualCoeff[r + 1], N + 1 columns) in LDS:
// every lane repeats the pivot search (sequential strict '>' scan, NaN never
// wins); the row swap and then each element a[j][k] -= a[i][k] * a[j][i-1] /
// a[i][i-1] of the step (no zero-pivot guard) is done by one lane, with the
// reference's operation order.  Columns left of the pivot are dead and skipped.
// Called by every lane of the wave (act: lane works on a live CU).
template <int N>
__device__ __forceinline__ void seg_eliminate(double* M, int li, int Ls, bool act) {
  constexpr int NC = N + 1;
#pragma unroll
  for (int i = 1; i < N; i++) {
    if (act) {
      double temp = fabs(M[(i - 1) * NC + i - 1]);
      int idx = i - 1;
#pragma unroll
      for (int r = i; r < N; r++) {
        const double f = fabs(M[r * NC + i - 1]);
        if (f > temp) {
          temp = f;
          idx = r;
        }
      }
      if (idx != i - 1 && li < N + 2 - i) {
        const int c = i - 1 + li;
        const double a = M[(i - 1) * NC + c], b = M[idx * NC + c];
        M[(i - 1) * NC + c] = b;
        M[idx * NC + c] = a;
      }
    }
    wave_sync();
    const int cols = N + 1 - i, E = (N - i) * cols;  // constants after unrolling
    if (act) {
      // at most two elements per lane (E <= 30, Ls >= 16); e / cols for e < 64
      // by a multiply-shift (exact for these small operands)
      constexpr int kMagic[7] = {0, 0, 513, 342, 257, 206, 171};  // ceil(1024 / cols)
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int e = li + q * Ls;
        if (e < E) {
          const int dr = (e * kMagic[N + 1 - i]) >> 10, r = i + dr, k = i + e - dr * cols;
          M[r * NC + k] = __dsub_rn(M[r * NC + k], __ddiv_rn(__dmul_rn(M[(i - 1) * NC + k], M[r * NC + i - 1]),
                                                             M[(i - 1) * NC + i - 1]));
        }
      }
    }
    wave_sync();
  }
}

// Back-substitution of solveEqual (affine.cl:832-856): fma where the
// reference's FP_CONTRACT fuses, all-zero result on a zero pivot; then the
// deltas fed to scaleDeltaMvs (affine.cl:860-883).
template <int NCP>
__device__ __forceinline__ void back_substitute(const double* M, int lw, int lh, double dd[6]) {
  constexpr int N = 2 * NCP, NC = N + 1;
  double p[N];
#pragma unroll
  for (int k = 0; k < N; k++) p[k] = 0.;
  p[N - 1] = __ddiv_rn(M[(N - 1) * NC + N], M[(N - 1) * NC + N - 1]);
  bool zero = false;
#pragma unroll
  for (int i = N - 2; i >= 0; i--) {
    if (!zero) {
      const double piv = M[i * NC + i];
      if (piv == 0.) {
        zero = true;
      } else {
        double temp = 0;
#pragma unroll
        for (int j = i + 1; j < N; j++) temp = fma(M[i * NC + j], p[j], temp);
        p[i] = __ddiv_rn(__dsub_rn(M[i * NC + N], temp), piv);
      }
    }
  }
  if (zero) {
#pragma unroll
    for (int k = 0; k < N; k++) p[k] = 0.;
  }
  const double w = (double)(1 << lw), h = (double)(1 << lh);
  dd[0] = p[0];
  dd[2] = p[2];
  dd[1] = __dadd_rn(__dmul_rn(p[1], w), p[0]);  // exact scaling by a power of two
  if constexpr (NCP == 3) {
    dd[3] = __dadd_rn(__dmul_rn(p[3], w), p[2]);
    dd[4] = __dadd_rn(__dmul_rn(p[4], h), p[0]);
    dd[5] = __dadd_rn(__dmul_rn(p[5], h), p[2]);
  } else {
    dd[3] = __dadd_rn(__dmul_rn(-p[3], w), p[2]);
    dd[4] = dd[5] = 0.;
  }
}

// Which reduced value feeds matrix element e = r * (N + 1) + c (eq_element's
// mapping as a table): bits 0-6 the value index, bit 7 set on the right-hand
// side column (scaled by 8).  2 CP: elements 0..19, 3 CP: 32..73.
struct EqMap {
  uint8_t v[80];
};
constexpr uint8_t eq_map_entry(int ncp, int r, int c) {
  if (ncp == 2) {
    if (c == 4) return (uint8_t)(0x80 | (10 + r));
    const int lo = r < c ? r : c, hi = r < c ? c : r;
    return (uint8_t)(lo == 0 ? hi : lo == 1 ? 3 + hi : lo == 2 ? 5 + hi : 9);
  }
  const int tr = (r == 2 || r == 3 || r == 5) ? 1 : 0, mr = (r == 1 || r == 3) ? 1 : (r >= 4 ? 2 : 0);
  if (c == 6) return (uint8_t)(0x80 | (18 + 3 * tr + mr));
  const int tc = (c == 2 || c == 3 || c == 5) ? 1 : 0, mc = (c == 1 || c == 3) ? 1 : (c >= 4 ? 2 : 0);
  const int prod = mr == 0 ? mc : mc == 0 ? mr : (mr == 1 && mc == 1) ? 3 : (mr == 2 && mc == 2) ? 5 : 4;
  return (uint8_t)(6 * (tr + tc) + prod);
}
constexpr EqMap make_eq_map() {
  EqMap m{};
  for (int e = 0; e < 20; e++) m.v[e] = eq_map_entry(2, e / 5, e % 5);
  for (int e = 0; e < 42; e++) m.v[32 + e] = eq_map_entry(3, e / 7, e % 7);
  return m;
}
static __constant__ EqMap kEqMap = make_eq_map();

// Build, eliminate and back-substitute one CU's system with its segment; the
// segment's first lane returns the deltas.  The int64 sums convert exactly
// (|value| < 2^53); the right-hand side is scaled by 8 exactly.
template <int NCP, bool KEEP_V = false>
__device__ __forceinline__ void seg_solve(long long* V, double* M, const uint8_t* eqmap, int li,
                                          int Ls, bool act, bool coop, int lw, int lh,
                                          double dd[6]) {
  constexpr int N = 2 * NCP, NC = N + 1;
  if (act) {
    for (int e = li; e < N * NC; e += Ls) {
      const int m = eqmap[(NCP == 2 ? 0 : 32) + e];
      const double sc = (m & 0x80) ? 8.0 : 1.0;
      M[e] = (double)V[m & 0x7F] * sc;
    }
    if (!KEEP_V && coop && li < kNumMom) {  // cooperative items accumulate with atomics
      int z = 0;
      opaque(z);  // a fresh zero, not a loop-carried (spilled) constant
      reinterpret_cast<int2*>(V)[li] = make_int2(z, z);
    }
  }
  wave_sync();
  seg_eliminate<N>(M, li, Ls, act);
  if (act && li == 0) {
    back_substitute<NCP>(M, lw, lh, dd);
    // the deltas for the CU's update lanes (M is dead now)
#pragma unroll
    for (int i = 0; i < 2 * NCP; i++) M[i] = dd[i];
  }
  wave_sync();
}

// Per-CU refinement state.  `live` drops to 0 when the CU is out of frame or
// when an update leaves its CPMVs unchanged -- or returns them to the previous
// iteration's: the next CPMVs are a function of the current ones alone (the
// prediction, gradients and solve depend on nothing else), so the iterations
// after a fixed point or a period-2 cycle only repeat predictions and costs
// already seen (never strictly better) -- skipping them leaves the result
// bit-identical.
struct CuState {
  int32_t cur[6];
  int32_t prev[6];  // the CPMVs of the previous iteration (period-2 cycle test)
  int32_t best[6];
  int64_t bestCost;
  int64_t bestCostSnap;  // bestCost as of the iteration's start (read by every lane of the CU)
  int32_t satd;
  int32_t inframe;
  int32_t live;
  int32_t rate;      // calc_affine_bits of cur (set at init and by the update)
  int32_t bestSatd;  // 2-CP pass: SATD of the best CPMVs
  int32_t bestHasS;  // 2-CP pass: the best CPMVs' gradient sums are in s_bestS
  int32_t seedSkip;  // 3-CP pass: iteration 0 reuses the 2-CP winner's prediction
  int32_t pad;
};

// Work-item classes (kernels): 0 affine_me_quad -- a 64x64 quadrant, 256
// threads; 1 affine_me_ctu -- a whole 128x128 CTU, 1024 threads; 2
// affine_me_half -- ONE 128x64 or 64x128 CU, 512 threads (two workgroups per
// CU: one's single-wave solve overlaps the other's prediction), its tile
// staged over the CU's extent only (160 x 96 or 96 x 160 of the square
// storage).
// 3 affine_me_ctu2 -- ONE 128x128 CU per 512-thread workgroup, two
// vertically adjacent sub-blocks per lane, two workgroups per CU (one's
// single-wave cost and solve phases overlap the other's prediction).
// 4 / 5 affine_me_half2w / affine_me_half2h -- ONE 128x64 / 64x128 CU per
// 256-thread workgroup, two stacked sub-blocks per lane, its tile staged over
// the CU's extent (160 x 96 / 96 x 160, sized for it), four workgroups per CU.
// 6 affine_me_quad2 -- a 64x64 quadrant's CUs of 32 to 128 sub-blocks, 256
// threads, two stacked sub-blocks per lane, autonomous wave tasks only (a CU
// of 32 / 64 / 128 sub-blocks on 16 / 32 / 64 lanes, four / two / one per
// wave): every per-wave step of an iteration (MV field, cost, equation
// reduction, solve, update) covers twice the sub-blocks it does in
// affine_me_quad, which keeps the 16-sub-block CUs and the 64x64 CUs.
enum { kKindQuad = 0, kKindCtu = 1, kKindHalf = 2, kKindCtu2 = 3, kKindHalf2W = 4, kKindHalf2H = 5, kKindQuad2 = 6 };
#ifndef VAME_QUAD2_STASH
#define VAME_QUAD2_STASH 0
#endif
template <int KIND>
struct Cfg {
  static constexpr bool HALF2 = KIND == kKindHalf2W || KIND == kKindHalf2H;
  static constexpr bool QUAD = KIND == kKindQuad || KIND == kKindQuad2;  // quadrant work items
  static constexpr int REGION = QUAD ? 64 : 128;  // largest region edge
  static constexpr int THREADS = QUAD || HALF2 ? 256 : KIND == kKindCtu ? 1024 : 512;
  static constexpr int SBL = KIND == kKindCtu2 || HALF2 || KIND == kKindQuad2 ? 2 : 1;  // sub-blocks per lane (stacked vertically)
  static constexpr int MAXCU = (KIND == kKindHalf || KIND == kKindCtu2 || HALF2) ? 1 : kMaxCu;  // CU state slots (LDS)
  static constexpr int ITEMCU = QUAD ? kItemCu : MAXCU;  // CU slots per item
  static constexpr bool AUTO = QUAD;                    // holds autonomous items
  static constexpr bool COOP = KIND != kKindQuad2;      // holds cooperative items
  static constexpr int MARGIN = 16;                     // reference-tile margin (samples)
  static constexpr int TILE = REGION + 2 * MARGIN;      // tile edge (samples; the staged extent's largest)
  static constexpr int TILE_W = KIND == kKindHalf2H ? 64 + 2 * MARGIN : TILE;  // allocated tile extent
  static constexpr int TILE_H = KIND == kKindHalf2W ? 64 + 2 * MARGIN : TILE;
  // tile pitch (samples) == 8 (mod 16): the window rows of sub-blocks 4 rows
  // apart land 16 banks apart (2-way at most for the packed-pair reads)
  static constexpr int TP = (TILE_W + 7) / 16 * 16 + 8;
  static constexpr int TILE_ELEMS = TILE_H * TP + 16;
  static constexpr int NSB = THREADS * SBL;             // sub-blocks per work item (max)
  // SBL = 2: the upper sub-block's prediction parked in LDS across the lower
  // one's (held in registers: +3 % time at c4); affine_me_half2* keep it in
  // registers, so that four workgroups fit a CU's LDS (parked in LDS, three
  // per CU: 8 % slower, HISTORY.md)
  // (affine_me_quad2: in registers, VAME_QUAD2_STASH=1 parks it in LDS)
  static constexpr bool STASH = KIND == kKindQuad2 ? VAME_QUAD2_STASH != 0 : !HALF2;
};

// Value i of a sub-block's contribution to its CU's normal equations
// (affine.cl:683-707: every sample of a sub-block uses the sub-block centre
// (u, v)), from the sub-block's five sums S.
//   2 CP, iC = (gx, u gx + v gy, gy, v gx - u gy) (affine.cl:691-694): the 10
//        distinct entries A00 A01 A02 A03 A11 A12 A13 A22 A23 A33 of the
//        symmetric matrix, then b0..b3 (before the << 3);
//   3 CP (affine.cl:684-689): the moments {1,u,v,uu,uv,vv} x {xx,xy,yy}, then
//        {1,u,v} x {xe,ye}; solve_cu forms the matrix from them.
__device__ __forceinline__ long long mul64(int a, int b) { return (long long)a * (long long)b; }

template <int NCP>
__device__ __forceinline__ long long eq_value(int i, const int (&S)[5], int u, int v) {
  // monomials fit int32 (u, v <= 126); every product is one i32 x i32 -> i64
  const int xx = S[0], xy = S[1], yy = S[2], xe = S[3], ye = S[4];
  const int uu = u * u, uv = u * v, vv = v * v;
  if constexpr (NCP == 2) {
    switch (i) {
      case 0: return xx;
      case 1: return mul64(u, xx) + mul64(v, xy);
      case 2: return xy;
      case 3: return mul64(v, xx) - mul64(u, xy);
      case 4: return mul64(uu, xx) + mul64(2 * uv, xy) + mul64(vv, yy);
      case 5: return mul64(u, xy) + mul64(v, yy);
      case 6: return mul64(uv, xx) + mul64(vv - uu, xy) - mul64(uv, yy);
      case 7: return yy;
      case 8: return mul64(v, xy) - mul64(u, yy);
      case 9: return mul64(vv, xx) - mul64(2 * uv, xy) + mul64(uu, yy);
      case 10: return xe;
      case 11: return mul64(u, xe) + mul64(v, ye);
      case 12: return ye;
      default: return mul64(v, xe) - mul64(u, ye);
    }
  } else {
    const int sidx = i < 18 ? i / 6 : (i < 21 ? 3 : 4);
    const int mono = i < 18 ? i % 6 : (i - 18) % 3;
    const int m = mono == 0 ? 1 : mono == 1 ? u : mono == 2 ? v : mono == 3 ? uu : mono == 4 ? uv : vv;
    return mul64(m, S[sidx]);
  }
}

// Segment sums over aligned segments of 2^LOGS lanes (LOGS <= 6; the host packs
// every wave with CUs of one size, so the segment size is wave-uniform): the
// LAST lane of every segment ends with the segment total.  row_shr steps inside
// a 16-lane DPP row, then row_bcast:15 / row_bcast:31 across rows (GFX9 DPP);
// a segment's last lane only ever adds lanes of its own segment, so no masking
// is needed.  One v_add_u32_dpp per step.
template <int LOGS>
__device__ __forceinline__ int seg_sum_c(int v) {
  if (LOGS > 0) v += dpp32<0x111, 0xF>(v);
  if (LOGS > 1) v += dpp32<0x112, 0xF>(v);
  if (LOGS > 2) v += dpp32<0x114, 0xF>(v);
  if (LOGS > 3) v += dpp32<0x118, 0xF>(v);
  if (LOGS > 4) v += dpp32<0x142, 0xA>(v);
  if (LOGS > 5) v += dpp32<0x143, 0xC>(v);
  return v;
}

// Reduction of a CU's equations over its sub-blocks (one per lane), as a
// transposing butterfly on whole int64 values (sums of |x| < 2^44 over <= 256
// lanes: exact).  The NV values of every lane are summed over the segment
// (the CU's lanes in this wave) by halving exchanges: at a step over lane bit
// b, the lanes with bit b clear keep the first half of their values and send
// the second half to the partner lane (lane ^ 2^b), which keeps the second
// half -- so each step halves the values a lane holds and doubles the lanes
// they are summed over.  Steps run cheapest first, while the counts are
// largest: bits 3 and 2 (two bank-masked DPP add pairs), bit 5
// (v_permlane32_swap), bit 4 (v_permlane16_swap), bits 1 and 0 (selects and a
// DPP quad_perm add; in practice plain row sums, the counts being 1 by then).  After the last step every value is held, fully summed, by exactly one
// lane of the segment, which stores it (autonomous items: int64 slots) or adds
// it (cooperative items: int64 LDS atomics across waves).  Integer sums: the
// order is free.

// Lane-bit selects: lane l gets (l >> B) & 1 ? if1 : if0.  Issued as the VOP3
// v_cndmask_b32 with the constant lane mask in an SGPR pair: the VOP2 form the
// compiler picks (condition in VCC) runs ~3x slower when two follow each other
// (profiles/ubench/valu_rate.hip: 7.7 vs 2.5 SIMD cycles per instruction in
// the reductions' select-select-DPP pattern).
constexpr unsigned long long kLaneBitMask[2] = {0xAAAAAAAAAAAAAAAAull, 0xCCCCCCCCCCCCCCCCull};
template <int B>
__device__ __forceinline__ int sel_bit(int if0, int if1) {
  int r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(kLaneBitMask[B]));
  return r;
}
template <int B>
__device__ __forceinline__ long long sel_bit64(long long if0, long long if1) {
  const int lo = sel_bit<B>((int)(unsigned long long)if0, (int)(unsigned long long)if1);
  const int hi = sel_bit<B>((int)((unsigned long long)if0 >> 32), (int)((unsigned long long)if1 >> 32));
  return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// value of lane ^ 2^B for the quad bits (B < 2): DPP quad_perm
template <int B>
__device__ __forceinline__ long long partner64(long long v) {
  static_assert(B == 0 || B == 1, "quad bits only");
  constexpr int ctrl = B == 1 ? 0x4E : 0xB1;  // quad_perm [2,3,0,1] / [1,0,3,2]
  const int lo = (int)(unsigned long long)v, hi = (int)((unsigned long long)v >> 32);
  const int rl = dpp32<ctrl, 0xF>(lo), rh = dpp32<ctrl, 0xF>(hi);
  return (long long)(((unsigned long long)(unsigned)rh << 32) | (unsigned)rl);
}
// Bits 3 / 2 of the lane are bank bits of the DPP row (banks 2-3 / 1-3), so
// one exchange is two bank-masked DPP adds into the same register: the lanes
// with the bit clear get a + partner(a), the others b + partner(b) (a lane's
// DPP source reads happen before any lane writes).  Each 64-bit add is
// v_add_co / v_addc_co with DPP; the carry in VCC stays within the lanes one
// masked pair enables.  Hazard waits are explicit (the backend does not look
// inside inline asm): one s_nop 1 ahead of the block covers a DPP read of a
// register the preceding VALU instruction wrote; inside the block every DPP
// source (a's and b's halves) was written before it, so no further waits
// (round 1 waited before each of the four: c3 -1 % without them).
template <int B>
__device__ __forceinline__ long long xchg_masked64(long long a, long long b) {
  unsigned al = (unsigned)(unsigned long long)a, ah = (unsigned)((unsigned long long)a >> 32);
  const unsigned bl = (unsigned)(unsigned long long)b, bh = (unsigned)((unsigned long long)b >> 32);
  if constexpr (B == 3) {
    asm("s_nop 1\n\tv_add_co_u32_dpp %0, vcc, %0, %0 row_ror:8 row_mask:0xf bank_mask:0x3\n\t"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_ror:8 row_mask:0xf bank_mask:0x3\n\t"
        "v_add_co_u32_dpp %0, vcc, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xc\n\t"
        "v_addc_co_u32_dpp %1, vcc, %3, %3, vcc row_ror:8 row_mask:0xf bank_mask:0xc"
        : "+v"(al), "+v"(ah)
        : "v"(bl), "v"(bh)
        : "vcc");
  } else {
    static_assert(B == 2, "bank bits only");
    asm("s_nop 1\n\tv_add_co_u32_dpp %0, vcc, %0, %0 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_add_co_u32_dpp %0, vcc, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
        "v_addc_co_u32_dpp %1, vcc, %3, %3, vcc row_shr:4 row_mask:0xf bank_mask:0xa"
        : "+v"(al), "+v"(ah)
        : "v"(bl), "v"(bh)
        : "vcc");
  }
  return (long long)(((unsigned long long)ah << 32) | al);
}

constexpr int ceil_half(int m) { return (m + 1) / 2; }

// Step order for a segment of 2^LOGS lanes: bits 3 2 5 4 1 0, restricted to
// bits < LOGS -- cheapest per pair-step first, while the counts are largest:
// a bank-masked DPP step (bits 3, 2) is ~11 SIMD cycles per int64 pair, a
// permlane swap step (bits 5, 4) ~14 (v_permlane32_swap issues at ~5.3
// cycles, profiles/r01_valu_rate.txt), a quad step (bits 1, 0) ~16.  The
// counts reach 1 before bits 1 / 0, which then become plain DPP row sums.
// (Round 1 ran 5 4 3 2 1 0; this order: c2 -0.6 %, c3 -0.3 %.)
template <int LOGS>
struct Schedule {
  static constexpr int bit(int i) {
    constexpr int all[6] = {3, 2, 5, 4, 1, 0};
    int n = 0;
    for (int k = 0; k < 6; k++)
      if (all[k] < LOGS) {
        if (n == i) return all[k];
        n++;
      }
    return -1;
  }
};

// One exchange of a halving step over lane bit B: a is the value the lanes
// with bit B clear keep, b the one the others keep; returns this lane's kept
// value summed with its partner's.
template <int B>
__device__ __forceinline__ long long pair_step(long long a, long long b) {
  if constexpr (B >= 4) {
    const unsigned al = (unsigned)(unsigned long long)a, ah = (unsigned)((unsigned long long)a >> 32);
    const unsigned bl = (unsigned)(unsigned long long)b, bh = (unsigned)((unsigned long long)b >> 32);
    // bit 5: lanes 0-31 end with a summed over (l, l^32), lanes 32-63 with b
    const auto rl = B == 5 ? __builtin_amdgcn_permlane32_swap(al, bl, false, false)
                           : __builtin_amdgcn_permlane16_swap(al, bl, false, false);
    const auto rh = B == 5 ? __builtin_amdgcn_permlane32_swap(ah, bh, false, false)
                           : __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
    return (long long)(((unsigned long long)rh[0] << 32) | rl[0]) +
           (long long)(((unsigned long long)rh[1] << 32) | rl[1]);
  } else if constexpr (B == 3 || B == 2) {
    return xchg_masked64<B>(a, b);
  } else {
    return sel_bit64<B>(a, b) + partner64<B>(sel_bit64<B>(b, a));
  }
}
// Halving step over lane bit B on the first M values of x (the rest unused):
// afterwards x[0 .. ceil(M/2)) holds this lane's kept half.
template <int B, int M>
__device__ __forceinline__ void halve64(long long* x) {
  constexpr int H = (M + 1) / 2;
#pragma unroll
  for (int j = 0; j < H; j++) x[j] = pair_step<B>(x[j], j + H < M ? x[j + H] : 0);
}
// Runs the halving steps while the count is > 1.  A remaining segment bit
// after the count reached 1 becomes a plain sum (row_shr:2^B), valid in the
// lanes whose bit is set.
template <int LOGS, int STEP, int M>
__device__ __forceinline__ void butterfly64(long long* x) {
  if constexpr (STEP < LOGS) {
    constexpr int B = Schedule<LOGS>::bit(STEP);
    if constexpr (M > 1) {
      halve64<B, M>(x);
      butterfly64<LOGS, STEP + 1, ceil_half(M)>(x);
    } else {
      static_assert(B <= 2, "plain steps only on DPP row bits");
      const int lo = (int)(unsigned long long)x[0], hi = (int)((unsigned long long)x[0] >> 32);
      const int rl = dpp32<0x110 + (1 << B), 0xF>(lo), rh = dpp32<0x110 + (1 << B), 0xF>(hi);
      x[0] += (long long)(((unsigned long long)(unsigned)rh << 32) | (unsigned)rl);
      butterfly64<LOGS, STEP + 1, M>(x);
    }
  }
}

// Count left per lane after the schedule.
template <int LOGS, int M>
constexpr int final_count() {
  int m = M;
  for (int i = 0; i < LOGS; i++)
    if (m > 1) m = ceil_half(m);
  return m;
}

// Window of value indices a lane holds after the schedule: [off, off + count),
// valid below `limit` (the upper half of an odd count carries a zero pad).
template <int LOGS, int K>
__device__ __forceinline__ void held_window(int lidx, int& off, int& limit) {
  off = 0;
  limit = K;
  int m = K;
#pragma unroll
  for (int i = 0; i < LOGS; i++) {
    if (m <= 1) break;
    const int b = Schedule<LOGS>::bit(i);
    const int h = ceil_half(m);
    if ((lidx >> b) & 1) {
      off += h;
    } else {
      limit = off + h;
    }
    m = h;
  }
}

// Value i of a lane's contribution: its sub-block's, or with SBL = 2 the sum
// of its two (vertically stacked: same u, rows v[0], v[1]) -- integer sums, so
// adding before the reduction is exact.
template <int NCP, int SBL>
__device__ __forceinline__ long long lane_value(int i, const int (&S)[SBL][5], int u, const int (&v)[SBL]) {
  long long r = eq_value<NCP>(i, S[0], u, v[0]);
#pragma unroll
  for (int j = 1; j < SBL; j++) r += eq_value<NCP>(i, S[j], u, v[j]);
  return r;
}

template <int NCP, int LOGS, bool COOP, int SBL>
__device__ __forceinline__ void reduce_equations_64(const int (&S)[SBL][5], int u, const int (&v)[SBL], bool owner,
                                                    long long* dst) {
  constexpr int NV = NCP == 2 ? kNumVal2 : kNumMom;
  long long x[NV];
  {
    // the first halving step is fused with the values' generation: values
    // j and j + NV/2 are formed and exchanged at once, so at most half of them
    // are live (for the 24 3-CP moments this removed the 3-CP passes' spills;
    // for the 14 2-CP values it is neutral to -0.2 % since the bank-masked
    // steps run first)
    constexpr int H = ceil_half(NV);
    constexpr int B0 = Schedule<LOGS>::bit(0);
#pragma unroll
    for (int j = 0; j < H; j++)
      x[j] = pair_step<B0>(lane_value<NCP, SBL>(j, S, u, v), j + H < NV ? lane_value<NCP, SBL>(j + H, S, u, v) : 0);
    butterfly64<LOGS, 1, H>(x);
  }
  constexpr int CNT = final_count<LOGS, NV>();
  const int lidx = __lane_id() & ((1 << LOGS) - 1);
  int off, limit;
  held_window<LOGS, NV>(lidx, off, limit);
  // the plain steps' bits (after the count reached 1) must be set
  constexpr int kPlain = [] {
    int m = NV, mask = 0;
    for (int i = 0; i < LOGS; i++) {
      if (m > 1)
        m = ceil_half(m);
      else
        mask |= 1 << Schedule<LOGS>::bit(i);
    }
    return mask;
  }();
  const bool ok = owner && (lidx & kPlain) == kPlain;
  if (ok) {
#pragma unroll
    for (int j = 0; j < CNT; j++) {
      const int idx = off + j;
      if (idx < limit) {
        if constexpr (COOP)
          atomicAdd(reinterpret_cast<unsigned long long*>(&dst[idx]), (unsigned long long)x[j]);
        else
          dst[idx] = x[j];  // int64 slots
      }
    }
  }
}

template <int NCP, int SBL>
__device__ __forceinline__ void reduce_equations(const int (&S)[SBL][5], int u, const int (&v)[SBL], int logS,
                                                 bool owner, bool coop, long long* dst) {
  if (coop) {  // cooperative items: whole-wave segments, partial sums meet in LDS atomics
    reduce_equations_64<NCP, 6, true, SBL>(S, u, v, owner, dst);
    return;
  }
  switch (logS) {  // wave-uniform; autonomous waves hold CUs of 16, 32 or 64 sub-blocks
    case 4: reduce_equations_64<NCP, 4, false, SBL>(S, u, v, owner, dst); break;
    case 5: reduce_equations_64<NCP, 5, false, SBL>(S, u, v, owner, dst); break;
    default: reduce_equations_64<NCP, 6, false, SBL>(S, u, v, owner, dst); break;
  }
}


// The LDS of one work item (a kernel's workgroup), laid out for kernel class
// KIND (BEST: a 2-CP pass feeds a 3-CP pass, MODE 3).  A kernel entry declares
// it; the quadrant kernel's bodies for one and for two sub-blocks per lane
// share one (affine_me_quad).  Members ordered by alignment (no padding: four
// quadrant workgroups need <= 40,960 B each).
template <int KIND, bool BEST>
struct Lds {
  using C = Cfg<KIND>;
  static constexpr int SBL = C::SBL;
  static constexpr bool STASH = SBL == 2 && C::STASH;
  alignas(16) uint16_t tile[C::TILE_ELEMS];
  uint4 coef[48];
  long long val[C::MAXCU][kNumMom];
  double mat[C::MAXCU][42];  // per CU: N x (N + 1) system, N <= 6
  CuState st[C::MAXCU];
  // row 0 / row 3 of every lane's prediction (packed pairs): of its sub-block,
  // or with two stacked sub-blocks per lane (SBL = 2) the upper one's top and
  // the lower one's bottom row (their inner rows stay in the lane)
  uint2 top[C::THREADS];
  uint2 bot[C::THREADS];
  // SBL = 2: the upper sub-block's prediction, parked in LDS from its SATD to
  // the gradient step (row r of lane t at [r][t]), so the lower one's
  // prediction runs with no extra live registers
  uint2 pred[STASH ? 4 : 1][STASH ? C::THREADS : 1];
  CuSlot cu[C::ITEMCU];
  // the five gradient sums of every sub-block at its CU's best 2-CP iteration
  // (3-CP seed reuse, see the 3-CP init); SBL = 2 keeps them in p.bestS
  int bestS[5][SBL == 1 && BEST ? C::NSB : 1];
  int hdr[2];  // item header, next wave task to claim
  uint8_t eqmap[76];  // EqMap entries 0..73
};

// MODE (one kernel per launch mode, so each holds only the pass copies it
// runs): 1 = 2-CP only, 2 = 3-CP only (seeds from p.prev), 3 = 2-CP then 3-CP.
// L: the work item's LDS (Lds<KIND>, or a layout that holds it).
template <int KIND, bool PROF, int MODE, typename L>
__device__ __forceinline__ void affine_me_body(const KParams& p, L& lds) {
  constexpr bool run2 = (MODE & 1) != 0, run3 = (MODE & 2) != 0;
  using C = Cfg<KIND>;
  constexpr int REGION = C::REGION;  // instrumentation slots: 128 = the 128-class kernels
  (void)REGION;
  static_assert((C::TP * 2) % 16 == 0 && C::TILE_W % 8 == 0, "16-byte tile rows");
  constexpr int SBL = C::SBL;
  constexpr bool STASH = SBL == 2 && C::STASH;
  using Own = Lds<KIND, run2 && run3>;  // the layout this body needs: L's arrays are at least as large
  static_assert(sizeof(L::tile) >= sizeof(Own::tile) && sizeof(L::top) >= sizeof(Own::top) &&
                    sizeof(L::bestS) >= sizeof(Own::bestS) && sizeof(L::pred) >= sizeof(Own::pred) &&
                    sizeof(L::val) >= sizeof(Own::val) && sizeof(L::mat) >= sizeof(Own::mat) &&
                    sizeof(L::st) >= sizeof(Own::st) && sizeof(L::cu) >= sizeof(Own::cu),
                "LDS layout too small for this kernel class");
  uint16_t* s_tile = lds.tile;
  uint2* s_top = lds.top;
  uint2* s_bot = lds.bot;
  auto& s_bestS = lds.bestS;
  auto& s_pred = lds.pred;
  auto& s_val = lds.val;
  auto& s_mat = lds.mat;
  uint4* s_coef = lds.coef;
  uint8_t* s_eqmap = lds.eqmap;
  CuState* s_st = lds.st;
  CuSlot* s_cu = lds.cu;
  int* s_hdr = lds.hdr;
  __shared__ long long s_dup[(VAME_DUP & 4) ? kNumMom : 1];  // timing-only builds

  const int tid = threadIdx.x;
  [[maybe_unused]] const int lane = tid & 63;  // (the phase-timing macros)
  const int wv = tid >> 6;
  constexpr int ph_off = 0;  // phase-timing slots (3-CP pass: +kNumPhases)
  (void)ph_off;
  PH_DECL
  PC_DECL

  // ---- XCD-aware block -> (group, item, ctu, pair).  A group is groupPairs
  // pairs x one chunk of CTU rows (a working set of a few hundred (ctu, pair)
  // combinations that the XCDs' L2s hold: at 1080p three whole pairs, at 2160p
  // part of one); within a group the order is item-major: all (ctu, pair)
  // blocks of template item 0 first, then item 1, ...; the host lists the
  // costlier items first, so the tail is made of short workgroups.  Each
  // (pair, chunk) has cpp combination slots, a multiple of 8, so slot j runs
  // on XCD j % 8 (blocks are dealt round-robin over the 8 XCDs) for every item
  // and pair: the items of one CTU re-read its reference tile and original
  // samples from the same L2, and the host's slot -> CTU table (`order`) gives
  // each XCD a compact strip of CTUs, so neighbouring tiles' margins come from
  // that L2 too.  Padding slots exit at once.
  const int b = blockIdx.x;
  const int gsz = p.nItems * p.groupPer;
  const int grp = b / gsz, gr = b % gsz;
  const int itemIdx = gr / p.groupPer;
  const int rest = gr % p.groupPer;
  const int pairIdx = (grp / p.nChunks) * p.groupPairs + rest / p.cpp;  // (POC, refIdx) pair of this launch
  if (pairIdx >= p.nPairs) return;  // padding (uniform, before any barrier)
  const int ctu = p.order[(grp % p.nChunks) * p.cpp + rest % p.cpp];
  if (ctu < 0) return;
  const PairArgs& pa = p.pair[pairIdx];
  const Item* it = p.items + itemIdx;
  const uint16_t* __restrict__ ref = pa.ref;
  const uint16_t* __restrict__ cur = pa.cur;
  const int W = p.W, H = p.H;
  const int ctuX = (ctu % p.ctusPerRow) * kCtu, ctuY = (ctu / p.ctusPerRow) * kCtu;

  // ---- one latency round: the region origin is read with scalar loads, so
  // the reference tile's loads are in flight together with the item's
  // descriptor loads, and one barrier publishes both
  const int tx0 = ctuX + (int)it->rx - C::MARGIN, ty0 = ctuY + (int)it->ry - C::MARGIN;  // tile origin
  const bool regionOut = tx0 + C::MARGIN >= W || ty0 + C::MARGIN >= H;
  // the staged extent: the whole square tile, or (affine_me_half) the CU's
  // region + margin, a 160 x 96 or 96 x 160 part of the square storage
  const int tileW = KIND == kKindHalf ? (int)it->rw + 2 * C::MARGIN : C::TILE_W;
  const int tileH = KIND == kKindHalf ? (int)it->rh + 2 * C::MARGIN : C::TILE_H;
  const int CPR = tileW / 8;  // chunks per tile row
  const int NCH = tileH * CPR;
  constexpr int PER = (C::TILE_H * (C::TILE_W / 8) + C::THREADS - 1) / C::THREADS;
  uint4 tv[PER];
  if constexpr ((VAME_DUP & 64) != 0) {  // timing-only: one extra staging round trip
    if (!regionOut) {
#pragma unroll
      for (int j = 0; j < PER; j++) {
        const int ch = tid + j * C::THREADS;
        if (ch < NCH) {
          const int ty = ch / CPR, cx = clampi((ch % CPR) * 8 + tx0, 0, W - 8);
          tv[j] = *reinterpret_cast<const uint4*>(ref + (size_t)clampi(ty0 + ty, 0, H - 1) * W + cx);
          *reinterpret_cast<uint4*>(&s_tile[(ch / CPR) * C::TP + (ch % CPR) * 8]) = tv[j];
        }
      }
    }
    __syncthreads();
  }
  // stage the reference region (+margin) into LDS, clamp-to-edge padded, in
  // 16-byte chunks; a region wholly outside the frame (the bottom CTU row at
  // 1080p) has no in-frame CU: nothing is predicted, its tile is never read
  if (!regionOut) {
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int ch = tid + j * C::THREADS;
      if (ch < NCH) {
        const int ty = ch / CPR, cx = (ch % CPR) * 8;
        const int fy = clampi(ty0 + ty, 0, H - 1), fx = tx0 + cx;
        const uint16_t* row = ref + (size_t)fy * W;
        if (fx >= 0 && fx + 7 < W) {
          tv[j] = *reinterpret_cast<const uint4*>(row + fx);
        } else {
          unsigned a[8];
#pragma unroll
          for (int m = 0; m < 8; m++) a[m] = row[clampi(fx + m, 0, W - 1)];
          tv[j] = make_uint4(a[0] | (a[1] << 16), a[2] | (a[3] << 16), a[4] | (a[5] << 16),
                             a[6] | (a[7] << 16));
        }
      }
    }
  }
  if (tid < C::ITEMCU) s_cu[tid] = it->cu[tid];
  if (tid < 48) s_coef[tid] = reinterpret_cast<const uint4*>(&kCoefTab)[tid];
  if (tid < 76) s_eqmap[tid] = kEqMap.v[tid];
  if (tid == 0) {
    s_hdr[0] = it->coop | (it->nTasks << 16);
    s_hdr[1] = 4;  // tasks 0 .. 3: waves 0 .. 3
  }
  for (int i = tid; i < C::MAXCU * kNumMom; i += C::THREADS) (&s_val[0][0])[i] = 0;
  PH_INIT
  if (!regionOut) {
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int ch = tid + j * C::THREADS;
      if (ch < NCH) *reinterpret_cast<uint4*>(&s_tile[(ch / CPR) * C::TP + (ch % CPR) * 8]) = tv[j];
    }
  }
  __syncthreads();
  PH_START
  const int hdr = __builtin_amdgcn_readfirstlane(s_hdr[0]);
  const int nTasks = (hdr >> 16) & 0xFF;
  const bool coop = C::COOP && (!C::AUTO || (hdr & 1) != 0);
  const bool claim = C::AUTO && (hdr & 2) != 0;  // autonomous: waves claim tasks as they finish
  PH_MARK(kPhStage)
  if (!coop && wv >= nTasks) {  // wave-uniform: an autonomous wave without CUs
    PH_FLUSH
    return;
  }

  // Tasks over the one staged tile: a cooperative item's tasks one after
  // another, an autonomous wave's tasks wv, wv + 4, ... (or, claiming, wv
  // and then the next unclaimed task when it finishes).  Each task's CU slots
  // are first moved into slots 0 .. (cooperative) or the wave's own slots
  // wv * kTaskCu .. (autonomous: its CU state, moments and systems; its
  // sub-blocks use the wave's own prediction rows, so its tasks need no
  // workgroup barrier).
  const int tidItem = tid;
  for (int task = coop ? 0 : __builtin_amdgcn_readfirstlane(wv);;) {
    // the thread's ids re-derived per task (opaque): as values carried
    // around the task loop, everything computed from them was hoisted out of
    // it and held in spill slots, whose writes reached HBM
    int tidTask = tidItem;
    opaque(tidTask);
    const int tid = tidTask, lane = tid & 63, wv = tid >> 6;
    // ---- CUs of this wave, this lane's CU and sub-blocks (fixed for the task)
    const int lidx = coop ? tid : lane;
    const CuSlot t0 = s_cu[coop ? 0 : wv * kTaskCu];
    int cuB = coop ? 0 : wv * kTaskCu;
    int cuE = cuB + t0.taskCus;
    int logL = t0.taskLogL;
    cuB = __builtin_amdgcn_readfirstlane(cuB);
    cuE = __builtin_amdgcn_readfirstlane(cuE);
    logL = __builtin_amdgcn_readfirstlane(logL);
    const int logS = min(logL, 6);                       // segment = lanes of one CU in one wave
    const int nCuW = coop ? (wv == 0 ? cuE : 0) : cuE - cuB;  // lanes doing per-CU work
    const int kLane = cuB + (lidx >> logL);
    const int myCu = kLane < cuE ? kLane : -1;
    Geo g;
    g.x = g.y = g.lw = g.lh = g.w = g.h = 0;
    const int local = lidx & ((1 << logL) - 1);  // this lane's sub-block (raster order in its CU)
    int sbIdx = 0, sx = 0, sy = 0, sbCols = 1;
    bool active = false;
    if (myCu >= 0) {
      const CuSlot cs = s_cu[myCu];
      g.lw = cs.lw;
      g.lh = cs.lh;
      g.w = 1 << g.lw;
      g.h = 1 << g.lh;
      g.x = ctuX + cs.x;
      g.y = ctuY + cs.y;
      // the lane's own prediction rows: a task's CUs take consecutive lanes
      // (of the workgroup, or of the running wave), in raster order within
      // each (SBL = 2: a lane per column and pair of sub-block rows, its two
      // sub-blocks at sy and sy + 4)
      sbIdx = tid;
      sbCols = 1 << (g.lw - 2);
      sx = (local & (sbCols - 1)) << 2;
      sy = (local >> (g.lw - 2)) << (SBL == 2 ? 3 : 2);
      active = (g.x + g.w <= W) && (g.y + g.h <= H);  // affine.cl:192-193
    }
    const bool leader = myCu >= 0 && (lane & ((1 << logS) - 1)) == (1 << logS) - 1;

    // one copy of the pass per CP count and item class: ncp and coop are
    // compile-time constants in each, so the 2-CP pass carries none of the 3-CP
    // selects and branches, and each copy keeps its spills outside its loops
    auto run_pass = [&](auto ncpTag, auto coopTag, auto keepTag) {
      constexpr int ncp = decltype(ncpTag)::value;
      constexpr bool coop = decltype(coopTag)::value;
      constexpr bool keepS = decltype(keepTag)::value;  // 2-CP pass that feeds a 3-CP pass
      constexpr int ph_off = ncp == 3 ? kNumPhases : 0;
      (void)ph_off;
      constexpr int kDup = (VAME_DUP & 32) && ncp != 3 ? 0 : VAME_DUP;  // timing-only builds
      const int niter = (ncp == 3 ? 4 : 5) + p.extra;

      // ---- per-CU initial CPMVs (2 CP: zero; 3 CP: derived from the 2-CP winner)
      if (lane < nCuW) {
        int k = __lane_id();  // == lane, recomputed: not a spilled loop-carried copy
        opaque(k);
        k += cuB;
        const CuSlot cs = s_cu[k];
        CuState& st = s_st[k];
        const int cx = ctuX + cs.x, cy = ctuY + cs.y;
        int c[6] = {0, 0, 0, 0, 0, 0};
        if (ncp == 3) {
          int prev[4];
          if (run2) {
            for (int i = 0; i < 4; i++) prev[i] = st.best[i];
          } else {
            const vame_cpmvs_dev& pv =
                p.prev[cs.align][(size_t)ctu * (cs.align ? kHalfCusPerCtu : kFullCusPerCtu) + cs.outOff];
            prev[0] = pv.ltx; prev[1] = pv.lty; prev[2] = pv.rtx; prev[3] = pv.rty;
          }
          // affine.cl:81-105
          const int sh = 7 + cs.lh - cs.lw;
          int vx2 = shl(prev[0], 7) - shl(prev[3] - prev[1], sh);
          int vy2 = shl(prev[1], 7) + shl(prev[2] - prev[0], sh);
          vx2 = (vx2 + 64 - (vx2 >= 0)) >> 7;
          vy2 = (vy2 + 64 - (vy2 >= 0)) >> 7;
          int lbx = clampi(vx2, -(1 << 17), (1 << 17) - 1);
          int lby = clampi(vy2, -(1 << 17), (1 << 17) - 1);
          lbx = shl(to_quarter(lbx), 2);
          lby = shl(to_quarter(lby), 2);
          clip_mv(lbx, lby, cx, cy, W, H);
          c[0] = prev[0]; c[1] = prev[1]; c[2] = prev[2]; c[3] = prev[3]; c[4] = lbx; c[5] = lby;
          // Seed reuse (exact): when the derived LB reproduces the 2-CP motion
          // field -- (LB - LT) << (7 - log2 h) == (-(RT - LT).y, (RT - LT).x)
          // << (7 - log2 w), i.e. no rounding or clipping in the derivation
          // (always so for square CUs) -- iteration 0's MV field, spread test,
          // prediction and gradients are those of the 2-CP winner, whose SATD
          // and per-sub-block gradient sums the 2-CP pass kept.  Iteration 0
          // then only re-prices the rate and rebuilds the 6-parameter equations.
          int skip = 0, satd0 = 0;
          if (run2 && st.bestHasS) {
            const int hx = shl(prev[2] - prev[0], 7 - cs.lw), hy = shl(prev[3] - prev[1], 7 - cs.lw);
            const int vx = shl(lbx - prev[0], 7 - cs.lh), vy = shl(lby - prev[1], 7 - cs.lh);
            if (vx == -hy && vy == hx) {
              skip = 1;
              satd0 = st.bestSatd;
            }
          }
          st.seedSkip = skip;
          st.satd = satd0;
        } else {
          st.satd = 0;
          st.bestHasS = 0;
        }
        // fresh constants (opaque): as loop-carried values the compiler kept
        // them in spill slots, whose scratch traffic reached HBM
        int never = (int)0x80000000;  // outside the clamped CPMV range: never matches
        int costInit = (int)kCostInit;
        opaque(never);
        opaque(costInit);
        for (int i = 0; i < 6; i++) {
          st.cur[i] = c[i];
          st.prev[i] = never;
          st.best[i] = c[i];
        }
        st.bestCost = (long long)costInit;
        st.bestCostSnap = (long long)costInit;
        st.rate = affine_bits(c, ncp);
        st.inframe = (cx + (1 << cs.lw) <= W) && (cy + (1 << cs.lh) <= H);
        st.live = st.inframe;
      }
      phase_sync(coop);

      for (int iter = 0; iter <= niter; iter++) {
        // =============== prediction + SATD (affine.cl:208-393) ===============
        // Everything a lane produces here is only read while its CU is live
        // (the CU's lanes are uniformly live or not), so the whole step runs
        // under `live`: the DPP neighbour reads at the CU's edges may see lanes
        // of other CUs, whose columns the border replication discards.
        // this lane's prediction and original rows (packed pairs), per sub-block
        // (SBL = 2: the originals are read again in the gradient step)
        uint2 Pr[SBL][4], Og[SBL][4];
        uint4 X[6];          // extended rows 0..3 (X[1..4]) and the neighbours' edges
        const bool live = active && s_st[myCu < 0 ? 0 : myCu].live;
        // 3-CP iteration 0 of a seed-reuse CU: SATD (set at init) and gradient
        // sums come from the 2-CP pass
        const bool reuse = ncp == 3 && iter == 0 && s_st[myCu < 0 ? 0 : myCu].seedSkip;
        if (live && !reuse && !(VAME_ABLATE & 8)) {
          PC_ADD
          Geo gp = g;
          int sxp = sx, syp = sy;
          opaque_geo(gp, sxp, syp);  // recomputed per phase (not hoisted: VGPRs)
          int cp[6];
          for (int i = 0; i < 6; i++) cp[i] = s_st[myCu].cur[i];
          const MvField f = mv_field(cp, ncp, gp.lw, gp.lh);
          if constexpr ((kDup & 128) != 0) {  // timing-only: the MV field again
            int cp2[6];
            for (int i = 0; i < 6; i++) cp2[i] = cp[i];
            int lw2 = gp.lw;
            opaque(cp2[0]);
            opaque(lw2);
            const MvField f2 = mv_field(cp2, ncp, lw2, gp.lh);
            if (ncp == 3)
              asm volatile("" ::"v"(f2.bx), "v"(f2.by), "v"(f2.hx), "v"(f2.hy), "v"(f2.vx), "v"(f2.vy),
                           "v"((int)f2.spread));
            else
              asm volatile("" ::"v"(f2.bx), "v"(f2.by), "v"(f2.hx), "v"(f2.hy), "v"((int)f2.spread));
          }
          int satdLane = 0;
#pragma unroll
          for (int j = 0; j < SBL; j++) {
            bool outside;
            satdLane += predict_sb<C::TILE, C::TP, PROF, (VAME_ABLATE & 1024) != 0 && ncp == 3, ncp>(
                f, sxp, syp + 4 * j, gp, s_tile, tx0, ty0, tileW - 9, tileH - 9, ref, cur, W, H, s_coef, Pr[j],
                Og[j], outside);
            if (SBL == 2 && j == 0) {
#pragma unroll
              for (int r = 0; r < 4; r++)
                if constexpr (STASH) s_pred[r][sbIdx] = Pr[0][r];
            }
#if VAME_COUNT_PRED
            {  // instrumentation: windows outside the tile, per kernel and pass, one atomic per wave
              const unsigned long long out = __builtin_amdgcn_ballot_w64(outside);
              if (out && __lane_id() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
                atomicAdd(&g_pred_count[2 + 2 * (REGION == 128) + (ncp == 3)], (unsigned long long)__popcll(out));
            }
            if (j > 0) PC_ADD
#endif
          }
          if (kDup & 1) {
            MvField f2 = f;
            opaque(f2.bx);
            uint2 P2[4], O2[4];
            bool out2;
            int s2 = predict_sb<C::TILE, C::TP, PROF>(f2, sxp, syp, gp, s_tile, tx0, ty0, tileW - 9, tileH - 9,
                                                      ref, cur, W, H, s_coef, P2, O2, out2);
            s2 += (int)(P2[0].x ^ P2[3].y ^ O2[1].x);
            asm volatile("" ::"v"(s2));
          }
          // extended rows (neighbour columns by DPP), edge rows published for
          // the sub-blocks above and below (SBL = 2: the gradient step forms
          // the extended rows of both sub-blocks)
          if constexpr (SBL == 1) {
#pragma unroll
            for (int r = 0; r < 4; r++)
              X[r + 1] = ext_row(Pr[0][r], dpp32<0x138, 0xF>((int)Pr[0][r].y), dpp32<0x130, 0xF>((int)Pr[0][r].x));
          }
          s_top[sbIdx] = Pr[0][0];
          s_bot[sbIdx] = Pr[SBL - 1][3];
          if constexpr ((kDup & 256) != 0) {  // timing-only: the extended rows and edge stores again
            int i2 = sbIdx;
            opaque(i2);
#pragma unroll
            for (int r = 0; r < 4; r++) {
              uint2 q = Pr[0][r];
              opaque(reinterpret_cast<int&>(q.x));
              const uint4 x2 = ext_row(q, dpp32<0x138, 0xF>((int)q.y), dpp32<0x130, 0xF>((int)q.x));
              asm volatile("" ::"v"(x2.x), "v"(x2.w));
            }
            s_top[i2] = Pr[0][0];
            s_bot[i2] = Pr[SBL - 1][3];
          }
          if constexpr ((kDup & 512) != 0) {  // timing-only: the SATD segment sum again
            int s2 = satdLane;
            opaque(s2);
            const int v2 = logS == 4 ? seg_sum_c<4>(s2) : logS == 5 ? seg_sum_c<5>(s2) : seg_sum_c<6>(s2);
            asm volatile("" ::"v"(v2));
          }
          const int v = logS == 4 ? seg_sum_c<4>(satdLane)
                        : logS == 5 ? seg_sum_c<5>(satdLane) : seg_sum_c<6>(satdLane);
          if (leader) {
            if (coop)
              atomicAdd(&s_st[myCu].satd, v);
            else
              s_st[myCu].satd = v;
          }
        }
        phase_sync(coop);
        PH_MARK(kPhPredict)

        // =============== cost, best update (affine.cl:416-457) ===============
        // The cost is the SATD sum plus floor(lambda * (bits + 2)), the rate
        // bits of the current CPMVs (calc_affine_bits, aux_functions.cl:2140-
        // 2189) kept in CuState by the update step; the strict best is kept.
        const bool lastIter = iter == niter;
        bool better = false;  // keepS: this lane's CU improved
        if constexpr ((kDup & 1024) != 0) {  // timing-only: the pricing again (before the real one)
          int bet2 = 0;
          if (myCu >= 0 && (keepS || local == 7)) {
            const CuState& st = s_st[myCu];
            int r2 = st.rate;
            opaque(r2);
            if (iter == 0 || st.live) {
              const float prod = __fmul_rn(pa.lambda, (float)(r2 + kRuiBits));
              const long long cost = (long long)st.satd + (long long)(int)floorf(prod);
              bet2 = cost < st.bestCost;
            }
          }
          if (!keepS) bet2 = __builtin_amdgcn_update_dpp(0, bet2, 0x157, 0xF, 0xF, false);
          asm volatile("" ::"v"(bet2));
        }
        if constexpr (!keepS) {
          // the CU's lane 7 prices and keeps the best; lanes 0-5 copy the CPMVs
          int bet = 0;
          if (myCu >= 0 && local == 7) {
            CuState& st = s_st[myCu];
            if (iter == 0 || st.live) {
              const float prod = __fmul_rn(pa.lambda, (float)(st.rate + kRuiBits));
              const long long cost = (long long)st.satd + (long long)(int)floorf(prod);
              if (cost < st.bestCost) {
                st.bestCost = cost;
                bet = 1;
              }
            }
            st.satd = 0;
          }
          bet = __builtin_amdgcn_update_dpp(0, bet, 0x157, 0xF, 0xF, false);  // row_newbcast:7
          if (myCu >= 0 && local < 6 && bet) s_st[myCu].best[local] = s_st[myCu].cur[local];
        } else {
          // 2-CP pass followed by a 3-CP pass: every lane of the CU prices it, so
          // each knows whether its CU improved and keeps its gradient sums for
          // the 3-CP seed reuse.  The comparison is against the best cost as of
          // the iteration's start: autonomous items read bestCost (the CU's
          // lanes are one wave, whose LDS reads precede lane 7's write);
          // cooperative items read bestCostSnap, refreshed in the solve phase.
          if (myCu >= 0) {
            CuState& st = s_st[myCu];
            if (iter == 0 || st.live) {
              const float prod = __fmul_rn(pa.lambda, (float)(st.rate + kRuiBits));
              const long long cost = (long long)st.satd + (long long)(int)floorf(prod);
              better = cost < (coop ? st.bestCostSnap : st.bestCost);
              if (better && local == 7) {
                st.bestCost = cost;
                st.bestSatd = st.satd;
                st.bestHasS = !lastIter && st.live;  // its gradient sums follow in this iteration
              }
            }
            if (local < 6 && better) st.best[local] = st.cur[local];
          }
        }
        PH_MARK(kPhCost)
        if (lastIter) {  // uniform; the results below are written by other lanes
          phase_sync(coop);
          break;
        }

        // =============== gradients + normal equations (affine.cl:477-752) ===============
        {
          int S[SBL][5];
#pragma unroll
          for (int j = 0; j < SBL; j++)
#pragma unroll
            for (int k = 0; k < 5; k++) S[j][k] = 0;
          // SBL = 2: the seed-reuse sums in global memory, per (pair, CTU): a
          // uniform base and 32-bit lane offsets (recomputed, not hoisted)
          char* gBest = SBL == 2 ? reinterpret_cast<char*>(p.bestS + ((size_t)(pairIdx * p.nCtus + ctu) * p.nItems +
                                                                      itemIdx) * 5 * C::NSB)
                                 : nullptr;
          auto gbest = [&](int k, int j) -> int32_t& {
            int i = sbIdx;
            opaque(i);
            return *reinterpret_cast<int32_t*>(gBest + (unsigned)(k * C::NSB + j * C::THREADS + i) * 4u);
          };
          if (reuse && live) {
#pragma unroll
            for (int j = 0; j < SBL; j++)
#pragma unroll
              for (int k = 0; k < 5; k++) S[j][k] = SBL == 1 ? s_bestS[k][sbIdx] : gbest(k, j);
          } else if (live && !(VAME_ABLATE & 2)) {
            // the neighbours' edge rows, extended by the left / right lanes' copies
            // the sub-blocks above / below, computed here (kept live across the
            // passes, the index was spilled)
            int nbIdx = sbIdx;
            if constexpr (SBL == 2) opaque(nbIdx);  // recomputed, not hoisted (VGPRs)
            const uint2 tb = s_bot[max(nbIdx - sbCols, 0)], bt = s_top[min(nbIdx + sbCols, C::THREADS - 1)];
            X[0] = ext_row(tb, dpp32<0x138, 0xF>((int)tb.y), dpp32<0x130, 0xF>((int)tb.x));
            if constexpr ((kDup & 256) != 0) {  // timing-only: the neighbours' edge rows again
              int n2 = nbIdx;
              opaque(n2);
              const uint2 tb2 = s_bot[max(n2 - sbCols, 0)], bt2 = s_top[min(n2 + sbCols, C::THREADS - 1)];
              const uint4 a2 = ext_row(tb2, dpp32<0x138, 0xF>((int)tb2.y), dpp32<0x130, 0xF>((int)tb2.x));
              const uint4 b2 = ext_row(bt2, dpp32<0x138, 0xF>((int)bt2.y), dpp32<0x130, 0xF>((int)bt2.x));
              asm volatile("" ::"v"(a2.x), "v"(a2.w), "v"(b2.x), "v"(b2.w));
            }
            Geo gg = g;
            int sxg = sx, syg = sy;
            if constexpr (SBL == 2) opaque_geo(gg, sxg, syg);
            if constexpr (SBL == 1) {
              X[5] = ext_row(bt, dpp32<0x138, 0xF>((int)bt.y), dpp32<0x130, 0xF>((int)bt.x));
              grad_sb(sxg, syg, gg, X, Og[0], S[0]);
            } else {
              // upper sub-block: rows X[1..4] its own, X[5] the lower one's top row;
              // lower sub-block: X[0] the upper one's bottom row, X[5] the lane
              // below's; the original rows read again (the frame base + 32-bit offsets)
#pragma unroll
              for (int j = 0; j < SBL; j++) {
                if (STASH && j == 0) {
#pragma unroll
                  for (int r = 0; r < 4; r++) Pr[0][r] = s_pred[r][sbIdx];
                }
#pragma unroll
                for (int r = 0; r < 4; r++)
                  X[r + 1] = ext_row(Pr[j][r], dpp32<0x138, 0xF>((int)Pr[j][r].y),
                                     dpp32<0x130, 0xF>((int)Pr[j][r].x));
                const uint2 nb = j + 1 < SBL ? Pr[j + 1][0] : bt;
                X[5] = ext_row(nb, dpp32<0x138, 0xF>((int)nb.y), dpp32<0x130, 0xF>((int)nb.x));
                {
                  const unsigned b0 = (unsigned)((gg.y + syg + 4 * j) * W + gg.x + sxg) * 2u, bw = (unsigned)W * 2u;
                  const char* base = reinterpret_cast<const char*>(cur);
#pragma unroll
                  for (int r = 0; r < 4; r++) Og[j][r] = *reinterpret_cast<const uint2*>(base + (b0 + (unsigned)r * bw));
                }
                grad_sb(sxg, syg + 4 * j, gg, X, Og[j], S[j]);
                if (j + 1 < SBL) X[0] = X[4];  // the lower sub-block's row above = the upper one's row 3
              }
            }
            if (kDup & 2) {
              int S2[5];
              int sxd = sxg;
              opaque(sxd);
              grad_sb(sxd, syg, gg, X, Og[0], S2);
              asm volatile("" ::"v"(S2[0] ^ S2[1] ^ S2[2] ^ S2[3] ^ S2[4]));
            }
            if (keepS && better && !(SBL == 2 && (VAME_ABLATE & 2048))) {  // the best iteration's sums, for the 3-CP seed reuse
#pragma unroll
              for (int j = 0; j < SBL; j++)
#pragma unroll
                for (int k = 0; k < 5; k++) {
                  if constexpr (SBL == 1)
                    s_bestS[k][sbIdx] = S[j][k];
                  else
                    gbest(k, j) = S[j][k];
                }
            }
          }
          PH_MARK(kPhGradient)
          if (!(VAME_ABLATE & 4)) {
            long long* dst = s_val[myCu < 0 ? 0 : myCu];
            int va[SBL];
#pragma unroll
            for (int j = 0; j < SBL; j++) va[j] = sy + 2 + 4 * j;
            if (ncp == 2)
              reduce_equations<2, SBL>(S, sx + 2, va, logS, myCu >= 0, coop, dst);
            else
              reduce_equations<3, SBL>(S, sx + 2, va, logS, myCu >= 0, coop, dst);
            if constexpr ((kDup & 4) != 0) {
              int ud = sx + 2;
              opaque(ud);
              if (ncp == 2)
                reduce_equations<2, SBL>(S, ud, va, logS, myCu >= 0, coop, s_dup);
              else
                reduce_equations<3, SBL>(S, ud, va, logS, myCu >= 0, coop, s_dup);
            }
          }
        }
        phase_sync(coop);
        PH_MARK(kPhReduce)

        // =============== solve + CPMV update (affine.cl:782-893), per CU segment ===============
        __builtin_amdgcn_s_setprio(kSolvePrio);
        if (!(VAME_ABLATE & 1)) {
          // the CU's lanes in its first wave solve it together
          int cuS = myCu, loc = local;
          opaque(cuS);  // recomputed, not loop-carried (VGPRs)
          opaque(loc);
          const bool solver = cuS >= 0 && loc < 64;
          const bool act = solver && s_st[cuS].live;
          const int Ls = 1 << logS;
          double dd[6] = {0, 0, 0, 0, 0, 0};
          long long* V = s_val[cuS < 0 ? 0 : cuS];
          double* M = s_mat[cuS < 0 ? 0 : cuS];
          const CuSlot cs = s_cu[cuS < 0 ? 0 : cuS];
          if constexpr ((kDup & 16) != 0) {  // timing-only: a throw-away solve first
            // on M itself, keeping V: the real solve below rebuilds M from V (no
            // extra LDS, so the occupancy is the product build's)
            double dd2[6] = {0, 0, 0, 0, 0, 0};
            double* M2 = M;
            if (ncp == 3)
              seg_solve<3, true>(V, M2, s_eqmap, loc, Ls, act, coop, cs.lw, cs.lh, dd2);
            else
              seg_solve<2, true>(V, M2, s_eqmap, loc, Ls, act, coop, cs.lw, cs.lh, dd2);
            asm volatile("" ::"v"(dd2[0]), "v"(dd2[1]), "v"(dd2[3]));
            wave_sync();
          }
          if (ncp == 3)
            seg_solve<3>(V, M, s_eqmap, loc, Ls, act, coop, cs.lw, cs.lh, dd);
          else
            seg_solve<2>(V, M, s_eqmap, loc, Ls, act, coop, cs.lw, cs.lh, dd);
          // affine.cl:860-893, one CPMV component per lane: lane j < 6 of the
          // CU applies scaleDeltaMvs to its delta (LT=(d0,d2), RT=(d1,d3),
          // LB=(d4,d5)), clampCpmvs and clipCpmvs, and the CU's lane 7 sums
          // the moved / cycle flags (DPP) into the CU's `live`
          if (keepS && coop && solver && loc == 7) {  // the next cost phase's view; fresh SATD sums
            CuState& st = s_st[cuS];
            st.bestCostSnap = st.bestCost;
            st.satd = 0;
          }
          bool liveNew = false;
          if constexpr ((kDup & 2048) != 0) {  // timing-only: the update again, without its stores
            if (act && loc < 8) {
              const CuState& st = s_st[cuS];
              int f = 0, q = 0;
              if (loc < 2 * ncp) {
                int j = loc;
                opaque(j);
                const double d = M[j == 1 ? 2 : j == 2 ? 1 : j];
                const int cj = st.cur[j], pj = st.prev[j];
                int v = (int)((unsigned)cj + (unsigned)scale_delta(d));
                v = clampi(v, kMvMin, kMvMax);
                const int pos = (j & 1) ? ctuY + cs.y : ctuX + cs.x, lim = (j & 1) ? H : W;
                v = clampi(v, shl(-128 - 8 - pos + 1, 4), shl(lim + 8 - pos - 1, 4));
                f = (v != cj ? 1 : 0) | (v != pj ? 16 : 0);
                q = to_quarter(v);
              }
              const int q2 = dpp32<0x112, 0xF>(q), q4 = dpp32<0x114, 0xF>(q);
              if (loc < 2 * ncp) f += eg_bits(q - (loc >= 4 ? q4 : loc >= 2 ? q2 : 0)) << 8;
              f += dpp32<0x111, 0xF>(f);
              f += dpp32<0x112, 0xF>(f);
              f += dpp32<0x114, 0xF>(f);
              asm volatile("" ::"v"(f));
            }
          }
          if (act && loc < 8) {
            CuState& st = s_st[cuS];
            int f = 0, q = 0;
            if (loc < 2 * ncp) {  // 2 CP: LB stays (0, 0)
              const int j = loc;
              const double d = M[j == 1 ? 2 : j == 2 ? 1 : j];
              const int cj = st.cur[j], pj = st.prev[j];
              int v = (int)((unsigned)cj + (unsigned)scale_delta(d));
              v = clampi(v, kMvMin, kMvMax);
              const int pos = (j & 1) ? ctuY + cs.y : ctuX + cs.x, lim = (j & 1) ? H : W;
              v = clampi(v, shl(-128 - 8 - pos + 1, 4), shl(lim + 8 - pos - 1, 4));  // clipMv
              f = (v != cj ? 1 : 0) | (v != pj ? 16 : 0);
              st.prev[j] = cj;
              st.cur[j] = v;
              q = to_quarter(v);
            }
            // the rate of the new CPMVs (calc_affine_bits, aux_functions.cl:2140-2189)
            // rides on the same lane sum: component j codes q_j - q_(j & 1) for
            // j >= 2 (RT - LT from lane j - 2, LB - LT from lane j - 4)
            {
              const int q2 = dpp32<0x112, 0xF>(q), q4 = dpp32<0x114, 0xF>(q);
              if (loc < 2 * ncp) f += eg_bits(q - (loc >= 4 ? q4 : loc >= 2 ? q2 : 0)) << 8;
            }
            f += dpp32<0x111, 0xF>(f);  // row_shr:1, 2, 4: lane 7 sums lanes 0..7
            f += dpp32<0x112, 0xF>(f);
            f += dpp32<0x114, 0xF>(f);
            if (loc == 7) {
              // moved, and not back to the previous (flag fields: bits 0-3 and 4-7)
              liveNew = (f & 15) != 0 && ((f >> 4) & 15) != 0;
              st.live = liveNew;
              st.rate = f >> 8;
            }
          }
          if (!coop) {  // leave once every CU of this wave is settled (wave-local)
            if (__ballot(liveNew) == 0) {
              __builtin_amdgcn_s_setprio(0);
              break;
            }
          }
        }
        __builtin_amdgcn_s_setprio(0);
        phase_sync(coop);
        PH_MARK(kPhSolve)
        if (coop) {  // leave once every CU of the item is settled (flags read after the sync)
          bool anyLive = false;
          for (int k = cuB; k < cuE; k++) anyLive |= s_st[k].live != 0;
          if (!anyLive) break;
        }
      }
      // =============== results (affine.cl:928-957) ===============
      if (lane < nCuW) {
        int k = __lane_id();  // == lane, recomputed: not a spilled loop-carried copy
        opaque(k);
        k += cuB;
        const CuState& st = s_st[k];
        const CuSlot cs = s_cu[k];
        const int mode = cs.align * 2 + (ncp - 2);
        const size_t idx = (size_t)ctu * (cs.align ? kHalfCusPerCtu : kFullCusPerCtu) + cs.outOff;
        pa.cost[mode][idx] = st.bestCost;
        vame_cpmvs_dev o;
        o.ncps = ncp;
        o.ltx = st.best[0]; o.lty = st.best[1]; o.rtx = st.best[2];
        o.rty = st.best[3]; o.lbx = st.best[4]; o.lby = st.best[5];
        pa.cpmv[mode][idx] = o;
      }
      phase_sync(coop);
      PH_MARK(kPhTail)
    };
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using T = std::true_type;
    using F = std::false_type;
    // keepS: the 2-CP pass feeds a 3-CP pass (seed reuse)
    using KeepS = std::integral_constant<bool, run3>;
    if (C::COOP && coop) {
      if constexpr (C::COOP) {
        if constexpr (run2) run_pass(I2{}, T{}, KeepS{});
        if constexpr (run3) run_pass(I3{}, T{}, F{});
      }
    } else {
      if constexpr (run2) run_pass(I2{}, F{}, KeepS{});
      if constexpr (run3) run_pass(I3{}, F{}, F{});
    }
    if (!C::QUAD) break;  // 128-class items: one task
    // the next task's CU slots into this task's (cooperative: after every wave's
    // last read of them, autonomous: the wave's own, read by this wave only)
    int next = task + (coop ? 1 : 4);
    if (claim) {
      int v = 0;
      if (lane == 0) v = atomicAdd(&s_hdr[1], 1);
      next = __builtin_amdgcn_readfirstlane(v);
    }
    if (next >= nTasks) break;
    if (coop) {
      if (tid < kTaskCu) s_cu[tid] = s_cu[min(next, C::ITEMCU / kTaskCu - 1) * kTaskCu + tid];
      __syncthreads();
    } else {
      if (lane < kTaskCu) s_cu[wv * kTaskCu + lane] = s_cu[min(next, C::ITEMCU / kTaskCu - 1) * kTaskCu + lane];
      wave_sync();
    }
    task = next;
  }
  PH_FLUSH
  PC_FLUSH
}

// Distinct entry points so profiles tell the work-item classes apart.
// Quadrant items: 4 workgroups per CU fit the LDS (~36-41 KB each), so cap the
// VGPRs at 128 to let all 16 waves be resident.  An item flagged SBL2 (Item
// coop bit 2: the CUs of 32-128 sub-blocks) runs the body with two stacked
// sub-blocks per lane, the others (16-sub-block and 64x64 CUs) with one; both
// bodies share the workgroup's LDS (one Lds<kKindQuad, ...>).
__device__ __forceinline__ bool quad_item_sbl2(const KParams& p) {
  const int b = blockIdx.x;
  const int gr = b % (p.nItems * p.groupPer);
  return (p.items[gr / p.groupPer].coop & 4) != 0;
}
//
// Which launch modes hand affine_me_quad SBL2 items (engine, VAME_SPLIT): by
// default only the 2-CP-only launches; in the others the SBL2 items go to
// affine_me_quad2 and affine_me_quad is built without the two-sub-block body,
// whose registers would otherwise spill into the one-sub-block body too
// (104 vs 0 B per lane in MODE 3).  Timing builds: 2 every mode, 1 / 0 none.
#ifndef VAME_SPLIT
#define VAME_SPLIT 3
#endif
template <int MODE>
constexpr bool kQuadMerged = VAME_SPLIT == 2 || (VAME_SPLIT == 3 && MODE == 1);
template <int MODE>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_quad(
    KParams p) {
  __shared__ Lds<kKindQuad, MODE == 3> lds;
  if constexpr (kQuadMerged<MODE>) {
    if (quad_item_sbl2(p)) {
      affine_me_body<kKindQuad2, false, MODE>(p, lds);
      return;
    }
  }
  affine_me_body<kKindQuad, false, MODE>(p, lds);
}
// Timing builds (VAME_SPLIT=1): the SBL2 items as a kernel of their own.
template <int MODE>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_quad2(
    KParams p) {
  __shared__ Lds<kKindQuad2, MODE == 3> lds;
  affine_me_body<kKindQuad2, false, MODE>(p, lds);
}
// ONE 128x128 CU per 512-thread workgroup, two stacked sub-blocks per lane,
// two workgroups per CU (~72 KB of LDS each; the 3-CP seed-reuse sums in
// global memory): 128 VGPRs so both fit.
template <int MODE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_ctu2(KParams p) {
  __shared__ Lds<kKindCtu2, MODE == 3> lds;
  affine_me_body<kKindCtu2, false, MODE>(p, lds);
}
// ONE 128x64 (w) / 64x128 (h) CU per 256-thread workgroup, two stacked
// sub-blocks per lane, four workgroups per CU (~40 KB of LDS each).
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_half2w(KParams p) {
  __shared__ Lds<kKindHalf2W, MODE == 3> lds;
  affine_me_body<kKindHalf2W, false, MODE>(p, lds);
}
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_half2h(KParams p) {
  __shared__ Lds<kKindHalf2H, MODE == 3> lds;
  affine_me_body<kKindHalf2H, false, MODE>(p, lds);
}
// Both orientations in one launch (an item's region width tells which), so
// the 128x64 and 64x128 CUs run side by side instead of one kernel after the
// other on the stream; the 64x128 layout's LDS holds the 128x64 one's.
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_half2(KParams p) {
  __shared__ Lds<kKindHalf2H, MODE == 3> lds;
  const int gr = blockIdx.x % (p.nItems * p.groupPer);
  const Item& it = p.items[gr / p.groupPer];
  if (it.rw > it.rh)
    affine_me_body<kKindHalf2W, false, MODE>(p, lds);
  else
    affine_me_body<kKindHalf2H, false, MODE>(p, lds);
}
// The same with PROF (vame_set_prof): the quadrant items (one sub-block per
// lane, every quadrant CU); the 128x128 CU in one 1024-thread workgroup per
// CU (~100 KB of LDS), one lane per sub-block; each 128x64 / 64x128 CU in a
// 512-thread workgroup, two per CU (~74 KB of LDS each).
template <int MODE>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_quad_prof(
    KParams p) {
  __shared__ Lds<kKindQuad, MODE == 3> lds;
  affine_me_body<kKindQuad, true, MODE>(p, lds);
}
template <int MODE>
__global__ __launch_bounds__(1024) void affine_me_ctu_prof(KParams p) {
  __shared__ Lds<kKindCtu, MODE == 3> lds;
  affine_me_body<kKindCtu, true, MODE>(p, lds);
}
template <int MODE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void affine_me_half_prof(KParams p) {
  __shared__ Lds<kKindHalf, MODE == 3> lds;
  affine_me_body<kKindHalf, true, MODE>(p, lds);
}

// The 2-CP-only (MODE 1) product kernels are compiled in a translation unit of
// their own, vame_kernels_2cp.hip, whose optimisation flags suit them (the
// Makefile); the engine's unit declares them instead of
// instantiating them.  Instrumentation builds keep every kernel in one unit:
// their device counters are per unit.
#if VAME_COUNT_PRED || VAME_PHASE_TIMING
#define VAME_SPLIT_TU 0
#else
#define VAME_SPLIT_TU 1
#endif
#define VAME_2CP_KERNELS(X)                 \
  X template __global__ void affine_me_quad<1>(KParams);   \
  X template __global__ void affine_me_quad2<1>(KParams);  \
  X template __global__ void affine_me_ctu2<1>(KParams);   \
  X template __global__ void affine_me_half2<1>(KParams);  \
  X template __global__ void affine_me_half2w<1>(KParams); \
  X template __global__ void affine_me_half2h<1>(KParams);

}  // namespace vame
