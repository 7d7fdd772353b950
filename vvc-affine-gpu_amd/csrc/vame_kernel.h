// vame_kernel.h -- HIP/CDNA4 device code of the affine-ME hot path.
//
// One workgroup (256 threads) = one work item: a 64x64 quadrant (or, for the
// 128-wide/high aligned sizes, the whole 128x128 CTU) of one CTU, for one
// reference frame, holding the candidate CUs of one or more CU-size groups.
// The workgroup runs the complete gradient-based CPMV refinement of
// affine.cl:195-917 for all of them -- 2 control points, then 3 control
// points seeded from the 2-CP winner of the same CU (affine.cl:81-105) --
// without leaving the CU:
//   * the reference frame region (+16 px margin, clamp-to-edge padded) is
//     staged once into LDS; every 9x9 filter window of every iteration is read
//     from there (windows outside the tile fall back to clamped global loads);
//   * predictions live in a per-CU-compact LDS buffer; gradients are computed
//     on the fly from it (no global gradient / equation scratch);
//   * the normal equations are reduced as 24 exact integer moments per CU
//     (wave butterflies + LDS int64 atomics) and solved by one lane per CU
//     with the reference's double-precision elimination, operation for
//     operation.
// Bit-exactness notes (SURVEY.md §8a traps): integer math is exact and
// order-free; the only float work is floor(lambda*bits) (single precision)
// and the FP64 solve (compiled with -ffp-contract=off, explicit fma where the
// reference's FP_CONTRACT=ON fuses, affine.cl:851); (int)double follows
// v_cvt_i32_f64 (NaN -> 0, saturate) explicitly.
#pragma once
#include <hip/hip_runtime.h>

#include "vame_tables.h"

namespace vame {

constexpr int kMaxCu = 32;   // CU slots per work item
constexpr int kMargin = 16;  // LDS reference-tile margin around the work-item region
constexpr int kThreads = 256;
constexpr int kNumMom = 24;  // {1,u,v,uu,uv,vv} x {xx,xy,yy} + {1,u,v} x {xe,ye}

// device view of vame_cpmvs / typedef.h Cpmvs (28 bytes)
struct vame_cpmvs_dev {
  int32_t ncps, ltx, lty, rtx, rty, lbx, lby;
};

struct CuSlot {     // 16 bytes
  int16_t x, y;     // CTU-relative position
  uint8_t lw, lh;   // log2 width / height
  uint8_t align;    // 0 FULL, 1 HALF
  uint8_t pad0;
  int16_t outOff;   // RETURN_STRIDE[group] + cuIdx
  int16_t sbBase;   // first sub-block (lane-major) of this CU inside the item
  int32_t pad1;
};

struct Item {
  int16_t nCu, nSb;  // CU slots, sub-blocks
  int16_t rx, ry;    // region origin (CTU-relative)
  CuSlot cu[kMaxCu];
};

struct KParams {
  const uint16_t* cur;
  const uint16_t* refs[4];
  int64_t* cost[4][4];        // [ref][FULL_2CP, FULL_3CP, HALF_2CP, HALF_3CP]
  vame_cpmvs_dev* cpmv[4][4];
  const vame_cpmvs_dev* prev[2];  // [align]: 3-CP seeds when the 2-CP pass is not run
  const Item* items;
  int nItems, nCtus, nRefs;
  int W, H, ctusPerRow;
  float lambda;
  int extra;
  int run2, run3;
};

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }
__device__ __forceinline__ int shl(int a, int s) { return (int)((unsigned)a << s); }

// aux_functions.cl:51-67 clipMv
__device__ __forceinline__ void clip_mv(int& x, int& y, int bx, int by, int W, int H) {
  x = clampi(x, shl(-128 - 8 - bx + 1, 4), shl(W + 8 - bx - 1, 4));
  y = clampi(y, shl(-128 - 8 - by + 1, 4), shl(H + 8 - by - 1, 4));
}

// aux_functions.cl:106-141 (bipred == 0)
__device__ __forceinline__ bool spread_over_limit(int a, int b, int c, int d) {
  const int s4 = 4 << 11;
  int w = (abs(4 * a + s4) >> 11) + 9, h = (abs(4 * b) >> 11) + 9;
  if (w * h > 165) return true;
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

__device__ __forceinline__ int cvt_i32_f64(double d) {  // v_cvt_i32_f64 semantics
  if (d != d) return 0;
  if (d >= 2147483647.0) return 2147483647;
  if (d <= -2147483648.0) return (int)0x80000000u;
  return (int)d;
}

// aux_functions.cl:2194-2215
__device__ __forceinline__ int scale_delta(double d) {
  double s = d >= 0 ? 1.0 : -1.0;
  return shl(cvt_i32_f64(d * 4.0 + s * 0.5), 2);
}

// segmented all-reduce over power-of-two lane groups of size S (<= 64); must be
// called by every lane of the wave (uniform control flow)
__device__ __forceinline__ long long seg_sum64(long long v, int S) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    long long o = __shfl_xor(v, d);
    if (d < S) v += o;
  }
  return v;
}
__device__ __forceinline__ int seg_sum32(int v, int S) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int o = __shfl_xor(v, d);
    if (d < S) v += o;
  }
  return v;
}

__device__ __forceinline__ void luma_coeffs(int frac, int* c) {
#pragma unroll
  for (int m = 0; m < 6; m++) c[m] = kLuma6[frac][m];
}

// affine.cl:782-856 (VTM solveEqual), same operation order as the reference.
__device__ void solve_equal(double (&a)[7][7], int n, double* p) {
  for (int k = 0; k < 6; k++) p[k] = 0.;
  for (int i = 1; i < n; i++) {
    double temp = fabs(a[i][i - 1]);
    int tempIdx = i;
    for (int j = i + 1; j < n + 1; j++) {
      if (fabs(a[j][i - 1]) > temp) {
        temp = fabs(a[j][i - 1]);
        tempIdx = j;
      }
    }
    if (tempIdx != i) {
      for (int j = 0; j < n + 1; j++) {
        a[0][j] = a[i][j];
        a[i][j] = a[tempIdx][j];
        a[tempIdx][j] = a[0][j];
      }
    }
    for (int j = i + 1; j < n + 1; j++)
      for (int k = i; k < n + 1; k++) {
        double num = __dmul_rn(a[i][k], a[j][i - 1]);
        double q = __ddiv_rn(num, a[i][i - 1]);
        a[j][k] = __dsub_rn(a[j][k], q);
      }
  }
  p[n - 1] = __ddiv_rn(a[n][n], a[n][n - 1]);
  for (int i = n - 2; i >= 0; i--) {
    if (a[i + 1][i] == 0.) {
      for (int k = 0; k < n; k++) p[k] = 0.;
      break;
    }
    double temp = 0;
    for (int j = i + 1; j < n; j++) temp = fma(a[i + 1][j], p[j], temp);  // FP_CONTRACT
    p[i] = __ddiv_rn(__dsub_rn(a[i + 1][n], temp), a[i + 1][i]);
  }
}

// Linear forms of the equation regressors in (1, u, v): iC_c = alpha_c . gx + beta_c . gy
// 2 CP (affine.cl:691-694): gx, u gx + v gy, gy, v gx - u gy
// 3 CP (affine.cl:684-689): gx, u gx, gy, u gy, v gx, v gy
__constant__ int8_t kAlpha2[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 0}, {0, 0, 1}};
__constant__ int8_t kBeta2[4][3] = {{0, 0, 0}, {0, 0, 1}, {1, 0, 0}, {0, -1, 0}};
__constant__ int8_t kAlpha3[6][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1}, {0, 0, 0}};
__constant__ int8_t kBeta3[6][3] = {{0, 0, 0}, {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 0}, {0, 0, 1}};

// product of two linear forms in (1,u,v) -> moment index {1,u,v,uu,uv,vv} weighted sum
__device__ __forceinline__ long long quad_form(const int8_t* p, const int8_t* q, const long long* m) {
  long long r = 0;
  r += (long long)(p[0] * q[0]) * m[0];
  r += (long long)(p[0] * q[1] + p[1] * q[0]) * m[1];
  r += (long long)(p[0] * q[2] + p[2] * q[0]) * m[2];
  r += (long long)(p[1] * q[1]) * m[3];
  r += (long long)(p[1] * q[2] + p[2] * q[1]) * m[4];
  r += (long long)(p[2] * q[2]) * m[5];
  return r;
}

struct CuState {  // 64 bytes
  int32_t cur[6];
  int32_t best[6];
  int64_t bestCost;
  uint32_t satd;
  int32_t inframe;
  int32_t pad[2];
};

template <int REGION>
struct Cfg {
  static constexpr int SBPL = REGION == 128 ? 4 : 1;        // sub-blocks per lane
  static constexpr int TILE = REGION + 2 * kMargin;         // tile edge (samples)
  static constexpr int TP = REGION == 128 ? 176 : 112;      // tile pitch, == 16 (mod 32)
  static constexpr int TILE_ELEMS = TILE * TP + 16;
};

template <int REGION>
__global__ __launch_bounds__(kThreads) void affine_me_kernel(KParams p) {
  using C = Cfg<REGION>;
  __shared__ __attribute__((aligned(16))) uint16_t s_tile[C::TILE_ELEMS];
  __shared__ __attribute__((aligned(16))) uint16_t s_pred[REGION * REGION];
  __shared__ __attribute__((aligned(16))) long long s_mom[kMaxCu][kNumMom];
  __shared__ CuState s_st[kMaxCu];
  __shared__ CuSlot s_cu[kMaxCu];
  __shared__ int s_hdr[4];

  const int tid = threadIdx.x;
  const int lane = tid & 63;

  // ---- XCD-aware block -> (ref, ctu, item): blocks b, b+8, ... share an XCD;
  // give each XCD a contiguous run of logical work (same CTUs -> L2 reuse).
  const int nb = gridDim.x, b = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = b & 7;
  const int logical = xcd * q8 + min(xcd, r8) + (b >> 3);
  const int itemIdx = logical % p.nItems;
  const int rest = logical / p.nItems;
  const int ctu = rest % p.nCtus;
  const int refIdx = rest / p.nCtus;
  const Item* it = p.items + itemIdx;
  const uint16_t* __restrict__ ref = p.refs[refIdx];
  const uint16_t* __restrict__ cur = p.cur;
  const int W = p.W, H = p.H;
  const int ctuX = (ctu % p.ctusPerRow) * kCtu, ctuY = (ctu / p.ctusPerRow) * kCtu;

  if (tid < kMaxCu) {
    s_cu[tid] = it->cu[tid];
  }
  if (tid == 0) {
    s_hdr[0] = it->nCu;
    s_hdr[1] = it->nSb;
    s_hdr[2] = it->rx;
    s_hdr[3] = it->ry;
  }
  __syncthreads();
  const int nCu = s_hdr[0], nSb = s_hdr[1];
  const int fx0 = ctuX + s_hdr[2], fy0 = ctuY + s_hdr[3];  // region origin (frame)
  const int tx0 = fx0 - kMargin, ty0 = fy0 - kMargin;     // tile origin (frame)

  // ---- stage the reference region (+margin) into LDS, clamp-to-edge padded
  {
    constexpr int CPR = C::TILE / 4;  // 8-byte chunks per row
    for (int ch = tid; ch < C::TILE * CPR; ch += kThreads) {
      int ty = ch / CPR, cx = (ch % CPR) * 4;
      int fy = clampi(ty0 + ty, 0, H - 1), fx = tx0 + cx;
      const uint16_t* row = ref + (size_t)fy * W;
      uint2 v;
      if (fx >= 0 && fx + 3 < W) {
        v = *reinterpret_cast<const uint2*>(row + fx);
      } else {
        unsigned a0 = row[clampi(fx, 0, W - 1)], a1 = row[clampi(fx + 1, 0, W - 1)];
        unsigned a2 = row[clampi(fx + 2, 0, W - 1)], a3 = row[clampi(fx + 3, 0, W - 1)];
        v.x = a0 | (a1 << 16);
        v.y = a2 | (a3 << 16);
      }
      *reinterpret_cast<uint2*>(&s_tile[ty * C::TP + cx]) = v;
    }
  }

  // ---- per-lane sub-block assignment (fixed for the whole item)
  int myCu = -1;  // CU slot of this lane's sub-block(s)
  {
    const int t0 = tid * C::SBPL;
    if (t0 < nSb) {
      int k = 0;
      for (int j = 1; j < nCu; j++)
        if (s_cu[j].sbBase <= t0) k = j;
      myCu = k;
    }
  }
  int cuW = 0, cuH = 0, cuLw = 0, cuLh = 0, cuX = 0, cuY = 0, predBase = 0, segS = 1;
  bool active = false;
  if (myCu >= 0) {
    const CuSlot cs = s_cu[myCu];
    cuLw = cs.lw;
    cuLh = cs.lh;
    cuW = 1 << cuLw;
    cuH = 1 << cuLh;
    cuX = ctuX + cs.x;
    cuY = ctuY + cs.y;
    predBase = cs.sbBase * 16;
    segS = min(((cuW * cuH) >> 4) / C::SBPL, 64);
    active = (cuX + cuW <= W) && (cuY + cuH <= H);  // affine.cl:192-193
  }

  for (int pass = 0; pass < 2; pass++) {
    const int ncp = pass == 0 ? 2 : 3;
    if ((pass == 0 && !p.run2) || (pass == 1 && !p.run3)) continue;
    const int niter = (ncp == 3 ? 4 : 5) + p.extra;

    // ---- per-CU initial CPMVs (2 CP: zero; 3 CP: derived from the 2-CP winner)
    if (tid < nCu) {
      const CuSlot cs = s_cu[tid];
      CuState& st = s_st[tid];
      const int cx = ctuX + cs.x, cy = ctuY + cs.y;
      int c[6] = {0, 0, 0, 0, 0, 0};
      if (ncp == 3) {
        int prev[6];
        if (p.run2) {
          for (int i = 0; i < 6; i++) prev[i] = st.best[i];
        } else {
          const vame_cpmvs_dev& pv =
              p.prev[cs.align][(size_t)ctu * (cs.align ? kHalfCusPerCtu : kFullCusPerCtu) + cs.outOff];
          prev[0] = pv.ltx; prev[1] = pv.lty; prev[2] = pv.rtx; prev[3] = pv.rty;
        }
        // affine.cl:81-105
        int sh = 7 + cs.lh - cs.lw;
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
      }
      for (int i = 0; i < 6; i++) {
        st.cur[i] = c[i];
        st.best[i] = c[i];
      }
      st.bestCost = kCostInit;
      st.satd = 0;
      st.inframe = (cx + (1 << cs.lw) <= W) && (cy + (1 << cs.lh) <= H);
      for (int i = 0; i < kNumMom; i++) s_mom[tid][i] = 0;
    }
    __syncthreads();

    for (int iter = 0; iter <= niter; iter++) {
      // =============== prediction + SATD (affine.cl:208-393) ===============
      int satdLane = 0;
      if (active) {
        const CuState& st = s_st[myCu];
        int cp[6];
        for (int i = 0; i < 6; i++) cp[i] = st.cur[i];
        // deriveMv{2,3}Cps_and_spread (aux_functions.cl:146-212)
        const int hx = shl(cp[2] - cp[0], 7 - cuLw), hy = shl(cp[3] - cp[1], 7 - cuLw);
        int vx, vy;
        if (ncp == 3) {
          vx = shl(cp[4] - cp[0], 7 - cuLh);
          vy = shl(cp[5] - cp[1], 7 - cuLh);
        } else {
          vx = -hy;
          vy = hx;
        }
        const bool spread = spread_over_limit(hx, hy, vx, vy);
        const int bx = shl(cp[0], 7), by = shl(cp[1], 7);
        for (int j = 0; j < C::SBPL; j++) {
          int local = (tid * C::SBPL + j) - s_cu[myCu].sbBase;
          int lcols = cuLw - 2;
          int sx = (local & ((1 << lcols) - 1)) << 2, sy = (local >> lcols) << 2;
          int px = spread ? (cuW >> 1) : sx + 2, py = spread ? (cuH >> 1) : sy + 2;
          int mx = bx + hx * px + vx * py, my = by + hy * px + vy * py;
          mx = (mx + 64 - (mx >= 0)) >> 7;
          my = (my + 64 - (my >= 0)) >> 7;
          clip_mv(mx, my, cuX, cuY, W, H);
          const int ix = mx >> 4, fxr = mx & 15, iy = my >> 4, fyr = my & 15;
          const int wx = cuX + sx + ix - 2, wy = cuY + sy + iy - 2;  // 9x9 window origin
          const int tx = wx - tx0, ty = wy - ty0;
          const bool inTile = (unsigned)tx <= (unsigned)(C::TILE - 9) &&
                              (unsigned)ty <= (unsigned)(C::TILE - 9);
          int cfx[6], cfy[6];
          luma_coeffs(fxr, cfx);
          luma_coeffs(fyr, cfy);
          int tmp[9][4];
#pragma unroll
          for (int i = 0; i < 9; i++) {
            int w9[9];
            if (inTile) {
              const int base = (ty + i) * C::TP + (tx & ~3);
              const uint2* src = reinterpret_cast<const uint2*>(&s_tile[base]);
              uint2 q0 = src[0], q1 = src[1], q2 = src[2];
              unsigned d[6] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y};
              const int s = tx & 3;
              if (s & 2) {
#pragma unroll
                for (int k = 0; k < 5; k++) d[k] = d[k + 1];
              }
              if (s & 1) {
#pragma unroll
                for (int k = 0; k < 5; k++) d[k] = __builtin_amdgcn_alignbit(d[k + 1], d[k], 16);
              }
#pragma unroll
              for (int m = 0; m < 9; m++) w9[m] = (d[m >> 1] >> ((m & 1) * 16)) & 0xFFFF;
            } else {
              const uint16_t* row = ref + (size_t)clampi(wy + i, 0, H - 1) * W;
#pragma unroll
              for (int m = 0; m < 9; m++) w9[m] = row[clampi(wx + m, 0, W - 1)];
            }
#pragma unroll
            for (int c = 0; c < 4; c++) {
              int sum = 0;
#pragma unroll
              for (int m = 0; m < 6; m++) sum += w9[c + m] * cfx[m];
              tmp[i][c] = (sum - 32768) >> 2;  // offset -IF_INTERNAL_OFFS<<2, shift 2
            }
          }
          int pr[16];
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
              int sum = 0;
#pragma unroll
              for (int m = 0; m < 6; m++) sum += tmp[r + m][c] * cfy[m];
              pr[r * 4 + c] = clampi((sum + 512 + (8192 << 6)) >> 10, 0, 1023);
            }
          // store prediction (CU-compact layout) and SATD vs the original
          int diff[16];
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int ofs = predBase + (sy + r) * cuW + sx;
            uint2 pk;
            pk.x = (unsigned)pr[r * 4 + 0] | ((unsigned)pr[r * 4 + 1] << 16);
            pk.y = (unsigned)pr[r * 4 + 2] | ((unsigned)pr[r * 4 + 3] << 16);
            *reinterpret_cast<uint2*>(&s_pred[ofs]) = pk;
            const uint2 o = *reinterpret_cast<const uint2*>(cur + (size_t)(cuY + sy + r) * W + cuX + sx);
            diff[r * 4 + 0] = (int)(o.x & 0xFFFF) - pr[r * 4 + 0];
            diff[r * 4 + 1] = (int)(o.x >> 16) - pr[r * 4 + 1];
            diff[r * 4 + 2] = (int)(o.y & 0xFFFF) - pr[r * 4 + 2];
            diff[r * 4 + 3] = (int)(o.y >> 16) - pr[r * 4 + 3];
          }
          // aux_functions.cl:1940-2043 (xCalcHADs4x4)
          int m[16], d[16];
          m[0] = diff[0] + diff[12]; m[1] = diff[1] + diff[13];
          m[2] = diff[2] + diff[14]; m[3] = diff[3] + diff[15];
          m[4] = diff[4] + diff[8];  m[5] = diff[5] + diff[9];
          m[6] = diff[6] + diff[10]; m[7] = diff[7] + diff[11];
          m[8] = diff[4] - diff[8];  m[9] = diff[5] - diff[9];
          m[10] = diff[6] - diff[10]; m[11] = diff[7] - diff[11];
          m[12] = diff[0] - diff[12]; m[13] = diff[1] - diff[13];
          m[14] = diff[2] - diff[14]; m[15] = diff[3] - diff[15];
          d[0] = m[0] + m[4];  d[1] = m[1] + m[5];  d[2] = m[2] + m[6];  d[3] = m[3] + m[7];
          d[4] = m[8] + m[12]; d[5] = m[9] + m[13]; d[6] = m[10] + m[14]; d[7] = m[11] + m[15];
          d[8] = m[0] - m[4];  d[9] = m[1] - m[5];  d[10] = m[2] - m[6]; d[11] = m[3] - m[7];
          d[12] = m[12] - m[8]; d[13] = m[13] - m[9]; d[14] = m[14] - m[10]; d[15] = m[15] - m[11];
          m[0] = d[0] + d[3];  m[1] = d[1] + d[2];  m[2] = d[1] - d[2];  m[3] = d[0] - d[3];
          m[4] = d[4] + d[7];  m[5] = d[5] + d[6];  m[6] = d[5] - d[6];  m[7] = d[4] - d[7];
          m[8] = d[8] + d[11]; m[9] = d[9] + d[10]; m[10] = d[9] - d[10]; m[11] = d[8] - d[11];
          m[12] = d[12] + d[15]; m[13] = d[13] + d[14]; m[14] = d[13] - d[14]; m[15] = d[12] - d[15];
          d[0] = m[0] + m[1];  d[1] = m[0] - m[1];  d[2] = m[2] + m[3];  d[3] = m[3] - m[2];
          d[4] = m[4] + m[5];  d[5] = m[4] - m[5];  d[6] = m[6] + m[7];  d[7] = m[7] - m[6];
          d[8] = m[8] + m[9];  d[9] = m[8] - m[9];  d[10] = m[10] + m[11]; d[11] = m[11] - m[10];
          d[12] = m[12] + m[13]; d[13] = m[12] - m[13]; d[14] = m[14] + m[15]; d[15] = m[15] - m[14];
          int sa = 0;
#pragma unroll
          for (int k = 1; k < 16; k++) sa += abs(d[k]);
          sa += abs(d[0]) >> 2;
          satdLane += (sa + 1) >> 1;
        }
      }
      {
        int v = seg_sum32(satdLane, segS);
        if (active && (lane & (segS - 1)) == 0) atomicAdd(&s_st[myCu].satd, (unsigned)v);
      }
      __syncthreads();

      // =============== cost, best update (affine.cl:416-457) ===============
      const bool lastIter = iter == niter;
      if (tid < nCu) {
        CuState& st = s_st[tid];
        if (iter == 0 || st.inframe) {
          const int bits = affine_bits(st.cur, ncp) + kRuiBits;
          const float prod = __fmul_rn(p.lambda, (float)bits);
          const long long cost = (long long)st.satd + (long long)(int)floorf(prod);
          st.satd = 0;
          if (cost < st.bestCost) {
            st.bestCost = cost;
            for (int i = 0; i < 6; i++) st.best[i] = st.cur[i];
          }
        }
        if (lastIter) {  // affine.cl:928-957
          const CuSlot cs = s_cu[tid];
          const int mode = cs.align * 2 + (ncp - 2);
          const size_t idx = (size_t)ctu * (cs.align ? kHalfCusPerCtu : kFullCusPerCtu) + cs.outOff;
          p.cost[refIdx][mode][idx] = st.bestCost;
          vame_cpmvs_dev o;
          o.ncps = ncp;
          o.ltx = st.best[0]; o.lty = st.best[1]; o.rtx = st.best[2];
          o.rty = st.best[3]; o.lbx = st.best[4]; o.lby = st.best[5];
          p.cpmv[refIdx][mode][idx] = o;
        }
      }
      if (lastIter) break;  // uniform

      // =============== gradients + normal-equation moments (affine.cl:477-708) ===============
      long long mom[kNumMom];
#pragma unroll
      for (int i = 0; i < kNumMom; i++) mom[i] = 0;
      if (active) {
        for (int j = 0; j < C::SBPL; j++) {
          int local = (tid * C::SBPL + j) - s_cu[myCu].sbBase;
          int lcols = cuLw - 2;
          int sx = (local & ((1 << lcols) - 1)) << 2, sy = (local >> lcols) << 2;
          // 6x6 prediction patch around the sub-block, rows clamped into the CU;
          // columns outside the CU only feed gradients that are replaced below.
          int P[6][6];
#pragma unroll
          for (int i = 0; i < 6; i++) {
            const int rr = clampi(sy - 1 + i, 0, cuH - 1);
            const uint16_t* prow = &s_pred[predBase + rr * cuW];
            const uint2 mid = *reinterpret_cast<const uint2*>(prow + sx);
            const uint2 lft = *reinterpret_cast<const uint2*>(prow + max(sx - 4, 0));
            const uint2 rgt = *reinterpret_cast<const uint2*>(prow + min(sx + 4, cuW - 4));
            P[i][0] = (int)(lft.y >> 16);
            P[i][1] = (int)(mid.x & 0xFFFF);
            P[i][2] = (int)(mid.x >> 16);
            P[i][3] = (int)(mid.y & 0xFFFF);
            P[i][4] = (int)(mid.y >> 16);
            P[i][5] = (int)(rgt.x & 0xFFFF);
          }
          int gx[4][4], gy[4][4];
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
              gx[r][c] = (P[r][c + 2] - P[r][c]) + 2 * (P[r + 1][c + 2] - P[r + 1][c]) +
                         (P[r + 2][c + 2] - P[r + 2][c]);
              gy[r][c] = (P[r + 2][c] - P[r][c]) + 2 * (P[r + 2][c + 1] - P[r][c + 1]) +
                         (P[r + 2][c + 2] - P[r][c + 2]);
            }
          // CU-border replication (affine.cl:506-540): rows first, then columns
          if (sy == 0) {
#pragma unroll
            for (int c = 0; c < 4; c++) { gx[0][c] = gx[1][c]; gy[0][c] = gy[1][c]; }
          }
          if (sy + 4 == cuH) {
#pragma unroll
            for (int c = 0; c < 4; c++) { gx[3][c] = gx[2][c]; gy[3][c] = gy[2][c]; }
          }
          if (sx == 0) {
#pragma unroll
            for (int r = 0; r < 4; r++) { gx[r][0] = gx[r][1]; gy[r][0] = gy[r][1]; }
          }
          if (sx + 4 == cuW) {
#pragma unroll
            for (int r = 0; r < 4; r++) { gx[r][3] = gx[r][2]; gy[r][3] = gy[r][2]; }
          }
          int sxx = 0, sxy = 0, syy = 0, sxe = 0, sye = 0;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const uint2 o = *reinterpret_cast<const uint2*>(cur + (size_t)(cuY + sy + r) * W + cuX + sx);
            const int ov[4] = {(int)(o.x & 0xFFFF), (int)(o.x >> 16), (int)(o.y & 0xFFFF), (int)(o.y >> 16)};
#pragma unroll
            for (int c = 0; c < 4; c++) {
              const int e = ov[c] - P[r + 1][c + 1];  // residual orig - pred (affine.cl:547-579)
              const int a = gx[r][c], g = gy[r][c];
              sxx += a * a;
              sxy += a * g;
              syy += g * g;
              sxe += a * e;
              sye += g * e;
            }
          }
          const long long u = sx + 2, v = sy + 2;  // sub-block centre (affine.cl:680-681)
          const long long mono[6] = {1, u, v, u * u, u * v, v * v};
          const int S3[3] = {sxx, sxy, syy};
#pragma unroll
          for (int s = 0; s < 3; s++)
#pragma unroll
            for (int k = 0; k < 6; k++) mom[s * 6 + k] += mono[k] * (long long)S3[s];
#pragma unroll
          for (int k = 0; k < 3; k++) {
            mom[18 + k] += mono[k] * (long long)sxe;
            mom[21 + k] += mono[k] * (long long)sye;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < kNumMom; i++) {
        long long v = seg_sum64(mom[i], segS);
        if (active && (lane & (segS - 1)) == 0)
          atomicAdd(reinterpret_cast<unsigned long long*>(&s_mom[myCu][i]), (unsigned long long)v);
      }
      __syncthreads();

      // =============== solve + CPMV update (affine.cl:726-893), one lane per CU ===============
      if (tid < nCu && s_st[tid].inframe) {
        CuState& st = s_st[tid];
        const CuSlot cs = s_cu[tid];
        long long M[kNumMom];
        for (int i = 0; i < kNumMom; i++) {
          M[i] = s_mom[tid][i];
          s_mom[tid][i] = 0;
        }
        const int n = 2 * ncp;
        double a[7][7];
        for (int i = 0; i < 7; i++)
          for (int j = 0; j < 7; j++) a[i][j] = 0.;
        for (int c = 0; c < n; c++) {
          const int8_t* al = ncp == 3 ? kAlpha3[c] : kAlpha2[c];
          const int8_t* be = ncp == 3 ? kBeta3[c] : kBeta2[c];
          for (int r = 0; r < n; r++) {
            const int8_t* al2 = ncp == 3 ? kAlpha3[r] : kAlpha2[r];
            const int8_t* be2 = ncp == 3 ? kBeta3[r] : kBeta2[r];
            long long A = quad_form(al, al2, M + 0);
            long long xy1 = quad_form(al, be2, M + 6), xy2 = quad_form(be, al2, M + 6);
            A += xy1 + xy2;
            A += quad_form(be, be2, M + 12);
            a[c + 1][r] = (double)A;
          }
          long long bsum = 0;
          for (int k = 0; k < 3; k++) bsum += (long long)al[k] * M[18 + k] + (long long)be[k] * M[21 + k];
          a[c + 1][n] = (double)(bsum * 8);
        }
        double pr[6];
        solve_equal(a, n, pr);
        double dd[6] = {0, 0, 0, 0, 0, 0};
        const double w = (double)(1 << cs.lw), h = (double)(1 << cs.lh);
        dd[0] = pr[0];
        dd[2] = pr[2];
        dd[1] = __dadd_rn(__dmul_rn(pr[1], w), pr[0]);  // exact scaling by a power of two
        if (ncp == 3) {
          dd[3] = __dadd_rn(__dmul_rn(pr[3], w), pr[2]);
          dd[4] = __dadd_rn(__dmul_rn(pr[4], h), pr[0]);
          dd[5] = __dadd_rn(__dmul_rn(pr[5], h), pr[2]);
        } else {
          dd[3] = __dadd_rn(__dmul_rn(-pr[3], w), pr[2]);
        }
        // affine.cl:884-893 (scaleDeltaMvs order: LT=(d0,d2), RT=(d1,d3), LB=(d4,d5))
        int c6[6];
        c6[0] = (int)((unsigned)st.cur[0] + (unsigned)scale_delta(dd[0]));
        c6[1] = (int)((unsigned)st.cur[1] + (unsigned)scale_delta(dd[2]));
        c6[2] = (int)((unsigned)st.cur[2] + (unsigned)scale_delta(dd[1]));
        c6[3] = (int)((unsigned)st.cur[3] + (unsigned)scale_delta(dd[3]));
        c6[4] = (int)((unsigned)st.cur[4] + (unsigned)scale_delta(dd[4]));
        c6[5] = (int)((unsigned)st.cur[5] + (unsigned)scale_delta(dd[5]));
        const int cx = ctuX + cs.x, cy = ctuY + cs.y;
        for (int i = 0; i < 6; i++) c6[i] = clampi(c6[i], kMvMin, kMvMax);
        clip_mv(c6[0], c6[1], cx, cy, W, H);
        clip_mv(c6[2], c6[3], cx, cy, W, H);
        clip_mv(c6[4], c6[5], cx, cy, W, H);
        for (int i = 0; i < 6; i++) st.cur[i] = c6[i];
      }
      __syncthreads();
    }
    __syncthreads();
  }
}

}  // namespace vame
