/*
 * vame_oracle.c -- CPU restatement of the reference affine-ME hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libvame.so, the vame CLI)
 * links or calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg do, and only as the checker / the CPU baseline.
 *
 * What it restates (reference = iagostorch/VVC-Affine-GPU, /root/reference):
 *   affine.cl:11-958      kernel affine_gradient_mult_sizes      (aligned CUs)
 *   affine.cl:960-1950    kernel affine_gradient_mult_sizes_HA   (half-aligned CUs)
 *   aux_functions.cl      the live helpers cited per function below
 *   constants.cl:12-61, 73-141, 150-435   VTM constants, filter taps, CU tables
 *
 * It is written per CU (one candidate CU at a time, plain loops), not per
 * work-item, so that it shares no structure with the HIP kernel it checks.
 * Integer arithmetic is exact and order-independent; the only floating point
 * is (a) the float lambda*bits cost (aux_functions.cl:2219) and (b) the
 * double Gaussian elimination (affine.cl:782-856).  This file is compiled with
 * -ffp-contract=off; the one product the reference's OpenCL default
 * FP_CONTRACT=ON fuses (temp += a*b in back-substitution, affine.cl:851) is an
 * explicit fma() here.  (int)double follows the AMDGPU v_cvt_i32_f64 rule
 * (NaN -> 0, saturate) that the reference gets on the GPU (T6 in SURVEY.md).
 *
 * Pinning: the oracle is checked against outputs of the reference kernels
 * themselves, compiled offline from /root/reference/affine.cl for gfx950 and
 * run on an MI355X by oracle/ref_harness.cpp (see oracle/Makefile and
 * tests/golden/README.md).
 *
 * Out-of-frame CUs (CU not fully inside the frame, affine.cl:192-193): the
 * reference does not predict them (SATD = 0) but still runs the gradient
 * update on uninitialised LDS.  Every later iteration's CPMVs are clipped by
 * clipCpmvs against the same bounds that clip the iteration-0 LB, so their
 * rate (monotone ExpGolomb of monotone quarter-pel rounding) can never be
 * strictly below iteration 0's; with the strict '<' of affine.cl:451 the
 * logged result is therefore always iteration 0.  The oracle computes exactly
 * that and skips the (result-free) refinement for those CUs.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { int32_t x, y; } omv;
typedef struct { int32_t nCPs; omv LT, RT, LB; } ocpmvs; /* == typedef.h Cpmvs (28 B) */

/* ------------------------------------------------------------------ tables */
/* constants.cl:73-113 (aligned sizes) and :125-139 (RETURN_STRIDE_LIST) */
static const int FW[12] = {128, 128, 64, 64, 64, 32, 32, 64, 16, 32, 16, 16};
static const int FH[12] = {128, 64, 128, 64, 32, 64, 32, 16, 64, 16, 32, 16};
static const int FSTRIDE[13] = {0, 1, 3, 5, 9, 17, 25, 41, 57, 73, 105, 137, 201};

/* constants.cl:316-421: half-aligned groups (w, h, count, return stride) */
static const int HW[24] = {64, 32, 64, 64, 16, 16, 32, 32, 32, 32, 32, 16, 16, 16,
                           16, 16, 16, 16, 32, 32, 32, 16, 16, 16};
static const int HH[24] = {32, 64, 16, 16, 64, 64, 32, 32, 16, 16, 16, 32, 32, 32,
                           16, 16, 16, 16, 32, 16, 16, 32, 32, 16};
static const int HN[24] = {4, 4, 8, 4, 8, 4, 8, 8, 16, 8, 16, 16, 8, 16,
                           32, 32, 16, 16, 4, 8, 4, 8, 4, 32};
static const int HSTRIDE[25] = {0, 4, 8, 16, 20, 28, 32, 40, 48, 64, 72, 88, 104, 112,
                                128, 160, 192, 208, 224, 228, 236, 240, 248, 252, 284};
/* constants.cl:207-313 (HA_ALL_X_POS / HA_ALL_Y_POS), CTU-relative */
static const uint8_t HX[24][32] = {
    {0, 64, 0, 64},
    {16, 80, 16, 80},
    {0, 64, 0, 64, 0, 64, 0, 64},
    {0, 64, 0, 64},
    {8, 40, 72, 104, 8, 40, 72, 104},
    {24, 88, 24, 88},
    {16, 80, 16, 80, 16, 80, 16, 80},
    {0, 32, 64, 96, 0, 32, 64, 96},
    {0, 32, 64, 96, 0, 32, 64, 96, 0, 32, 64, 96, 0, 32, 64, 96},
    {0, 32, 64, 96, 0, 32, 64, 96},
    {16, 80, 16, 80, 16, 80, 16, 80, 16, 80, 16, 80, 16, 80, 16, 80},
    {8, 40, 72, 104, 8, 40, 72, 104, 8, 40, 72, 104, 8, 40, 72, 104},
    {24, 88, 24, 88, 24, 88, 24, 88},
    {0, 16, 32, 48, 64, 80, 96, 112, 0, 16, 32, 48, 64, 80, 96, 112},
    {0, 16, 32, 48, 64, 80, 96, 112, 0, 16, 32, 48, 64, 80, 96, 112,
     0, 16, 32, 48, 64, 80, 96, 112, 0, 16, 32, 48, 64, 80, 96, 112},
    {8, 40, 72, 104, 8, 40, 72, 104, 8, 40, 72, 104, 8, 40, 72, 104,
     8, 40, 72, 104, 8, 40, 72, 104, 8, 40, 72, 104, 8, 40, 72, 104},
    {0, 16, 32, 48, 64, 80, 96, 112, 0, 16, 32, 48, 64, 80, 96, 112},
    {24, 88, 24, 88, 24, 88, 24, 88, 24, 88, 24, 88, 24, 88, 24, 88},
    {16, 80, 16, 80},
    {16, 80, 16, 80, 16, 80, 16, 80},
    {16, 80, 16, 80},
    {8, 40, 72, 104, 8, 40, 72, 104},
    {24, 88, 24, 88},
    {8, 24, 40, 72, 88, 104, 8, 40, 72, 104, 8, 24, 40, 72, 88, 104,
     8, 24, 40, 72, 88, 104, 8, 40, 72, 104, 8, 24, 40, 72, 88, 104}};
static const uint8_t HY[24][32] = {
    {16, 16, 80, 80},
    {0, 0, 64, 64},
    {8, 8, 40, 40, 72, 72, 104, 104},
    {24, 24, 88, 88},
    {0, 0, 0, 0, 64, 64, 64, 64},
    {0, 0, 64, 64},
    {0, 0, 32, 32, 64, 64, 96, 96},
    {16, 16, 16, 16, 80, 80, 80, 80},
    {8, 8, 8, 8, 40, 40, 40, 40, 72, 72, 72, 72, 104, 104, 104, 104},
    {24, 24, 24, 24, 88, 88, 88, 88},
    {0, 0, 16, 16, 32, 32, 48, 48, 64, 64, 80, 80, 96, 96, 112, 112},
    {0, 0, 0, 0, 32, 32, 32, 32, 64, 64, 64, 64, 96, 96, 96, 96},
    {0, 0, 32, 32, 64, 64, 96, 96},
    {16, 16, 16, 16, 16, 16, 16, 16, 80, 80, 80, 80, 80, 80, 80, 80},
    {8, 8, 8, 8, 8, 8, 8, 8, 40, 40, 40, 40, 40, 40, 40, 40,
     72, 72, 72, 72, 72, 72, 72, 72, 104, 104, 104, 104, 104, 104, 104, 104},
    {0, 0, 0, 0, 16, 16, 16, 16, 32, 32, 32, 32, 48, 48, 48, 48,
     64, 64, 64, 64, 80, 80, 80, 80, 96, 96, 96, 96, 112, 112, 112, 112},
    {24, 24, 24, 24, 24, 24, 24, 24, 88, 88, 88, 88, 88, 88, 88, 88},
    {0, 0, 16, 16, 32, 32, 48, 48, 64, 64, 80, 80, 96, 96, 112, 112},
    {16, 16, 80, 80},
    {8, 8, 40, 40, 72, 72, 104, 104},
    {24, 24, 88, 88},
    {16, 16, 16, 16, 80, 80, 80, 80},
    {16, 16, 80, 80},
    {8, 8, 8, 8, 8, 8, 24, 24, 24, 24, 40, 40, 40, 40, 40, 40,
     72, 72, 72, 72, 72, 72, 88, 88, 88, 88, 104, 104, 104, 104, 104, 104}};

/* constants.cl:40-58 m_lumaFilter4x4 (6-tap affine filter stored as 8 taps) */
static const int LUMA[16][8] = {
    {0, 0, 0, 64, 0, 0, 0, 0},     {0, 1, -3, 63, 4, -2, 1, 0},
    {0, 1, -5, 62, 8, -3, 1, 0},   {0, 2, -8, 60, 13, -4, 1, 0},
    {0, 3, -10, 58, 17, -5, 1, 0}, {0, 3, -11, 52, 26, -8, 2, 0},
    {0, 2, -9, 47, 31, -10, 3, 0}, {0, 3, -11, 45, 34, -10, 3, 0},
    {0, 3, -11, 40, 40, -11, 3, 0},{0, 3, -10, 34, 45, -11, 3, 0},
    {0, 3, -10, 31, 47, -9, 2, 0}, {0, 2, -8, 26, 52, -11, 3, 0},
    {0, 1, -5, 17, 58, -10, 3, 0}, {0, 1, -4, 13, 60, -8, 2, 0},
    {0, 1, -3, 8, 62, -5, 1, 0},   {0, 1, -2, 4, 63, -3, 1, 0}};

#define MAX_COST_INIT ((int64_t)1 << 30) /* constants.cl:61 MAX_LONG = 1<<62 folds to 1<<30 (T1) */
#define MV_MAXV ((1 << 17) - 1)           /* constants.cl:35 */
#define MV_MINV (-(1 << 17))              /* constants.cl:36 */

/* ------------------------------------------------------------- helpers */
static inline int32_t shl(int32_t a, int s) { return (int32_t)((uint32_t)a << s); }
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int ilog2(int v) { int l = 0; while ((1 << (l + 1)) <= v) l++; return l; }
static inline int iabs(int v) { return v < 0 ? -v : v; }

/* aux_functions.cl:38-47 roundMv (shift 7, roundAndClipMv :90-101) */
static inline int round_mv(int v, int shift) {
  int off = 1 << (shift - 1);
  return (v + off - (v >= 0)) >> shift;
}

/* aux_functions.cl:51-67 clipMv (clipMvInPic), block position = CU position */
static inline omv clip_mv(omv m, int bx, int by, int W, int H) {
  int horMax = shl(W + 8 - bx - 1, 4), horMin = shl(-128 - 8 - bx + 1, 4);
  int verMax = shl(H + 8 - by - 1, 4), verMin = shl(-128 - 8 - by + 1, 4);
  omv r;
  r.x = clampi(m.x, horMin, horMax);
  r.y = clampi(m.y, verMin, verMax);
  return r;
}

/* aux_functions.cl:106-141 isSubblockVectorSpreadOverLimit, bipred == 0 branch */
static int spread_over_limit(int a, int b, int c, int d) {
  const int s4 = 4 << 11;
  int w = iabs(4 * a + s4), h = iabs(4 * b);
  w = (w >> 11) + 9;
  h = (h >> 11) + 9;
  if (w * h > 15 * 11) return 1;
  w = iabs(4 * c);
  h = iabs(4 * d + s4);
  w = (w >> 11) + 9;
  h = (h >> 11) + 9;
  if (w * h > 11 * 15) return 1;
  return 0;
}

/* aux_functions.cl:146-212 deriveMv{2,3}Cps_and_spread; then roundAndClipMv */
static omv subblock_mv(const ocpmvs *cp, int nCP, int w, int h, int sx, int sy,
                       int cux, int cuy, int W, int H, int *spread) {
  int lw = ilog2(w), lh = ilog2(h);
  int hx = shl(cp->RT.x - cp->LT.x, 7 - lw);
  int hy = shl(cp->RT.y - cp->LT.y, 7 - lw);
  int vx, vy;
  if (nCP == 3) {
    vx = shl(cp->LB.x - cp->LT.x, 7 - lh);
    vy = shl(cp->LB.y - cp->LT.y, 7 - lh);
  } else {
    vx = -hy;
    vy = hx;
  }
  int bx = shl(cp->LT.x, 7), by = shl(cp->LT.y, 7);
  int px, py;
  *spread = spread_over_limit(hx, hy, vx, vy);
  if (*spread) {
    px = w >> 1;
    py = h >> 1;
  } else {
    px = sx + 2;
    py = sy + 2;
  }
  omv m;
  m.x = bx + hx * px + vx * py;
  m.y = by + hy * px + vy * py;
  m.x = round_mv(m.x, 7);
  m.y = round_mv(m.y, 7);
  return clip_mv(m, cux, cuy, W, H);
}

/* affine.cl:246-345 + aux_functions.cl:1096-1239 (horizontal_vertical_filter_new,
 * PROF disabled).  Reference window clamped to the frame edges (the select()
 * cascade of affine.cl:288-326 is clamp-to-edge).  Taps 0 and 7 are zero for
 * every phase, so the live support is 9x9 at (X0-2, Y0-2). */
static void predict_4x4(const uint16_t *ref, int W, int H, int x0, int y0, omv mv,
                        int out[16]) {
  int ix = mv.x >> 4, fx = mv.x & 15, iy = mv.y >> 4, fy = mv.y & 15;
  int bx = x0 + ix - 3, by = y0 + iy - 3; /* 11x11 window origin */
  int tmp[11][4];
  for (int r = 0; r < 11; r++) {
    int yy = clampi(by + r, 0, H - 1);
    for (int c = 0; c < 4; c++) {
      int sum = 0;
      for (int k = 0; k < 8; k++) {
        int xx = clampi(bx + c + k, 0, W - 1);
        sum += (int)ref[(size_t)yy * W + xx] * LUMA[fx][k];
      }
      tmp[r][c] = (sum + (-8192 * 4)) >> 2; /* shift 6-4, offset -IF_INTERNAL_OFFS<<2 */
    }
  }
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      int sum = 0;
      for (int k = 0; k < 8; k++) sum += tmp[r + k][c] * LUMA[fy][k];
      int v = (sum + 512 + (8192 << 6)) >> 10; /* shift 6+4, offset 1<<9 + OFFS<<6 */
      out[r * 4 + c] = clampi(v, 0, 1023);    /* clipPel, aux_functions.cl:403 */
    }
}

/* ---- PROF (prediction refinement with optical flow), aux_functions.cl:215-605
 * and the enablePROF branch of horizontal_vertical_filter_new (:1096-1239).
 * The reference hard-codes enablePROF = 0 (affine.cl:168, :1132); vame offers
 * it as an option (vame_set_prof), restated here from those functions. */

/* aux_functions.cl:11-30 roundValue16, one component */
static inline int round_value(int v, int shift) {
  return (v + (1 << (shift - 1)) - (v >= 0)) >> shift;
}

/* aux_functions.cl:218-404 get{Horizontal,Vertical}DeltasPROF{2,3}Cps: the
 * per-sample MV offsets of a 4x4 sub-block from its centre (the same for every
 * sub-block of a CU), 1/16-pel << 8, rounded by 8 bits and clamped to +-31. */
static void prof_deltas(const ocpmvs *cp, int nCP, int w, int h, int dH[16], int dV[16]) {
  int lw = ilog2(w), lh = ilog2(h);
  int hx = shl(cp->RT.x - cp->LT.x, 7 - lw), hy = shl(cp->RT.y - cp->LT.y, 7 - lw);
  int vx, vy;
  if (nCP == 3) {
    vx = shl(cp->LB.x - cp->LT.x, 7 - lh);
    vy = shl(cp->LB.y - cp->LT.y, 7 - lh);
  } else { /* 4-parameter model: the vertical gradient is the rotated horizontal one */
    vx = -hy;
    vy = hx;
  }
  int qhx = shl(hx, 2), qvx = shl(vx, 2), qhy = shl(hy, 2), qvy = shl(vy, 2);
  int mh[16], mv[16];
  mh[0] = shl(hx + vx, 1) - shl(qhx + qvx, 1);
  mv[0] = shl(hy + vy, 1) - shl(qhy + qvy, 1);
  for (int c = 1; c < 4; c++) {
    mh[c] = mh[c - 1] + qhx;
    mv[c] = mv[c - 1] + qhy;
  }
  for (int r = 1; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      mh[r * 4 + c] = mh[(r - 1) * 4 + c] + qvx;
      mv[r * 4 + c] = mv[(r - 1) * 4 + c] + qvy;
    }
  for (int i = 0; i < 16; i++) {
    dH[i] = clampi(round_value(mh[i], 8), -31, 31);
    dV[i] = clampi(round_value(mv[i], 8), -31, 31);
  }
}

/* horizontal_vertical_filter_new with applyPROF (aux_functions.cl:1096-1239):
 * the vertical pass is not the last one (shift 6, no offset, no clip), then
 * PROF (aux_functions.cl:471-605): the 4x4 block padded to 6x6 with reference
 * samples around the integer position nearest the fractional one, scaled to
 * the internal precision ((s << 4) - 8192); gradients of the >> 6 samples;
 * dI = gx*dH + gy*dV clamped to [-8192, 8191]; (p + dI + 8 + 8192) >> 4,
 * clipped to 10 bits. */
static void predict_4x4_prof(const uint16_t *ref, int W, int H, int x0, int y0, omv mv,
                             const int dH[16], const int dV[16], int out[16]) {
  int ix = mv.x >> 4, fx = mv.x & 15, iy = mv.y >> 4, fy = mv.y & 15;
  int bx = x0 + ix - 3, by = y0 + iy - 3; /* 11x11 window origin */
#define WIN(r, c) ((int)ref[(size_t)clampi(by + (r), 0, H - 1) * W + clampi(bx + (c), 0, W - 1)])
  int tmp[11][4];
  for (int r = 0; r < 11; r++)
    for (int c = 0; c < 4; c++) {
      int sum = 0;
      for (int k = 0; k < 8; k++) sum += WIN(r, c + k) * LUMA[fx][k];
      tmp[r][c] = (sum + (-8192 * 4)) >> 2;
    }
  int P[6][6]; /* padded block; corners unused */
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      int sum = 0;
      for (int k = 0; k < 8; k++) sum += tmp[r + k][c] * LUMA[fy][k];
      P[r + 1][c + 1] = sum >> 6; /* not last: shift IF_FILTER_PREC, offset 0 */
    }
  const int xo = fx >> 3, yo = fy >> 3; /* aux_functions.cl:491-492 */
  for (int k = 0; k < 4; k++) {       /* columns left / right of the block */
    P[k + 1][0] = (WIN(3 + yo + k, 2 + xo) << 4) - 8192;
    P[k + 1][5] = (WIN(3 + yo + k, 7 + xo) << 4) - 8192;
  }
  for (int k = 0; k < 6; k++) { /* rows above / below */
    P[0][k] = (WIN(2 + yo, 2 + xo + k) << 4) - 8192;
    P[5][k] = (WIN(7 + yo, 2 + xo + k) << 4) - 8192;
  }
#undef WIN
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      int gx = (P[r + 1][c + 2] >> 6) - (P[r + 1][c] >> 6);
      int gy = (P[r + 2][c + 1] >> 6) - (P[r][c + 1] >> 6);
      int di = clampi(gx * dH[r * 4 + c] + gy * dV[r * 4 + c], -8192, 8191);
      out[r * 4 + c] = clampi((P[r + 1][c + 1] + di + 8 + 8192) >> 4, 0, 1023);
    }
}

/* aux_functions.cl:1940-2043 satd_4x4 (VTM xCalcHADs4x4 + JVET_R0164) */
static int satd4x4(const int *o, const int *p) {
  int diff[16], m[16], d[16];
  for (int k = 0; k < 16; k++) diff[k] = o[k] - p[k];
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
  int satd = 0;
  for (int k = 0; k < 16; k++) satd += iabs(d[k]);
  satd -= iabs(d[0]);
  satd += iabs(d[0]) >> 2;
  return (satd + 1) >> 1;
}

/* aux_functions.cl:2057-2075 changeAffinePrecInternal2Amvr(., QUARTER): 1/16 -> 1/4 */
static inline int to_quarter(int v) { return v >= 0 ? (v + 1) >> 2 : (v + 2) >> 2; }

/* aux_functions.cl:2117-2129 xGetExpGolombNumberOfBits */
static int eg_bits(int value) {
  unsigned len = 1;
  unsigned t = value <= 0 ? (((unsigned)(-value)) << 1) + 1 : (unsigned)value << 1;
  while (t > 128) {
    len += 14;
    t >>= 7;
  }
  int l = 0;
  while ((t >> (l + 1)) != 0) l++;
  return (int)len + (l << 1);
}

/* aux_functions.cl:2140-2189 calc_affine_bits with a zero predictor
 * (affine.cl:431-434: the 2-CP predictor predCpmvs is all-zero, 3-CP uses zeroCpmvs) */
static int affine_bits(const ocpmvs *c, int nCP) {
  int ltx = to_quarter(c->LT.x), lty = to_quarter(c->LT.y);
  int b = eg_bits(ltx) + eg_bits(lty);
  b += eg_bits(to_quarter(c->RT.x) - ltx) + eg_bits(to_quarter(c->RT.y) - lty);
  if (nCP == 3) b += eg_bits(to_quarter(c->LB.x) - ltx) + eg_bits(to_quarter(c->LB.y) - lty);
  return b;
}

/* aux_functions.cl:2219-2221 getCost: floor(lambda * bits) in single precision */
static inline int64_t rate_cost(int bits, float lambda) {
  volatile float prod = lambda * (float)bits;
  return (int64_t)(int)floorf(prod);
}

/* (int)double as AMDGPU v_cvt_i32_f64: truncate, NaN -> 0, saturate */
static inline int32_t cvt_i32_f64(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return 2147483647;
  if (d <= -2147483648.0) return (int32_t)0x80000000u;
  return (int32_t)d;
}

/* aux_functions.cl:2194-2215 scaleDeltaMvs: (int)(d*4 + SIGN(d)*0.5) << 2 */
static inline int32_t scale_delta(double d) {
  double s = d >= 0 ? 1.0 : -1.0; /* SIGN(): NaN -> -1 */
  double v = d * 4.0 + s * 0.5;   /* d*4 exact: fused or not is identical */
  return shl(cvt_i32_f64(v), 2);
}

/* affine.cl:782-856: VTM solveEqual, verbatim operation order.  a[1..n][0..n]. */
static void solve_equal(double a[7][7], int n, double *p) {
  for (int k = 0; k < n; k++) p[k] = 0.;
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
        double num = a[i][k] * a[j][i - 1];
        double q = num / a[i][i - 1];
        a[j][k] = a[j][k] - q;
      }
  }
  p[n - 1] = a[n][n] / a[n][n - 1];
  for (int i = n - 2; i >= 0; i--) {
    if (a[i + 1][i] == 0.) {
      for (int k = 0; k < n; k++) p[k] = 0.;
      break;
    }
    double temp = 0;
#ifdef VAME_ORACLE_NO_FMA /* T5 probe build: the uncontracted alternative */
    for (int j = i + 1; j < n; j++) temp = temp + a[i + 1][j] * p[j];
#else
    for (int j = i + 1; j < n; j++) temp = fma(a[i + 1][j], p[j], temp); /* FP_CONTRACT */
#endif
    p[i] = (a[i + 1][n] - temp) / a[i + 1][i];
  }
}

/* affine.cl:81-105: 3-CP seed (LB derived from the 2-CP LT/RT, 4->6 param) */
static ocpmvs seed_3cp(ocpmvs prev, int w, int h, int cux, int cuy, int W, int H) {
  int sh = 7 + ilog2(h) - ilog2(w);
  int vx2 = shl(prev.LT.x, 7) - shl(prev.RT.y - prev.LT.y, sh);
  int vy2 = shl(prev.LT.y, 7) + shl(prev.RT.x - prev.LT.x, sh);
  vx2 = (vx2 + 64 - (vx2 >= 0)) >> 7;
  vy2 = (vy2 + 64 - (vy2 >= 0)) >> 7;
  omv lb;
  lb.x = clampi(vx2, -(1 << 17), (1 << 17) - 1);
  lb.y = clampi(vy2, -(1 << 17), (1 << 17) - 1);
  /* roundAffinePrecInternal2Amvr(., QUARTER), aux_functions.cl:2078-2113 */
  lb.x = shl(to_quarter(lb.x), 2);
  lb.y = shl(to_quarter(lb.y), 2);
  prev.LB = clip_mv(lb, cux, cuy, W, H);
  return prev;
}

/* One candidate CU: the whole iteration loop of affine.cl:195-917. */
static void run_cu(const uint16_t *ref, const uint16_t *cur, int W, int H, float lambda,
                   int nCP, int extra, int prof, int cux, int cuy, int w, int h, ocpmvs init,
                   int64_t *out_cost, ocpmvs *out_cp, int16_t *pred, int16_t *gx,
                   int16_t *gy) {
  const int inframe = (cux + w <= W) && (cuy + h <= H);
  const int niter = (nCP == 3 ? 4 : 5) + extra;
  const int n = 2 * nCP;
  ocpmvs curr = init, best = init;
  int64_t bestCost = MAX_COST_INIT;
  for (int it = 0; it <= niter; it++) {
    int64_t satd = 0;
    if (inframe) {
      int dH[16], dV[16];
      if (prof) prof_deltas(&curr, nCP, w, h, dH, dV);
      for (int sy = 0; sy < h; sy += 4)
        for (int sx = 0; sx < w; sx += 4) {
          int spread;
          omv mv = subblock_mv(&curr, nCP, w, h, sx, sy, cux, cuy, W, H, &spread);
          int p[16], o[16];
          if (prof && !spread) /* applyPROF = enablePROF && !isSpread (aux_functions.cl:1101) */
            predict_4x4_prof(ref, W, H, cux + sx, cuy + sy, mv, dH, dV, p);
          else
            predict_4x4(ref, W, H, cux + sx, cuy + sy, mv, p);
          for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) {
              o[r * 4 + c] = cur[(size_t)(cuy + sy + r) * W + cux + sx + c];
              pred[(sy + r) * w + sx + c] = (int16_t)p[r * 4 + c];
            }
          satd += satd4x4(o, p);
        }
    }
    int64_t cost = satd + rate_cost(affine_bits(&curr, nCP) + 2, lambda); /* ruiBits=2 */
    if (cost < bestCost) {
      bestCost = cost;
      best = curr;
    }
    if (it == niter || !inframe) break;

    /* Sobel gradients with CU-border replication (affine.cl:477-540) */
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++) {
        int rr = clampi(r, 1, h - 2), cc = clampi(c, 1, w - 2);
        const int16_t *P = pred;
#define PP(y, x) ((int)P[(y) * w + (x)])
        gx[r * w + c] = (int16_t)(PP(rr - 1, cc + 1) - PP(rr - 1, cc - 1) + 2 * PP(rr, cc + 1) -
                                  2 * PP(rr, cc - 1) + PP(rr + 1, cc + 1) - PP(rr + 1, cc - 1));
        gy[r * w + c] = (int16_t)(PP(rr + 1, cc - 1) - PP(rr - 1, cc - 1) + 2 * PP(rr + 1, cc) -
                                  2 * PP(rr - 1, cc) + PP(rr + 1, cc + 1) - PP(rr - 1, cc + 1));
#undef PP
      }
    /* normal equations (affine.cl:671-708) */
    int64_t A[7][7];
    memset(A, 0, sizeof(A));
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++) {
        int g0 = gx[r * w + c], g1 = gy[r * w + c];
        int cy = ((r >> 2) << 2) + 2, cx = ((c >> 2) << 2) + 2;
        int e = (int)cur[(size_t)(cuy + r) * W + cux + c] - (int)pred[r * w + c];
        int iC[6];
        if (nCP == 3) {
          iC[0] = g0; iC[1] = cx * g0; iC[2] = g1; iC[3] = cx * g1; iC[4] = cy * g0; iC[5] = cy * g1;
        } else {
          iC[0] = g0; iC[1] = cx * g0 + cy * g1; iC[2] = g1; iC[3] = cy * g0 - cx * g1;
        }
        for (int col = 0; col < n; col++) {
          for (int row = 0; row < n; row++) A[col + 1][row] += (int64_t)iC[col] * (int64_t)iC[row];
          A[col + 1][n] += ((int64_t)iC[col] * (int64_t)e) * 8;
        }
      }
    double D[7][7];
    memset(D, 0, sizeof(D));
    for (int i = 1; i <= n; i++)
      for (int j = 0; j < 7; j++) D[i][j] = (double)A[i][j];
    double p[6];
    solve_equal(D, n, p);
    double dd[6] = {0, 0, 0, 0, 0, 0};
    dd[0] = p[0];
    dd[2] = p[2];
    if (nCP == 3) {
      dd[1] = p[1] * w + p[0]; /* exact: w is a power of two */
      dd[3] = p[3] * w + p[2];
      dd[4] = p[4] * h + p[0];
      dd[5] = p[5] * h + p[2];
    } else {
      dd[1] = p[1] * w + p[0];
      dd[3] = -p[3] * w + p[2];
    }
    /* affine.cl:884-893 (LT.y <- d2, RT.x <- d1 per scaleDeltaMvs ordering) */
    curr.LT.x = (int32_t)((uint32_t)curr.LT.x + (uint32_t)scale_delta(dd[0]));
    curr.LT.y = (int32_t)((uint32_t)curr.LT.y + (uint32_t)scale_delta(dd[2]));
    curr.RT.x = (int32_t)((uint32_t)curr.RT.x + (uint32_t)scale_delta(dd[1]));
    curr.RT.y = (int32_t)((uint32_t)curr.RT.y + (uint32_t)scale_delta(dd[3]));
    curr.LB.x = (int32_t)((uint32_t)curr.LB.x + (uint32_t)scale_delta(dd[4]));
    curr.LB.y = (int32_t)((uint32_t)curr.LB.y + (uint32_t)scale_delta(dd[5]));
    /* clampCpmvs (aux :2224) then clipCpmvs (aux :70-86) */
    curr.LT.x = clampi(curr.LT.x, MV_MINV, MV_MAXV); curr.LT.y = clampi(curr.LT.y, MV_MINV, MV_MAXV);
    curr.RT.x = clampi(curr.RT.x, MV_MINV, MV_MAXV); curr.RT.y = clampi(curr.RT.y, MV_MINV, MV_MAXV);
    curr.LB.x = clampi(curr.LB.x, MV_MINV, MV_MAXV); curr.LB.y = clampi(curr.LB.y, MV_MINV, MV_MAXV);
    curr.LT = clip_mv(curr.LT, cux, cuy, W, H);
    curr.RT = clip_mv(curr.RT, cux, cuy, W, H);
    curr.LB = clip_mv(curr.LB, cux, cuy, W, H);
  }
  best.nCPs = nCP;
  *out_cost = bestCost;
  *out_cp = best;
}

/* ------------------------------------------------------------------ API */
/* main_aux_functions.h:1587-1597 + constants.h:73-79 (resolution table) */
int vame_oracle_num_ctus(int W, int H) {
  static const int R[5][3] = {{3840, 2160, 510}, {1920, 1080, 135}, {1280, 720, 60},
                              {832, 480, 28},    {416, 240, 8}};
  for (int i = 0; i < 5; i++)
    if (R[i][0] == W && R[i][1] == H) return R[i][2];
  return 0;
}

int vame_oracle_cus_per_ctu(int align) { return align ? 284 : 201; }

/* One reference launch: affine_gradient_mult_sizes(_HA) compiled with -DnCP=nCP.
 * align 0 = FULL (aligned), 1 = HALF.  prev (nCP==3 only): the same-alignment
 * 2-CP result of this (POC, ref), indexed like the outputs.  Outputs are
 * indexed ctu*{201|284} + STRIDE[group] + cuIdx (affine.cl:936, :1929). */
int vame_oracle_affine_me_ex(const uint16_t *ref, const uint16_t *cur, int W, int H,
                             float lambda, int align, int nCP, int extra, int prof,
                             const ocpmvs *prev, int64_t *cost, ocpmvs *cpmvs, int nthreads) {
  int nCtus = vame_oracle_num_ctus(W, H);
  if (!nCtus || (nCP != 2 && nCP != 3) || (align != 0 && align != 1) || extra < 0) return -1;
  if (nCP == 3 && !prev) return -2;
  const int T = align ? 284 : 201, G = align ? 24 : 12;
  const int ctusPerRow = (W + 127) / 128; /* T8: integer ceil */
  const int nwork = nCtus * G;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    int16_t *pred = (int16_t *)malloc(3 * 128 * 128 * sizeof(int16_t));
    int16_t *gx = pred + 128 * 128, *gy = gx + 128 * 128;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int wk = 0; wk < nwork; wk++) {
      int ctu = wk / G, g = wk % G;
      int ctuX = (ctu % ctusPerRow) * 128, ctuY = (ctu / ctusPerRow) * 128;
      int w = align ? HW[g] : FW[g], h = align ? HH[g] : FH[g];
      int ncu = align ? HN[g] : (128 * 128) / (w * h);
      int stride = align ? HSTRIDE[g] : FSTRIDE[g];
      for (int k = 0; k < ncu; k++) {
        int cx, cy;
        if (align) {
          cx = HX[g][k];
          cy = HY[g][k];
        } else {
          cx = (k % (128 / w)) * w;
          cy = (k / (128 / w)) * h;
        }
        int idx = ctu * T + stride + k;
        ocpmvs init;
        memset(&init, 0, sizeof(init));
        if (nCP == 3) init = seed_3cp(prev[idx], w, h, ctuX + cx, ctuY + cy, W, H);
        run_cu(ref, cur, W, H, lambda, nCP, extra, prof, ctuX + cx, ctuY + cy, w, h, init,
               &cost[idx], &cpmvs[idx], pred, gx, gy);
      }
    }
    free(pred);
  }
  return 0;
}

/* The reference's launch (PROF off, as affine.cl hard-codes it). */
int vame_oracle_affine_me(const uint16_t *ref, const uint16_t *cur, int W, int H,
                          float lambda, int align, int nCP, int extra,
                          const ocpmvs *prev, int64_t *cost, ocpmvs *cpmvs, int nthreads) {
  return vame_oracle_affine_me_ex(ref, cur, W, H, lambda, align, nCP, extra, 0, prev, cost,
                                  cpmvs, nthreads);
}

/* ---- known-answer hooks for tests (each wraps one helper above) ---- */
void vame_oracle_prof_deltas(const ocpmvs *cp, int nCP, int w, int h, int *dH16, int *dV16) {
  prof_deltas(cp, nCP, w, h, dH16, dV16);
}
void vame_oracle_predict_4x4_prof(const uint16_t *ref, int W, int H, int x0, int y0, int mvx,
                                  int mvy, const int *dH16, const int *dV16, int *out16) {
  omv m = {mvx, mvy};
  predict_4x4_prof(ref, W, H, x0, y0, m, dH16, dV16, out16);
}
int vame_oracle_satd4x4(const int *orig16, const int *pred16) { return satd4x4(orig16, pred16); }
int vame_oracle_eg_bits(int v) { return eg_bits(v); }
int vame_oracle_to_quarter(int v) { return to_quarter(v); }
int vame_oracle_affine_bits(const ocpmvs *c, int nCP) { return affine_bits(c, nCP); }
int64_t vame_oracle_rate_cost(int bits, float lambda) { return rate_cost(bits, lambda); }
int vame_oracle_scale_delta(double d) { return scale_delta(d); }
int vame_oracle_spread(int a, int b, int c, int d) { return spread_over_limit(a, b, c, d); }
void vame_oracle_predict_4x4(const uint16_t *ref, int W, int H, int x0, int y0, int mvx,
                             int mvy, int *out16) {
  omv m = {mvx, mvy};
  predict_4x4(ref, W, H, x0, y0, m, out16);
}
void vame_oracle_seed_3cp(const ocpmvs *prev, int w, int h, int cux, int cuy, int W, int H,
                          ocpmvs *out) {
  *out = seed_3cp(*prev, w, h, cux, cuy, W, H);
}
void vame_oracle_solve(const double *a49, int n, double *p) {
  double a[7][7];
  memcpy(a, a49, sizeof(a));
  solve_equal(a, n, p);
}
/* CTU-relative CU geometry per (align, group): used by tests to cross-check tables */
int vame_oracle_group_geometry(int align, int g, int *w, int *h, int *ncu, int *stride,
                               int *xs, int *ys) {
  if ((align == 0 && (g < 0 || g >= 12)) || (align == 1 && (g < 0 || g >= 24))) return -1;
  *w = align ? HW[g] : FW[g];
  *h = align ? HH[g] : FH[g];
  *ncu = align ? HN[g] : (128 * 128) / ((*w) * (*h));
  *stride = align ? HSTRIDE[g] : FSTRIDE[g];
  for (int k = 0; k < *ncu; k++) {
    xs[k] = align ? HX[g][k] : (k % (128 / *w)) * *w;
    ys[k] = align ? HY[g][k] : (k / (128 / *w)) * *h;
  }
  return 0;
}
