// prof_kat.cl -- TEST INFRASTRUCTURE ONLY.  A known-answer kernel written for
// vame: it calls the REFERENCE's own PROF functions, compiled from
// /root/reference/aux_functions.cl where it lies (nothing copied), on test
// vectors, so the oracle's restatement of the PROF branch (which affine.cl
// hard-disables with `int enablePROF=0`, affine.cl:168 / :1132) is pinned to
// the reference's code rather than to itself.
//   aux_functions.cl:218-404   get{Horizontal,Vertical}DeltasPROF{2,3}Cps
//   aux_functions.cl:1096-1239 horizontal_vertical_filter_new(..., enablePROF=1)
//   aux_functions.cl:471-605   PROF
// Per case g: win[g] = 11x11 reference window (affine.cl:246-326 layout),
// prm[g] = {nCPs, LT.x, LT.y, RT.x, RT.y, LB.x, LB.y, width, height, xFrac, yFrac, isSpread};
// out[g] = {deltaHor[16], deltaVer[16], prediction[16]}.
#include "aux_functions.cl"

__kernel void prof_kat(__global const int* win, __global const int* prm, __global int* out,
                       const int n) {
  const int g = get_global_id(0);
  if (g >= n) return;
  int w[11 * 11];
  for (int i = 0; i < 121; i++) w[i] = win[g * 121 + i];
  __global const int* q = prm + g * 12;
  Cpmvs cp;
  cp.nCPs = q[0];
  cp.LT.x = q[1]; cp.LT.y = q[2];
  cp.RT.x = q[3]; cp.RT.y = q[4];
  cp.LB.x = q[5]; cp.LB.y = q[6];
  const int pw = q[7], ph = q[8], xFrac = q[9], yFrac = q[10], spread = q[11];
  int16 dH, dV;
  if (cp.nCPs == 3) {
    dH = getHorizontalDeltasPROF3Cps(cp, pw, ph, 0, 0, false);
    dV = getVerticalDeltasPROF3Cps(cp, pw, ph, 0, 0, false);
  } else {
    dH = getHorizontalDeltasPROF2Cps(cp, pw, ph, 0, 0, false);
    dV = getVerticalDeltasPROF2Cps(cp, pw, ph, 0, 0, false);
  }
  const int16 p = horizontal_vertical_filter_new(w, (int2)(0, 0), 11, 11, 4, 4, xFrac, yFrac,
                                                 spread, dH, dV, 1);
  vstore16(dH, 0, out + g * 48);
  vstore16(dV, 0, out + g * 48 + 16);
  vstore16(p, 0, out + g * 48 + 32);
}
