// vame_hostlogic.cpp -- per-POC host logic the reference runs around its
// kernel launches: the GOP-8 QP/lambda model and the 4-slot reference list.
// Pure C++ (no device work); exported through include/vame.h.
#include <cmath>

#include "../../include/vame.h"

namespace {

// constants.h:94-103 fullLambdas[qp] (float)
const float kFullLambdas[60] = {
    0.f,        0.f,        0.f,        0.f,        0.f,        0.f,        0.f,
    0.f,        0.f,        0.f,        0.f,        2.769291f,  3.108425f,  3.489089f,
    3.916370f,  4.395976f,  4.934316f,  5.538583f,  6.216849f,  6.978177f,  7.832739f,
    8.791952f,  9.868633f,  11.077166f, 12.433698f, 13.956355f, 15.665478f, 17.583905f,
    19.737266f, 22.154332f, 24.867397f, 27.912709f, 31.330957f, 35.167810f, 39.474532f,
    44.308664f, 49.734793f, 55.825418f, 62.661913f, 70.335619f, 78.949063f, 88.617327f,
    99.469587f, 111.650836f, 125.323826f, 140.671239f, 157.898127f, 177.234655f,
    198.939174f, 223.301672f, 250.647653f, 281.342477f, 315.796254f, 354.469310f,
    397.878347f, 446.603345f, 501.295305f, 562.684955f, 631.592507f, 708.938619f};

}  // namespace

extern "C" {

// main_aux_functions.h:1482-1497 computeDeltaQp (GOP-8 low-delay QP model)
int vame_poc_qp(int qp, int poc) {
  static const int pocOffset[8] = {1, 5, 4, 5, 4, 5, 4, 5};
  const int m = ((poc % 8) + 8) % 8;
  const double scale = m == 0 ? 0 : 0.259, offset = m == 0 ? 0 : -6.5;
  int q = qp + pocOffset[m];
  double d = q * scale + offset + 0.5;
  d = std::fmax(0.0, std::fmin(3.0, d));  // clip3(0, 3, .) then floor (main_aux_functions.h:1473)
  return q + (int)std::floor(d);
}

// main.cpp:585: lambda = fullLambdas[computeDeltaQp(QP, POC)]
float vame_lambda(int qp, int poc) {
  const int q = vame_poc_qp(qp, poc);
  if (q < 0 || q >= 60) return -1.f;
  return kFullLambdas[q];
}

// main.cpp:591-707 -- replays the circular reference buffer (labels only: every
// device copy there is paired with the label move) from POC 1 to `poc`.
int vame_ref_list(int poc, int* pocs) {
  if (poc < 1 || !pocs) return VAME_E_INVALID;
  int L[4] = {-1, -1, -1, -1}, LT[4] = {0, 0, 0, 0};
  for (int p = 1; p <= poc; p++) {
    const int numRefs = p < 4 ? p : 4;
    if (p < 5) {
      int tempA = L[0], tempB;
      L[0] = p - 1;
      if (numRefs > 1) {
        tempB = L[1];
        L[1] = tempA;
        if (numRefs > 2) {
          tempA = L[2];
          L[2] = tempB;
          if (numRefs > 3) L[3] = tempA;
        }
      }
      LT[3] = L[3] % 8 == 0 ? 1 : 0;
    } else {
      int tempA = L[0], tempB;
      L[0] = p - 1;
      int update = LT[1] == 0 ? 1 : (tempA % 8 == 0 && tempA != L[0] ? 1 : 0);
      if (update) {
        tempB = L[1];
        L[1] = tempA;
        update = LT[2] == 0 ? 1 : (tempB % 8 == 0 && tempB != L[1] ? 1 : 0);
        if (update) {
          tempA = L[2];
          L[2] = tempB;
          update = LT[3] == 0 ? 1 : (tempA % 8 == 0 && tempA != L[3] ? 1 : 0);
          if (update) L[3] = tempA;
        }
      }
      LT[3] = L[3] % 8 == 0 ? 1 : 0;
      LT[2] = (L[2] % 8 == 0 && LT[3]) ? 1 : 0;
      LT[1] = (L[1] % 8 == 0 && LT[2]) ? 1 : 0;
    }
  }
  const int n = poc < 4 ? poc : 4;
  for (int r = 0; r < n; r++) pocs[r] = L[r];
  return n;
}

}  // extern "C"
