// vame_tables.h -- CU-candidate geometry and VVC constants shared by host and
// device code of the affine-ME engine.
//
// Restates (as data) the reference's tables:
//   constants.cl:73-113   aligned CU sizes (WIDTH_LIST / HEIGHT_LIST)
//   constants.cl:125-139  RETURN_STRIDE_LIST (output index of each size)
//   constants.cl:207-435  half-aligned groups: positions, sizes, counts, strides
//   constants.cl:40-58    m_lumaFilter4x4 (6-tap affine luma filter, 16 phases)
//   constants.h:73-79     supported resolutions / CTU counts
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define VAME_HD __host__ __device__
#else
#define VAME_HD
#endif

namespace vame {

constexpr int kCtu = 128;
constexpr int kFullGroups = 12;
constexpr int kHalfGroups = 24;
constexpr int kFullCusPerCtu = 201;  // TOTAL_ALIGNED_CUS_PER_CTU
constexpr int kHalfCusPerCtu = 284;  // TOTAL_HALF_ALIGNED_CUS_PER_CTU

// ---- aligned ("FULL") groups: CU k of group g sits at raster position k
constexpr int kFullW[kFullGroups] = {128, 128, 64, 64, 64, 32, 32, 64, 16, 32, 16, 16};
constexpr int kFullH[kFullGroups] = {128, 64, 128, 64, 32, 64, 32, 16, 64, 16, 32, 16};
constexpr int kFullStride[kFullGroups + 1] = {0, 1, 3, 5, 9, 17, 25, 41, 57, 73, 105, 137, 201};

// ---- half-aligned ("HALF") groups
constexpr int kHalfW[kHalfGroups] = {64, 32, 64, 64, 16, 16, 32, 32, 32, 32, 32, 16,
                                     16, 16, 16, 16, 16, 16, 32, 32, 32, 16, 16, 16};
constexpr int kHalfH[kHalfGroups] = {32, 64, 16, 16, 64, 64, 32, 32, 16, 16, 16, 32,
                                     32, 32, 16, 16, 16, 16, 32, 16, 16, 32, 32, 16};
constexpr int kHalfN[kHalfGroups] = {4, 4, 8, 4, 8, 4, 8, 8, 16, 8, 16, 16,
                                     8, 16, 32, 32, 16, 16, 4, 8, 4, 8, 4, 32};
constexpr int kHalfStride[kHalfGroups + 1] = {0,   4,   8,   16,  20,  28,  32,  40,  48,
                                              64,  72,  88,  104, 112, 128, 160, 192, 208,
                                              224, 228, 236, 240, 248, 252, 284};
// CTU-relative positions, divided by 8 (every half-aligned offset is a multiple of 8)
constexpr uint8_t kHalfX8[kHalfGroups][32] = {
    {0, 8, 0, 8},
    {2, 10, 2, 10},
    {0, 8, 0, 8, 0, 8, 0, 8},
    {0, 8, 0, 8},
    {1, 5, 9, 13, 1, 5, 9, 13},
    {3, 11, 3, 11},
    {2, 10, 2, 10, 2, 10, 2, 10},
    {0, 4, 8, 12, 0, 4, 8, 12},
    {0, 4, 8, 12, 0, 4, 8, 12, 0, 4, 8, 12, 0, 4, 8, 12},
    {0, 4, 8, 12, 0, 4, 8, 12},
    {2, 10, 2, 10, 2, 10, 2, 10, 2, 10, 2, 10, 2, 10, 2, 10},
    {1, 5, 9, 13, 1, 5, 9, 13, 1, 5, 9, 13, 1, 5, 9, 13},
    {3, 11, 3, 11, 3, 11, 3, 11},
    {0, 2, 4, 6, 8, 10, 12, 14, 0, 2, 4, 6, 8, 10, 12, 14},
    {0, 2, 4, 6, 8, 10, 12, 14, 0, 2, 4, 6, 8, 10, 12, 14,
     0, 2, 4, 6, 8, 10, 12, 14, 0, 2, 4, 6, 8, 10, 12, 14},
    {1, 5, 9, 13, 1, 5, 9, 13, 1, 5, 9, 13, 1, 5, 9, 13,
     1, 5, 9, 13, 1, 5, 9, 13, 1, 5, 9, 13, 1, 5, 9, 13},
    {0, 2, 4, 6, 8, 10, 12, 14, 0, 2, 4, 6, 8, 10, 12, 14},
    {3, 11, 3, 11, 3, 11, 3, 11, 3, 11, 3, 11, 3, 11, 3, 11},
    {2, 10, 2, 10},
    {2, 10, 2, 10, 2, 10, 2, 10},
    {2, 10, 2, 10},
    {1, 5, 9, 13, 1, 5, 9, 13},
    {3, 11, 3, 11},
    {1, 3, 5, 9, 11, 13, 1, 5, 9, 13, 1, 3, 5, 9, 11, 13,
     1, 3, 5, 9, 11, 13, 1, 5, 9, 13, 1, 3, 5, 9, 11, 13}};
constexpr uint8_t kHalfY8[kHalfGroups][32] = {
    {2, 2, 10, 10},
    {0, 0, 8, 8},
    {1, 1, 5, 5, 9, 9, 13, 13},
    {3, 3, 11, 11},
    {0, 0, 0, 0, 8, 8, 8, 8},
    {0, 0, 8, 8},
    {0, 0, 4, 4, 8, 8, 12, 12},
    {2, 2, 2, 2, 10, 10, 10, 10},
    {1, 1, 1, 1, 5, 5, 5, 5, 9, 9, 9, 9, 13, 13, 13, 13},
    {3, 3, 3, 3, 11, 11, 11, 11},
    {0, 0, 2, 2, 4, 4, 6, 6, 8, 8, 10, 10, 12, 12, 14, 14},
    {0, 0, 0, 0, 4, 4, 4, 4, 8, 8, 8, 8, 12, 12, 12, 12},
    {0, 0, 4, 4, 8, 8, 12, 12},
    {2, 2, 2, 2, 2, 2, 2, 2, 10, 10, 10, 10, 10, 10, 10, 10},
    {1, 1, 1, 1, 1, 1, 1, 1, 5, 5, 5, 5, 5, 5, 5, 5,
     9, 9, 9, 9, 9, 9, 9, 9, 13, 13, 13, 13, 13, 13, 13, 13},
    {0, 0, 0, 0, 2, 2, 2, 2, 4, 4, 4, 4, 6, 6, 6, 6,
     8, 8, 8, 8, 10, 10, 10, 10, 12, 12, 12, 12, 14, 14, 14, 14},
    {3, 3, 3, 3, 3, 3, 3, 3, 11, 11, 11, 11, 11, 11, 11, 11},
    {0, 0, 2, 2, 4, 4, 6, 6, 8, 8, 10, 10, 12, 12, 14, 14},
    {2, 2, 10, 10},
    {1, 1, 5, 5, 9, 9, 13, 13},
    {3, 3, 11, 11},
    {2, 2, 2, 2, 10, 10, 10, 10},
    {2, 2, 10, 10},
    {1, 1, 1, 1, 1, 1, 3, 3, 3, 3, 5, 5, 5, 5, 5, 5,
     9, 9, 9, 9, 9, 9, 11, 11, 11, 11, 13, 13, 13, 13, 13, 13}};

// ---- 6-tap affine luma filter, taps 1..6 of the 8-tap table (taps 0 and 7 are
// zero for every phase), one int8 per tap, phase-major.
constexpr int8_t kLuma6[16][6] = {
    {0, 0, 64, 0, 0, 0},     {1, -3, 63, 4, -2, 1},   {1, -5, 62, 8, -3, 1},
    {2, -8, 60, 13, -4, 1},  {3, -10, 58, 17, -5, 1}, {3, -11, 52, 26, -8, 2},
    {2, -9, 47, 31, -10, 3}, {3, -11, 45, 34, -10, 3}, {3, -11, 40, 40, -11, 3},
    {3, -10, 34, 45, -11, 3}, {3, -10, 31, 47, -9, 2}, {2, -8, 26, 52, -11, 3},
    {1, -5, 17, 58, -10, 3}, {1, -4, 13, 60, -8, 2},  {1, -3, 8, 62, -5, 1},
    {1, -2, 4, 63, -3, 1}};

// ---- VTM constants used by the search (constants.cl:12-37)
constexpr int kMvMax = (1 << 17) - 1;  // MV_MAX (MV_BITS = 18)
constexpr int kMvMin = -(1 << 17);     // MV_MIN
constexpr int64_t kCostInit = int64_t(1) << 30;  // MAX_LONG = 1<<62 evaluated as int: 1<<30
constexpr int kRuiBits = 2;                      // LOW_DELAY_P (affine.cl:442-446)

// ---- resolutions accepted by the reference host (constants.h:73-79)
VAME_HD inline int num_ctus(int w, int h) {
  if (w == 3840 && h == 2160) return 510;
  if (w == 1920 && h == 1080) return 135;
  if (w == 1280 && h == 720) return 60;
  if (w == 832 && h == 480) return 28;
  if (w == 416 && h == 240) return 8;
  return 0;
}

}  // namespace vame
