// vame_engine.hip -- C ABI of the MI355X affine-ME engine (include/vame.h).
//
// Replaces the reference's OpenCL host launch boundary (main.cpp:473-552 buffer
// management, :754-966 clSetKernelArg/clEnqueueNDRangeKernel for the four
// kernel objects).  The host side here only builds the work-item templates,
// packs one kernel-argument struct and enqueues on the caller's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/vame.h"
#include "vame_kernel.h"

using namespace vame;

static_assert(sizeof(vame_cpmvs) == 28, "Cpmvs layout (typedef.h)");
static_assert(sizeof(vame_cpmvs_dev) == 28, "Cpmvs layout (typedef.h)");
static_assert(sizeof(CuSlot) == 16, "CuSlot layout");

static thread_local char g_hip_err[256] = "";

#define VAME_HIP(x)                                                               \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      snprintf(g_hip_err, sizeof(g_hip_err), "%s (%s:%d)", hipGetErrorString(e_), \
               __FILE__, __LINE__);                                               \
      return VAME_E_DEVICE;                                                       \
    }                                                                             \
  } while (0)

struct vame_ctx {
  int device, W, H, nCtus, ctusPerRow;
  // device-resident work-item templates: [quadFull | quadHalf] and big (FULL 128-class)
  Item* dQuad = nullptr;
  Item* dBig = nullptr;
  int nQuadFull = 0, nQuadHalf = 0, nBig = 0;
  hipStream_t side = nullptr;   // second stream: 128-class items run beside the quadrant items
  hipEvent_t evFork = nullptr, evJoin = nullptr;
  // optional per-kernel timing: (start, end) event pairs per kernel class
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[2];
  size_t evUsed[2] = {0, 0};
};

namespace {

int ilog2(int v) {
  int l = 0;
  while ((1 << (l + 1)) <= v) l++;
  return l;
}

struct CuDesc {
  int x, y, w, h, align, outOff;
};

// One work item.  sbpl = sub-blocks per lane of the kernel class (1 quadrant,
// 4 CTU).  Quadrant items whose CUs all fit one wave (<= 64 sub-blocks) are
// "autonomous": CUs are first-fit packed into <= 4 waves of 64 lanes and every
// wave refines its own CUs; other items are "cooperative" (CUs span waves,
// workgroup barriers per phase).  In both modes larger CUs come first inside
// their lane range, so every CU's first lane is aligned to its own
// power-of-two lane count, which the segmented wave reductions rely on.
Item make_item(int rx, int ry, std::vector<CuDesc> cus, int sbpl) {
  std::stable_sort(cus.begin(), cus.end(),
                   [](const CuDesc& a, const CuDesc& b) { return a.w * a.h > b.w * b.h; });
  if ((int)cus.size() > kMaxCu) abort();
  Item it;
  memset(&it, 0, sizeof(it));
  it.nCu = (int16_t)cus.size();
  it.rx = (int16_t)rx;
  it.ry = (int16_t)ry;
  bool coop = sbpl > 1;
  for (auto& c : cus) coop |= c.w * c.h / 16 > 64;
  std::vector<int> waveOf(cus.size(), 0);
  int nWaves = 1;
  if (!coop) {
    int fill[kMaxWaves] = {0, 0, 0, 0};
    nWaves = 0;
    for (size_t k = 0; k < cus.size(); k++) {
      const int nsb = cus[k].w * cus[k].h / 16;
      int w = 0;
      while (w < nWaves && fill[w] + nsb > 64) w++;
      if (w == nWaves) nWaves++;
      if (nWaves > kMaxWaves) abort();
      fill[w] += nsb;
      waveOf[k] = w;
    }
    // CU slots grouped by wave (stable: still largest first inside a wave)
    std::vector<size_t> order(cus.size());
    for (size_t k = 0; k < order.size(); k++) order[k] = k;
    std::stable_sort(order.begin(), order.end(),
                     [&](size_t a, size_t b) { return waveOf[a] < waveOf[b]; });
    std::vector<CuDesc> c2;
    std::vector<int> w2;
    for (size_t k : order) {
      c2.push_back(cus[k]);
      w2.push_back(waveOf[k]);
    }
    cus.swap(c2);
    waveOf.swap(w2);
  }
  it.coop = coop ? 1 : 0;
  it.nWaves = (int16_t)(coop ? kMaxWaves : nWaves);
  int sb = 0, waveSb0 = 0, prevWave = -1;
  for (size_t k = 0; k < cus.size(); k++) {
    CuSlot& s = it.cu[k];
    s.x = (int16_t)cus[k].x;
    s.y = (int16_t)cus[k].y;
    s.lw = (uint8_t)ilog2(cus[k].w);
    s.lh = (uint8_t)ilog2(cus[k].h);
    s.align = (uint8_t)cus[k].align;
    s.outOff = (int16_t)cus[k].outOff;
    s.sbBase = (int16_t)sb;
    if (coop) {
      s.laneBase = (int16_t)(sb / sbpl);
    } else {
      const int w = waveOf[k];
      if (w != prevWave) {
        it.wave[w].cuBegin = (int16_t)k;
        waveSb0 = sb;
        prevWave = w;
      }
      it.wave[w].cuEnd = (int16_t)(k + 1);
      it.wave[w].nSb = (int16_t)(sb + cus[k].w * cus[k].h / 16 - waveSb0);
      s.laneBase = (int16_t)(sb - waveSb0);
    }
    sb += cus[k].w * cus[k].h / 16;
  }
  it.nSb = (int16_t)sb;
  if (sb > kThreads * sbpl) abort();
  return it;
}

// Work-item templates (identical for every CTU):
//   big      : FULL 128x128 / 128x64 / 64x128 groups, whole CTU, 1024 sub-blocks
//   quadFull : FULL groups <= 64x64, one item per (group, 64x64 quadrant), 256 sub-blocks
//   quadHalf : HALF groups, per quadrant, first-fit-decreasing packed to <= 256 sub-blocks
void build_templates(std::vector<Item>& big, std::vector<Item>& quadFull,
                     std::vector<Item>& quadHalf) {
  for (int g = 0; g < kFullGroups; g++) {
    const int w = kFullW[g], h = kFullH[g], n = (kCtu * kCtu) / (w * h), cols = kCtu / w;
    if (w == 128 || h == 128) {
      std::vector<CuDesc> c;
      for (int k = 0; k < n; k++) c.push_back({(k % cols) * w, (k / cols) * h, w, h, 0, kFullStride[g] + k});
      big.push_back(make_item(0, 0, c, Cfg<128>::SBPL));
      continue;
    }
    for (int q = 0; q < 4; q++) {
      const int qx = (q & 1) * 64, qy = (q >> 1) * 64;
      std::vector<CuDesc> c;
      for (int k = 0; k < n; k++) {
        const int x = (k % cols) * w, y = (k / cols) * h;
        if (x >= qx && x < qx + 64 && y >= qy && y < qy + 64) c.push_back({x, y, w, h, 0, kFullStride[g] + k});
      }
      quadFull.push_back(make_item(qx, qy, c, Cfg<64>::SBPL));
    }
  }
  for (int q = 0; q < 4; q++) {
    const int qx = (q & 1) * 64, qy = (q >> 1) * 64;
    struct Grp { int sbTotal, sbPerCu; std::vector<CuDesc> cus; };
    std::vector<Grp> groups;
    for (int g = 0; g < kHalfGroups; g++) {
      Grp gr;
      gr.sbPerCu = kHalfW[g] * kHalfH[g] / 16;
      gr.sbTotal = 0;
      for (int k = 0; k < kHalfN[g]; k++) {
        const int x = kHalfX8[g][k] * 8, y = kHalfY8[g][k] * 8;
        if (x >= qx && x < qx + 64 && y >= qy && y < qy + 64) {
          gr.cus.push_back({x, y, kHalfW[g], kHalfH[g], 1, kHalfStride[g] + k});
          gr.sbTotal += gr.sbPerCu;
        }
      }
      if (!gr.cus.empty()) groups.push_back(gr);
    }
    std::stable_sort(groups.begin(), groups.end(),
                     [](const Grp& a, const Grp& b) { return a.sbTotal > b.sbTotal; });
    std::vector<std::pair<int, std::vector<CuDesc>>> bins;
    for (auto& gr : groups) {
      bool placed = false;
      for (auto& bn : bins)
        if (bn.first + gr.sbTotal <= kThreads && (int)(bn.second.size() + gr.cus.size()) <= kMaxCu) {
          bn.first += gr.sbTotal;
          bn.second.insert(bn.second.end(), gr.cus.begin(), gr.cus.end());
          placed = true;
          break;
        }
      if (!placed) bins.push_back({gr.sbTotal, gr.cus});
    }
    for (auto& bn : bins) quadHalf.push_back(make_item(qx, qy, bn.second, Cfg<64>::SBPL));
  }
}

void fill_common(KParams& kp, const vame_ctx* c, float lambda, int extra) {
  kp.W = c->W;
  kp.H = c->H;
  kp.nCtus = c->nCtus;
  kp.ctusPerRow = c->ctusPerRow;
  kp.lambda = lambda;
  kp.extra = extra;
}

// timing hooks (no-ops unless vame_set_timing(ctx, 1))
int time_begin(vame_ctx* c, int cls, hipStream_t s) {
  if (!c->timing) return VAME_OK;
  auto& v = c->ev[cls];
  if (c->evUsed[cls] == v.size()) {
    std::pair<hipEvent_t, hipEvent_t> e;
    VAME_HIP(hipEventCreate(&e.first));
    VAME_HIP(hipEventCreate(&e.second));
    v.push_back(e);
  }
  VAME_HIP(hipEventRecord(v[c->evUsed[cls]].first, s));
  return VAME_OK;
}
int time_end(vame_ctx* c, int cls, hipStream_t s) {
  if (!c->timing) return VAME_OK;
  VAME_HIP(hipEventRecord(c->ev[cls][c->evUsed[cls]].second, s));
  c->evUsed[cls]++;
  return VAME_OK;
}

#define VAME_TRY(x)        \
  do {                     \
    int rc_ = (x);         \
    if (rc_) return rc_;   \
  } while (0)

int launch(vame_ctx* c, KParams kp, bool quadFull, bool quadHalf, bool bigItems,
           hipStream_t stream) {
  // 128-class items (big LDS, 1 workgroup per CU) go first on a side stream so
  // they overlap with the quadrant items instead of forming a tail.
  const bool fork = bigItems && (quadFull || quadHalf);
  if (bigItems) {
    KParams kb = kp;
    kb.items = c->dBig;
    kb.nItems = c->nBig;
    const unsigned grid = (unsigned)(kb.nItems * kb.nCtus * kb.nRefs);
    hipStream_t s = stream;
    if (fork) {
      VAME_HIP(hipEventRecord(c->evFork, stream));
      VAME_HIP(hipStreamWaitEvent(c->side, c->evFork, 0));
      s = c->side;
    }
    VAME_TRY(time_begin(c, 1, s));
    hipLaunchKernelGGL(affine_me_ctu, dim3(grid), dim3(kThreads), 0, s, kb);
    VAME_HIP(hipGetLastError());
    VAME_TRY(time_end(c, 1, s));
    if (fork) VAME_HIP(hipEventRecord(c->evJoin, s));
  }
  if (quadFull || quadHalf) {
    KParams kq = kp;
    kq.items = quadFull ? c->dQuad : c->dQuad + c->nQuadFull;
    kq.nItems = (quadFull ? c->nQuadFull : 0) + (quadHalf ? c->nQuadHalf : 0);
    const unsigned grid = (unsigned)(kq.nItems * kq.nCtus * kq.nRefs);
    VAME_TRY(time_begin(c, 0, stream));
    hipLaunchKernelGGL(affine_me_quad, dim3(grid), dim3(kThreads), 0, stream, kq);
    VAME_HIP(hipGetLastError());
    VAME_TRY(time_end(c, 0, stream));
  }
  if (fork) VAME_HIP(hipStreamWaitEvent(stream, c->evJoin, 0));
  return VAME_OK;
}

}  // namespace

extern "C" {

int vame_num_ctus(int width, int height) { return num_ctus(width, height); }
int vame_cus_per_ctu(int align) {
  return align == 0 ? kFullCusPerCtu : align == 1 ? kHalfCusPerCtu : 0;
}
int vame_num_groups(int align) { return align == 0 ? kFullGroups : align == 1 ? kHalfGroups : 0; }

int vame_group_geometry(int align, int g, int* w, int* h, int* ncu, int* stride, int* xs, int* ys) {
  if (!w || !h || !ncu || !stride || !xs || !ys) return VAME_E_INVALID;
  if (align == 0 && g >= 0 && g < kFullGroups) {
    *w = kFullW[g];
    *h = kFullH[g];
    *ncu = (kCtu * kCtu) / (*w * *h);
    *stride = kFullStride[g];
    for (int k = 0; k < *ncu; k++) {
      xs[k] = (k % (kCtu / *w)) * *w;
      ys[k] = (k / (kCtu / *w)) * *h;
    }
    return VAME_OK;
  }
  if (align == 1 && g >= 0 && g < kHalfGroups) {
    *w = kHalfW[g];
    *h = kHalfH[g];
    *ncu = kHalfN[g];
    *stride = kHalfStride[g];
    for (int k = 0; k < *ncu; k++) {
      xs[k] = kHalfX8[g][k] * 8;
      ys[k] = kHalfY8[g][k] * 8;
    }
    return VAME_OK;
  }
  return VAME_E_INVALID;
}

int vame_create(vame_ctx** out, int device, int width, int height) {
  if (!out) return VAME_E_INVALID;
  *out = nullptr;
  const int nCtus = num_ctus(width, height);
  if (!nCtus) return VAME_E_INVALID;
  int ndev = 0;
  VAME_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return VAME_E_INVALID;
  VAME_HIP(hipSetDevice(device));
  std::vector<Item> big, qf, qh;
  build_templates(big, qf, qh);
  vame_ctx* c = new vame_ctx();
  c->device = device;
  c->W = width;
  c->H = height;
  c->nCtus = nCtus;
  c->ctusPerRow = (width + kCtu - 1) / kCtu;  // T8: integer ceil
  c->nBig = (int)big.size();
  c->nQuadFull = (int)qf.size();
  c->nQuadHalf = (int)qh.size();
  std::vector<Item> quad(qf);
  quad.insert(quad.end(), qh.begin(), qh.end());
  hipError_t e = hipMalloc(&c->dQuad, quad.size() * sizeof(Item));
  if (e == hipSuccess) e = hipMalloc(&c->dBig, big.size() * sizeof(Item));
  if (e == hipSuccess) e = hipMemcpy(c->dQuad, quad.data(), quad.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->dBig, big.data(), big.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->evFork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->evJoin, hipEventDisableTiming);
  if (e != hipSuccess) {
    snprintf(g_hip_err, sizeof(g_hip_err), "%s", hipGetErrorString(e));
    vame_destroy(c);
    return VAME_E_DEVICE;
  }
  *out = c;
  return VAME_OK;
}

void vame_destroy(vame_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->dQuad) (void)hipFree(c->dQuad);
  if (c->dBig) (void)hipFree(c->dBig);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->evFork) (void)hipEventDestroy(c->evFork);
  if (c->evJoin) (void)hipEventDestroy(c->evJoin);
  for (int k = 0; k < 2; k++)
    for (auto& e : c->ev[k]) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
  delete c;
}

int vame_affine_me(vame_ctx* c, const uint16_t* ref, const uint16_t* cur, float lambda, int align,
                   int nCP, int extra, const vame_cpmvs* prev, int64_t* cost, vame_cpmvs* cpmvs,
                   void* stream) {
  if (!c || !ref || !cur || !cost || !cpmvs) return VAME_E_INVALID;
  if ((align != 0 && align != 1) || (nCP != 2 && nCP != 3) || extra < 0 || extra > 64)
    return VAME_E_INVALID;
  if (nCP == 3 && !prev) return VAME_E_INVALID;
  VAME_HIP(hipSetDevice(c->device));
  KParams kp;
  memset(&kp, 0, sizeof(kp));
  fill_common(kp, c, lambda, extra);
  kp.cur = cur;
  kp.refs[0] = ref;
  kp.nRefs = 1;
  kp.run2 = nCP == 2;
  kp.run3 = nCP == 3;
  const int mode = align * 2 + (nCP - 2);
  kp.cost[0][mode] = cost;
  kp.cpmv[0][mode] = reinterpret_cast<vame_cpmvs_dev*>(cpmvs);
  kp.prev[align] = reinterpret_cast<const vame_cpmvs_dev*>(prev);
  return launch(c, kp, align == 0, align == 1, align == 0, (hipStream_t)stream);
}

int vame_affine_me_poc(vame_ctx* c, const uint16_t* cur, const uint16_t* const* refs, int nrefs,
                       float lambda, int mode_mask, int extra, const vame_poc_result* out,
                       void* stream) {
  if (!c || !cur || !refs || !out) return VAME_E_INVALID;
  if (nrefs < 1) return VAME_E_INVALID;
  if (nrefs > 4) return VAME_E_UNSUPPORTED;
  if (!(mode_mask & VAME_MODE_2CP) || (mode_mask & ~3) || extra < 0 || extra > 64)
    return VAME_E_INVALID;
  const bool run3 = (mode_mask & VAME_MODE_3CP) != 0;
  for (int r = 0; r < nrefs; r++) {
    if (!refs[r]) return VAME_E_INVALID;
    for (int m = 0; m < 4; m++) {
      const bool need = (m & 1) ? run3 : true;
      if (need && (!out->cost[r][m] || !out->cpmvs[r][m])) return VAME_E_INVALID;
    }
  }
  VAME_HIP(hipSetDevice(c->device));
  KParams kp;
  memset(&kp, 0, sizeof(kp));
  fill_common(kp, c, lambda, extra);
  kp.cur = cur;
  kp.nRefs = nrefs;
  kp.run2 = 1;
  kp.run3 = run3;
  for (int r = 0; r < nrefs; r++) {
    kp.refs[r] = refs[r];
    for (int m = 0; m < 4; m++) {
      kp.cost[r][m] = out->cost[r][m];
      kp.cpmv[r][m] = reinterpret_cast<vame_cpmvs_dev*>(out->cpmvs[r][m]);
    }
  }
  return launch(c, kp, true, true, true, (hipStream_t)stream);
}

int vame_set_timing(vame_ctx* c, int enable) {
  if (!c) return VAME_E_INVALID;
  c->timing = enable != 0;
  c->evUsed[0] = c->evUsed[1] = 0;
  return VAME_OK;
}

int vame_get_timing(vame_ctx* c, int cls, double* total_ms, int* launches, int reset) {
  if (!c || cls < 0 || cls > 1 || !total_ms || !launches) return VAME_E_INVALID;
  VAME_HIP(hipSetDevice(c->device));
  double t = 0;
  for (size_t i = 0; i < c->evUsed[cls]; i++) {
    float ms = 0;
    VAME_HIP(hipEventSynchronize(c->ev[cls][i].second));
    VAME_HIP(hipEventElapsedTime(&ms, c->ev[cls][i].first, c->ev[cls][i].second));
    t += ms;
  }
  *total_ms = t;
  *launches = (int)c->evUsed[cls];
  if (reset) c->evUsed[cls] = 0;
  return VAME_OK;
}

const char* vame_strerror(int code) {
  switch (code) {
    case VAME_OK: return "ok";
    case VAME_E_INVALID: return "invalid argument";
    case VAME_E_DEVICE: return "HIP runtime error";
    case VAME_E_NOMEM: return "out of memory";
    case VAME_E_UNSUPPORTED: return "unsupported";
    default: return "unknown error";
  }
}

const char* vame_last_hip_error(void) { return g_hip_err; }
const char* vame_version(void) { return "vame 0.1 (gfx950)"; }

}  // extern "C"
