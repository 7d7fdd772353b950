// vame_engine.hip -- C ABI of the MI355X affine-ME engine (include/vame.h).
//
// Replaces the reference's OpenCL host launch boundary (main.cpp:473-552 buffer
// management, :754-966 clSetKernelArg/clEnqueueNDRangeKernel for the four
// kernel objects).  The host side here only builds the work-item templates,
// packs one kernel-argument struct and enqueues on the caller's stream.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/vame.h"
#include "vame_kernel.h"

#if VAME_SPLIT_TU
namespace vame {
VAME_2CP_KERNELS(extern)  // defined in vame_kernels_2cp.hip
}
#endif

using namespace vame;

static_assert(sizeof(vame_cpmvs) == 28, "Cpmvs layout (typedef.h)");
static_assert(sizeof(vame_cpmvs_dev) == 28, "Cpmvs layout (typedef.h)");

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

constexpr int kTimingClasses = 7;

struct vame_ctx {
  int device, W, H, nCtus, ctusPerRow;
  // device-resident work-item templates: the quadrant items of four sets
  // [s][FULL | HALF | both alignments] at dQuad + quadOff[s][a]: 3 the SBL1
  // and SBL2 items together (one affine_me_quad launch: the 2-CP-only
  // launches), 0 / 1 the SBL1 / SBL2 items apart (affine_me_quad beside
  // affine_me_quad2: the 2+3-CP launches), 2 the PROF packing (every quadrant
  // CU one sub-block per lane, affine_me_quad_prof); and the 128-class CUs,
  // each a workgroup of its own: the 128x128 CU (dBig1: affine_me_ctu2;
  // affine_me_ctu_prof under PROF) and every 128x64 / 64x128 CU (dHalfW /
  // dHalfH: affine_me_half2w / _half2h; both in dHalf for affine_me_half_prof
  // under PROF)
  Item* dQuad = nullptr;
  int quadOff[4][3] = {}, quadN[4][3] = {};
  Item* dBig1 = nullptr;
  Item* dHalf = nullptr;
  Item* dHalfW = nullptr;
  Item* dHalfH = nullptr;
  int nBig1 = 0, nHalf = 0, nHalfW = 0, nHalfH = 0;
  // The 3-CP seed-reuse sums of the kernels with two sub-blocks per lane
  // (affine_me_ctu2, _half2w, _half2h, affine_me_quad2: 5 int32 per sub-block
  // of every (pair, CTU, item) of a launch; vame_kernel.h KParams::bestS), sized
  // for maxPairs pairs per launch and allocated by vame_create /
  // vame_set_max_pairs -- never inside a launch, so a captured call holds no
  // allocation.  bestOff[k]: the region of kernel k (ctu2, half2w, half2h,
  // quad2).  It is one
  // buffer per context: a call that uses it on another stream than the last
  // one waits for bestEv, recorded after that call.
  int32_t* bestS = nullptr;
  size_t bestOff[4] = {0, 0, 0, 0};
  int maxPairs = kMaxPairs;
  hipEvent_t bestEv = nullptr;
  hipStream_t bestStream = nullptr;
  bool bestPending = false;
  // block order (block_grid), per kernel class (0 quadrant, 1 128-class):
  // slot -> CTU table, group size, CTU chunks, slots per (pair, chunk)
  int32_t* dOrder[2] = {nullptr, nullptr};
  int groupCombos[2] = {408, 408}, nChunks[2] = {1, 1}, cpp[2] = {0, 0};
  // Streams of a call (VAME_STREAMS).  Kernels of one stream run one after
  // the other on MI355X even without the AQL barrier bit
  // (hipExtAnyOrderLaunch: profiles/ubench/anyorder_overlap.hip, three 50-us
  // kernels take 155 us on one stream, ~90 on three), so by default (2) the
  // quadrant kernel runs on a side stream forked from the caller's and the
  // 128-class kernels on the caller's stream, issued first;
  // 1: every kernel on the caller's stream, the quadrant kernel first with
  // the barrier bit, the others after it in any order.
  int streams = 2;
  hipStream_t side = nullptr;
  hipStream_t side2 = nullptr;  // timing builds VAME_Q1_SIDE=2: affine_me_quad on a stream of its own
  hipEvent_t evFork = nullptr, evJoin = nullptr, evJoin2 = nullptr;
  // VAME_SYNC (default 1): the join as a stream memory operation -- the side
  // stream writes a sequence number to a signal-memory word
  // (hipStreamWriteValue32, ordered after its earlier work), the caller's
  // stream waits for it (hipStreamWaitValue32) -- ~6 us per cross-stream hop
  // on MI355X against ~12 with an event record + hipStreamWaitEvent
  // (profiles/ubench/stream_hop.hip).  The fork stays an event: its slower
  // hop is the head start that lets the 128-class workgroups, issued on the
  // caller's stream, take their CUs before the quadrant kernel fills the GPU.
  // 0, a word that cannot be allocated, or a caller's stream under capture:
  // events.
  int valueSync = 1;
  uint32_t* syncWord = nullptr;
  uint32_t joinSeq = 0;
  // optional per-kernel timing: (start, end) event pairs per kernel class
  // (0 affine_me_quad, 1 128x128 CUs in affine_me_ctu_prof, 2 128x64 / 64x128
  // CUs in affine_me_half_prof, 3 128x128 CUs in affine_me_ctu2, 4 / 5 128x64 /
  // 64x128 CUs in affine_me_half2w / _half2h, 6 affine_me_quad2)
  int timing = 0;
  // PROF on (vame_set_prof): the *_prof kernels
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[kTimingClasses];
  size_t evUsed[kTimingClasses] = {};
  // vame_pack_records: the segment table of the last pack (host copy kept
  // until the next call) and its device copy
  std::vector<struct PackSeg> packSegs;
  struct PackSeg* dPackSegs = nullptr;
  size_t dPackCap = 0;
  hipEvent_t packEv = nullptr;  // after the last pack kernel (it read the device table)
};

// One segment of a record pack: the n records of one (POC, refIdx, PRED),
// costs to slab[off .. off + n), CPMV components after them.
struct PackSeg {
  const int64_t* cost;
  const int32_t* cpmv;  // vame_cpmvs, 7 int32 per record
  long long off;
  int n, ncp;
};

// Compact wire form (shard.pack's specification): thread i of segment
// blockIdx.y moves record i -- its cost as int32, its 2 * ncp CPMV components
// -- and flags a record the form cannot hold (cost outside [0, 2^31), a 2-CP
// LB other than (0, 0)).
__global__ __launch_bounds__(256) void pack_records_kernel(const PackSeg* segs, int32_t* slab, int32_t* bad) {
  const PackSeg sg = segs[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= sg.n) return;
  const long long c = sg.cost[i];
  const int32_t* r = sg.cpmv + (size_t)i * 7;
  int flag = (c < 0 || c >= (1ll << 31)) ? 1 : 0;
  slab[sg.off + i] = (int32_t)c;
  int32_t* d = slab + sg.off + sg.n + (size_t)i * 2 * sg.ncp;
  if (sg.ncp == 2) {
    d[0] = r[1]; d[1] = r[2]; d[2] = r[3]; d[3] = r[4];
    flag |= (r[5] | r[6]) != 0;
  } else {
    d[0] = r[1]; d[1] = r[2]; d[2] = r[3]; d[3] = r[4]; d[4] = r[5]; d[5] = r[6];
  }
  if (__builtin_amdgcn_ballot_w64(flag != 0) && flag) atomicOr(bad, 1);
}

namespace {

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

static_assert(kFullCusPerCtu <= 512 && kHalfCusPerCtu <= 512, "CuSlot::outOff");
// The quadrant packing (measured alternatives in HISTORY.md): autonomous items
// of kMaxTasks wave tasks over one staged tile, waves claiming the next task
// from an LDS counter as they finish; one cooperative item per quadrant
// chaining its cooperative groups; a launch of both alignments on items
// mixing them, every quadrant's first (largest-task) autonomous item first.

int ilog2(int v) {
  int l = 0;
  while ((1 << (l + 1)) <= v) l++;
  return l;
}

struct CuDesc {
  int x, y, w, h, align, outOff;
};

int nsb_of(const CuDesc& c) { return c.w * c.h / 16; }

void set_slot(CuSlot& s, const CuDesc& c) {
  s.x = (int16_t)c.x;
  s.y = (int16_t)c.y;
  s.lw = (uint8_t)ilog2(c.w);
  s.lh = (uint8_t)ilog2(c.h);
  s.align = (uint8_t)c.align;
  s.outOff = (uint16_t)c.outOff;
}

// Cooperative item: tasks of CUs of one size, each CU spanning nsb >= 64
// lanes (one per sub-block) of the workgroup (workgroup barriers per phase,
// LDS atomics), run one after another over the item's one staged tile.  A
// single task holds slots 0 .. (up to kMaxCu), a chain's task t slots
// t * kTaskCu ...
Item make_coop_item(int rx, int ry, const std::vector<std::vector<CuDesc>>& tasks, int threads) {
  Item it;
  memset(&it, 0, sizeof(it));
  it.rx = (int16_t)rx;
  it.ry = (int16_t)ry;
  it.coop = 1;
  if (tasks.empty() || (int)tasks.size() > kMaxTasks) abort();
  it.nTasks = (int16_t)tasks.size();
  const int stride = tasks.size() > 1 ? kTaskCu : kMaxCu;
  for (size_t t = 0; t < tasks.size(); t++) {
    const int nsb = nsb_of(tasks[t][0]);
    const int n = (int)tasks[t].size();
    for (auto& c : tasks[t])
      if (nsb_of(c) != nsb) abort();
    if (nsb < 64 || n * nsb > threads || n > stride) abort();
    for (int i = 0; i < n; i++) set_slot(it.cu[t * stride + i], tasks[t][i]);
    it.cu[t * stride].taskCus = (uint8_t)n;
    it.cu[t * stride].taskLogL = (uint16_t)ilog2(nsb);
    it.nCu = (int16_t)(t * stride + n);
  }
  return it;
}
Item make_coop_item(int rx, int ry, const std::vector<CuDesc>& cus, int threads) {
  return make_coop_item(rx, ry, std::vector<std::vector<CuDesc>>{cus}, threads);
}

// Autonomous item: up to kMaxTasks wave tasks, each CUs of ONE size (one lane
// per sub-block, or per two stacked sub-blocks with sbl = 2: 16, 32 or 64
// lanes per CU), so a task's segment size is uniform.  Wave w runs task w,
// then claims the next unclaimed one as it finishes, over the one staged
// tile: task t holds CU slots t * kTaskCu .. (its first slot carries the
// task's CU count and lanes per CU) and the running wave's prediction rows.
// Unused slots stay zero (lw 0).
Item make_auto_item(int rx, int ry, const std::vector<std::vector<CuDesc>>& tasks, int sbl) {
  Item it;
  memset(&it, 0, sizeof(it));
  it.rx = (int16_t)rx;
  it.ry = (int16_t)ry;
  it.coop = sbl == 2 ? 2 | 4 : 2;  // bit 1: waves claim tasks; bit 2: two sub-blocks per lane
  if (tasks.empty() || (int)tasks.size() > kMaxTasks) abort();
  it.nTasks = (int16_t)tasks.size();
  it.nCu = (int16_t)(tasks.size() * kTaskCu);
  for (size_t t = 0; t < tasks.size(); t++) {
    const int lanes = nsb_of(tasks[t][0]) / sbl;
    const int n = (int)tasks[t].size();
    for (auto& c : tasks[t])
      if (nsb_of(c) / sbl != lanes) abort();
    if (n * lanes > 64 || lanes < 16 || n > kTaskCu) abort();  // the kernel's segment sums handle 16 / 32 / 64
    for (int i = 0; i < n; i++) set_slot(it.cu[t * kTaskCu + i], tasks[t][i]);
    it.cu[t * kTaskCu].taskCus = (uint8_t)n;
    it.cu[t * kTaskCu].taskLogL = (uint16_t)ilog2(lanes);
  }
  return it;
}

// CUs of one quadrant: wave tasks of one size class (largest first, at most
// kTaskCu CUs and 64 lanes each), then items of kMaxTasks consecutive tasks.
// Returns the number of items appended.
#ifndef VAME_Q2_TASKS  // timing builds: wave tasks per affine_me_quad2 item
#define VAME_Q2_TASKS 16
#endif
size_t pack_autonomous(int qx, int qy, std::vector<CuDesc> cus, std::vector<Item>& out, int sbl) {
  const int perItem = sbl == 2 ? VAME_Q2_TASKS : kMaxTasks;
  std::stable_sort(cus.begin(), cus.end(),
                   [](const CuDesc& a, const CuDesc& b) { return nsb_of(a) > nsb_of(b); });
  std::vector<std::vector<CuDesc>> waves;
  for (auto& c : cus) {
    if (waves.empty() || nsb_of(waves.back()[0]) != nsb_of(c) || (int)waves.back().size() == kTaskCu ||
        (int)(waves.back().size() + 1) * nsb_of(c) / sbl > 64)
      waves.push_back({});
    waves.back().push_back(c);
  }
  for (size_t w = 0; w < waves.size(); w += perItem) {
    std::vector<std::vector<CuDesc>> grp(waves.begin() + w,
                                         waves.begin() + std::min(waves.size(), w + perItem));
    out.push_back(make_auto_item(qx, qy, grp, sbl));
  }
  return (waves.size() + perItem - 1) / perItem;
}

// The quadrant items of one kernel: for launches of FULL CUs only, HALF CUs
// only, and both alignments.
struct QuadSet {
  std::vector<Item> full, half, both;
};

// Work-item templates (identical for every CTU):
//   big      : the FULL 128x128 CU, whole CTU, cooperative
//   half     : each 128x64 / 64x128 CU alone, its own region
//   q1       : affine_me_quad (one sub-block per lane), per 64x64 quadrant:
//              the cooperative CUs (FULL 64x64; without q2 also FULL 64x32 /
//              32x64 and HALF 64x32 + 32x64) chained in one item, then
//              autonomous items of kMaxTasks wave tasks over the CUs of 16
//              sub-blocks (without q2: of <= 64)
//   q2       : (nullptr: not used, the PROF packing) affine_me_quad2 (two
//              stacked sub-blocks per lane): autonomous items over the CUs of
//              32 to 128 sub-blocks
// In the items of a launch of both alignments the alignments mix: every
// quadrant's cooperative chain first, then every quadrant's first
// (largest-task) autonomous item, then the seconds, ...: the kernel's last
// workgroups are its shortest.
void build_templates(std::vector<Item>& big, std::vector<Item>& halfItems, QuadSet& q1, QuadSet* q2) {
  for (int g = 0; g < kFullGroups; g++) {
    const int w = kFullW[g], h = kFullH[g], n = (kCtu * kCtu) / (w * h), cols = kCtu / w;
    if (w == 128 || h == 128) {
      std::vector<CuDesc> c;
      for (int k = 0; k < n; k++) c.push_back({(k % cols) * w, (k / cols) * h, w, h, 0, kFullStride[g] + k});
      if (w != h) {
        if (VAME_ABLATE & 256) continue;  // timing-only builds: no 128x64 / 64x128 items
        for (auto& cu : c) {  // one CU per item, the region = the CU
          Item it = make_coop_item(cu.x, cu.y, {cu}, Cfg<kKindHalf>::THREADS);
          it.rw = (int16_t)w;
          it.rh = (int16_t)h;
          halfItems.push_back(it);
        }
      } else {
        big.push_back(make_coop_item(0, 0, c, Cfg<kKindCtu>::THREADS));
      }
    }
  }
  // the largest CU an autonomous task of each kernel holds (sub-blocks)
  const int max1 = q2 ? 16 : 64, min2 = 32, max2 = 128;
  struct Both {
    std::vector<Item> coop, autos;
    std::vector<int> rank;  // an autonomous item's index within its quadrant
  } both1, both2;
  for (int q = 0; q < 4; q++) {
    const int qx = (q & 1) * 64, qy = (q >> 1) * 64;
    auto inq = [&](int x, int y) { return x >= qx && x < qx + 64 && y >= qy && y < qy + 64; };
    std::vector<CuDesc> a1[2], a2[2];              // autonomous CUs per alignment, per kernel
    std::vector<std::vector<CuDesc>> coop[2];      // cooperative tasks (q1), per alignment
    auto place = [&](const std::vector<CuDesc>& c, int align) {
      if (c.empty()) return;
      const int nsb = nsb_of(c[0]);
      if (nsb <= max1)
        a1[align].insert(a1[align].end(), c.begin(), c.end());
      else if (q2 && nsb >= min2 && nsb <= max2)
        a2[align].insert(a2[align].end(), c.begin(), c.end());
      else
        coop[align].push_back(c);  // a task per group
    };
    for (int g = 0; g < kFullGroups; g++) {
      const int w = kFullW[g], h = kFullH[g], n = (kCtu * kCtu) / (w * h), cols = kCtu / w;
      if (w == 128 || h == 128) continue;
      std::vector<CuDesc> c;
      for (int k = 0; k < n; k++) {
        const int x = (k % cols) * w, y = (k / cols) * h;
        if (inq(x, y)) c.push_back({x, y, w, h, 0, kFullStride[g] + k});
      }
      place(c, 0);
    }
    std::vector<CuDesc> halfBig;  // the HALF 64x32 + 32x64 CUs: one cooperative task
    for (int g = 0; g < kHalfGroups; g++) {
      std::vector<CuDesc> c;
      for (int k = 0; k < kHalfN[g]; k++) {
        const int x = kHalfX8[g][k] * 8, y = kHalfY8[g][k] * 8;
        if (!inq(x, y)) continue;
        if (x + kHalfW[g] > qx + 64 || y + kHalfH[g] > qy + 64) abort();
        c.push_back({x, y, kHalfW[g], kHalfH[g], 1, kHalfStride[g] + k});
      }
      if (!c.empty() && nsb_of(c[0]) > max1 && !(q2 && nsb_of(c[0]) <= max2))
        halfBig.insert(halfBig.end(), c.begin(), c.end());
      else
        place(c, 1);
    }
    if (!halfBig.empty()) coop[1].push_back(halfBig);
    // one-alignment sets: the cooperative chain, then the autonomous items
    for (int al = 0; al < 2; al++) {
      std::vector<Item>& o1 = al ? q1.half : q1.full;
      if (!coop[al].empty()) o1.push_back(make_coop_item(qx, qy, coop[al], Cfg<kKindQuad>::THREADS));
      pack_autonomous(qx, qy, a1[al], o1, 1);
      if (q2) pack_autonomous(qx, qy, a2[al], al ? q2->half : q2->full, 2);
    }
    // both alignments
    std::vector<std::vector<CuDesc>> t(coop[0]);
    t.insert(t.end(), coop[1].begin(), coop[1].end());
    if (!t.empty()) both1.coop.push_back(make_coop_item(qx, qy, t, Cfg<kKindQuad>::THREADS));
    for (int k = 0; k < (q2 ? 2 : 1); k++) {
      Both& b = k ? both2 : both1;
      std::vector<CuDesc> cus(k ? a2[0] : a1[0]);
      const std::vector<CuDesc>& h = k ? a2[1] : a1[1];
      cus.insert(cus.end(), h.begin(), h.end());
      const size_t n = pack_autonomous(qx, qy, cus, b.autos, k ? 2 : 1);
      for (size_t i = 0; i < n; i++) b.rank.push_back((int)i);
    }
  }
  for (int k = 0; k < (q2 ? 2 : 1); k++) {
    Both& b = k ? both2 : both1;
    std::vector<Item>& out = k ? q2->both : q1.both;
    out = b.coop;
    std::vector<size_t> idx(b.autos.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return b.rank[x] < b.rank[y]; });
    for (size_t i : idx) out.push_back(b.autos[i]);
  }
}

// The seed-reuse regions of the two-sub-block kernels for `pairs` pairs per
// launch: [ctu2 | half2w | half2h | quad2], each [pairs * nCtus * items][5][NSB]
// int32 (vame_kernel.h: p.bestS + ((pair * nCtus + ctu) * nItems + item) * 5 *
// NSB; quad2: sized for its largest item set).
size_t best_layout(const vame_ctx* c, int pairs, size_t off[4]) {
  const size_t per = (size_t)pairs * c->nCtus * 5;
  int nq2 = 0;  // the SBL2 items index the region by their item index
  for (int a = 0; a < 3; a++) nq2 = std::max({nq2, c->quadN[1][a], c->quadN[3][a]});
  off[0] = 0;
  off[1] = off[0] + per * c->nBig1 * Cfg<kKindCtu2>::NSB;
  off[2] = off[1] + per * c->nHalfW * Cfg<kKindHalf2W>::NSB;
  off[3] = off[2] + per * c->nHalfH * Cfg<kKindHalf2H>::NSB;
  return off[3] + per * nq2 * Cfg<kKindQuad2>::NSB;
}

int alloc_best(vame_ctx* c, int pairs) {
  if (c->bestS) {
    VAME_HIP(hipDeviceSynchronize());  // no launch may still use the old buffer
    VAME_HIP(hipFree(c->bestS));
    c->bestS = nullptr;
  }
  c->bestPending = false;
  const size_t words = best_layout(c, pairs, c->bestOff);
  if (hipMalloc(&c->bestS, words * sizeof(int32_t)) != hipSuccess) {
    (void)hipGetLastError();
    c->bestS = nullptr;
    return VAME_E_NOMEM;
  }
  c->maxPairs = pairs;
  return VAME_OK;
}

void fill_common(KParams& kp, const vame_ctx* c, int extra) {
  kp.W = c->W;
  kp.H = c->H;
  kp.nCtus = c->nCtus;
  kp.ctusPerRow = c->ctusPerRow;
  kp.extra = extra;
}

// Per-kernel timing (vame_set_timing(ctx, 1)): the kernel's own dispatch
// packet carries the start / stop events (hipExtLaunchKernel), so timing adds
// no marker packets to the streams and the interval is the dispatch's own
// execution, as rocprofv3 reports it (timed dispatches still cost ~0.8 % of a
// c2 step, with or without the events' system-scope fence, as did the event
// records around each launch used before).  Returns the (start, stop) pair for the
// next launch of kernel class `cls`, or nulls with timing off.
int time_events(vame_ctx* c, int cls, hipEvent_t& start, hipEvent_t& stop) {
  start = stop = nullptr;
  if (!((c->timing >> cls) & 1)) return VAME_OK;
  auto& v = c->ev[cls];
  if (c->evUsed[cls] == v.size()) {
    std::pair<hipEvent_t, hipEvent_t> e;
    VAME_HIP(hipEventCreate(&e.first));
    VAME_HIP(hipEventCreate(&e.second));
    v.push_back(e);
  }
  start = v[c->evUsed[cls]].first;
  stop = v[c->evUsed[cls]].second;
  c->evUsed[cls]++;
  return VAME_OK;
}

// Makes c->device current for one C-ABI call and restores the caller's device
// on every return path: the entry points must not change the calling thread's
// current device (a torch thread holding engines on two GPUs would otherwise
// see torch.cuda.current_device() move under it).
struct DeviceGuard {
  int prev = -1;
  hipError_t err;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int now = -1;
    if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
  }
};

#define VAME_TRY(x)        \
  do {                     \
    int rc_ = (x);         \
    if (rc_) return rc_;   \
  } while (0)

// Block order (affine_me_body): groups of about c->groupCombos (ctu, pair)
// combinations, whose tiles and original samples the XCDs' L2s hold while
// every item of a CTU passes -- the 3 pairs of a 1080p 2-frame step, or one
// chunk of CTU rows of one 2160p pair -- and within a group, the (ctu, pair)
// combinations of each template item in slots padded to a multiple of 8 per
// (pair, chunk), so every item of a CTU lands on the same XCD (padding blocks
// exit at once).  Returns the grid size.
unsigned block_grid(const vame_ctx* c, int cls, KParams& k) {
  k.order = c->dOrder[cls];
  k.nChunks = c->nChunks[cls];
  k.cpp = c->cpp[cls];
  k.groupPairs = k.nChunks > 1 ? 1 : std::max(1, std::min(k.nPairs, c->groupCombos[cls] / k.cpp));
  k.groupPer = k.groupPairs * k.cpp;
  const int groups = (k.nPairs + k.groupPairs - 1) / k.groupPairs * k.nChunks;
  return (unsigned)(groups * k.nItems * k.groupPer);
}

// The slot -> CTU table of the block order: the frame's CTU rows cut into
// chunks of at most groupCombos CTUs; within a chunk the CTUs in raster order,
// padded to a multiple of 8 slots, so slot j runs on XCD j % 8 (workgroups
// are dealt round-robin over the XCDs) and raster neighbours sit on different
// XCDs: the per-XCD load follows the frame's content evenly.  (Runs of
// adjacent CTUs per XCD and compact per-XCD strips measured slower or equal:
// HISTORY.md.)
std::vector<int32_t> build_order(int nCtus, int cols, int groupCombos, int& nChunks, int& cpp) {
  const int rows = nCtus / cols;
  nChunks = (nCtus + groupCombos - 1) / groupCombos;
  const int rowsPer = (rows + nChunks - 1) / nChunks;
  nChunks = (rows + rowsPer - 1) / rowsPer;
  cpp = (rowsPer * cols + 7) / 8 * 8;
  std::vector<int32_t> order((size_t)nChunks * cpp, -1);
  for (int ch = 0; ch < nChunks; ch++) {
    const int r0 = ch * rowsPer, r1 = std::min(rows, r0 + rowsPer);
    int32_t* o = order.data() + (size_t)ch * cpp;
    for (int k = 0; k < (r1 - r0) * cols; k++) o[k] = r0 * cols + k;
  }
  return order;
}

// The kernel instance of a launch mode (vame_kernel.h MODE: 1 = 2-CP only,
// 2 = 3-CP only, 3 = 2-CP then 3-CP).
using KernelFn = void (*)(KParams);
// the 128x64 and 64x128 CUs in one launch (affine_me_half2) in 2-CP-only
// launches (c2 0.883 vs 0.888 ms), affine_me_half2w then affine_me_half2h in
// the others (c4 290.9 vs 292.5 ms: the merged kernel's two bodies spill 88 vs
// 20 B per lane), profiles/r06_quad2_ab.txt.  Timing builds: VAME_HALF_MERGE=2
// merged in every mode, 0 in none.
#ifndef VAME_HALF_MERGE
#define VAME_HALF_MERGE 1
#endif
inline bool half_merged(int mode) { return VAME_HALF_MERGE == 2 || (VAME_HALF_MERGE == 1 && mode == 1); }

template <int KIND>
KernelFn kernel_for(int mode) {
  if constexpr (KIND == kKindHalf2W) {
    return mode == 1 ? affine_me_half2w<1> : mode == 2 ? affine_me_half2w<2> : affine_me_half2w<3>;
  } else if constexpr (KIND == kKindHalf2H) {
    return mode == 1 ? affine_me_half2h<1> : mode == 2 ? affine_me_half2h<2> : affine_me_half2h<3>;
  } else if constexpr (KIND == kKindCtu2) {
    return mode == 1 ? affine_me_ctu2<1> : mode == 2 ? affine_me_ctu2<2> : affine_me_ctu2<3>;
  } else if constexpr (KIND == kKindQuad2) {
    return mode == 1 ? affine_me_quad2<1> : mode == 2 ? affine_me_quad2<2> : affine_me_quad2<3>;
  } else if constexpr (KIND == kKindHalf2W + 100) {  // both orientations (affine_me_half2)
    if constexpr (VAME_HALF_MERGE == 2)
      return mode == 1 ? affine_me_half2<1> : mode == 2 ? affine_me_half2<2> : affine_me_half2<3>;
    else
      return mode == 1 ? affine_me_half2<1> : nullptr;  // half_merged(): 2-CP-only launches
  } else if constexpr (KIND == kKindCtu) {  // PROF only
    return mode == 1 ? affine_me_ctu_prof<1> : mode == 2 ? affine_me_ctu_prof<2> : affine_me_ctu_prof<3>;
  } else if constexpr (KIND == kKindHalf) {  // PROF only
    return mode == 1 ? affine_me_half_prof<1> : mode == 2 ? affine_me_half_prof<2> : affine_me_half_prof<3>;
  } else {
    return mode == 1 ? affine_me_quad<1> : mode == 2 ? affine_me_quad<2> : affine_me_quad<3>;
  }
}
KernelFn quad_kernel(bool prof, int mode) {
  if (prof) return mode == 1 ? affine_me_quad_prof<1> : mode == 2 ? affine_me_quad_prof<2> : affine_me_quad_prof<3>;
  return kernel_for<kKindQuad>(mode);
}

// Launch one kernel: with the dispatch-carried timing events and AQL flags, or
// (the caller's stream under capture) as a plain launch, which the graph records.
template <typename K>
hipError_t launch_kernel(K kernel, unsigned grid, unsigned threads, hipStream_t s, hipEvent_t t0, hipEvent_t t1,
                         int flags, const KParams& kp, bool capture) {
  if (grid == 0) return hipSuccess;  // no work items (a kernel class without CUs)
  if (capture)
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, kp);
  else
    hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, t0, t1, flags, kp);
  return hipGetLastError();
}


// where affine_me_quad runs beside the 128-class kernels (VAME_Q1_SIDE
// timing builds: 1 = after affine_me_quad2 on the quadrant stream)
#ifndef VAME_Q1_SIDE
#define VAME_Q1_SIDE 0
#endif
constexpr bool kQ1Side = VAME_Q1_SIDE == 1;  // 2: on a second side stream
// The quadrant kernels, by launch mode (default, VAME_SPLIT=3, vame_kernel.h
// kQuadMerged): a 2-CP-only launch runs one affine_me_quad kernel over the
// SBL1 and SBL2 items (the short c2 step needs the two kinds of items side by
// side: c2 0.889 vs 0.953 ms as two kernels), a 2+3-CP launch the SBL2 items
// in affine_me_quad2 on the quadrant stream beside affine_me_quad with the
// SBL1 items on the caller's stream (c4 291.3 vs 298.8 ms in one kernel, whose
// two bodies spill more: 104 vs 28 B per lane), profiles/r06_quad2_ab.txt.
// Timing builds: 2 / 1 one structure for every mode, 0 every quadrant CU one
// sub-block per lane (the packing of rounds 4-5, which PROF keeps).

// The launches of one call.  By default (VAME_STREAMS=2) the 128-class
// kernels run on the caller's stream and the quadrant kernel on a side stream
// forked from it: the 128-class workgroups, issued first and ahead of the
// fork's cross-stream hop, take their CUs before the quadrant workgroups fill
// the GPU, and the quadrant workgroups then fill the room beside them (a
// 512-thread affine_me_ctu2 workgroup leaves a CU room for two quadrant
// workgroups, a 256-thread half2 one for three).  Kernels of one stream run
// one after the other, so only separate streams overlap them.  The launches
// of one batch (maxPairs pairs each) fork once and join once: launch k + 1's
// kernels follow launch k's on their own streams.  Under capture (the
// caller's stream is being captured into a graph) the fork and join are
// events, the graph's edges.
int launch_direct(vame_ctx* c, const std::vector<KParams>& kps, bool quadFull, bool quadHalf, bool bigItems,
                  hipStream_t stream, bool capture) {
  if (VAME_ABLATE & 16) bigItems = false;  // timing-only builds
  if (VAME_ABLATE & 32) quadFull = quadHalf = false;
  if (kps.empty()) return VAME_OK;
  const int mode = (kps[0].run2 ? 1 : 0) | (kps[0].run3 ? 2 : 0);  // the kernel instance (MODE)
  if (mode == 0) return VAME_OK;
  const bool fork = c->streams == 2 && bigItems && (quadFull || quadHalf);
  const hipStream_t sQuad = fork ? c->side : stream;
  if (fork && !c->side) return VAME_E_INVALID;
  int issued = 0;  // VAME_STREAMS=1: kernels after a call's first may start before it ends
  auto order_flag = [&]() { return c->streams == 1 && issued++ > 0 ? hipExtAnyOrderLaunch : 0; };
  const bool valueSync = c->valueSync != 0 && c->syncWord && !capture;
  auto events = [&](int cls, hipEvent_t& t0, hipEvent_t& t1) -> int {
    t0 = t1 = nullptr;
    return capture ? VAME_OK : time_events(c, cls, t0, t1);
  };
  auto join = [&]() -> int {
    if (valueSync) {
      const uint32_t v = ++c->joinSeq;
      VAME_HIP(hipStreamWriteValue32(c->side, c->syncWord, v, 0));
      VAME_HIP(hipStreamWaitValue32(stream, c->syncWord, v, hipStreamWaitValueGte, 0xFFFFFFFFu));
    } else {
      VAME_HIP(hipEventRecord(c->evJoin, c->side));
      VAME_HIP(hipStreamWaitEvent(stream, c->evJoin, 0));
    }
    if (c->side2) {
      VAME_HIP(hipEventRecord(c->evJoin2, c->side2));
      VAME_HIP(hipStreamWaitEvent(stream, c->evJoin2, 0));
    }
    return VAME_OK;
  };
  if (fork) {
    VAME_HIP(hipEventRecord(c->evFork, stream));
    VAME_HIP(hipStreamWaitEvent(c->side, c->evFork, 0));
    if (c->side2) VAME_HIP(hipStreamWaitEvent(c->side2, c->evFork, 0));
  }
  // the 128x128 CUs: affine_me_ctu2 (two sub-blocks per lane), under PROF
  // affine_me_ctu_prof
  auto big = [&](const KParams& kp) -> int {
    KParams kb = kp;
    kb.items = c->dBig1;
    kb.nItems = c->nBig1;
    kb.bestS = c->bestS + c->bestOff[0];
    const unsigned grid = block_grid(c, 1, kb);
    hipEvent_t t0, t1;
    if (c->prof) {
      VAME_TRY(events(1, t0, t1));
      VAME_HIP(launch_kernel(kernel_for<kKindCtu>(mode), grid, Cfg<kKindCtu>::THREADS, stream, t0, t1,
                             order_flag(), kb, capture));
    } else {
      VAME_TRY(events(3, t0, t1));
      VAME_HIP(launch_kernel(kernel_for<kKindCtu2>(mode), grid, Cfg<kKindCtu2>::THREADS, stream, t0, t1,
                             order_flag(), kb, capture));
    }
    return VAME_OK;
  };
  // then the 128x64 and 64x128 CUs: affine_me_half2w / _half2h, under PROF
  // affine_me_half_prof
  auto half = [&](const KParams& kp) -> int {
    if (c->prof) {
      KParams kh = kp;
      kh.items = c->dHalf;
      kh.nItems = c->nHalf;
      const unsigned grid = block_grid(c, 1, kh);
      hipEvent_t t0, t1;
      VAME_TRY(events(2, t0, t1));
      VAME_HIP(launch_kernel(kernel_for<kKindHalf>(mode), grid, Cfg<kKindHalf>::THREADS, stream, t0, t1,
                             order_flag(), kh, capture));
      return VAME_OK;
    }
    if (half_merged(mode)) {  // one launch over both orientations: dHalfW then dHalfH, adjacent
      KParams kh = kp;
      kh.items = c->dHalfW;
      kh.nItems = c->nHalfW + c->nHalfH;
      kh.bestS = c->bestS + c->bestOff[1];  // [pair, CTU, item of 4]: the two regions' span
      const unsigned grid = block_grid(c, 1, kh);
      hipEvent_t t0, t1;
      VAME_TRY(events(4, t0, t1));
      VAME_HIP(launch_kernel(kernel_for<kKindHalf2W + 100>(mode), grid, Cfg<kKindHalf2W>::THREADS, stream, t0,
                             t1, order_flag(), kh, capture));
      return VAME_OK;
    }
    for (int o = 0; o < 2; o++) {
      KParams kh = kp;
      kh.items = o ? c->dHalfH : c->dHalfW;
      kh.nItems = o ? c->nHalfH : c->nHalfW;
      kh.bestS = c->bestS + c->bestOff[1 + o];
      const unsigned grid = block_grid(c, 1, kh);
      hipEvent_t t0, t1;
      VAME_TRY(events(4 + o, t0, t1));
      VAME_HIP(launch_kernel(o ? kernel_for<kKindHalf2H>(mode) : kernel_for<kKindHalf2W>(mode), grid,
                             Cfg<kKindHalf2W>::THREADS, stream, t0, t1, order_flag(), kh, capture));
    }
    return VAME_OK;
  };
  // the quadrant items: set 0 (affine_me_quad), 1 (affine_me_quad2) or, under
  // PROF, 2 (every quadrant CU in affine_me_quad_prof)
  const int aset = quadFull && quadHalf ? 2 : quadFull ? 0 : 1;
  auto quad = [&](const KParams& kp, int set, hipStream_t s) -> int {
    KParams kq = kp;
    kq.items = c->dQuad + c->quadOff[set][aset];
    kq.nItems = c->quadN[set][aset];
    kq.bestS = c->bestS + c->bestOff[3];
    const unsigned grid = block_grid(c, 0, kq);
    hipEvent_t t0, t1;
    VAME_TRY(events(set == 1 ? 6 : 0, t0, t1));
    if (set == 1)
      VAME_HIP(launch_kernel(kernel_for<kKindQuad2>(mode), grid, Cfg<kKindQuad2>::THREADS, s, t0, t1, order_flag(),
                             kq, capture));
    else
      VAME_HIP(launch_kernel(quad_kernel(c->prof, mode), grid, Cfg<kKindQuad>::THREADS, s, t0, t1, order_flag(),
                             kq, capture));
    return VAME_OK;
  };
  const bool anyQuad = quadFull || quadHalf;
  // the split packing: affine_me_quad2 on the quadrant stream, affine_me_quad
  // after the 128-class kernels on the caller's stream (one stream: both
  // quadrant kernels first)
  const bool kSplit = VAME_SPLIT == 1 || (VAME_SPLIT == 3 && mode != 1);  // the SBL2 items apart
  auto quads = [&](const KParams& kp, hipStream_t s1) -> int {
    if (c->prof || VAME_SPLIT == 0) return quad(kp, 2, sQuad);
    if (!kSplit) return quad(kp, 3, sQuad);
    VAME_TRY(quad(kp, 1, sQuad));
    if (s1 == sQuad || !fork) VAME_TRY(quad(kp, 0, s1));
    return VAME_OK;
  };
  auto all = [&]() -> int {
    for (const KParams& kp : kps) {
      if (!fork && anyQuad) VAME_TRY(quads(kp, stream));  // one stream: the quadrant kernels first
      if (bigItems) {
        VAME_TRY(big(kp));
        VAME_TRY(half(kp));
      }
      if (fork) {
        VAME_TRY(quads(kp, kQ1Side ? sQuad : stream));
        if (!kQ1Side && !c->prof && kSplit) VAME_TRY(quad(kp, 0, c->side2 ? c->side2 : stream));
      }
    }
    return fork ? join() : VAME_OK;
  };
  const int rc = all();
  if (rc != VAME_OK && fork) {
    // a launch failed after earlier kernels went to the side stream: order
    // them before the caller's stream anyway, so the caller never frees or
    // reuses result buffers they still write (best effort, the first error is
    // the one reported)
    (void)join();
  }
  return rc;
}

int launch(vame_ctx* c, const std::vector<KParams>& kps, bool quadFull, bool quadHalf, bool bigItems,
           hipStream_t stream) {
  if (kps.empty()) return VAME_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  VAME_HIP(hipStreamIsCapturing(stream, &cs));
  if (cs == hipStreamCaptureStatusInvalidated) return VAME_E_INVALID;
  const bool capture = cs == hipStreamCaptureStatusActive;
  // the seed-reuse sums (allocated with the context): one buffer per context,
  // so a call on another stream than the last user's waits for it first
  const bool useBest = !c->prof && kps[0].run2 && kps[0].run3;  // quad2 and the 128-class kernels
  if (useBest && !c->bestS) return VAME_E_NOMEM;
  if (useBest && !capture && c->bestPending && c->bestStream != stream)
    VAME_HIP(hipStreamWaitEvent(stream, c->bestEv, 0));
  const int rc = launch_direct(c, kps, quadFull, quadHalf, bigItems, stream, capture);
  if (useBest && !capture) {
    VAME_HIP(hipEventRecord(c->bestEv, stream));  // after the join: every kernel of the call
    c->bestStream = stream;
    c->bestPending = true;
  }
  return rc;
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
  DeviceGuard guard(device);
  VAME_HIP(guard.err);
  std::vector<Item> big1, hf, bigP, hfP;
  QuadSet qs[4];  // SBL1 items, SBL2 items; the PROF packing; the product's merged set
  build_templates(big1, hf, qs[0], &qs[1]);
  build_templates(bigP, hfP, qs[2], nullptr);
  // one affine_me_quad launch over both: the cooperative (64x64) items first,
  // then the SBL2 items, then the 16-sub-block items (the shortest last)
  for (int a = 0; a < 3; a++) {
    const std::vector<Item>& v1 = a == 0 ? qs[0].full : a == 1 ? qs[0].half : qs[0].both;
    const std::vector<Item>& v2 = a == 0 ? qs[1].full : a == 1 ? qs[1].half : qs[1].both;
    std::vector<Item>& m = a == 0 ? qs[3].full : a == 1 ? qs[3].half : qs[3].both;
    for (const Item& it : v1)
      if (it.coop & 1) m.push_back(it);
    m.insert(m.end(), v2.begin(), v2.end());
    for (const Item& it : v1)
      if (!(it.coop & 1)) m.push_back(it);
  }
  std::vector<Item> hfw, hfh;  // the single-CU half items by orientation
  for (const Item& it : hf) (it.cu[0].lw > it.cu[0].lh ? hfw : hfh).push_back(it);
  // the kernels index bestS by these counts (best_layout); the templates hold
  // one 128x128 item and two of each orientation
  if (big1.size() != 1 || (!(VAME_ABLATE & 256) && (hfw.size() != 2 || hfh.size() != 2))) return VAME_E_INVALID;
  vame_ctx* c = new vame_ctx();
  c->device = device;
  c->W = width;
  c->H = height;
  c->nCtus = nCtus;
  c->ctusPerRow = (width + kCtu - 1) / kCtu;  // T8: integer ceil
  c->nBig1 = (int)big1.size();
  c->nHalf = (int)hf.size();
  c->nHalfW = (int)hfw.size();
  c->nHalfH = (int)hfh.size();
  std::vector<Item> quad;  // [set][FULL | HALF | both alignments]
  for (int k = 0; k < 4; k++)
    for (int a = 0; a < 3; a++) {
      const std::vector<Item>& v = a == 0 ? qs[k].full : a == 1 ? qs[k].half : qs[k].both;
      c->quadOff[k][a] = (int)quad.size();
      c->quadN[k][a] = (int)v.size();
      quad.insert(quad.end(), v.begin(), v.end());
    }
  // the runtime knobs (include/vame.h; results are bit-identical under every
  // setting, the defaults are the measured best)
  c->streams = env_int("VAME_STREAMS", 2) == 1 ? 1 : 2;
  c->valueSync = env_int("VAME_SYNC", 1) != 0 ? 1 : 0;
  c->groupCombos[0] = c->groupCombos[1] = std::max(8, env_int("VAME_GROUP_COMBOS", 408));
  hipError_t e = hipSuccess;
  auto upload = [&](Item*& d, const std::vector<Item>& v) {
    if (e == hipSuccess && !v.empty()) e = hipMalloc(&d, v.size() * sizeof(Item));
    if (e == hipSuccess && !v.empty()) e = hipMemcpy(d, v.data(), v.size() * sizeof(Item), hipMemcpyHostToDevice);
  };
  upload(c->dQuad, quad);
  upload(c->dBig1, big1);
  upload(c->dHalf, hf);
  {  // the 128x64 items, then the 64x128 ones, adjacent (affine_me_half2 runs both)
    std::vector<Item> hwh(hfw);
    hwh.insert(hwh.end(), hfh.begin(), hfh.end());
    upload(c->dHalfW, hwh);
    if (c->dHalfW) c->dHalfH = c->dHalfW + hfw.size();
  }
  for (int k = 0; k < 2 && e == hipSuccess; k++) {
    const std::vector<int32_t> order = build_order(nCtus, c->ctusPerRow, c->groupCombos[k], c->nChunks[k], c->cpp[k]);
    e = hipMalloc(&c->dOrder[k], order.size() * sizeof(int32_t));
    if (e == hipSuccess)
      e = hipMemcpy(c->dOrder[k], order.data(), order.size() * sizeof(int32_t), hipMemcpyHostToDevice);
  }
  // the side stream the default launch structure uses, created here, not
  // during a launch (a launch may be under stream capture): a process has
  // GPU_MAX_HW_QUEUES = 4 hardware queues and HIP shares them between its
  // streams beyond that, so an idle stream created here could put the
  // caller's own copy streams on the quadrant kernel's queue (the CLI's
  // compute, upload and download streams + the side stream are four)
  if (e == hipSuccess && c->streams == 2) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  if (e == hipSuccess && c->streams == 2 && VAME_SPLIT != 2 && VAME_Q1_SIDE == 2)
    e = hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->evJoin, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->evJoin2, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->evFork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->bestEv, hipEventDisableTiming);
  if (e == hipSuccess && c->valueSync) {
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&c->syncWord), 8, hipMallocSignalMemory) != hipSuccess ||
        hipMemset(c->syncWord, 0, 8) != hipSuccess) {
      (void)hipGetLastError();
      if (c->syncWord) (void)hipFree(c->syncWord);
      c->syncWord = nullptr;
      c->valueSync = 0;  // events instead
    }
  }
  if (e != hipSuccess) {
    snprintf(g_hip_err, sizeof(g_hip_err), "%s", hipGetErrorString(e));
    vame_destroy(c);
    return VAME_E_DEVICE;
  }
  // the seed-reuse sums for kMaxPairs pairs per launch (vame_set_max_pairs
  // resizes them): ~1 GB at 3840x2160, 260 MB at 1920x1080
  const int rc = alloc_best(c, kMaxPairs);
  if (rc != VAME_OK) {
    vame_destroy(c);
    return rc;
  }
  *out = c;
  return VAME_OK;
}

int vame_set_max_pairs(vame_ctx* c, int max_pairs) {
  if (!c || max_pairs < 1 || max_pairs > kMaxPairs) return VAME_E_INVALID;
  if (max_pairs == c->maxPairs && c->bestS) return VAME_OK;
  DeviceGuard guard(c->device);
  VAME_HIP(guard.err);
  return alloc_best(c, max_pairs);
}

int vame_get_max_pairs(vame_ctx* c) { return c ? c->maxPairs : VAME_E_INVALID; }

void vame_destroy(vame_ctx* c) {
  if (!c) return;
  DeviceGuard guard(c->device);
  for (Item* d : {c->dQuad, c->dBig1, c->dHalf, c->dHalfW})  // dHalfH lies inside dHalfW's block
    if (d) (void)hipFree(d);
  if (c->bestS) (void)hipFree(c->bestS);
  for (int k = 0; k < 2; k++)
    if (c->dOrder[k]) (void)hipFree(c->dOrder[k]);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->side2) (void)hipStreamDestroy(c->side2);
  for (hipEvent_t e : {c->evJoin, c->evJoin2, c->evFork, c->bestEv, c->packEv})
    if (e) (void)hipEventDestroy(e);
  if (c->syncWord) (void)hipFree(c->syncWord);
  if (c->dPackSegs) (void)hipFree(c->dPackSegs);
  for (int k = 0; k < kTimingClasses; k++)
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
  DeviceGuard guard(c->device);
  VAME_HIP(guard.err);
  KParams kp;
  memset(&kp, 0, sizeof(kp));
  fill_common(kp, c, extra);
  kp.pair[0].cur = cur;
  kp.pair[0].ref = ref;
  kp.pair[0].lambda = lambda;
  kp.nPairs = 1;
  kp.run2 = nCP == 2;
  kp.run3 = nCP == 3;
  const int mode = align * 2 + (nCP - 2);
  kp.pair[0].cost[mode] = cost;
  kp.pair[0].cpmv[mode] = reinterpret_cast<vame_cpmvs_dev*>(cpmvs);
  kp.prev[align] = reinterpret_cast<const vame_cpmvs_dev*>(prev);
  return launch(c, std::vector<KParams>{kp}, align == 0, align == 1, align == 0, (hipStream_t)stream);
}

int vame_template_coverage(int half128, int align, int32_t* hits, int32_t* items3) {
  if (!hits || (align != 0 && align != 1) || half128 == 0) return VAME_E_INVALID;
  std::vector<Item> big, hf, bigP, hfP;
  QuadSet q1, q2, qp;
  build_templates(big, hf, q1, &q2);
  build_templates(bigP, hfP, qp, nullptr);
  // the split packing (affine_me_quad + affine_me_quad2) and the PROF packing
  // must each cover alike
  std::vector<Item> qf(q1.full), qh(q1.half), qb(q1.both);
  qf.insert(qf.end(), q2.full.begin(), q2.full.end());
  qh.insert(qh.end(), q2.half.begin(), q2.half.end());
  qb.insert(qb.end(), q2.both.begin(), q2.both.end());
  for (const std::vector<Item>* pv : {&qp.full, &qp.half, &qp.both}) {
    std::vector<int32_t> a((size_t)(align ? kHalfCusPerCtu : kFullCusPerCtu), 0),
        b((size_t)(align ? kHalfCusPerCtu : kFullCusPerCtu), 0);
    const std::vector<Item>& split = pv == &qp.full ? qf : pv == &qp.half ? qh : qb;
    for (int k = 0; k < 2; k++)
      for (const Item& it : k ? split : *pv)
        for (int i = 0; i < it.nCu; i++)
          if (it.cu[i].lw != 0 && it.cu[i].align == align) (k ? b : a)[it.cu[i].outOff]++;
    if (a != b) return VAME_E_INVALID;
  }
  const int n = align ? kHalfCusPerCtu : kFullCusPerCtu;
  // the one-alignment item set and the both-alignment one must cover alike
  std::vector<int32_t> both(n, 0);
  for (int i = 0; i < n; i++) hits[i] = 0;
  for (const auto* v : {&big, &hf, &qf, &qh, &qb})
    for (const Item& it : *v)
      for (int k = 0; k < it.nCu; k++) {
        const CuSlot& s = it.cu[k];
        if (s.lw == 0 || s.align != align) continue;  // lw 0: an unused slot
        if (s.outOff >= n) return VAME_E_INVALID;
        (v == &qb ? both[s.outOff] : hits[s.outOff])++;
      }
  for (const auto* v : {&big, &hf})
    for (const Item& it : *v)
      for (int k = 0; k < it.nCu; k++)
        if (it.cu[k].lw != 0 && it.cu[k].align == align) both[it.cu[k].outOff]++;
  for (int i = 0; i < n; i++)
    if (both[i] != hits[i]) return VAME_E_INVALID;
  if (items3) {
    items3[0] = (int32_t)qb.size();  // affine_me_quad + affine_me_quad2 items of a both-alignment launch
    items3[1] = (int32_t)big.size();
    items3[2] = (int32_t)hf.size();
  }
  return VAME_OK;
}

int vame_pred_mask(int mode_mask) {
  const int ncp = (mode_mask & VAME_MODE_3CP) ? 3 : 1;  // 2CP [+ 3CP] per alignment
  const int sel = (mode_mask >> 2) & 3;                  // neither selection bit: both
  return ((sel == 0 || (sel & 1)) ? ncp : 0) | ((sel == 0 || (sel & 2)) ? ncp << 2 : 0);
}

int vame_affine_me_batch(vame_ctx* c, const vame_poc_job* jobs, int njobs, int mode_mask,
                         int extra, void* stream) {
  if (!c || !jobs || njobs < 1) return VAME_E_INVALID;
  if (!(mode_mask & VAME_MODE_2CP) || (mode_mask & ~15) || extra < 0 || extra > 64)
    return VAME_E_INVALID;
  const bool run3 = (mode_mask & VAME_MODE_3CP) != 0;
  const int preds = vame_pred_mask(mode_mask);  // alignment selection: only those items launch
  const bool doFull = (preds & 1) != 0, doHalf = (preds & 4) != 0;
  for (int j = 0; j < njobs; j++) {
    const vame_poc_job& jb = jobs[j];
    if (!jb.cur || !jb.refs || !jb.out || jb.nrefs < 1) return VAME_E_INVALID;
    if (jb.nrefs > 4) return VAME_E_UNSUPPORTED;
    for (int r = 0; r < jb.nrefs; r++) {
      if (!jb.refs[r]) return VAME_E_INVALID;
      for (int m = 0; m < 4; m++) {
        const bool need = ((preds >> m) & 1) != 0;
        if (need && (!jb.out->cost[r][m] || !jb.out->cpmvs[r][m])) return VAME_E_INVALID;
      }
    }
  }
  DeviceGuard guard(c->device);
  VAME_HIP(guard.err);
  // every (POC, refIdx) pair of the batch, maxPairs per launch
  std::vector<KParams> kps;
  KParams kp;
  memset(&kp, 0, sizeof(kp));
  fill_common(kp, c, extra);
  kp.run2 = 1;
  kp.run3 = run3;
  for (int j = 0; j < njobs; j++) {
    const vame_poc_job& jb = jobs[j];
    for (int r = 0; r < jb.nrefs; r++) {
      PairArgs& pa = kp.pair[kp.nPairs++];
      pa.cur = jb.cur;
      pa.ref = jb.refs[r];
      pa.lambda = jb.lambda;
      for (int m = 0; m < 4; m++) {
        pa.cost[m] = jb.out->cost[r][m];
        pa.cpmv[m] = reinterpret_cast<vame_cpmvs_dev*>(jb.out->cpmvs[r][m]);
      }
      const bool last = j == njobs - 1 && r == jb.nrefs - 1;
      if (kp.nPairs == c->maxPairs || last) {
        kps.push_back(kp);
        kp.nPairs = 0;
      }
    }
  }
  return launch(c, kps, doFull, doHalf, doFull, (hipStream_t)stream);
}

int vame_affine_me_poc(vame_ctx* c, const uint16_t* cur, const uint16_t* const* refs, int nrefs,
                       float lambda, int mode_mask, int extra, const vame_poc_result* out,
                       void* stream) {
  if (!out) return VAME_E_INVALID;
  const vame_poc_job job{cur, refs, nrefs, lambda, out};
  return vame_affine_me_batch(c, &job, 1, mode_mask, extra, stream);
}

int vame_pack_records(vame_ctx* c, const vame_poc_job* jobs, int njobs, int mode_mask, int32_t* slab,
                      long long words, int32_t* bad, void* stream) {
  if (!c || !jobs || njobs < 0 || !slab || !bad || words < 0) return VAME_E_INVALID;
  if (!(mode_mask & VAME_MODE_2CP) || (mode_mask & ~15)) return VAME_E_INVALID;
  const int preds = vame_pred_mask(mode_mask);
  DeviceGuard guard(c->device);
  VAME_HIP(guard.err);
  // the previous pack kernel read the device table (and the upload the host
  // one): both are rewritten below
  if (c->packEv) VAME_HIP(hipEventSynchronize(c->packEv));
  std::vector<PackSeg>& segs = c->packSegs;
  segs.clear();
  long long off = 0;
  int maxn = 0;
  for (int j = 0; j < njobs; j++) {
    const vame_poc_job& jb = jobs[j];
    if (!jb.out || jb.nrefs < 1 || jb.nrefs > 4) return VAME_E_INVALID;
    for (int r = 0; r < jb.nrefs; r++)
      for (int m = 0; m < 4; m++) {
        if (!((preds >> m) & 1)) continue;
        if (!jb.out->cost[r][m] || !jb.out->cpmvs[r][m]) return VAME_E_INVALID;
        PackSeg sg;
        sg.cost = jb.out->cost[r][m];
        sg.cpmv = reinterpret_cast<const int32_t*>(jb.out->cpmvs[r][m]);
        sg.n = c->nCtus * ((m >> 1) ? kHalfCusPerCtu : kFullCusPerCtu);
        sg.ncp = (m & 1) ? 3 : 2;
        sg.off = off;
        off += (long long)sg.n * (1 + 2 * sg.ncp);
        maxn = std::max(maxn, sg.n);
        segs.push_back(sg);
      }
  }
  if (off > words) return VAME_E_INVALID;
  hipStream_t s = (hipStream_t)stream;
  if (!c->packEv) VAME_HIP(hipEventCreateWithFlags(&c->packEv, hipEventDisableTiming));
  if (segs.size() > c->dPackCap) {
    if (c->dPackSegs) VAME_HIP(hipFree(c->dPackSegs));
    c->dPackSegs = nullptr;
    c->dPackCap = 0;
    VAME_HIP(hipMalloc(&c->dPackSegs, segs.size() * sizeof(PackSeg)));
    c->dPackCap = segs.size();
  }
  if (!segs.empty()) {
    VAME_HIP(hipMemcpyAsync(c->dPackSegs, segs.data(), segs.size() * sizeof(PackSeg), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(pack_records_kernel, dim3((maxn + 255) / 256, (unsigned)segs.size()), dim3(256), 0, s,
                       c->dPackSegs, slab, bad);
    VAME_HIP(hipGetLastError());
    VAME_HIP(hipEventRecord(c->packEv, s));  // after the kernel: the next call waits for its table reads
  }
  if (words > off) VAME_HIP(hipMemsetAsync(slab + off, 0, (size_t)(words - off) * sizeof(int32_t), s));
  return VAME_OK;
}

int vame_set_prof(vame_ctx* c, int enable) {
  if (!c) return VAME_E_INVALID;
  c->prof = enable != 0;
  return VAME_OK;
}

int vame_set_timing(vame_ctx* c, int enable) {
  if (!c) return VAME_E_INVALID;
  // kernel classes timed (bit k: class k, see vame_ctx::timing): 2 = the
  // quadrant kernels (classes 0 and 6), any other non-zero value every class;
  // VAME_TIMING_KEEP (16) keeps the launches recorded so far (a caller timing
  // a sample of its steps toggles timing between them)
  const bool keep = (enable & VAME_TIMING_KEEP) != 0;
  enable &= ~VAME_TIMING_KEEP;
  c->timing = enable == 2 ? (1 | 64) : enable != 0 ? (1 << kTimingClasses) - 1 : 0;
  if (!keep)
    for (size_t& u : c->evUsed) u = 0;
  return VAME_OK;
}

int vame_get_timing(vame_ctx* c, int cls, double* total_ms, int* launches, int reset) {
  if (!c || cls < 0 || cls >= kTimingClasses || !total_ms || !launches) return VAME_E_INVALID;
  DeviceGuard guard(c->device);
  VAME_HIP(guard.err);
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

#if VAME_PHASE_TIMING
// profiling-only builds: per-phase shader-clock sums [kernel: quad, ctu, half,
// ctu2, half2w, half2h][kPhSlots] (see vame_kernel.h)
int vame_debug_phase_cycles(unsigned long long* out, int reset) {
  if (!out) return VAME_E_INVALID;
  VAME_HIP(hipDeviceSynchronize());
  VAME_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_cycles), sizeof(g_phase_cycles)));
  if (reset) {
    unsigned long long z[7 * kPhSlots] = {};
    VAME_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof(z)));
  }
  return VAME_OK;
}
#endif
#if VAME_COUNT_PRED
// instrumentation builds: sub-block predictions run, [quad, ctu], and those of
// them whose window left the staged tile, [2 + quad 2-CP, quad 3-CP, ctu 2-CP,
// ctu 3-CP], and of those the ones a 4 / 8 / 16 px wider margin would hold,
// [6 + quad x3, ctu x3], then the wave lane slots [12 + kernel], [14 + kernel],
// [16 + kernel] (see vame_kernel.h)
int vame_debug_pred_count(unsigned long long* out20, int reset) {
  if (!out20) return VAME_E_INVALID;
  VAME_HIP(hipDeviceSynchronize());
  VAME_HIP(hipMemcpyFromSymbol(out20, HIP_SYMBOL(g_pred_count), sizeof(unsigned long long) * 20));
  if (reset) {
    unsigned long long z[20] = {};
    VAME_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_pred_count), z, sizeof(z)));
  }
  return VAME_OK;
}
#endif
const char* vame_version(void) { return "vame 0.1 (gfx950)"; }

}  // extern "C"
