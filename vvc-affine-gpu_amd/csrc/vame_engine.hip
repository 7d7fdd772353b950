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

struct vame_ctx {
  int device, W, H, nCtus, ctusPerRow;
  // device-resident work-item templates: [quadFull | quadHalf] and the FULL
  // 128-class CUs in two packings: dBig3 -- the 128x128, 128x64 and 64x128
  // groups as 1024-thread CTU items (affine_me_ctu); or dBig1 (the 128x128
  // item) + dHalf (each 128x64 / 64x128 CU alone, affine_me_half)
  Item* dQuad = nullptr;
  Item* dBig3 = nullptr;
  Item* dBig1 = nullptr;
  Item* dBig2 = nullptr;  // dBig3 without the 128x128 item (that one runs in affine_me_ctu2)
  Item* dHalf = nullptr;
  Item* dHalfW = nullptr;  // dHalf's 128x64 / 64x128 items (affine_me_half2w / _half2h)
  Item* dHalfH = nullptr;
  int nQuadFull = 0, nQuadHalf = 0, nQuadBoth = 0, nBig3 = 0, nBig1 = 0, nBig2 = 0, nHalf = 0, nHalfW = 0,
      nHalfH = 0;
  // VAME_HALF2 (default 1): the 128x64 / 64x128 CUs of the half packing in
  // affine_me_half2w / _half2h (256 threads, two stacked sub-blocks per lane,
  // four workgroups per CU) instead of affine_me_half (512 threads, one per lane)
  bool half2 = true;
  // VAME_CTU2: where the 128x128 CUs run -- 2 (default): in affine_me_ctu2
  // (512 threads, two stacked sub-blocks per lane, two workgroups per CU,
  // room beside them for quadrant workgroups); 1: there in the launches that
  // use the half packing, in the CTU items in the others; 0: always in CTU
  // items.  The 3-CP seed-reuse sums of the two-sub-block kernels live in
  // bestS (allocated on first use)
  int ctu2 = 2;
  int32_t* bestS = nullptr;
  // which packing a launch uses (VAME_HALF128): 1 (default) always dBig1 +
  // dHalf (every 128x64 / 64x128 CU a workgroup of its own), 0 always dBig3
  // (1024-thread CTU items, a whole CU each), 2 dBig1 + dHalf for launches of
  // at least halfMinPairs (POC, refIdx) pairs (VAME_HALF_MIN_PAIRS, default
  // 16), dBig3 below.  With the quadrant kernel on its own stream the small
  // workgroups share CUs with it (c2 0.931 vs 0.987 ms)
  int halfMode = 1, halfMinPairs = 16;
  // VAME_QUAD_FIRST (one-stream mode, default 1): the quadrant kernel issued
  // first (it carries the call's barrier bit, the 128-class kernels follow it
  // in any order)
  bool quadFirst = true;
  // block order (block_grid), per kernel class (0 quadrant, 1 128-class):
  // slot -> CTU table, group size, CTU chunks, slots per (pair, chunk)
  int32_t* dOrder[2] = {nullptr, nullptr};
  int groupCombos[2] = {408, 408}, nChunks[2] = {1, 1}, cpp[2] = {0, 0};
  // side streams of a call (VAME_STREAMS > 1): [0] the quadrant kernel, [1]
  // / [2] the 128x64 / 64x128 kernels; forked from the caller's stream and
  // joined back into it
  hipStream_t side[3] = {nullptr, nullptr, nullptr};
  hipEvent_t evFork = nullptr, evJoin[3] = {nullptr, nullptr, nullptr};
  // VAME_SYNC (default 1): the joins as stream memory operations -- the side
  // stream writes a sequence number to a signal-memory word
  // (hipStreamWriteValue32, ordered after its earlier work), the caller's
  // stream waits for it (hipStreamWaitValue32) -- ~6 us per cross-stream hop
  // on MI355X against ~12 with an event record + hipStreamWaitEvent
  // (profiles/ubench/stream_hop.hip).  The fork stays an event: its slower
  // hop is the head start that lets the 128-class workgroups, issued on the
  // caller's stream, take their CUs before the quadrant kernel fills the GPU
  // (with the fork as a value too, VAME_SYNC=2, the c2 step takes 0.99 ms
  // instead of 0.935: the 128x128 kernel then waits for CUs until the
  // quadrant kernel ends).  0, words that cannot be allocated, or stream
  // capture (VAME_GRAPH): events.  syncWord[0] the fork, [1 + i] side stream
  // i's join.
  int valueSync = 1;
  bool quadAlt = false;  // VAME_QUAD_ALT (see launch_direct)
  bool halfFirst = false;  // VAME_HALF_FIRST=1: the 128x64 / 64x128 kernels before the 128x128 one
  uint32_t* syncWord[4] = {nullptr, nullptr, nullptr, nullptr};
  uint32_t forkSeq = 0, joinSeq[3] = {0, 0, 0};
  // optional per-kernel timing: (start, end) event pairs per kernel class
  // (0 quadrant, 1 CTU items, 2 128x64 / 64x128 CUs in affine_me_half, 3
  // 128x128 CUs in affine_me_ctu2, 4 / 5 128x64 / 64x128 CUs in
  // affine_me_half2w / _half2h)
  int timing = 0;
  // PROF on (vame_set_prof): the *_prof kernels
  bool prof = false;
  // VAME_JOIN_EACH=1: join the two streams after every launch of a batch
  bool joinEach = false;
  // Streams of a call (VAME_STREAMS).  Kernels of one stream run one after
  // the other on MI355X even without the AQL barrier bit
  // (hipExtAnyOrderLaunch: profiles/ubench/anyorder_overlap.hip, three 50-us
  // kernels take 155 us on one stream, ~90 on three), so the kernel classes
  // of a call go to streams of their own: 4 (default) -- the quadrant kernel
  // on side stream 0, the 128x128 CUs (affine_me_ctu2 / CTU items) on the
  // caller's stream, the 128x64 and 64x128 kernels on side streams 1 and 2;
  // 3 -- both of those on side stream 1; 2 -- every 128-class kernel on the
  // caller's stream; 1 -- every kernel on the caller's stream, all but the
  // call's first without the barrier bit.  The side streams fork from the
  // caller's stream and join back into it at the end of the call.
  int streams = 4;
  // VAME_GRAPH=1: a call's launch sequence (fork, kernels, join) is captured
  // once into a hipGraph (on capStream) and replayed on the caller's stream
  // whenever the same call -- the same kernel arguments -- repeats, e.g. the
  // bench's steps; calls with kernel timing on launch directly
  bool useGraph = false;
  hipStream_t capStream = nullptr;
  struct GraphEntry {
    std::vector<unsigned char> key;
    hipGraphExec_t exec;
  };
  std::vector<GraphEntry> graphs;  // most recent last, at most kMaxGraphs
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[6];
  size_t evUsed[6] = {0, 0, 0, 0, 0, 0};
  // vame_pack_records: the segment table of the last pack (host copy kept
  // until the next call) and its device copy
  std::vector<struct PackSeg> packSegs;
  struct PackSeg* dPackSegs = nullptr;
  size_t dPackCap = 0;
  hipEvent_t packEv = nullptr;  // the last table upload (the host table is rewritten after it)
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

// wave tasks per autonomous quadrant item (VAME_TASKS, 1..16)
int tasks_per_item() { return std::min(kMaxTasks, std::max(1, env_int("VAME_TASKS", 16))); }
static_assert(kFullCusPerCtu <= 512 && kHalfCusPerCtu <= 512, "CuSlot::outOff");
// one cooperative item per quadrant chaining its cooperative groups (VAME_CHAIN)
bool chain_coop() { return env_int("VAME_CHAIN", 1) != 0; }
// launches of both alignments use items mixing them (VAME_MIX)
bool mix_aligns() { return env_int("VAME_MIX", 1) != 0; }
// autonomous waves claim their next task from an LDS counter as they finish
// (VAME_CLAIM=0: wave w runs tasks w, w + 4, ...)
bool claim_tasks() { return env_int("VAME_CLAIM", 1) != 0; }

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

// Autonomous item: up to kMaxTasks wave tasks, each CUs of ONE size (<= 64
// sub-blocks, one lane per sub-block), so a task's segment size is uniform.
// Wave w runs task w, then (claim) the next unclaimed one as it finishes, or
// tasks w + 4, w + 8, ..., over the one staged tile: task t holds CU
// slots t * kTaskCu .. (its first slot carries the task's CU count and lanes
// per CU) and the running wave's prediction rows.  Unused slots stay zero
// (lw 0).
Item make_auto_item(int rx, int ry, const std::vector<std::vector<CuDesc>>& tasks, bool claim) {
  Item it;
  memset(&it, 0, sizeof(it));
  it.rx = (int16_t)rx;
  it.ry = (int16_t)ry;
  it.coop = claim ? 2 : 0;
  if (tasks.empty() || (int)tasks.size() > kMaxTasks) abort();
  it.nTasks = (int16_t)tasks.size();
  it.nCu = (int16_t)(tasks.size() * kTaskCu);
  for (size_t t = 0; t < tasks.size(); t++) {
    const int nsb = nsb_of(tasks[t][0]);
    const int n = (int)tasks[t].size();
    for (auto& c : tasks[t])
      if (nsb_of(c) != nsb) abort();
    if (n * nsb > 64 || nsb < 16 || n > kTaskCu) abort();  // the kernel's segment sums handle 16 / 32 / 64
    for (int i = 0; i < n; i++) set_slot(it.cu[t * kTaskCu + i], tasks[t][i]);
    it.cu[t * kTaskCu].taskCus = (uint8_t)n;
    it.cu[t * kTaskCu].taskLogL = (uint16_t)ilog2(nsb);
  }
  return it;
}

// CUs of one quadrant and one alignment, <= 64 sub-blocks: wave tasks of one
// size class (largest first), then items of `perItem` consecutive tasks.
void pack_autonomous(int qx, int qy, std::vector<CuDesc> cus, std::vector<Item>& out, int perItem) {
  std::stable_sort(cus.begin(), cus.end(),
                   [](const CuDesc& a, const CuDesc& b) { return nsb_of(a) > nsb_of(b); });
  std::vector<std::vector<CuDesc>> waves;
  for (auto& c : cus) {
    if (waves.empty() || nsb_of(waves.back()[0]) != nsb_of(c) ||
        (int)(waves.back().size() + 1) * nsb_of(c) > 64)
      waves.push_back({});
    waves.back().push_back(c);
  }
  for (size_t w = 0; w < waves.size(); w += perItem) {
    std::vector<std::vector<CuDesc>> grp(waves.begin() + w,
                                         waves.begin() + std::min(waves.size(), w + perItem));
    out.push_back(make_auto_item(qx, qy, grp, claim_tasks()));
  }
}

// Work-item templates (identical for every CTU):
//   big      : FULL 128x128 group (and, without `half`, the 128x64 / 64x128
//              groups), whole CTU, cooperative
//   half     : with `half`, each 128x64 / 64x128 CU alone, its own region
//              (affine_me_half, 512 threads)
//   quadFull : FULL groups <= 64x64 per 64x64 quadrant: 64x64 / 64x32 / 32x64
//              cooperative (one item chaining the three groups, or with
//              `chainCoop` off one item per group), the rest autonomous in
//              items of `tasks` wave tasks
//   quadHalf : HALF groups per quadrant (no HALF CU crosses a quadrant):
//              64x32 + 32x64 cooperative, the rest autonomous
//   quadBoth : the items of a launch of both alignments: with `mixed`, per
//              quadrant one cooperative chain of the FULL and HALF tasks and
//              autonomous items over both alignments' CUs; else quadFull +
//              quadHalf
void build_templates(std::vector<Item>& big, std::vector<Item>& halfItems, std::vector<Item>& quadFull,
                     std::vector<Item>& quadHalf, std::vector<Item>& quadBoth, bool half, int tasks,
                     bool chainCoop, bool mixed) {
  for (int g = 0; g < kFullGroups; g++) {
    const int w = kFullW[g], h = kFullH[g], n = (kCtu * kCtu) / (w * h), cols = kCtu / w;
    if (w == 128 || h == 128) {
      std::vector<CuDesc> c;
      for (int k = 0; k < n; k++) c.push_back({(k % cols) * w, (k / cols) * h, w, h, 0, kFullStride[g] + k});
      if ((VAME_ABLATE & 256) && w != h) continue;
      if (half && w != h) {
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
  std::vector<Item> bothCoop, bothAuto;
  std::vector<int> autoRank;  // an autonomous item's index within its quadrant
  for (int q = 0; q < 4; q++) {
    const int qx = (q & 1) * 64, qy = (q >> 1) * 64;
    auto inq = [&](int x, int y) { return x >= qx && x < qx + 64 && y >= qy && y < qy + 64; };
    std::vector<CuDesc> fullSmall, halfSmall, halfBig;
    std::vector<std::vector<CuDesc>> fullCoop;  // a task per group
    for (int g = 0; g < kFullGroups; g++) {
      const int w = kFullW[g], h = kFullH[g], n = (kCtu * kCtu) / (w * h), cols = kCtu / w;
      if (w == 128 || h == 128) continue;
      std::vector<CuDesc> c;
      for (int k = 0; k < n; k++) {
        const int x = (k % cols) * w, y = (k / cols) * h;
        if (inq(x, y)) c.push_back({x, y, w, h, 0, kFullStride[g] + k});
      }
      if (w * h / 16 <= 64)
        fullSmall.insert(fullSmall.end(), c.begin(), c.end());
      else
        fullCoop.push_back(c);
    }
    for (int g = 0; g < kHalfGroups; g++)
      for (int k = 0; k < kHalfN[g]; k++) {
        const int x = kHalfX8[g][k] * 8, y = kHalfY8[g][k] * 8;
        if (!inq(x, y)) continue;
        if (x + kHalfW[g] > qx + 64 || y + kHalfH[g] > qy + 64) abort();
        const CuDesc c{x, y, kHalfW[g], kHalfH[g], 1, kHalfStride[g] + k};
        (nsb_of(c) > 64 ? halfBig : halfSmall).push_back(c);
      }
    // cooperative tasks: one chained item, or an item per task
    auto coop = [&](const std::vector<std::vector<CuDesc>>& t, std::vector<Item>& out) {
      if (chainCoop)
        out.push_back(make_coop_item(qx, qy, t, Cfg<kKindQuad>::THREADS));
      else
        for (auto& cus : t) out.push_back(make_coop_item(qx, qy, cus, Cfg<kKindQuad>::THREADS));
    };
    coop(fullCoop, quadFull);
    pack_autonomous(qx, qy, fullSmall, quadFull, tasks);
    if (!halfBig.empty()) quadHalf.push_back(make_coop_item(qx, qy, halfBig, Cfg<kKindQuad>::THREADS));
    pack_autonomous(qx, qy, halfSmall, quadHalf, tasks);
    if (mixed) {  // both alignments in one item set: every quadrant's cooperative chain first
      std::vector<std::vector<CuDesc>> t(fullCoop);
      if (!halfBig.empty()) t.push_back(halfBig);
      coop(t, bothCoop);
      std::vector<CuDesc> small(fullSmall);
      small.insert(small.end(), halfSmall.begin(), halfSmall.end());
      const size_t n0 = bothAuto.size();
      pack_autonomous(qx, qy, small, bothAuto, tasks);
      for (size_t k = n0; k < bothAuto.size(); k++) autoRank.push_back((int)(k - n0));
    }
  }
  if (mixed) {
    quadBoth = bothCoop;
    // every quadrant's first (largest-task) autonomous item, then the seconds,
    // ...: the kernel's last workgroups are its shortest (VAME_ITEM_ORDER=0:
    // quadrant by quadrant)
    if (env_int("VAME_ITEM_ORDER", 1) == 1) {
      std::vector<size_t> idx(bothAuto.size());
      for (size_t k = 0; k < idx.size(); k++) idx[k] = k;
      std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return autoRank[a] < autoRank[b]; });
      for (size_t k : idx) quadBoth.push_back(bothAuto[k]);
    } else {
      quadBoth.insert(quadBoth.end(), bothAuto.begin(), bothAuto.end());
    }
  } else {
    quadBoth = quadFull;
    quadBoth.insert(quadBoth.end(), quadHalf.begin(), quadHalf.end());
  }
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
// chunks of at most groupCombos CTUs; within a chunk, slot j runs on XCD j % 8
// (workgroups are dealt round-robin over the XCDs).  xcdOrder picks which
// CTUs share an XCD: 0 deals the chunk's CTUs one by one in raster order
// (neighbours on different XCDs: the per-XCD load follows the frame's content
// evenly); R >= 2 deals runs of R raster-adjacent CTUs (neighbours share the
// margins of their reference tiles in one L2); 1 gives XCD x the x-th eighth
// of the chunk in column-major order (compact strips: fewest fetches, but an
// XCD's load follows the content of its strip).
std::vector<int32_t> build_order(int nCtus, int cols, int groupCombos, int xcdOrder, int& nChunks,
                                 int& cpp) {
  const int rows = nCtus / cols;
  nChunks = (nCtus + groupCombos - 1) / groupCombos;
  const int rowsPer = (rows + nChunks - 1) / nChunks;
  nChunks = (rows + rowsPer - 1) / rowsPer;
  const int R = std::max(1, xcdOrder == 1 ? 1 : xcdOrder);
  const int maxN = rowsPer * cols;
  const int perXcd = xcdOrder == 1 ? (maxN + 7) / 8 : ((maxN + R - 1) / R + 7) / 8 * R;
  cpp = perXcd * 8;
  std::vector<int32_t> order((size_t)nChunks * cpp, -1);
  for (int ch = 0; ch < nChunks; ch++) {
    const int r0 = ch * rowsPer, r1 = std::min(rows, r0 + rowsPer);
    std::vector<int> L;
    if (xcdOrder == 1)
      for (int x = 0; x < cols; x++)
        for (int y = r0; y < r1; y++) L.push_back(y * cols + x);
    else
      for (int y = r0; y < r1; y++)
        for (int x = 0; x < cols; x++) L.push_back(y * cols + x);
    const int n = (int)L.size();
    int32_t* o = order.data() + (size_t)ch * cpp;
    if (xcdOrder == 1) {
      const int s = (n + 7) / 8;  // CTUs per XCD in this chunk
      for (int x = 0; x < 8; x++)
        for (int i = 0; i < s && x * s + i < n; i++) o[8 * i + x] = L[x * s + i];
    } else {  // run k -> XCD k % 8; XCD x's i-th slot = element i % R of its (i / R)-th run
      for (int x = 0; x < 8; x++)
        for (int i = 0; i < perXcd; i++) {
          const int e = (x + 8 * (i / R)) * R + i % R;
          if (e < n) o[8 * i + x] = L[e];
        }
    }
  }
  return order;
}



// The kernel instance of a launch mode (vame_kernel.h MODE: 1 = 2-CP only,
// 2 = 3-CP only, 3 = 2-CP then 3-CP).
using KernelFn = void (*)(KParams);
template <int KIND>
KernelFn kernel_for(bool prof, int mode) {
  if constexpr (KIND == kKindHalf2W) {
    (void)prof;
    return mode == 1 ? affine_me_half2w<1> : mode == 2 ? affine_me_half2w<2> : affine_me_half2w<3>;
  } else if constexpr (KIND == kKindHalf2H) {
    (void)prof;
    return mode == 1 ? affine_me_half2h<1> : mode == 2 ? affine_me_half2h<2> : affine_me_half2h<3>;
  } else if constexpr (KIND == kKindCtu2) {
    (void)prof;  // PROF runs the 128x128 CUs in affine_me_ctu_prof (launch_direct)
    return mode == 1 ? affine_me_ctu2<1> : mode == 2 ? affine_me_ctu2<2> : affine_me_ctu2<3>;
  } else if constexpr (KIND == kKindCtu) {
    if (prof) return mode == 1 ? affine_me_ctu_prof<1> : mode == 2 ? affine_me_ctu_prof<2> : affine_me_ctu_prof<3>;
    return mode == 1 ? affine_me_ctu<1> : mode == 2 ? affine_me_ctu<2> : affine_me_ctu<3>;
  } else if constexpr (KIND == kKindHalf) {
    if (prof) return mode == 1 ? affine_me_half_prof<1> : mode == 2 ? affine_me_half_prof<2> : affine_me_half_prof<3>;
    return mode == 1 ? affine_me_half<1> : mode == 2 ? affine_me_half<2> : affine_me_half<3>;
  } else {
    if (prof) return mode == 1 ? affine_me_quad_prof<1> : mode == 2 ? affine_me_quad_prof<2> : affine_me_quad_prof<3>;
    return mode == 1 ? affine_me_quad<1> : mode == 2 ? affine_me_quad<2> : affine_me_quad<3>;
  }
}

constexpr size_t kMaxGraphs = 8;

// Launch one kernel: with the dispatch-carried timing events and AQL flags, or
// (stream capture) as a plain launch, which a graph records.
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

int launch_direct(vame_ctx* c, const std::vector<KParams>& kps, bool quadFull, bool quadHalf, bool bigItems,
                  hipStream_t stream, bool capture) {
  // The 128-class kernels run on the caller's stream and the quadrant kernel
  // on a side stream forked from it (VAME_STREAMS, see vame_ctx): the
  // 128-class workgroups, issued first and ahead of the fork's cross-stream
  // hop, take their CUs before the quadrant workgroups fill the GPU, and the
  // quadrant workgroups then fill the room beside them (a 512-thread
  // affine_me_ctu2 workgroup leaves a CU room for two quadrant workgroups, a
  // 256-thread half2 one for three).  Kernels of one stream run one after the
  // other, so only separate streams overlap them.  The launches of one batch
  // (32 pairs each) fork once and join once: launch k + 1's kernels follow
  // launch k's on their own streams.
  if (VAME_ABLATE & 16) bigItems = false;  // timing-only builds
  if (VAME_ABLATE & 32) quadFull = quadHalf = false;
  if (kps.empty()) return VAME_OK;
  const int mode = (kps[0].run2 ? 1 : 0) | (kps[0].run3 ? 2 : 0);  // the kernel instance (MODE)
  if (mode == 0) return VAME_OK;
  auto use_half = [&](const KParams& kp) {
    return c->halfMode == 1 || (c->halfMode == 2 && kp.nPairs >= c->halfMinPairs);
  };
  bool anyHalf = false;
  for (const KParams& kp : kps) anyHalf |= bigItems && use_half(kp);
  // the side streams this call uses: 0 the quadrant kernel, 1 / 2 the
  // 128x64 / 64x128 kernels (VAME_STREAMS, see vame_ctx)
  bool used[3] = {false, false, false};
  hipStream_t sBig = stream, sQuad = stream, sHalf[2] = {stream, stream};
  if (c->streams == 5 && bigItems && (quadFull || quadHalf)) {  // the 128-class kernels on the side stream
    sBig = sHalf[0] = sHalf[1] = c->side[0];
    used[0] = true;
  } else if (c->streams > 1 && bigItems && (quadFull || quadHalf)) {
    sQuad = c->side[0];
    used[0] = true;
  }
  // VAME_QUAD_ALT=1 (two-stream mode): a batch's quadrant kernels alternate
  // between side streams 0 and 1, so launch k + 1's quadrant workgroups can
  // fill the CUs that launch k's tail leaves idle (c3 / c4: within +-0.1 %,
  // off by default)
  const bool quadAlt = c->streams == 2 && c->quadAlt && used[0] && kps.size() > 1;
  if (quadAlt) used[1] = true;
  if (c->streams > 2 && c->streams < 5 && anyHalf) {
    sHalf[0] = c->side[1];
    sHalf[1] = c->side[c->streams > 3 ? 2 : 1];
    used[1] = true;
    used[2] = c->streams > 3;
  }
  const bool fork = used[0] || used[1] || used[2];
  int issued = 0;  // VAME_STREAMS=1: kernels after a call's first may start before it ends
  auto order_flag = [&]() { return c->streams == 1 && issued++ > 0 ? hipExtAnyOrderLaunch : 0; };
  const bool valueSync = c->valueSync != 0 && !capture;
  auto fork_sides = [&]() -> int {
    if (c->valueSync == 2 && valueSync) {
      const uint32_t v = ++c->forkSeq;
      VAME_HIP(hipStreamWriteValue32(stream, c->syncWord[0], v, 0));
      for (int i = 0; i < 3; i++)
        if (used[i]) VAME_HIP(hipStreamWaitValue32(c->side[i], c->syncWord[0], v, hipStreamWaitValueGte, 0xFFFFFFFFu));
      return VAME_OK;
    }
    VAME_HIP(hipEventRecord(c->evFork, stream));
    for (int i = 0; i < 3; i++)
      if (used[i]) VAME_HIP(hipStreamWaitEvent(c->side[i], c->evFork, 0));
    return VAME_OK;
  };
  auto join_sides = [&]() -> int {
    for (int i = 0; i < 3; i++)
      if (used[i]) {
        if (valueSync) {
          const uint32_t v = ++c->joinSeq[i];
          VAME_HIP(hipStreamWriteValue32(c->side[i], c->syncWord[1 + i], v, 0));
          VAME_HIP(hipStreamWaitValue32(stream, c->syncWord[1 + i], v, hipStreamWaitValueGte, 0xFFFFFFFFu));
        } else {
          VAME_HIP(hipEventRecord(c->evJoin[i], c->side[i]));
          VAME_HIP(hipStreamWaitEvent(stream, c->evJoin[i], 0));
        }
      }
    return VAME_OK;
  };
  for (int i = 0; i < 3; i++)
    if (used[i] && !c->side[i]) return VAME_E_INVALID;  // (vame_create made the streams the knobs use)
  if (fork) VAME_TRY(fork_sides());
  auto big = [&](const KParams& kp) -> int {
    KParams kb = kp;
    const bool ctu2 = !c->prof && (c->ctu2 == 2 || (c->ctu2 == 1 && use_half(kp)));
    if (ctu2 && kp.run2 && kp.run3 && !c->bestS) return VAME_E_INVALID;  // seed-reuse scratch missing
    if (ctu2) {  // the 128x128 CUs in affine_me_ctu2, the rest (short launches) in CTU items
      kb.items = c->dBig1;
      kb.nItems = c->nBig1;
      kb.bestS = c->bestS;
      const unsigned grid = block_grid(c, 1, kb);
      hipEvent_t t0, t1;
      VAME_TRY(time_events(c, 3, t0, t1));
      VAME_HIP(launch_kernel(kernel_for<kKindCtu2>(false, mode), grid, Cfg<kKindCtu2>::THREADS, sBig, t0, t1,
                             order_flag(), kb, capture));
      if (use_half(kp)) return VAME_OK;
      kb = kp;
      kb.items = c->dBig2;
      kb.nItems = c->nBig2;
    } else {
      kb.items = use_half(kp) ? c->dBig1 : c->dBig3;
      kb.nItems = use_half(kp) ? c->nBig1 : c->nBig3;
    }
    const unsigned grid = block_grid(c, 1, kb);
    hipEvent_t t0, t1;
    VAME_TRY(time_events(c, 1, t0, t1));
    VAME_HIP(launch_kernel(kernel_for<kKindCtu>(c->prof, mode), grid, Cfg<kKindCtu>::THREADS, sBig, t0, t1,
                           order_flag(), kb, capture));
    return VAME_OK;
  };
  auto half = [&](const KParams& kp) -> int {  // after the 128x128 items, on their stream
    if (c->half2 && !c->prof) {  // 128x64 then 64x128 CUs, 256-thread workgroups
      if (kp.run2 && kp.run3 && !c->bestS) return VAME_E_INVALID;  // seed-reuse scratch missing
      for (int o = 0; o < 2; o++) {
        KParams kh = kp;
        kh.items = o ? c->dHalfH : c->dHalfW;
        kh.nItems = o ? c->nHalfH : c->nHalfW;
        kh.bestS = c->bestS ? c->bestS + (size_t)kMaxPairs * c->nCtus * 5 * (Cfg<kKindCtu2>::NSB +
                                                                              o * 2 * Cfg<kKindHalf2W>::NSB)
                            : nullptr;
        const unsigned grid = block_grid(c, 1, kh);
        hipEvent_t t0, t1;
        VAME_TRY(time_events(c, 4 + o, t0, t1));
        VAME_HIP(launch_kernel(o ? kernel_for<kKindHalf2H>(false, mode) : kernel_for<kKindHalf2W>(false, mode),
                               grid, Cfg<kKindHalf2W>::THREADS, sHalf[o], t0, t1, order_flag(), kh, capture));
      }
      return VAME_OK;
    }
    KParams kh = kp;
    kh.items = c->dHalf;
    kh.nItems = c->nHalf;
    const unsigned grid = block_grid(c, 1, kh);
    hipEvent_t t0, t1;
    VAME_TRY(time_events(c, 2, t0, t1));
    VAME_HIP(launch_kernel(kernel_for<kKindHalf>(c->prof, mode), grid, Cfg<kKindHalf>::THREADS, sHalf[0], t0, t1,
                           order_flag(), kh, capture));
    return VAME_OK;
  };
  auto quad = [&](const KParams& kp) -> int {
    KParams kq = kp;
    if (quadFull && quadHalf) {
      kq.items = c->dQuad + c->nQuadFull + c->nQuadHalf;
      kq.nItems = c->nQuadBoth;
    } else {
      kq.items = quadFull ? c->dQuad : c->dQuad + c->nQuadFull;
      kq.nItems = quadFull ? c->nQuadFull : c->nQuadHalf;
    }
    const unsigned grid = block_grid(c, 0, kq);
    hipEvent_t t0, t1;
    VAME_TRY(time_events(c, 0, t0, t1));
    VAME_HIP(launch_kernel(kernel_for<kKindQuad>(c->prof, mode), grid, Cfg<kKindQuad>::THREADS,
                           quadAlt && (&kp - kps.data()) % 2 ? c->side[1] : sQuad, t0, t1, order_flag(), kq,
                           capture));
    return VAME_OK;
  };
  auto all = [&]() -> int {
    for (size_t k = 0; k < kps.size(); k++) {
      const bool quadFirst = c->streams == 1 && c->quadFirst;  // VAME_QUAD_FIRST (one-stream mode)
      if (quadFirst && (quadFull || quadHalf)) VAME_TRY(quad(kps[k]));
      if (bigItems && use_half(kps[k]) && c->halfFirst) VAME_TRY(half(kps[k]));
      if (bigItems) VAME_TRY(big(kps[k]));
      if (bigItems && use_half(kps[k]) && !c->halfFirst) VAME_TRY(half(kps[k]));
      if (!quadFirst && (quadFull || quadHalf)) VAME_TRY(quad(kps[k]));
      if (fork && (c->joinEach || k + 1 == kps.size())) {
        VAME_TRY(join_sides());
        if (k + 1 < kps.size()) VAME_TRY(fork_sides());  // VAME_JOIN_EACH: fork again for the next launch
      }
    }
    return VAME_OK;
  };
  const int rc = all();
  if (rc != VAME_OK && fork) {
    // a launch failed after earlier kernels went to the side streams: order
    // them before the caller's stream anyway, so the caller never frees or
    // reuses result buffers they still write (best effort, the first error is
    // the one reported)
    (void)join_sides();
  }
  return rc;
}

int launch(vame_ctx* c, const std::vector<KParams>& kps, bool quadFull, bool quadHalf, bool bigItems,
           hipStream_t stream) {
  if ((c->ctu2 || c->half2) && !c->bestS && bigItems && !kps.empty() && kps[0].run2 && kps[0].run3) {
    // the 3-CP seed-reuse sums of the kernels with two sub-blocks per lane,
    // 5 int32 per sub-block: per (pair, CTU) of a launch the 128x128 CU
    // (affine_me_ctu2), then the two 128x64 and the two 64x128 CUs (_half2w / _half2h)
    VAME_HIP(hipMalloc(&c->bestS, (size_t)kMaxPairs * c->nCtus * 5 *
                                      (Cfg<kKindCtu2>::NSB + 4 * Cfg<kKindHalf2W>::NSB) * sizeof(int32_t)));
  }
  if (!c->useGraph || c->timing || kps.empty()) return launch_direct(c, kps, quadFull, quadHalf, bigItems, stream, false);
  // the call's identity: its kernel arguments and launch selection
  std::vector<unsigned char> key(kps.size() * sizeof(KParams) + 4);
  for (size_t k = 0; k < kps.size(); k++) memcpy(key.data() + k * sizeof(KParams), &kps[k], sizeof(KParams));
  unsigned char* tail = key.data() + kps.size() * sizeof(KParams);
  tail[0] = quadFull;
  tail[1] = quadHalf;
  tail[2] = bigItems;
  tail[3] = c->prof;
  for (size_t i = 0; i < c->graphs.size(); i++) {
    if (c->graphs[i].key == key) {
      vame_ctx::GraphEntry e = std::move(c->graphs[i]);
      c->graphs.erase(c->graphs.begin() + (long)i);
      c->graphs.push_back(std::move(e));  // most recently used last
      VAME_HIP(hipGraphLaunch(c->graphs.back().exec, stream));
      return VAME_OK;
    }
  }
  // capture on the engine's own stream (the caller's may be the null stream,
  // which cannot be captured); the fork / join to the side stream become graph edges
  VAME_HIP(hipStreamBeginCapture(c->capStream, hipStreamCaptureModeThreadLocal));
  const int rc = launch_direct(c, kps, quadFull, quadHalf, bigItems, c->capStream, true);
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(c->capStream, &g);
  if (rc != VAME_OK || ec != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    if (rc != VAME_OK) return rc;
    VAME_HIP(ec);
  }
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  VAME_HIP(ei);
  if (c->graphs.size() == kMaxGraphs) {
    (void)hipGraphExecDestroy(c->graphs.front().exec);
    c->graphs.erase(c->graphs.begin());
  }
  c->graphs.push_back({std::move(key), exec});
  VAME_HIP(hipGraphLaunch(exec, stream));
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
  DeviceGuard guard(device);
  VAME_HIP(guard.err);
  std::vector<Item> big3, big1, big2, hf, qf, qh, qb, unused;
  const int tasks = tasks_per_item();
  build_templates(big3, unused, qf, qh, qb, false, tasks, chain_coop(), mix_aligns());
  for (const Item& it : big3)  // the CTU items without the 128x128 one
    if (it.cu[0].lw != it.cu[0].lh) big2.push_back(it);
  qf.clear();
  qh.clear();
  qb.clear();
  build_templates(big1, hf, qf, qh, qb, true, tasks, chain_coop(), mix_aligns());
  std::vector<Item> hfw, hfh;  // the single-CU half items by orientation
  for (const Item& it : hf) (it.cu[0].lw > it.cu[0].lh ? hfw : hfh).push_back(it);
  if (hfw.empty() || hfh.empty()) return VAME_E_INVALID;
  vame_ctx* c = new vame_ctx();
  c->device = device;
  c->W = width;
  c->H = height;
  c->nCtus = nCtus;
  c->ctusPerRow = (width + kCtu - 1) / kCtu;  // T8: integer ceil
  c->nBig3 = (int)big3.size();
  c->nBig1 = (int)big1.size();
  c->nBig2 = (int)big2.size();
  c->ctu2 = std::min(2, std::max(0, env_int("VAME_CTU2", 2)));
  c->nHalf = (int)hf.size();
  c->nHalfW = (int)hfw.size();
  c->nHalfH = (int)hfh.size();
  c->half2 = env_int("VAME_HALF2", 1) != 0;
  c->halfMode = std::min(2, std::max(0, env_int("VAME_HALF128", 1)));
  c->halfMinPairs = std::max(1, env_int("VAME_HALF_MIN_PAIRS", 16));
  c->nQuadFull = (int)qf.size();
  c->nQuadHalf = (int)qh.size();
  c->nQuadBoth = (int)qb.size();
  std::vector<Item> quad(qf);  // [FULL][HALF][both alignments]
  quad.insert(quad.end(), qh.begin(), qh.end());
  quad.insert(quad.end(), qb.begin(), qb.end());
  hipError_t e = hipMalloc(&c->dQuad, quad.size() * sizeof(Item));
  // tuning knobs of the block order (defaults measured on MI355X)
  const int xcdOrder = env_int("VAME_XCD_ORDER", 0);
  c->joinEach = env_int("VAME_JOIN_EACH", 0) != 0;
  c->streams = std::min(5, std::max(1, env_int("VAME_STREAMS", 2)));
  c->useGraph = env_int("VAME_GRAPH", 0) != 0;
  c->quadFirst = env_int("VAME_QUAD_FIRST", 1) != 0;
  c->groupCombos[0] = std::max(8, env_int("VAME_GROUP_COMBOS", 408));
  c->groupCombos[1] = std::max(8, env_int("VAME_GROUP_COMBOS_BIG", c->groupCombos[0]));
  for (int k = 0; k < 2 && e == hipSuccess; k++) {
    const std::vector<int32_t> order =
        build_order(nCtus, c->ctusPerRow, c->groupCombos[k], xcdOrder, c->nChunks[k], c->cpp[k]);
    e = hipMalloc(&c->dOrder[k], order.size() * sizeof(int32_t));
    if (e == hipSuccess)
      e = hipMemcpy(c->dOrder[k], order.data(), order.size() * sizeof(int32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMalloc(&c->dBig3, big3.size() * sizeof(Item));
  if (e == hipSuccess) e = hipMalloc(&c->dBig1, big1.size() * sizeof(Item));
  if (e == hipSuccess) e = hipMalloc(&c->dBig2, big2.size() * sizeof(Item));
  if (e == hipSuccess) e = hipMemcpy(c->dBig2, big2.data(), big2.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->dQuad, quad.data(), quad.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->dBig3, big3.data(), big3.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->dBig1, big1.data(), big1.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess && !hfw.empty()) e = hipMalloc(&c->dHalfW, hfw.size() * sizeof(Item));
  if (e == hipSuccess && !hfw.empty())
    e = hipMemcpy(c->dHalfW, hfw.data(), hfw.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess && !hfh.empty()) e = hipMalloc(&c->dHalfH, hfh.size() * sizeof(Item));
  if (e == hipSuccess && !hfh.empty())
    e = hipMemcpy(c->dHalfH, hfh.data(), hfh.size() * sizeof(Item), hipMemcpyHostToDevice);
  if (e == hipSuccess && !hf.empty()) e = hipMalloc(&c->dHalf, hf.size() * sizeof(Item));
  if (e == hipSuccess && !hf.empty())
    e = hipMemcpy(c->dHalf, hf.data(), hf.size() * sizeof(Item), hipMemcpyHostToDevice);
  c->valueSync = std::min(2, std::max(0, env_int("VAME_SYNC", 1)));
  c->quadAlt = env_int("VAME_QUAD_ALT", 0) != 0;
  c->halfFirst = env_int("VAME_HALF_FIRST", 0) != 0;
  // only the side streams the knobs use (side stream 0 by default; 1 for
  // VAME_STREAMS=3 / VAME_QUAD_ALT, 2 for VAME_STREAMS=4), created here, not
  // during a launch (a launch may be under stream capture): a process has
  // GPU_MAX_HW_QUEUES = 4 hardware queues and HIP shares them between its
  // streams beyond that, so an idle stream created here could put the
  // caller's own copy streams on the quadrant kernel's queue (the CLI's
  // compute, upload and download streams + side stream 0 are four)
  const int nSide = c->streams == 4 ? 3 : (c->streams == 3 || (c->streams == 2 && c->quadAlt)) ? 2 : 1;
  for (int i = 0; i < nSide && e == hipSuccess; i++) {
    e = hipStreamCreateWithFlags(&c->side[i], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->evJoin[i], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->evFork, hipEventDisableTiming);
  for (int i = 0; i < 4 && e == hipSuccess && c->valueSync; i++) {
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&c->syncWord[i]), 8, hipMallocSignalMemory) != hipSuccess ||
        hipMemset(c->syncWord[i], 0, 8) != hipSuccess) {
      (void)hipGetLastError();
      c->valueSync = 0;  // events instead
    }
  }
  if (e == hipSuccess && c->useGraph) e = hipStreamCreateWithFlags(&c->capStream, hipStreamNonBlocking);
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
  DeviceGuard guard(c->device);
  if (c->dQuad) (void)hipFree(c->dQuad);
  if (c->dBig3) (void)hipFree(c->dBig3);
  if (c->dBig1) (void)hipFree(c->dBig1);
  if (c->dBig2) (void)hipFree(c->dBig2);
  if (c->bestS) (void)hipFree(c->bestS);
  if (c->dHalf) (void)hipFree(c->dHalf);
  if (c->dHalfW) (void)hipFree(c->dHalfW);
  if (c->dHalfH) (void)hipFree(c->dHalfH);
  for (int k = 0; k < 2; k++)
    if (c->dOrder[k]) (void)hipFree(c->dOrder[k]);
  for (auto& g : c->graphs) (void)hipGraphExecDestroy(g.exec);
  if (c->capStream) (void)hipStreamDestroy(c->capStream);
  for (int i = 0; i < 3; i++) {
    if (c->side[i]) (void)hipStreamDestroy(c->side[i]);
    if (c->evJoin[i]) (void)hipEventDestroy(c->evJoin[i]);
  }
  if (c->evFork) (void)hipEventDestroy(c->evFork);
  for (uint32_t* w : c->syncWord)
    if (w) (void)hipFree(w);
  if (c->dPackSegs) (void)hipFree(c->dPackSegs);
  if (c->packEv) (void)hipEventDestroy(c->packEv);
  for (int k = 0; k < 6; k++)
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
  if (!hits || (align != 0 && align != 1)) return VAME_E_INVALID;
  std::vector<Item> big, hf, qf, qh, qb;
  build_templates(big, hf, qf, qh, qb, half128 != 0, tasks_per_item(), chain_coop(), mix_aligns());
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
    items3[0] = (int32_t)qb.size();
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
  // every (POC, refIdx) pair of the batch, kMaxPairs per launch
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
      if (kp.nPairs == kMaxPairs || last) {
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
  if (c->packEv) VAME_HIP(hipEventSynchronize(c->packEv));  // the previous upload read the table
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
    VAME_HIP(hipEventRecord(c->packEv, s));
    hipLaunchKernelGGL(pack_records_kernel, dim3((maxn + 255) / 256, (unsigned)segs.size()), dim3(256), 0, s,
                       c->dPackSegs, slab, bad);
    VAME_HIP(hipGetLastError());
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
  // kernel classes timed: bit 0 quadrant, bit 1 CTU items, bit 2 half items;
  // VAME_TIMING_KEEP (16) keeps the launches recorded so far (a caller timing
  // a sample of its steps toggles timing between them)
  const bool keep = (enable & VAME_TIMING_KEEP) != 0;
  enable &= ~VAME_TIMING_KEEP;
  c->timing = enable == 2 ? 1 : enable != 0 ? 63 : 0;
  if (!keep)
    for (size_t& u : c->evUsed) u = 0;
  return VAME_OK;
}

int vame_get_timing(vame_ctx* c, int cls, double* total_ms, int* launches, int reset) {
  if (!c || cls < 0 || cls > 5 || !total_ms || !launches) return VAME_E_INVALID;
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
    unsigned long long z[6 * kPhSlots] = {};
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
