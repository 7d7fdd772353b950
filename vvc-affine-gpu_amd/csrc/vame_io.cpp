// vame_io.cpp -- host-side input and output contracts of the reference's ./main,
// native and multi-threaded.  No device work; exported through include/vame.h.
//
//  * Frame ingest (main.cpp:293-330): the reference reads N_FRAMES x H lines of
//    W comma-separated integers from the original and reference CSVs with
//    getline(',') + stoi, one value at a time.  Here the file is mmapped, split
//    into byte ranges at line starts, and parsed by a thread per range.
//    Raw little-endian uint16 frames (`*.u16` / `*.yuv`) take a memcpy path.
//  * Decision log (main_aux_functions.h:387-525 reportAffineResultsMaster_new,
//    :1547-1585 removeOldTraces): one CSV per (PRED, CU size), header
//    "POC,List,Ref,CTU,idx,X,Y,Cost,LT_X,LT_Y,RT_X,RT_Y,LB_X,LB_Y", rows appended
//    per (POC, refIdx) in (group, CTU, cuIdx) order.  Rows are formatted with
//    std::to_chars by a thread per CTU range and appended with one fwrite per
//    group, so the bytes are identical to the reference's fprintf loop.
//    vame_log_writer_* logs a whole POC per call on a persistent thread pool
//    with the files kept open (the CLI's path): the rows of every (refIdx,
//    PRED, group, CTU chunk) are formatted in parallel, then each file gets
//    its rows with one writev, files in parallel.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vame.h"
#include "vame_tables.h"

using namespace vame;

namespace {

// Host CPUs this process may use: its affinity mask, capped by a cgroup-v2
// CPU quota (cpu.max) and by OMP_NUM_THREADS when set -- a GPU box can show
// hundreds of CPUs while granting a process a 16-CPU share, and threads beyond
// the share only get throttled.
int host_threads() {
  static const int n = [] {
    int c = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) c = CPU_COUNT(&set);
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long period = 0;
      if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
        c = std::min<long>(c, std::max(1L, (atol(q) + period - 1) / period));
      fclose(f);
    }
    if (const char* e = getenv("OMP_NUM_THREADS"))
      if (atoi(e) > 0) c = std::min(c, atoi(e));
    return std::max(1, c);
  }();
  return n;
}

int pick_threads(int requested, long work_items) {
  int t = requested > 0 ? requested : host_threads();
  t = std::max(1, std::min(t, 64));
  return (int)std::max(1L, std::min<long>(t, work_items));
}

// Persistent workers for the log writer: run(n, f) calls f(i) for i < n on
// the workers and the calling thread, and returns when all are done.  Callers
// on several threads take turns (run_mu_); in a child forked after the pool
// started -- which has none of its threads -- run() works serially; the
// owner must not destroy a pool there (forked(): its condition variables
// still count the parent's waiting threads, and destroying them would wait
// for those forever), and leaks it instead.
class Pool {
 public:
  explicit Pool(int nthreads) : pid_(getpid()), th_(new std::vector<std::thread>) {
    for (int t = 1; t < nthreads; t++) th_->emplace_back([this] { loop(); });
  }
  bool forked() const { return getpid() != pid_; }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : *th_) t.join();
  }
  void run(int n, const std::function<void(int)>& f) {
    if (th_->empty() || n <= 1 || forked()) {
      for (int i = 0; i < n; i++) f(i);
      return;
    }
    std::lock_guard<std::mutex> turn(run_mu_);
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &f;
      n_ = n;
      next_.store(0);
      active_ = (int)th_->size();
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return active_ == 0; });
    job_ = nullptr;
  }

 private:
  void work() {
    for (int i; (i = next_.fetch_add(1)) < n_;) (*job_)(i);
  }
  void loop() {
    unsigned long long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> g(mu_);
      if (--active_ == 0) done_.notify_all();
    }
  }
  const pid_t pid_;
  std::unique_ptr<std::vector<std::thread>> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int n_ = 0, active_ = 0;
  std::atomic<int> next_{0};
  unsigned long long gen_ = 0;
  bool stop_ = false;
};

template <class F>
void parallel_for(int nthreads, int n, F&& f) {
  if (nthreads <= 1 || n <= 1) {
    for (int i = 0; i < n; i++) f(i, 0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nthreads);
  for (int t = 0; t < nthreads; t++)
    th.emplace_back([&, t] {
      for (int i = t; i < n; i += nthreads) f(i, t);
    });
  for (auto& x : th) x.join();
}

bool ends_with(const char* s, const char* suf) {
  size_t a = strlen(s), b = strlen(suf);
  return a >= b && strcmp(s + a - b, suf) == 0;
}

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  ~Mapped() {
    if (p && n) munmap((void*)p, n);
    if (fd >= 0) close(fd);
  }
};

int map_file(const char* path, Mapped& m) {
  m.fd = open(path, O_RDONLY);
  if (m.fd < 0) return VAME_E_INVALID;
  struct stat st;
  if (fstat(m.fd, &st) != 0) return VAME_E_INVALID;
  m.n = (size_t)st.st_size;
  if (m.n == 0) return VAME_OK;
  void* p = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
  if (p == MAP_FAILED) {
    m.n = 0;
    return VAME_E_NOMEM;
  }
  madvise(p, m.n, MADV_SEQUENTIAL);
  m.p = (const char*)p;
  return VAME_OK;
}

// One CSV line = W values.  Per value, as getline(',') + stoi does
// (main.cpp:318-325): skip leading whitespace, optional sign, digits; anything
// after the digits up to the next ',' is ignored.  Returns false if the line
// holds fewer than W values or a value has no digits (stoi would throw).
bool parse_line(const char* s, const char* e, int W, uint16_t* out) {
  for (int w = 0; w < W; w++) {
    if (s >= e) return false;
    while (s < e && (*s == ' ' || *s == '\t' || *s == '\r')) s++;
    bool neg = false;
    if (s < e && (*s == '-' || *s == '+')) neg = *s++ == '-';
    if (s >= e || *s < '0' || *s > '9') return false;
    // std::stoi semantics (main.cpp:324): a value outside int's range throws
    // out_of_range there, so it is rejected here (bounded: no overflow)
    const long long lim = neg ? 2147483648ll : 2147483647ll;
    long long v = 0;
    while (s < e && *s >= '0' && *s <= '9') {
      v = v * 10 + (*s++ - '0');
      if (v > lim) return false;
    }
    out[w] = (uint16_t)(neg ? -v : v);  // stored into unsigned short (main.cpp:324-325)
    while (s < e && *s != ',') s++;
    if (s < e) s++;  // the ','
  }
  return true;
}

// ---- decision-log naming (main_aux_functions.h:392-425, 1555-1570)
const char* kPredTag[4] = {"_FULL_2CPs_", "_FULL_3CPs_", "_HALF_2CPs_", "_HALF_3CPs_"};
const char* kHeader = "POC,List,Ref,CTU,idx,X,Y,Cost,LT_X,LT_Y,RT_X,RT_Y,LB_X,LB_Y\n";

std::string size_name(int align, int g) {
  const int w = align ? kHalfW[g] : kFullW[g], h = align ? kHalfH[g] : kFullH[g];
  return std::to_string(w) + "x" + std::to_string(h);
}

std::string log_path(const char* prefix, int pred, int g) {
  return std::string(prefix) + kPredTag[pred] + size_name(pred >> 1, g) + ".csv";
}

// CU position inside the frame, as the log writer computes it
// (main_aux_functions.h:460-479): FULL = raster order of the size, HALF = the
// host tables HA_ALL_X_POS / HA_ALL_Y_POS (constants.h:327-364, equal to the
// kernel tables restated in vame_tables.h).
inline void cu_pos(int align, int g, int cu, int ctu, int ctuCols, int& x, int& y) {
  if (!align) {
    y = (cu * kFullW[g]) / 128 * kFullH[g];
    x = (cu * kFullW[g]) % 128;
  } else {
    y = kHalfY8[g][cu] * 8;
    x = kHalfX8[g][cu] * 8;
  }
  y += (ctu / ctuCols) * 128;
  x += (ctu % ctuCols) * 128;
}

// Decimal text of an integer, as printf's %d / %ld: two digits per step from
// a pair table, 32-bit arithmetic whenever the value fits (costs are < 2^31).
constexpr char kPairs[201] =
    "0001020304050607080910111213141516171819202122232425262728293031323334353637383940414243444546474849"
    "5051525354555657585960616263646566676869707172737475767778798081828384858687888990919293949596979899";
inline char* put_u32(char* p, uint32_t v) {
  const int n = v < 10 ? 1 : v < 100 ? 2 : v < 1000 ? 3 : v < 10000 ? 4 : v < 100000 ? 5
              : v < 1000000 ? 6 : v < 10000000 ? 7 : v < 100000000 ? 8 : v < 1000000000 ? 9 : 10;
  char* q = p + n;
  while (v >= 100) {
    const uint32_t r = v % 100;
    v /= 100;
    q -= 2;
    memcpy(q, kPairs + 2 * r, 2);
  }
  if (v >= 10) {
    memcpy(q - 2, kPairs + 2 * v, 2);
  } else {
    q[-1] = (char)('0' + v);
  }
  return p + n;
}
inline char* put(char* p, long long v) {
  if (v >= -2147483647ll && v <= 4294967295ll) {
    if (v < 0) {
      *p++ = '-';
      return put_u32(p, (uint32_t)(-v));
    }
    return put_u32(p, (uint32_t)v);
  }
  return std::to_chars(p, p + 24, v).ptr;
}

// Rows of one (group, CTU range) in the reference's fprintf format
// "%d,%d,%d,%d,%d,%d,%d,%ld,%d,%d,%d,%d,%d,%d\n" (main_aux_functions.h:491).
// A reusable text buffer (grown without the zero fill of std::string::resize).
struct Buf {
  std::unique_ptr<char[]> d;
  size_t cap = 0, len = 0;
  char* reserve(size_t n) {
    if (n > cap) {
      d.reset(new char[n]);
      cap = n;
    }
    return d.get();
  }
};

void format_rows(Buf& buf, int align, int g, int ctu0, int ctu1, int ctuCols, int poc,
                 int ref, const int64_t* cost, const vame_cpmvs* cp) {
  const int ncu = align ? kHalfN[g] : (kFullStride[g + 1] - kFullStride[g]);
  const int stride = align ? kHalfStride[g] : kFullStride[g];
  const int T = align ? kHalfCusPerCtu : kFullCusPerCtu;
  // a row is at most 4 x 11 + 3 x 5 + 20 + 6 x 11 + 14 separators < 160 bytes
  char* const p0 = buf.reserve((size_t)(ctu1 - ctu0) * ncu * 160);
  char* p = p0;
  char pre[32];
  char* pe = put(pre, poc);
  *pe++ = ',';
  *pe++ = '0';  // List (always L0, main_aux_functions.h:388)
  *pe++ = ',';
  pe = put(pe, ref);
  *pe++ = ',';
  const size_t npre = (size_t)(pe - pre);
  for (int ctu = ctu0; ctu < ctu1; ctu++) {
    for (int cu = 0; cu < ncu; cu++) {
      int x, y;
      cu_pos(align, g, cu, ctu, ctuCols, x, y);
      const size_t i = (size_t)ctu * T + stride + cu;
      memcpy(p, pre, npre);
      p += npre;
      p = put(p, ctu);
      *p++ = ',';
      p = put(p, cu);
      *p++ = ',';
      p = put(p, x);
      *p++ = ',';
      p = put(p, y);
      *p++ = ',';
      p = put(p, cost[i]);
      const vame_cpmvs& c = cp[i];
      const int32_t v[6] = {c.LT.x, c.LT.y, c.RT.x, c.RT.y, c.LB.x, c.LB.y};
      for (int k = 0; k < 6; k++) {
        *p++ = ',';
        p = put(p, v[k]);
      }
      *p++ = '\n';
    }
  }
  buf.len = (size_t)(p - p0);
}

}  // namespace

// A POC-at-a-time decision-log writer (include/vame.h vame_log_writer_*).
struct vame_log_writer {
  std::string prefix;
  int W = 0, H = 0, nCtus = 0, ctuCols = 0;
  std::unique_ptr<Pool> pool;
  // files: per pred, group -> file index (duplicate HALF names share a file)
  std::vector<int> fileOf[4];
  std::vector<std::string> paths;
  std::vector<int> predOf;
  std::vector<int> fds;
  std::vector<Buf> bufs;  // per task, reused across POCs
  // deferred mode (vame_log_writer_set_deferred): each file's rows held in
  // memory, in blocks, until vame_log_writer_flush_at places them
  struct Held {
    std::vector<std::unique_ptr<char[]>> blocks;
    size_t last = 0;   // bytes used in the last block
    long long total = 0;
  };
  static constexpr size_t kHeldBlock = size_t(32) << 20;
  bool deferred = false;
  bool started = false;  // a POC was logged (the mode is fixed from then on)
  std::vector<Held> held;
  ~vame_log_writer() {
    for (int fd : fds)
      if (fd >= 0) close(fd);
    if (pool && pool->forked()) (void)pool.release();  // see Pool: leaked in a forked child
  }
};

namespace {
constexpr int kLogChunk = 64;  // CTUs per formatting task
}

extern "C" {

vame_log_writer* vame_log_writer_create(const char* prefix, int width, int height, int nthreads) {
  if (!prefix) return nullptr;
  const int nCtus = num_ctus(width, height);
  if (!nCtus) return nullptr;
  auto* w = new vame_log_writer;
  w->prefix = prefix;
  w->W = width;
  w->H = height;
  w->nCtus = nCtus;
  w->ctuCols = (width + kCtu - 1) / kCtu;
  w->pool.reset(new Pool(pick_threads(nthreads, 1 << 20)));
  std::map<std::string, int> idx;
  for (int m = 0; m < 4; m++) {
    const int ng = (m >> 1) ? kHalfGroups : kFullGroups;
    for (int g = 0; g < ng; g++) {
      const std::string p = log_path(prefix, m, g);
      auto it = idx.find(p);
      if (it == idx.end()) {
        it = idx.emplace(p, (int)w->paths.size()).first;
        w->paths.push_back(p);
        w->predOf.push_back(m);
      }
      w->fileOf[m].push_back(it->second);
    }
  }
  w->fds.assign(w->paths.size(), -1);
  return w;
}

long long vame_log_writer_poc(vame_log_writer* w, int poc, int nrefs, int pred_mask,
                              const int64_t* const* cost, const vame_cpmvs* const* cpmvs) {
  return vame_log_writer_refs(w, poc, 0, nrefs, pred_mask, cost, cpmvs);
}

long long vame_log_writer_refs(vame_log_writer* w, int poc, int ref0, int nrefs, int pred_mask,
                               const int64_t* const* cost, const vame_cpmvs* const* cpmvs) {
  if (!w || ref0 < 0 || nrefs <= 0 || ref0 + nrefs > 4 || !cost || !cpmvs || (pred_mask & ~15))
    return VAME_E_INVALID;
  for (int r = 0; r < nrefs; r++)
    for (int m = 0; m < 4; m++)
      if (((pred_mask >> m) & 1) && (!cost[r * 4 + m] || !cpmvs[r * 4 + m])) return VAME_E_INVALID;
  const int nchunks = (w->nCtus + kLogChunk - 1) / kLogChunk;
  // tasks in file order: refIdx, PRED, group, CTU chunk
  struct Task {
    int r, m, g, c;
  };
  std::vector<Task> tasks;
  for (int r = 0; r < nrefs; r++)
    for (int m = 0; m < 4; m++) {
      if (!((pred_mask >> m) & 1)) continue;
      const int ng = (m >> 1) ? kHalfGroups : kFullGroups;
      for (int g = 0; g < ng; g++)
        for (int c = 0; c < nchunks; c++) tasks.push_back({r, m, g, c});
    }
  if (w->bufs.size() < tasks.size()) w->bufs.resize(tasks.size());
  w->started = true;
  w->pool->run((int)tasks.size(), [&](int i) {
    const Task& t = tasks[i];
    format_rows(w->bufs[i], t.m >> 1, t.g, t.c * kLogChunk, std::min(w->nCtus, (t.c + 1) * kLogChunk),
                w->ctuCols, poc, ref0 + t.r, cost[t.r * 4 + t.m], cpmvs[t.r * 4 + t.m]);
  });
  // per file, its tasks in order (a file belongs to one PRED; HALF names
  // shared by several groups take them in group order, as the reference's
  // per-group appends do)
  std::vector<std::vector<int>> per(w->paths.size());
  for (size_t i = 0; i < tasks.size(); i++) per[w->fileOf[tasks[i].m][tasks[i].g]].push_back((int)i);
  std::vector<long long> wrote(w->paths.size(), 0);
  std::atomic<int> bad{0};
  w->pool->run((int)w->paths.size(), [&](int f) {
    if (per[f].empty()) return;
    if (w->deferred) {  // into the file's held blocks, in order
      vame_log_writer::Held& h = w->held[f];
      for (int i : per[f]) {
        const char* q = w->bufs[i].d.get();
        size_t left = w->bufs[i].len;
        wrote[f] += (long long)left;
        h.total += (long long)left;
        while (left) {
          if (h.blocks.empty() || h.last == vame_log_writer::kHeldBlock) {
            h.blocks.emplace_back(new char[vame_log_writer::kHeldBlock]);
            h.last = 0;
          }
          const size_t k = std::min(left, vame_log_writer::kHeldBlock - h.last);
          memcpy(h.blocks.back().get() + h.last, q, k);
          h.last += k;
          q += k;
          left -= k;
        }
      }
      return;
    }
    int& fd = w->fds[f];
    if (fd < 0) fd = open(w->paths[f].c_str(), O_WRONLY | O_APPEND | O_CREAT, 0644);
    if (fd < 0) {
      bad = 1;
      return;
    }
    std::vector<iovec> iov;
    for (int i : per[f])
      if (w->bufs[i].len) iov.push_back({(void*)w->bufs[i].d.get(), w->bufs[i].len});
    size_t k = 0;
    while (k < iov.size()) {
      const int cnt = (int)std::min<size_t>(iov.size() - k, 512);
      size_t want = 0;
      for (int j = 0; j < cnt; j++) want += iov[k + j].iov_len;
      const ssize_t n = writev(fd, &iov[k], cnt);
      if (n < 0 || (size_t)n != want) {  // short write: finish the batch by plain writes
        size_t done = n < 0 ? 0 : (size_t)n;
        for (int j = 0; j < cnt; j++) {
          const size_t len = iov[k + j].iov_len;
          if (done >= len) {
            done -= len;
            continue;
          }
          const char* q = (const char*)iov[k + j].iov_base + done;
          size_t left = len - done;
          done = 0;
          while (left) {
            const ssize_t m = write(fd, q, left);
            if (m <= 0) {
              bad = 1;
              return;
            }
            q += m;
            left -= (size_t)m;
          }
        }
      }
      wrote[f] += (long long)want;
      k += (size_t)cnt;
    }
  });
  if (bad) return VAME_E_INVALID;
  long long total = 0;
  for (long long b : wrote) total += b;
  return total;
}

int vame_log_writer_set_deferred(vame_log_writer* w, int deferred) {
  if (!w || w->started) return VAME_E_INVALID;  // rows already appended or held
  w->deferred = deferred != 0;
  w->held.resize(w->paths.size());
  return VAME_OK;
}

int vame_log_writer_num_files(vame_log_writer* w) { return w ? (int)w->paths.size() : VAME_E_INVALID; }

int vame_log_writer_file_name(vame_log_writer* w, int f, char* buf, int buflen) {
  if (!w || f < 0 || f >= (int)w->paths.size() || !buf || buflen <= (int)w->paths[f].size())
    return VAME_E_INVALID;
  memcpy(buf, w->paths[f].c_str(), w->paths[f].size() + 1);
  return VAME_OK;
}

int vame_log_writer_sizes(vame_log_writer* w, long long* sizes) {
  if (!w || !sizes) return VAME_E_INVALID;
  for (size_t f = 0; f < w->paths.size(); f++) sizes[f] = f < w->held.size() ? w->held[f].total : 0;
  return VAME_OK;
}

long long vame_log_writer_flush_at(vame_log_writer* w, const long long* offsets) {
  if (!w || !offsets) return VAME_E_INVALID;
  std::atomic<int> bad{0};
  long long total = 0;
  w->held.resize(w->paths.size());
  // one task per held block (not per file: the 40 files' sizes differ by two
  // orders of magnitude, the 16x16 groups' files hold most of the bytes), each
  // written at its own offset -- the files opened once, never truncated
  struct Piece {
    int f;
    const char* q;
    size_t n;
    long long off;
  };
  std::vector<Piece> pieces;
  std::vector<int> fds(w->paths.size(), -1);
  for (size_t f = 0; f < w->paths.size(); f++) {
    vame_log_writer::Held& h = w->held[f];
    if (!h.total) continue;
    fds[f] = open(w->paths[f].c_str(), O_WRONLY | O_CREAT, 0644);
    if (fds[f] < 0) {
      bad = 1;
      break;
    }
    long long off = offsets[f];
    for (size_t b = 0; b < h.blocks.size(); b++) {
      const size_t n = b + 1 == h.blocks.size() ? h.last : vame_log_writer::kHeldBlock;
      pieces.push_back({(int)f, h.blocks[b].get(), n, off});
      off += (long long)n;
    }
    total += h.total;
  }
  if (!bad)
    w->pool->run((int)pieces.size(), [&](int i) {
      const Piece& pc = pieces[i];
      const char* q = pc.q;
      size_t left = pc.n;
      long long off = pc.off;
      while (left) {
        const ssize_t k = pwrite(fds[pc.f], q, left, (off_t)off);
        if (k <= 0) {
          bad = 1;
          return;
        }
        q += k;
        off += k;
        left -= (size_t)k;
      }
    });
  for (int fd : fds)
    if (fd >= 0) close(fd);
  for (auto& h : w->held) h = vame_log_writer::Held();
  return bad ? VAME_E_INVALID : total;
}

int vame_log_writer_destroy(vame_log_writer* w) {
  delete w;
  return VAME_OK;
}

int vame_read_frames(const char* path, int width, int height, int nframes, uint16_t* out,
                     int nthreads) {
  return vame_read_frames_range(path, width, height, 0, nframes, out, nthreads);
}

int vame_read_frames_range(const char* path, int width, int height, int first_frame, int nframes,
                           uint16_t* out, int nthreads) {
  return vame_read_frames_span(path, width, height, first_frame, nframes, 0, 0, -1, out, nthreads);
}

long long vame_count_lines(const char* path, long long begin, long long end, int nthreads) {
  if (!path || begin < 0) return VAME_E_INVALID;
  Mapped m;
  if (int rc = map_file(path, m)) return rc;
  const size_t e = end < 0 ? m.n : std::min((size_t)end, m.n);
  if ((size_t)begin >= e) return 0;
  const size_t len = e - (size_t)begin;
  const int T = pick_threads(nthreads, (long)(len >> 20) + 1);
  std::vector<long long> nl(T, 0);
  parallel_for(T, T, [&](int t, int) {
    const char* q = m.p + begin + len * t / T;
    const char* qe = m.p + begin + len * (t + 1) / T;
    long long c = 0;
    while (q < qe) {
      const char* r = (const char*)memchr(q, '\n', (size_t)(qe - q));
      if (!r) break;
      c++;
      q = r + 1;
    }
    nl[t] = c;
  });
  long long c = 0;
  for (long long v : nl) c += v;
  return c;
}

int vame_count_lines_ranges(const char* path, const long long* begin, const long long* end, int n,
                            long long* counts, int nthreads) {
  if (!path || n < 0 || (n > 0 && (!begin || !end || !counts))) return VAME_E_INVALID;
  for (int i = 0; i < n; i++)
    if (begin[i] < 0 || end[i] < begin[i]) return VAME_E_INVALID;
  Mapped m;
  if (int rc = map_file(path, m)) return rc;
  // pieces of <= 4 MiB over all ranges, dealt to the threads in turn
  constexpr size_t kPiece = size_t(4) << 20;
  struct Piece {
    int range;
    size_t b, e;
  };
  std::vector<Piece> pieces;
  for (int i = 0; i < n; i++) {
    counts[i] = 0;
    const size_t b = std::min((size_t)begin[i], m.n), e = std::min((size_t)end[i], m.n);
    for (size_t o = b; o < e; o += kPiece) pieces.push_back({i, o, std::min(e, o + kPiece)});
  }
  std::vector<long long> per(pieces.size(), 0);
  const int T = pick_threads(nthreads, (long)pieces.size());
  parallel_for(T, (int)pieces.size(), [&](int k, int) {
    const char* q = m.p + pieces[k].b;
    const char* qe = m.p + pieces[k].e;
    long long c = 0;
    while (q < qe) {
      const char* r = (const char*)memchr(q, '\n', (size_t)(qe - q));
      if (!r) break;
      c++;
      q = r + 1;
    }
    per[k] = c;
  });
  for (size_t k = 0; k < pieces.size(); k++) counts[pieces[k].range] += per[k];
  return VAME_OK;
}

int vame_read_frames_span(const char* path, int width, int height, int first_frame, int nframes,
                          long long span_begin, long long lines_before, long long span_end,
                          uint16_t* out, int nthreads) {
  const int first = first_frame;
  if (!path || !out || width <= 0 || height <= 0 || first < 0 || nframes <= 0 || span_begin < 0 ||
      lines_before < 0)
    return VAME_E_INVALID;
  Mapped m;
  int rc = map_file(path, m);
  if (rc) return rc;
  const size_t fsz = (size_t)width * height;
  if (ends_with(path, ".u16") || ends_with(path, ".yuv")) {  // raw 16-bit side path
    if (m.n < fsz * ((size_t)first + nframes) * 2) return VAME_E_INVALID;
    memcpy(out, m.p + fsz * first * 2, fsz * nframes * 2);
    return VAME_OK;
  }
  // text lines [line0, nlines) are frames first .. first + nframes - 1; the
  // bytes [b0, n) hold them, with lines_before newlines ahead of b0
  const long line0 = (long)first * height;
  const long nlines = ((long)first + nframes) * height;
  const char* base = m.p;
  const size_t n = span_end < 0 ? m.n : std::min((size_t)span_end, m.n);
  const size_t b0 = (size_t)span_begin;
  if (m.n == 0 || b0 >= n || line0 < lines_before) return VAME_E_INVALID;
  const size_t len = n - b0;
  // pass 1: newline count per byte range
  const int T = pick_threads(nthreads, (long)(len >> 20) + 1);
  std::vector<size_t> cut(T + 1);
  for (int t = 0; t <= T; t++) cut[t] = b0 + len * t / T;
  std::vector<long> nl(T, 0);
  parallel_for(T, T, [&](int t, int) {
    long c = 0;
    for (const char* q = base + cut[t]; q < base + cut[t + 1];) {
      const char* r = (const char*)memchr(q, '\n', (size_t)(base + cut[t + 1] - q));
      if (!r) break;
      c++;
      q = r + 1;
    }
    nl[t] = c;
  });
  // the line that holds byte cut[t] (lines start at 0 and after each '\n')
  std::vector<long> firstLine(T + 1, (long)lines_before);
  for (int t = 0; t < T; t++) firstLine[t + 1] = firstLine[t] + nl[t];
  const long total_lines = firstLine[T] + (n == m.n && base[n - 1] != '\n' ? 1 : 0);
  if (total_lines < nlines) return VAME_E_INVALID;
  // pass 2: parse the lines that START in each range
  std::vector<int> bad(T, 0);
  parallel_for(T, T, [&](int t, int) {
    const char* q = base + cut[t];
    long li = firstLine[t];
    if (cut[t] > 0 && base[cut[t] - 1] != '\n') {  // skip the tail of a line started earlier
      const char* r = (const char*)memchr(q, '\n', (size_t)(base + cut[t + 1] - q));
      if (!r) return;
      q = r + 1;
      li++;  // firstLine[t] is the line that straddles cut[t]; q starts the next one
    }
    const char* end = base + cut[t + 1];
    while (q < end && li < nlines) {
      const char* r = (const char*)memchr(q, '\n', (size_t)(base + m.n - q));
      const char* le = r ? r : base + m.n;
      if (li >= line0 && !parse_line(q, le, width, out + (size_t)(li - line0) * width)) {
        bad[t] = 1;
        return;
      }
      li++;
      if (!r) break;
      q = r + 1;
    }
  });
  for (int t = 0; t < T; t++)
    if (bad[t]) return VAME_E_INVALID;
  return VAME_OK;
}

int vame_log_remove_old(const char* prefix) {
  if (!prefix) return VAME_E_INVALID;
  // main_aux_functions.h:1555-1570: every PRED type x the 12 FULL size names
  static const char* types[4] = {"FULL_2CPs", "FULL_3CPs", "HALF_2CPs", "HALF_3CPs"};
  for (int t = 0; t < 4; t++)
    for (int g = 0; g < kFullGroups; g++) {
      std::string p = std::string(prefix) + "_" + types[t] + "_" + size_name(0, g) + ".csv";
      remove(p.c_str());
    }
  return VAME_OK;
}

int vame_log_write_headers(const char* prefix, int pred) {
  if (!prefix || pred < 0 || pred > 3) return VAME_E_INVALID;
  const int ng = (pred >> 1) ? kHalfGroups : kFullGroups;
  for (int g = 0; g < ng; g++) {  // main_aux_functions.h:410-433 ("w" + header per group)
    std::string p = log_path(prefix, pred, g);
    FILE* f = fopen(p.c_str(), "w");
    if (!f) return VAME_E_INVALID;
    fputs(kHeader, f);
    fclose(f);
  }
  return VAME_OK;
}

long long vame_log_append(const char* prefix, int pred, int width, int height, int poc, int ref,
                          const int64_t* cost, const vame_cpmvs* cpmvs, int nthreads) {
  if (!prefix || pred < 0 || pred > 3 || !cost || !cpmvs) return VAME_E_INVALID;
  const int nCtus = num_ctus(width, height);
  if (!nCtus) return VAME_E_INVALID;
  const int align = pred >> 1;
  const int ng = align ? kHalfGroups : kFullGroups;
  const int ctuCols = (width + kCtu - 1) / kCtu;  // ceil((float)W/128), exact here (T8)
  // tasks = (group, CTU chunk); each produces one byte string
  const int chunk = 64;
  const int nchunks = (nCtus + chunk - 1) / chunk;
  const int ntasks = ng * nchunks;
  std::vector<Buf> out(ntasks);
  // threads of this call only: the entry point stays reentrant and fork-safe
  parallel_for(pick_threads(nthreads, ntasks), ntasks, [&](int i, int) {
    const int g = i / nchunks, c = i % nchunks;
    format_rows(out[i], align, g, c * chunk, std::min(nCtus, (c + 1) * chunk), ctuCols, poc, ref,
                cost, cpmvs);
  });
  long long total = 0;
  for (int g = 0; g < ng; g++) {  // append in group order (duplicate HALF names share a file)
    std::string p = log_path(prefix, pred, g);
    FILE* f = fopen(p.c_str(), "a");
    if (!f) return VAME_E_INVALID;
    for (int c = 0; c < nchunks; c++) {
      const Buf& s = out[g * nchunks + c];
      if (s.len && fwrite(s.d.get(), 1, s.len, f) != s.len) {
        fclose(f);
        return VAME_E_INVALID;
      }
      total += (long long)s.len;
    }
    fclose(f);
  }
  return total;
}

int vame_log_file_count(int pred) {
  if (pred < 0 || pred > 3) return VAME_E_INVALID;
  const int align = pred >> 1, ng = align ? kHalfGroups : kFullGroups;
  std::vector<std::string> names;
  for (int g = 0; g < ng; g++) names.push_back(size_name(align, g));
  std::sort(names.begin(), names.end());
  return (int)(std::unique(names.begin(), names.end()) - names.begin());
}

}  // extern "C"
