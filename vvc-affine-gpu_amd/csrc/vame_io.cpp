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
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vame.h"
#include "vame_tables.h"

using namespace vame;

namespace {

int pick_threads(int requested, long work_items) {
  int t = requested > 0 ? requested : (int)std::thread::hardware_concurrency();
  t = std::max(1, std::min(t, 64));
  return (int)std::max(1L, std::min<long>(t, work_items));
}

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

inline char* put(char* p, long long v) { return std::to_chars(p, p + 24, v).ptr; }

// Rows of one (group, CTU range) in the reference's fprintf format
// "%d,%d,%d,%d,%d,%d,%d,%ld,%d,%d,%d,%d,%d,%d\n" (main_aux_functions.h:491).
void format_rows(std::string& buf, int align, int g, int ctu0, int ctu1, int ctuCols, int poc,
                 int ref, const int64_t* cost, const vame_cpmvs* cp) {
  const int ncu = align ? kHalfN[g] : (kFullStride[g + 1] - kFullStride[g]);
  const int stride = align ? kHalfStride[g] : kFullStride[g];
  const int T = align ? kHalfCusPerCtu : kFullCusPerCtu;
  buf.resize((size_t)(ctu1 - ctu0) * ncu * 160);
  char* p = &buf[0];
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
  buf.resize((size_t)(p - &buf[0]));
}

}  // namespace

extern "C" {

int vame_read_frames(const char* path, int width, int height, int nframes, uint16_t* out,
                     int nthreads) {
  if (!path || !out || width <= 0 || height <= 0 || nframes <= 0) return VAME_E_INVALID;
  Mapped m;
  int rc = map_file(path, m);
  if (rc) return rc;
  const size_t fsz = (size_t)width * height;
  if (ends_with(path, ".u16") || ends_with(path, ".yuv")) {  // raw 16-bit side path
    if (m.n < fsz * nframes * 2) return VAME_E_INVALID;
    memcpy(out, m.p, fsz * nframes * 2);
    return VAME_OK;
  }
  const long nlines = (long)nframes * height;
  const char* base = m.p;
  const size_t n = m.n;
  if (n == 0) return VAME_E_INVALID;
  // pass 1: newline count per byte range
  const int T = pick_threads(nthreads, (long)(n >> 20) + 1);
  std::vector<size_t> cut(T + 1);
  for (int t = 0; t <= T; t++) cut[t] = n * t / T;
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
  // line index of the first line starting in range t: lines start at 0 and after each '\n'
  std::vector<long> first(T + 1, 0);
  for (int t = 0; t < T; t++) first[t + 1] = first[t] + nl[t];
  const long total_lines = first[T] + (base[n - 1] != '\n' ? 1 : 0);
  if (total_lines < nlines) return VAME_E_INVALID;
  // pass 2: parse the lines that START in each range (line 0 starts at byte 0)
  std::vector<int> bad(T, 0);
  parallel_for(T, T, [&](int t, int) {
    const char* q = base + cut[t];
    long li = first[t];
    if (t > 0) {  // skip the tail of a line started in an earlier range
      if (base[cut[t] - 1] != '\n') {
        const char* r = (const char*)memchr(q, '\n', (size_t)(base + cut[t + 1] - q));
        if (!r) return;
        q = r + 1;
        li++;  // first[t] is the line that straddles cut[t]; q starts the next one
      }
    }
    const char* end = base + cut[t + 1];
    while (q < end && li < nlines) {
      const char* r = (const char*)memchr(q, '\n', (size_t)(base + n - q));
      const char* le = r ? r : base + n;
      if (!parse_line(q, le, width, out + (size_t)li * width)) {
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
  std::vector<std::string> out(ntasks);
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
      const std::string& s = out[g * nchunks + c];
      if (fwrite(s.data(), 1, s.size(), f) != s.size()) {
        fclose(f);
        return VAME_E_INVALID;
      }
      total += (long long)s.size();
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
