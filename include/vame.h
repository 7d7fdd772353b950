/*
 * vame.h -- C ABI of the MI355X affine motion-estimation engine (libvame.so).
 *
 * Drop-in boundary for the reference's hot path (iagostorch/VVC-Affine-GPU):
 * what the reference host does with clSetKernelArg + clEnqueueNDRangeKernel on
 *   affine_gradient_mult_sizes     (affine.cl:11,  aligned CUs)      and
 *   affine_gradient_mult_sizes_HA  (affine.cl:960, half-aligned CUs)
 * compiled with -DnCP=2|3 (main.cpp:389-392) and launched at main.cpp:827-966
 * is one call of vame_affine_me() here.  The gradient / equation scratch
 * buffers of the reference signature (args 5-7) and its unused debug args
 * (11-12) disappear: all scratch lives in LDS and registers.
 *
 * Plain pointers and sizes only.  Frame / result pointers are DEVICE pointers
 * (hipMalloc'd or torch.cuda tensors) unless a function says otherwise; every
 * call is asynchronous on `stream` (a hipStream_t, NULL = default stream).
 * Results use the reference's return-array layout (affine.cl:936, :1929):
 *   index = ctu * {201 | 284} + RETURN_STRIDE[group] + cuIdx
 * so the host's decision-log writer (main_aux_functions.h:387-525) is unchanged.
 * A context is bound to one device and is not thread-safe; use one per GPU per
 * host thread.  Functions return 0 or a negative VAME_E* code.
 */
#ifndef VAME_H
#define VAME_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* typedef.h:1-8 Mv / Cpmvs, same 28-byte layout.  1/16-pel units. */
typedef struct { int32_t x, y; } vame_mv;
typedef struct { int32_t nCPs; vame_mv LT, RT, LB; } vame_cpmvs;

enum { VAME_ALIGN_FULL = 0, VAME_ALIGN_HALF = 1 };
/* mode_mask bits of the fused calls: 2CP (required), 3CP (seeded by 2CP), and
 * an optional alignment selection -- FULL and/or HALF; neither bit = both, as
 * the reference codes them (the vame CLI's --align) */
enum { VAME_MODE_2CP = 1, VAME_MODE_3CP = 2, VAME_MODE_FULL = 4, VAME_MODE_HALF = 8 };
/* The PREDs (bit m = FULL_2CP, FULL_3CP, HALF_2CP, HALF_3CP) a valid mode_mask
 * codes: the vame_poc_result entries it writes, the log files it feeds. */
int vame_pred_mask(int mode_mask);

enum {
  VAME_OK = 0,
  VAME_E_INVALID = -1,     /* bad argument (resolution, nCP, align, null pointer ...) */
  VAME_E_DEVICE = -2,      /* HIP runtime error (see vame_last_hip_error) */
  VAME_E_NOMEM = -3,
  VAME_E_UNSUPPORTED = -4  /* e.g. more than 4 reference frames */
};

typedef struct vame_ctx vame_ctx;

/* Output slots of the fused per-POC call: [ref][FULL_2CP, FULL_3CP, HALF_2CP, HALF_3CP].
 * cost/cpmvs of slot (r, m) must hold nCtus*{201|284} entries (or be NULL when the
 * mode is not requested).  Mirrors the four return_* memory objects per refIdx
 * of main.cpp:484-504. */
typedef struct {
  int64_t* cost[4][4];
  vame_cpmvs* cpmvs[4][4];
} vame_poc_result;

/* Create a context on HIP device `device` for frames of width x height (one of
 * the reference's resolutions: constants.h:73-79 / main.cpp:257-265).
 * Every device buffer the launches use is allocated here (the reference
 * allocates its buffers before the POC loop, main.cpp:473-552), among them the
 * 3-CP seed-reuse scratch for 32 pairs per launch (~1 GB at 3840x2160; see
 * vame_set_max_pairs): no launch allocates, so a call may be captured into a
 * hipGraph on the caller's stream.  Runtime knobs, read here (results are
 * bit-identical under every setting; the defaults are the measured best on
 * MI355X):
 *   VAME_STREAMS       2 (default): the quadrant kernel on a side stream of the
 *                      context, forked from and joined into the caller's stream;
 *                      1: every kernel on the caller's stream
 *   VAME_SYNC          1 (default): the join as a stream memory operation;
 *                      0: an event
 *   VAME_GROUP_COMBOS  (CTU, pair) combinations per block-order group (408) */
int vame_create(vame_ctx** out, int device, int width, int height);
void vame_destroy(vame_ctx* ctx);
/* (POC, refIdx) pairs per launch of the fused calls, 1..32 (default 32): the
 * seed-reuse scratch is re-sized for it (synchronizes the device; outside any
 * capture), batches are cut into launches of at most that many pairs.  A
 * caller coding a few pairs per call (the CLI: one POC, <= 4 pairs) keeps the
 * scratch at 1/8 of the default.  vame_get_max_pairs returns the setting. */
int vame_set_max_pairs(vame_ctx* ctx, int max_pairs);
int vame_get_max_pairs(vame_ctx* ctx);

/* One reference launch (affine.cl:11 or :960 built with -DnCP=nCP).
 *   ref, cur : W*H uint16 samples (10-bit), device memory
 *   lambda   : motion lambda (float kernel arg 4, main.cpp:585/831)
 *   prev     : nCP==3 only: the same-alignment 2-CP result of this (POC, ref)
 *              (gPrevCpmvs, main.cpp:777/908); NULL for nCP==2
 *   cost     : nCtus*{201|284} int64 best RD cost per candidate CU
 *   cpmvs    : same count, best CPMVs (LB = 0 for 2 CPs)                       */
int vame_affine_me(vame_ctx* ctx, const uint16_t* ref, const uint16_t* cur, float lambda,
                   int align, int nCP, int extra_grad_iter, const vame_cpmvs* prev,
                   int64_t* cost, vame_cpmvs* cpmvs, void* stream);

/* Fused per-POC call: every ref x {FULL, HALF} x {2CP -> 3CP} in one pass
 * (the whole refIdx loop of main.cpp:746-966).  3-CP seeds come from the 2-CP
 * result of the same CU inside the kernel (no round trip through memory). */
int vame_affine_me_poc(vame_ctx* ctx, const uint16_t* cur, const uint16_t* const* refs,
                       int nrefs, float lambda, int mode_mask, int extra_grad_iter,
                       const vame_poc_result* out, void* stream);

/* Batched fused call: several POCs (each one vame_affine_me_poc) in as few
 * launches as possible (vame_get_max_pairs() (POC, refIdx) pairs per launch,
 * default 32), so consecutive
 * POCs share one grid -- no launch gaps or tails between them.  Results are
 * identical to one vame_affine_me_poc per job. */
typedef struct {
  const uint16_t* cur;              /* orig of the POC */
  const uint16_t* const* refs;      /* its nrefs (1..4) reference frames, refIdx order */
  int nrefs;
  float lambda;
  const vame_poc_result* out;
} vame_poc_job;
int vame_affine_me_batch(vame_ctx* ctx, const vame_poc_job* jobs, int njobs, int mode_mask,
                         int extra_grad_iter, void* stream);

/* The compact wire form of the jobs' decision records, for the frame-shard
 * gather into rank 0 (vame/shard.py pack() is its
 * specification): for each job in order, refIdx 0..nrefs-1, each PRED of
 * vame_pred_mask(mode_mask) in PRED order: the nCtus*{201|284} costs as
 * int32, then the records' CPMV components (LT, RT, and LB for 3-CP: 4 or 6
 * int32 each).  `slab` (device, `words` int32) is zero-filled past the
 * records; `*bad` (device int32) is OR-ed with 1 when a record does not fit
 * the form (cost outside [0, 2^31), 2-CP LB != 0).  One kernel on `stream`;
 * the jobs' cur / refs / lambda are not read.  VAME_E_INVALID when the records
 * exceed `words`. */
int vame_pack_records(vame_ctx* ctx, const vame_poc_job* jobs, int njobs, int mode_mask, int32_t* slab,
                      long long words, int32_t* bad, void* stream);

/* PROF (prediction refinement with optical flow).  The reference carries the
 * code but hard-disables it (`int enablePROF=0`, affine.cl:168 / :1132;
 * aux_functions.cl:215-605, :1096-1239); enable != 0 turns it on for the
 * context's later launches (both entry points), exactly as the reference's
 * functions compute it with enablePROF = 1.  Default off = reference behaviour. */
int vame_set_prof(vame_ctx* ctx, int enable);

/* Device-side kernel timing (the reference's per-PRED kernelExecutionTime,
 * main.cpp:856-866): when enabled, every kernel launch carries hipEvents in its
 * own dispatch on the stream it runs on.  kernel_class 0 = quadrant work items
 * (affine_me_quad); 3 = the 128x128 CUs (affine_me_ctu2); 4 / 5 = the 128x64 /
 * 64x128 CUs (affine_me_half2w / _half2h); under PROF 1 = the 128x128 CUs
 * (affine_me_ctu_prof), 2 = the 128x64 / 64x128 CUs (affine_me_half_prof).
 * enable = 2 times the quadrant kernel only (its dispatches carry the events;
 * the 128-class launches run untimed).  vame_get_timing waits for the recorded
 * launches and returns their summed duration and count since the last reset.
 * enable | VAME_TIMING_KEEP changes what later launches record without
 * dropping the launches recorded so far (timing a sample of a run's steps).
 * Launches on a stream under capture carry no events. */
enum { VAME_TIMING_KEEP = 16 };
int vame_set_timing(vame_ctx* ctx, int enable);
int vame_get_timing(vame_ctx* ctx, int kernel_class, double* total_ms, int* launches, int reset);

/* Work-item templates (no device work): how many times the engine's work
 * items -- quadrant, 128x128 and 128x64 / 64x128 items, as vame_create builds
 * them -- cover each of the CTU's candidate CUs of `align`: hits[0 ..
 * {201|284}) indexed by the output offset RETURN_STRIDE[group] + cuIdx
 * (affine.cl:936 / :1929).  A valid partition covers every CU exactly once
 * (the quadrant items of one-alignment launches; VAME_E_INVALID if those of
 * both-alignment launches cover differently).  half128 must be non-zero (the
 * one packing: every 128x64 / 64x128 CU a work item of its own).  Also returns
 * the item counts per kernel class (quad -- of a both-alignment launch --,
 * 128x128, 128x64 + 64x128) in items3 when non-NULL. */
int vame_template_coverage(int half128, int align, int32_t* hits, int32_t* items3);

/* Geometry / host helpers (no device work). */
int vame_num_ctus(int width, int height);   /* 0 if unsupported */
int vame_cus_per_ctu(int align);            /* 201 / 284 */
int vame_num_groups(int align);             /* 12 / 24 */
/* CU group g: size, count, return stride, CTU-relative positions (xs/ys >= 64 entries) */
int vame_group_geometry(int align, int g, int* w, int* h, int* ncu, int* stride, int* xs,
                        int* ys);
/* Motion lambda of a POC (main.cpp:585 -> main_aux_functions.h:1482-1497, constants.h:94-103) */
float vame_lambda(int qp, int poc);
int vame_poc_qp(int qp, int poc);
/* Reference-picture list of a POC (main.cpp:591-707): fills pocs[0..min(4,poc)-1]
 * with the POC held by each refIdx slot; returns the number of refs. */
int vame_ref_list(int poc, int* pocs);

/* ---- Host I/O contracts of the reference's ./main (no device work) ---- */

/* Frame ingest (main.cpp:293-330): reads `nframes` frames of width x height
 * samples into `out` (host, nframes*W*H uint16).  CSV layout as the reference
 * reads it: one frame line per text line, ',' separated, frames stacked; each
 * value parsed like stoi and stored as unsigned short.  Paths ending in .u16 /
 * .yuv are raw little-endian 16-bit frames.  nthreads <= 0: all host cores.
 * Returns 0, or VAME_E_INVALID for a missing file / short file / bad value. */
int vame_read_frames(const char* path, int width, int height, int nframes, uint16_t* out,
                     int nthreads);
/* The same for frames first .. first + nframes - 1 of the file (a frame-sharded
 * rank reads only the frames its POC block uses). */
int vame_read_frames_range(const char* path, int width, int height, int first, int nframes,
                           uint16_t* out, int nthreads);
/* The same, reading only the bytes [span_begin, span_end) of a CSV (span_end < 0:
 * to the end), which must hold every line of those frames, with lines_before =
 * the number of '\n' in [0, span_begin) -- so a rank whose frames lie deep in
 * a large file does not scan the bytes ahead of them.  vame_count_lines counts
 * the '\n' of [begin, end) (end < 0: to the end; ranks count disjoint chunks
 * and exchange the counts). */
long long vame_count_lines(const char* path, long long begin, long long end, int nthreads);
/* The '\n' counts of n byte ranges [begin[i], end[i]) of one file, into
 * counts[i], in one pass over one mapping with one set of threads (a rank's
 * chunks of a CSV: calling vame_count_lines per chunk paid a mapping and a
 * thread start per 16 MB chunk).  Returns VAME_OK, or VAME_E_INVALID for a
 * missing file, a negative or reversed range. */
int vame_count_lines_ranges(const char* path, const long long* begin, const long long* end, int n,
                            long long* counts, int nthreads);
int vame_read_frames_span(const char* path, int width, int height, int first, int nframes,
                          long long span_begin, long long lines_before, long long span_end,
                          uint16_t* out, int nthreads);

/* Decision log (main_aux_functions.h:387-525, 1547-1585).  pred = 0 FULL_2CP,
 * 1 FULL_3CP, 2 HALF_2CP, 3 HALF_3CP (constants.h:15-21).  Files are
 * <prefix>_<FULL|HALF>_<2|3>CPs_<W>x<H>.csv with the reference's header.
 *   vame_log_remove_old    : removeOldTraces (:1547) -- deletes the old files
 *   vame_log_write_headers : creates/truncates the files of one pred with the
 *                            header (done by the reference at POC 1, refIdx 0)
 *   vame_log_append        : appends the rows of one (POC, refIdx, pred) from
 *                            HOST result arrays in the reference's index layout;
 *                            returns the number of bytes written (< 0: error)
 *   vame_log_file_count    : distinct files of a pred (12 FULL, 8 HALF)        */
int vame_log_remove_old(const char* prefix);
int vame_log_write_headers(const char* prefix, int pred);
long long vame_log_append(const char* prefix, int pred, int width, int height, int poc, int ref,
                          const int64_t* cost, const vame_cpmvs* cpmvs, int nthreads);
int vame_log_file_count(int pred);

/* The same log, a whole POC per call (the CLI's path): a writer holds a
 * persistent thread pool and the open files of one prefix.  One call appends
 * the rows of every refIdx r < nrefs and PRED m in pred_mask (bit m), from the
 * host arrays cost[r*4 + m] / cpmvs[r*4 + m] (entries of PREDs outside the
 * mask may be NULL); the files receive exactly the bytes of the reference's
 * per-(POC, refIdx, PRED) appends in main.cpp:942-958 order (refIdx outer,
 * PRED inner).  Headers stay with vame_log_write_headers (POC 1, before the
 * first call).  Returns the bytes written (< 0: error).
 *   vame_log_writer_create : NULL on a bad prefix / unsupported resolution;
 *                            nthreads <= 0: all host cores                   */
typedef struct vame_log_writer vame_log_writer;
vame_log_writer* vame_log_writer_create(const char* prefix, int width, int height, int nthreads);
long long vame_log_writer_poc(vame_log_writer* w, int poc, int nrefs, int pred_mask,
                              const int64_t* const* cost, const vame_cpmvs* const* cpmvs);
/* The same for refIdx ref0 .. ref0 + nrefs - 1 only (arrays indexed
 * (r - ref0)*4 + m): a POC whose refIdx range is cut between two frame-shard
 * ranks is logged by each for its own refs, in the same order. */
long long vame_log_writer_refs(vame_log_writer* w, int poc, int ref0, int nrefs, int pred_mask,
                               const int64_t* const* cost, const vame_cpmvs* const* cpmvs);
int vame_log_writer_destroy(vame_log_writer* w);
/* Deferred mode, for a frame-shard rank whose rows belong in the middle of
 * the files: after vame_log_writer_set_deferred(w, 1) (before its first POC;
 * VAME_E_INVALID once rows were logged) the writer keeps each
 * file's rows in host memory instead of appending them.  Its files are
 * numbered 0 .. vame_log_writer_num_files - 1 (vame_log_writer_file_name);
 * vame_log_writer_sizes reports the bytes held per file, and
 * vame_log_writer_flush_at writes every file's rows at offsets[f] (pwrite;
 * the file is created if missing and never truncated), files in parallel,
 * returning the bytes written -- so the ranks of a node, once they know each
 * other's sizes, place their blocks into the one set of files at once. */
int vame_log_writer_set_deferred(vame_log_writer* w, int deferred);
int vame_log_writer_num_files(vame_log_writer* w);
int vame_log_writer_file_name(vame_log_writer* w, int f, char* buf, int buflen);
int vame_log_writer_sizes(vame_log_writer* w, long long* sizes);
long long vame_log_writer_flush_at(vame_log_writer* w, const long long* offsets);

const char* vame_strerror(int code);
const char* vame_last_hip_error(void);
const char* vame_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VAME_H */
