/* vame_synth.c -- native generator of the synthetic 10-bit test sequences
 * (vame/synth.py is the specification; tests/test_synth.py checks the two
 * agree bit for bit).  Bench / test data only, not part of the product path:
 * the reference's data/ CSVs are absent, and a 240-frame
 * 3840x2160 sequence (BASELINE configs[4]) takes hours in numpy.
 *
 * Every value is built from integer hashing and +, -, *, /, floor on binary64
 * in the same order as the numpy code (compiled with -ffp-contract=off), so
 * the bytes are identical.  The camera parameters (cos / sin) come from the
 * caller, so no libm transcendental is involved here.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t mix64(uint64_t z) { /* SplitMix64 finaliser */
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline uint64_t hash2(int64_t ix, int64_t iy, uint64_t salt) {
  return mix64((uint64_t)ix * 0x9E3779B97F4A7C15ull + (uint64_t)iy * 0xC2B2AE3D27D4EB4Full + salt);
}

static inline double lattice(int64_t ix, int64_t iy, uint64_t salt) {
  return (double)(hash2(ix, iy, salt) >> 11) * (1.0 / 9007199254740992.0);
}

static inline double value_noise(double x, double y, double scale, uint64_t salt) {
  const double u = x / scale, v = y / scale;
  const double iu = floor(u), iv = floor(v);
  const double fu = u - iu, fv = v - iv;
  const int64_t ju = (int64_t)iu, jv = (int64_t)iv;
  const double a = lattice(ju, jv, salt), b = lattice(ju + 1, jv, salt);
  const double c = lattice(ju, jv + 1, salt), d = lattice(ju + 1, jv + 1, salt);
  const double top = a + (b - a) * fu;
  const double bot = c + (d - c) * fu;
  return top + (bot - top) * fv - 0.5;
}

static inline double tri(double t) { return fabs(t - floor(t) - 0.5) - 0.25; }

static const double kOct[5][2] = {{61.0, 420.0}, {29.0, 230.0}, {13.0, 120.0}, {6.5, 60.0}, {3.1, 28.0}};
static const double kGrat[3][4] = {{0.8, 0.6, 37.0, 240.0}, {-0.28, 0.96, 17.0, 160.0}, {0.96, -0.28, 91.0, 200.0}};

static inline double canvas(double x, double y, int W, int H, uint64_t seed) {
  double f = 512.0;
  for (int k = 0; k < 5; k++) f += kOct[k][1] * value_noise(x, y, kOct[k][0], seed * 131u + (uint64_t)k);
  for (int k = 0; k < 3; k++) f += kGrat[k][3] * tri((x * kGrat[k][0] + y * kGrat[k][1]) / kGrat[k][2]);
  const double fx0 = 0.30 * W, fy0 = 0.25 * H;
  if (x >= fx0 && x < fx0 + 96 && y >= fy0 && y < fy0 + 96) f = 600.0;
  const double bx0 = W - 64.0, by0 = H - 64.0;
  if (x >= bx0 && y >= by0) {
    const double s = floor((x - bx0) / 8.0) + floor((y - by0) / 8.0);
    f = fmod(s, 2.0) == 0.0 ? 980.0 : 40.0;
  }
  return f;
}

/* uniform integer in [-amp, amp] per pixel: ((h >> 32) * (2 amp + 1)) >> 32 - amp */
static inline int pixel_noise(int x, int y, uint64_t salt, int amp) {
  const uint64_t h = hash2(x, y, salt);
  return (int)(((h >> 32) * (uint64_t)(2 * amp + 1)) >> 32) - amp;
}

/* Original POC `poc` of the sequence `seed` (H x W).  zoom / ca / sa / tx / ty:
 * the camera of synth.camera(poc). */
void vame_synth_frame(int W, int H, uint64_t seed, int poc, double zoom, double ca, double sa,
                      double tx, double ty, uint16_t* out) {
  const double cx = W / 2.0, cy = H / 2.0;
  const uint64_t nsalt = seed * 1000003u + (uint64_t)poc;
#pragma omp parallel for schedule(static)
  for (int yy = 0; yy < H; yy++) {
    for (int xx = 0; xx < W; xx++) {
      const double px = ((double)xx - cx - tx) / zoom;
      const double py = ((double)yy - cy - ty) / zoom;
      const double sx = ca * px + sa * py + cx;
      const double sy = -sa * px + ca * py + cy;
      double f = floor(canvas(sx, sy, W, H, seed) + 0.5) + pixel_noise(xx, yy, nsalt, 2);
      f = f < 0 ? 0 : f > 1023 ? 1023 : f;
      out[(size_t)yy * W + xx] = (uint16_t)f;
    }
  }
}

/* Reconstruction of `frame` (POC poc): frame + uniform noise in [-amp, amp], clamped. */
void vame_synth_recon(const uint16_t* frame, int W, int H, uint64_t seed, int poc, int amp,
                      uint16_t* out) {
  const uint64_t salt = (seed ^ 0xC0FFEEu) * 7919u + (uint64_t)poc;
#pragma omp parallel for schedule(static)
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      int v = frame[(size_t)y * W + x] + (amp ? pixel_noise(x, y, salt, amp) : 0);
      v = v < 0 ? 0 : v > 1023 ? 1023 : v;
      out[(size_t)y * W + x] = (uint16_t)v;
    }
}

/* Frames in the reference CSV layout (main.cpp:313-328): one line per frame
 * row, ',' separated, frames stacked.  Rows are formatted in parallel into
 * per-row buffers and written in order.  Returns 0 or -1. */
int vame_synth_write_csv(const char* path, const uint16_t* frames, int n, int W, int H) {
  FILE* fp = fopen(path, "wb");
  if (!fp) return -1;
  const int rows = n * H, chunk = 256;
  char* buf = (char*)malloc((size_t)chunk * (size_t)W * 6 + 16);
  size_t* len = (size_t*)malloc(sizeof(size_t) * chunk);
  int rc = (buf && len) ? 0 : -1;
  for (int r0 = 0; r0 < rows && rc == 0; r0 += chunk) {
    const int nr = rows - r0 < chunk ? rows - r0 : chunk;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nr; i++) {
      const uint16_t* src = frames + (size_t)(r0 + i) * W;
      char* d = buf + (size_t)i * W * 6;
      char* p = d;
      for (int x = 0; x < W; x++) {
        unsigned v = src[x];
        char tmp[6];
        int k = 0;
        do {
          tmp[k++] = (char)('0' + v % 10);
          v /= 10;
        } while (v);
        while (k) *p++ = tmp[--k];
        *p++ = x + 1 < W ? ',' : '\n';
      }
      len[i] = (size_t)(p - d);
    }
    for (int i = 0; i < nr && rc == 0; i++)
      if (fwrite(buf + (size_t)i * W * 6, 1, len[i], fp) != len[i]) rc = -1;
  }
  free(buf);
  free(len);
  if (fclose(fp) != 0) rc = -1;
  return rc;
}
