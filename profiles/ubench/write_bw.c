// Host write bandwidth of one rank's log block into shared files (the
// frame-shard merge, vame_log_writer_flush_at): B bytes into F files at a
// byte offset, T threads, 32 MiB pieces, by (0) pwrite, (1) fallocate +
// mmap(MAP_SHARED) + memcpy, (2) the same with MAP_POPULATE, (3) with
// madvise(MADV_POPULATE_WRITE).  The files hold one rank's bytes after O bytes of
// another rank's (written first, untimed).
//   gcc -O2 -o write_bw write_bw.c -lpthread && ./write_bw <dir> <MB> <files> <threads> <mode>
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>
static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }
typedef struct { int fd; size_t off, n; const char* src; int mode; } Piece;
static Piece* P; static int NP, next_piece; static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static void* work(void* a) {
  (void)a;
  for (;;) {
    pthread_mutex_lock(&mu); int k = next_piece++; pthread_mutex_unlock(&mu);
    if (k >= NP) return 0;
    Piece* p = &P[k];
    if (p->mode == 0) {
      size_t d = 0;
      while (d < p->n) { ssize_t r = pwrite(p->fd, p->src + d, p->n - d, p->off + d); if (r <= 0) { perror("pwrite"); exit(1); } d += r; }
    } else {
      const size_t pg = 4096, a0 = p->off & ~(pg - 1), lead = p->off - a0;
      char* m = mmap(0, p->n + lead, PROT_READ | PROT_WRITE, MAP_SHARED | (p->mode == 2 ? MAP_POPULATE : 0), p->fd, a0);
      if (m == MAP_FAILED) { perror("mmap"); exit(1); }
#ifdef MADV_POPULATE_WRITE
      if (p->mode == 3 && madvise(m, p->n + lead, MADV_POPULATE_WRITE) != 0) { perror("madvise"); exit(1); }
#endif
      memcpy(m + lead, p->src, p->n);
      munmap(m, p->n + lead);
    }
  }
}
int main(int argc, char** argv) {
  const char* dir = argv[1]; size_t B = (size_t)atol(argv[2]) << 20; int F = atoi(argv[3]), T = atoi(argv[4]), mode = atoi(argv[5]);
  const size_t piece = 32u << 20, O = 12345677;  // a previous rank's bytes, odd length
  char* src = malloc(B); for (size_t i = 0; i < B; i++) src[i] = "0123456789,\n"[i % 12];
  int* fd = malloc(F * sizeof(int)); size_t per = B / F;
  for (int f = 0; f < F; f++) {
    char name[512]; snprintf(name, sizeof name, "%s/wbw_%d.csv", dir, f);
    unlink(name); fd[f] = open(name, O_RDWR | O_CREAT, 0644);
    size_t d = 0; while (d < O) { ssize_t r = pwrite(fd[f], src, O - d < per ? O - d : per, d); d += r; }
  }
  P = malloc(sizeof(Piece) * (B / piece + 2 * F + 2)); NP = 0;
  double t0 = now();
  for (int f = 0; f < F; f++) {
    if (mode >= 1 && fallocate(fd[f], 0, O, per) != 0) { perror("fallocate"); return 1; }
    for (size_t o = 0; o < per; o += piece) P[NP++] = (Piece){fd[f], O + o, o + piece < per ? piece : per - o, src + (size_t)f * per + o, mode};
  }
  pthread_t th[128]; for (int t = 0; t < T; t++) pthread_create(&th[t], 0, work, 0);
  for (int t = 0; t < T; t++) pthread_join(th[t], 0);
  double t1 = now();
  printf("mode %d (%s): %zu MB into %d files, %d threads: %.3f s, %.1f GB/s\n", mode, mode == 0 ? "pwrite" : mode == 1 ? "fallocate+mmap" : mode == 2 ? "+MAP_POPULATE" : "+MADV_POPULATE_WRITE",
         B >> 20, F, T, t1 - t0, B / (t1 - t0) / 1e9);
  for (int f = 0; f < F; f++) { char name[512]; snprintf(name, sizeof name, "%s/wbw_%d.csv", dir, f); close(fd[f]); unlink(name); }
  return 0;
}
