/* tools/scalar_mt.c -- the scalar service under concurrent callers: T threads (1, 2, 4, 8, 16)
 * each call pdb_crc32c_value on an sstable-block-sized input (4172 B: contents + type of a db_bench
 * data block) for ~1 s, the way an engine's reader threads each verify one block per point read
 * (table/format.cc:96-104).  Every answer is checked against the thread's first one.  Prints one
 * JSON line: calls/s in aggregate and us per call per thread, for each T.
 * Build: gcc -O2 -pthread -o tools/_scalar_mt tools/scalar_mt.c -Iinclude -Lpebblesdb_amd/_lib \
 *   -lpdb_crc32c -Wl,-rpath,'$ORIGIN/../pebblesdb_amd/_lib' */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "pdb_crc32c.h"

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

enum { kLen = 4172, kMaxT = 16 };
static uint8_t g_buf[kMaxT][kLen + 64];
static volatile int g_go = 0;

typedef struct {
  int t;
  double seconds;
  long calls;
  long bad;
} Arg;

static void* body(void* p) {
  Arg* a = (Arg*)p;
  const uint8_t* d = g_buf[a->t] + (a->t & 15);
  const uint32_t want = pdb_crc32c_value(d, kLen);
  while (!g_go) {
  }
  const double t0 = now_s();
  long n = 0, bad = 0;
  while (now_s() - t0 < 1.0) {
    for (int k = 0; k < 64; ++k) bad += pdb_crc32c_value(d, kLen) != want;
    n += 64;
  }
  a->seconds = now_s() - t0;
  a->calls = n;
  a->bad = bad;
  return NULL;
}

int main(void) {
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int t = 0; t < kMaxT; ++t)
    for (int i = 0; i < kLen + 64; ++i) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      g_buf[t][i] = (uint8_t)x;
    }
  if (pdb_crc32c_init(0) != 0) {
    fprintf(stderr, "init failed: %s\n", pdb_last_error());
    return 1;
  }
  static const int ts[] = {1, 2, 4, 8, 16};
  printf("{\"tool\": \"scalar_mt\", \"bytes\": %d, \"runs\": [", kLen);
  for (size_t r = 0; r < sizeof(ts) / sizeof(ts[0]); ++r) {
    const int T = ts[r];
    pthread_t th[kMaxT];
    Arg a[kMaxT];
    g_go = 0;
    for (int t = 0; t < T; ++t) {
      a[t].t = t;
      pthread_create(&th[t], NULL, body, &a[t]);
    }
    const double w0 = now_s();
    g_go = 1;
    long calls = 0, bad = 0;
    double tsum = 0;
    for (int t = 0; t < T; ++t) {
      pthread_join(th[t], NULL);
      calls += a[t].calls;
      bad += a[t].bad;
      tsum += a[t].seconds;
    }
    const double wall = now_s() - w0;
    printf("%s{\"threads\": %d, \"calls_per_s\": %.0f, \"us_per_call_per_thread\": %.3f, \"bad\": %ld}",
           r ? ", " : "", T, calls / wall, tsum * 1e6 / calls, bad);
    fflush(stdout);
  }
  printf("]}\n");
  return 0;
}
