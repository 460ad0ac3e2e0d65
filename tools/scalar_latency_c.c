/* tools/scalar_latency_c.c -- per-call cost of the scalar drop-in pdb_crc32c_extend
 * (leveldb::crc32c::Extend) from C, without Python/ctypes overhead: the cost a C++ caller such as
 * the reference's db_bench sees per call (log_writer.cc:121, table_builder.cc:197-199).
 * Prints one JSON line.  Build: gcc -O2 -o tools/_scalar_latency_c tools/scalar_latency_c.c \
 *   -Iinclude -Lpebblesdb_amd/_lib -lpdb_crc32c -Wl,-rpath,'$ORIGIN/../pebblesdb_amd/_lib' */
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

int main(void) {
  static const size_t sizes[] = {1, 16, 1024, 1100, 4096, 4101, 4172, 16384, 32768, 65536, 1u << 20};
  const size_t nsz = sizeof(sizes) / sizeof(sizes[0]);
  const size_t maxn = 1u << 20;
  uint8_t* buf = (uint8_t*)malloc(maxn + 64);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < maxn + 64; ++i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    buf[i] = (uint8_t)x;
  }
  if (pdb_crc32c_init(0) != 0) {
    fprintf(stderr, "init failed: %s\n", pdb_last_error());
    return 1;
  }
  printf("{\"metric\": \"pdb_crc32c_extend latency from C (host bytes -> CRC)\", \"sizes\": {");
  uint32_t sink = 0;
  for (size_t k = 0; k < nsz; ++k) {
    const size_t n = sizes[k];
    for (int i = 0; i < 50; ++i) sink ^= pdb_crc32c_extend(sink, buf + 3, n);
    const int reps = n >= (1u << 20) ? 200 : (n >= 32768 ? 2000 : 20000);
    const double t0 = now_s();
    for (int i = 0; i < reps; ++i) sink ^= pdb_crc32c_extend(i, buf + (i & 7), n);
    const double dt = (now_s() - t0) / reps;
    printf("%s\"%zu\": {\"us_per_call\": %.3f, \"reps\": %d", k ? ", " : "", n, dt * 1e6, reps);
    printf("}");
    fflush(stdout);
  }
  printf("}, \"sink\": %u}\n", sink);
  return 0;
}
