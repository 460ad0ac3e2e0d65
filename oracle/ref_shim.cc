// oracle/ref_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// A C-linkage wrapper around the REFERENCE's own CRC32C, compiled together
// with /root/reference/src/util/crc32c.cc (left where it lies; never copied)
// by oracle/build_ref.sh into oracle/_ref/libpdbref.so.  Used to (1) generate
// the golden vectors in tests/golden/ and (2) time the reference CPU path as
// bench.py's cpu_baseline (kind "reference").  Nothing in pebblesdb_amd/ loads it.
//
// Wrapped interface: leveldb::crc32c::{Extend,Value,Mask,Unmask}
// (reference util/crc32c.h:14-40).
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include <string>

#include "util/crc32c.h"

namespace {
struct Blk {
  uint64_t off;
  uint32_t len;
  uint32_t init;
};
struct Job {
  const char* base;
  const Blk* blk;
  size_t lo, hi;
  uint32_t flags;
  uint32_t* out;
};
void* Work(void* a) {
  Job* j = static_cast<Job*>(a);
  for (size_t i = j->lo; i < j->hi; ++i) {
    uint32_t init = (j->flags & 2u) ? j->blk[i].init : 0u;
    uint32_t c = leveldb::crc32c::Extend(init, j->base + j->blk[i].off, j->blk[i].len);
    j->out[i] = (j->flags & 1u) ? leveldb::crc32c::Mask(c) : c;
  }
  return nullptr;
}
}  // namespace

extern "C" {
uint32_t ref_crc32c_extend(uint32_t init, const char* p, size_t n) {
  return leveldb::crc32c::Extend(init, p, n);
}
uint32_t ref_crc32c_value(const char* p, size_t n) { return leveldb::crc32c::Value(p, n); }
uint32_t ref_crc32c_mask(uint32_t c) { return leveldb::crc32c::Mask(c); }
uint32_t ref_crc32c_unmask(uint32_t c) { return leveldb::crc32c::Unmask(c); }

int ref_crc32c_batch(const char* base, const void* blk, size_t nblk, uint32_t flags,
                     uint32_t* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  Job jobs[256];
  const Blk* b = static_cast<const Blk*>(blk);
  for (int t = 0; t < nthreads; ++t)
    jobs[t] = Job{base, b, nblk * t / nthreads, nblk * (t + 1) / nthreads, flags, out};
  for (int t = 1; t < nthreads; ++t)
    if (pthread_create(&th[t], nullptr, Work, &jobs[t]) != 0) return -1;
  Work(&jobs[0]);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], nullptr);
  return 0;
}

// db_bench's `crc32c` benchmark loop (reference db/db_bench.cc:1112-1129): Value() over the same
// 4096 x 'x' buffer until `total` bytes; returns seconds, the last CRC in *crc (0xa46ab21f).
double ref_crc32c_dbbench_loop(uint64_t total, uint32_t* crc) {
  const std::string data(4096, 'x');
  uint64_t bytes = 0;
  uint32_t c = 0;
  timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  while (bytes < total) {
    c = leveldb::crc32c::Value(data.data(), data.size());
    bytes += data.size();
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (crc) *crc = c;
  return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
}
