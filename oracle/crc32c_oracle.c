/*
 * oracle/crc32c_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference CRC32C (Castagnoli) used by PebblesDB's
 * sstable block trailers.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this file's library; the product path
 * (pebblesdb_amd/) never links or calls it.
 *
 * What it restates (file:line under /root/reference/src):
 *   - util/crc32c.cc:25-32   crc32_software(): init ^ 0xFFFFFFFF, align prefix
 *                            init_bytes = min(n, (4 - addr%4)%4), ^ 0xFFFFFFFF out
 *   - util/crc32c.cc:585-625 crc32c_sb8_64_bit(): Intel slicing-by-8, reflected,
 *                            byte loop over init_bytes, 8-byte main loop that
 *                            XORs the running crc into the first LE32 word and
 *                            looks the 8 bytes up in tables o88..o32, byte tail.
 *   - util/crc32c.cc:116-128 table comment: poly 0x1EDC6F41 reflected
 *                            (= 0x82F63B78); tables o32..o88 are T0..T7 where
 *                            T0 is the byte table and Tk[b] = T(k-1)[b] shifted
 *                            by one more zero byte.  Tables are GENERATED here,
 *                            not copied (util/crc32c.cc:130-556 holds literals).
 *   - util/crc32c.h:20-40    Value = Extend(0,..); Mask = ror32(crc,15)+0xa282ead8;
 *                            Unmask inverse.
 *   - table/table_builder.cc:187-205  block trailer = [type][Mask(crc(contents||type))]
 *   - table/format.cc:96-104          verify: Unmask(DecodeFixed32(data+n+1)) == Value(data,n+1)
 *
 * Parity pinning: tests/golden/*.json hold the reference's own known answers
 * (util/crc32c_test.cc:13-60) plus vectors produced by the reference's own
 * util/crc32c.cc compiled here (oracle/build_ref.sh -> oracle/_ref/).  The
 * tests check this restatement against every one of them.
 *
 * Two independent formulations are provided: a bit-serial CRC (the definition)
 * and the slicing-by-8 restatement (the reference's algorithm); tests assert
 * they agree, and the slicing-by-8 one is the timed CPU baseline.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_POLY_REFLECTED 0x82F63B78u
#define ORACLE_MASK_DELTA 0xa282ead8u

static uint32_t g_tab[8][256];
static int g_tab_ready = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY_REFLECTED : (c >> 1);
    g_tab[0][b] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t b = 0; b < 256; ++b)
      g_tab[t][b] = (g_tab[t - 1][b] >> 8) ^ g_tab[0][g_tab[t - 1][b] & 0xffu];
  g_tab_ready = 1;
}

static void ensure_tables(void) {
  if (!g_tab_ready) pthread_once(&g_once, build_tables);
}

/* Bit-serial definition: reflected CRC-32C, init/xorout 0xFFFFFFFF. */
uint32_t oracle_crc32c_extend_bitwise(uint32_t init_crc, const uint8_t* p, size_t n) {
  uint32_t c = init_crc ^ 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY_REFLECTED : (c >> 1);
  }
  return c ^ 0xFFFFFFFFu;
}

static inline uint32_t le32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4); /* little-endian host, as the reference assumes (crc32c.cc:604) */
  return v;
}

/* Restatement of crc32c_sb8_64_bit (util/crc32c.cc:585-625).  Note the
 * reference narrows `length` to uint32_t (crc32c.cc:589); the restatement keeps
 * size_t and the tests stay below 4 GiB per call, where both agree. */
static uint32_t sb8_body(uint32_t crc, const uint8_t* p, size_t length, size_t init_bytes) {
  size_t running = ((length - init_bytes) / 8) * 8;
  size_t end_bytes = length - init_bytes - running;
  for (size_t i = 0; i < init_bytes; ++i) crc = g_tab[0][(crc ^ *p++) & 0xffu] ^ (crc >> 8);
  for (size_t i = 0; i < running / 8; ++i) {
    uint32_t lo = crc ^ le32(p);
    uint32_t hi = le32(p + 4);
    p += 8;
    crc = g_tab[7][lo & 0xff] ^ g_tab[6][(lo >> 8) & 0xff] ^ g_tab[5][(lo >> 16) & 0xff] ^
          g_tab[4][lo >> 24] ^ g_tab[3][hi & 0xff] ^ g_tab[2][(hi >> 8) & 0xff] ^
          g_tab[1][(hi >> 16) & 0xff] ^ g_tab[0][hi >> 24];
  }
  for (size_t i = 0; i < end_bytes; ++i) crc = g_tab[0][(crc ^ *p++) & 0xffu] ^ (crc >> 8);
  return crc;
}

/* Restatement of crc32_software + Extend (util/crc32c.cc:25-32, 101-103). */
uint32_t oracle_crc32c_extend(uint32_t init_crc, const uint8_t* p, size_t n) {
  ensure_tables();
  uintptr_t x = (uintptr_t)p;
  size_t init = (size_t)(((x + 3) & ~(uintptr_t)3) - x);
  if (init > n) init = n;
  return sb8_body(init_crc ^ 0xFFFFFFFFu, p, n, init) ^ 0xFFFFFFFFu;
}

uint32_t oracle_crc32c_value(const uint8_t* p, size_t n) { return oracle_crc32c_extend(0, p, n); }

/* util/crc32c.h:29-40 */
uint32_t oracle_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + ORACLE_MASK_DELTA; }
uint32_t oracle_crc32c_unmask(uint32_t m) {
  uint32_t rot = m - ORACLE_MASK_DELTA;
  return (rot >> 17) | (rot << 15);
}

/* Batch over a descriptor list {off,len,init} (the same 16-byte layout as the
 * product's pdb_blk).  flags: bit0 = mask output, bit1 = use per-block init. */
typedef struct {
  uint64_t off;
  uint32_t len;
  uint32_t init;
} oracle_blk;

typedef struct {
  const uint8_t* base;
  const oracle_blk* blk;
  size_t lo, hi;
  uint32_t flags;
  uint32_t* out;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    uint32_t init = (j->flags & 2u) ? j->blk[i].init : 0u;
    uint32_t c = oracle_crc32c_extend(init, j->base + j->blk[i].off, j->blk[i].len);
    j->out[i] = (j->flags & 1u) ? oracle_crc32c_mask(c) : c;
  }
  return NULL;
}

/* Multi-threaded batch: disjoint contiguous block ranges per thread (the
 * reference's CRC is pure/reentrant: util/crc32c.h:14-17). */
int oracle_crc32c_batch(const uint8_t* base, const oracle_blk* blk, size_t nblk, uint32_t flags,
                        uint32_t* out, int nthreads) {
  ensure_tables();
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((size_t)nthreads > nblk) nthreads = nblk ? (int)nblk : 1;
  pthread_t th[256];
  batch_job jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].base = base;
    jobs[t].blk = blk;
    jobs[t].lo = nblk * (size_t)t / (size_t)nthreads;
    jobs[t].hi = nblk * (size_t)(t + 1) / (size_t)nthreads;
    jobs[t].flags = flags;
    jobs[t].out = out;
  }
  for (int t = 1; t < nthreads; ++t)
    if (pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0) return -1;
  batch_worker(&jobs[0]);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* Fixed-stride batch: block i at base + i*stride, len bytes. */
int oracle_crc32c_batch_fixed(const uint8_t* base, uint64_t stride, uint32_t len, size_t nblk,
                              uint32_t flags, uint32_t* out, int nthreads) {
  ensure_tables();
  (void)flags;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  /* Reuse the descriptor worker with a small on-stack chunking loop. */
  enum { CH = 4096 };
  oracle_blk tmp[CH];
  for (size_t lo = 0; lo < nblk; lo += CH) {
    size_t m = nblk - lo < CH ? nblk - lo : CH;
    for (size_t i = 0; i < m; ++i) {
      tmp[i].off = (uint64_t)(lo + i) * stride;
      tmp[i].len = len;
      tmp[i].init = 0;
    }
    int rc = oracle_crc32c_batch(base, tmp, m, flags & 1u, out + lo, nthreads);
    if (rc) return rc;
  }
  return 0;
}

/* Synthetic data: splitmix64 over a counter; byte j is byte (j%8) of word j/8
 * (little-endian).  The same generator exists in numpy (tests/golden/gen) and
 * on the device (pebblesdb_amd/csrc), so fixtures store only seeds. */
static inline uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_fill_splitmix(uint8_t* dst, size_t nbytes, uint64_t seed, uint64_t byte_offset) {
  for (size_t j = 0; j < nbytes; ++j) {
    uint64_t g = byte_offset + j;
    uint64_t w = splitmix64_at(seed, g >> 3);
    dst[j] = (uint8_t)(w >> (8 * (g & 7)));
  }
}
