// crc32c_tables.cpp -- host-side generation of the slice-by-4 tables and the GF(2) shift
// operators the kernels stage into LDS.  Everything is generated from the reflected polynomial;
// no table literal is copied from the reference (util/crc32c.cc:130-556).
#include <string.h>

#include "crc32c_math.h"
#include "crc32c_internal.h"

namespace pdb {
namespace {

// 32x32 GF(2) matrix as 32 column vectors: M * v = XOR of cols[i] for set bits i of v.
struct Gf2Mat {
  uint32_t col[32];
};

uint32_t mat_vec(const Gf2Mat& m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; ++i, v >>= 1)
    if (v & 1u) r ^= m.col[i];
  return r;
}

Gf2Mat mat_mul(const Gf2Mat& a, const Gf2Mat& b) {  // (a*b)v = a(b v)
  Gf2Mat r;
  for (int i = 0; i < 32; ++i) r.col[i] = mat_vec(a, b.col[i]);
  return r;
}

// Operator for one zero byte: c' = T0[c & 0xff] ^ (c >> 8).
Gf2Mat one_zero_byte(const uint32_t* t0) {
  Gf2Mat m;
  for (int i = 0; i < 32; ++i) {
    uint32_t c = 1u << i;
    m.col[i] = t0[c & 0xffu] ^ (c >> 8);
  }
  return m;
}

Gf2Mat mat_pow(Gf2Mat base, uint64_t e) {
  Gf2Mat r;
  for (int i = 0; i < 32; ++i) r.col[i] = 1u << i;
  while (e) {
    if (e & 1) r = mat_mul(base, r);
    base = mat_mul(base, base);
    e >>= 1;
  }
  return r;
}

}  // namespace

void build_byte_table(uint32_t t0[256]) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ PDB_CRC32C_POLY_REFLECTED : (c >> 1);
    t0[b] = c;
  }
}

uint32_t host_shift(uint32_t c, uint64_t nbytes) {
  uint32_t t0[256];
  build_byte_table(t0);
  return mat_vec(mat_pow(one_zero_byte(t0), nbytes), c);
}

// One zero byte backwards: the state c with T0[c & 0xff] ^ (c >> 8) == c'.  The top byte of c'
// is the top byte of T0[c & 0xff] (c >> 8 has none), and T0's top bytes are a permutation of
// 0..255, so the low byte of c is found by lookup and the rest follows.
static uint32_t unshift_byte(const uint32_t* t0, uint32_t c1) {
  uint32_t idx = 0;
  while ((t0[idx] >> 24) != (c1 >> 24)) ++idx;
  return ((c1 ^ t0[idx]) << 8) | idx;
}

// Fills `out` (PDB_TABLE_WORDS u32): [T0|T1|T2|T3] then the PDB_NCAT catalog operators, each as
// 4 sub-tables j=0..3 of 256 entries: op[j][b] = shift(b << 8j, D); then the unshifted seeds
// U[z] = shift^-z(0xFFFFFFFF), z = 0..16 (PDB_UNSHIFT_OFF); then the record kernel's operators
// (PDB_SPANOP_OFF, same layout).
void build_device_tables(uint32_t* out) {
  uint32_t t[4][256];
  build_byte_table(t[0]);
  for (int k = 1; k < 4; ++k)
    for (int b = 0; b < 256; ++b) t[k][b] = (t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xffu];
  memcpy(out, t, sizeof(t));

  const Gf2Mat z1 = one_zero_byte(t[0]);
  for (int o = 0; o < PDB_NCAT; ++o) {
    Gf2Mat m = mat_pow(z1, kPdbCatDist[o]);
    uint32_t* op = out + 1024 + o * 1024;
    for (int j = 0; j < 4; ++j)
      for (uint32_t b = 0; b < 256; ++b) op[j * 256 + b] = mat_vec(m, b << (8 * j));
  }
  for (int o = 0; o < PDB_SPANOP_N; ++o) {
    Gf2Mat m = mat_pow(z1, kPdbSpanOpDist[o]);
    uint32_t* op = out + PDB_SPANOP_OFF + o * 1024;
    for (int j = 0; j < 4; ++j)
      for (uint32_t b = 0; b < 256; ++b) op[j * 256 + b] = mat_vec(m, b << (8 * j));
  }
  uint32_t* un = out + PDB_UNSHIFT_OFF;
  memset(un, 0, PDB_UNSHIFT_WORDS * sizeof(uint32_t));
  uint32_t c = 0xFFFFFFFFu;
  for (uint32_t z = 0; z <= 16; ++z) {
    un[z] = c;
    c = unshift_byte(t[0], c);
  }
  for (uint32_t z = 0; z <= 16; ++z)  // shift(U[z], z) == 0xFFFFFFFF
    if (mat_vec(mat_pow(z1, z), un[z]) != 0xFFFFFFFFu) __builtin_trap();
}

// 64 operators (PDB_POW2_WORDS u32): op k = shift by 2^k bytes, 4 x 256 entries each, for the
// long-span combine (any distance = product of the operators of its set bits).
void build_pow2_tables(uint32_t* out) {
  uint32_t t0[256];
  build_byte_table(t0);
  Gf2Mat m = one_zero_byte(t0);
  for (int k = 0; k < 64; ++k) {
    uint32_t* op = out + k * 1024;
    for (int j = 0; j < 4; ++j)
      for (uint32_t b = 0; b < 256; ++b) op[j * 256 + b] = mat_vec(m, b << (8 * j));
    m = mat_mul(m, m);
  }
}

}  // namespace pdb
