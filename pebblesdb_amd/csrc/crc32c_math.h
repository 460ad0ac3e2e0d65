// crc32c_math.h -- GF(2) algebra of CRC32C (Castagnoli, reflected) shared by the host table
// builder and the HIP kernels.
//
// Conventions ("raw state" = the register the reference's crc32c_sb8_64_bit carries between
// calls, i.e. crc ^ 0xFFFFFFFF; util/crc32c.cc:27,31):
//   byte step      c' = T0[(c ^ b) & 0xff] ^ (c >> 8)          (util/crc32c.cc:601,623)
//   shift(c, D)    = raw state after D zero bytes from state c; linear in c.
//   Tk[b]          = shift(b, k+1);  T0 is the byte table, T1..T7 = the reference's
//                    o40..o88 slices (util/crc32c.cc:130-556, generated here, not copied).
//   word step      x = c ^ LE32(w); c' = T3[x0] ^ T2[x1] ^ T1[x2] ^ T0[x3]  (= shift(x, 4))
//   injection      processing M from state c == processing (M with its first 4 bytes XORed
//                  with LE32(c)) from state 0, for |M| >= 4.
//   concatenation  R(A||B) = shift(R(A), |B|) ^ R(B), with R the raw CRC from state 0.
//   Extend(init,M) = ~S(~init, M)   (util/crc32c.cc:25-32)
//   Mask(c)        = ror32(c,15) + 0xa282ead8 (util/crc32c.h:29-32)
#pragma once
#include <stdint.h>

#define PDB_CRC32C_POLY_REFLECTED 0x82F63B78u /* 0x1EDC6F41 reflected (util/crc32c.cc:116-128) */
#define PDB_CRC32C_MASK_DELTA 0xa282ead8u     /* util/crc32c.h:24 */

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PDB_HD __host__ __device__ __forceinline__
#else
#define PDB_HD static inline
#endif

PDB_HD uint32_t pdb_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + PDB_CRC32C_MASK_DELTA; }
PDB_HD uint32_t pdb_unmask(uint32_t m) {
  uint32_t rot = m - PDB_CRC32C_MASK_DELTA;
  return (rot >> 17) | (rot << 15);
}

// ---- LDS image geometry (shared by host table packer and kernels) -----------------------------
//
// MAIN region [0, 0x20000): the four slice-by-4 tables T0..T3, each replicated 32x so that lane
// l reads replica (l & 31) -> LDS bank (l & 31) for every ds_read_b32: conflict-free random
// lookups.  Entry b of table k, replica r lives at byte
//     ((k >> 1) << 16) | (b << 8) | ((k & 1) << 7) | (r << 2)
// i.e. the data byte lands in address bits 8..15, so one v_perm_b32 builds the address.
//
// OPS region [0x20000, 0x20000 + PDB_NOPS*4096): PDB_NOPS = 8 operator slots (4 x 256 u32
// each, one copy).  Slots 0..5 hold the wave-tree operators "shift by P << k bytes" (P = bytes a
// lane owns contiguously: 64, 32 or 16 depending on the kernel's load pattern); slot 6 holds the
// per-lane Horner operator (the gap between two pieces a lane owns); slot 7 a second fold
// operator (the generic stream kernel's "shift 32").  Each kernel stages the
// operators it needs from the catalog below.
#define PDB_LANES 64
#define PDB_CHUNK 64 /* bytes per lane per round in the generic kernel */
#define PDB_MAIN_BYTES 0x20000u
#define PDB_NOPS 8
#define PDB_SLOT_HORNER 6
#define PDB_OPS_BYTES (PDB_NOPS * 4096u)
#define PDB_LDS_BYTES (PDB_MAIN_BYTES + PDB_OPS_BYTES) /* 163840 = the whole 160 KiB LDS of a CU */
/* Operator catalog (device table source): distance in bytes of catalog entry i. */
#define PDB_NCAT 11
#define PDB_CAT_TREE16 0   /* 16, 32, ..., 512   (entries 0..5) */
#define PDB_CAT_TREE32 1   /* 32, ..., 1024      (entries 1..6) */
#define PDB_CAT_TREE64 2   /* 64, ..., 2048      (entries 2..7) */
#define PDB_CAT_S1024 6    /* 1024: chain fold, 4 x 16-B pieces per lane per 4 KiB */
#define PDB_CAT_S2048 7    /* 2048: chain fold, 2 x 32-B pieces per lane per 4 KiB */
#define PDB_CAT_H1008 8    /* 1024 - 16: 4 x 16-B pieces per lane per 4 KiB */
#define PDB_CAT_H2016 9    /* 2048 - 32: 2 x 32-B pieces per lane per 4 KiB */
#define PDB_CAT_H4032 10   /* 4096 - 64: generic kernel, rounds of 64 x 64 B */
static const unsigned long long kPdbCatDist[PDB_NCAT] = {16,   32,   64,   128,  256, 512,
                                                           1024, 2048, 1008, 2016, 4032};
/* Long spans (pdb_crc32c_extend*): 64 power-of-two shift operators in device memory, and the
 * segment geometry of the parallel split + tree combine. */
#define PDB_POW2_WORDS (64u * 1024u)
#define PDB_SPAN_MIN_SEG_LOG2 16      /* segments of >= 64 KiB */
#define PDB_SPAN_MAX_SEGS_LOG2 14     /* <= 16384 segments: the combine tree fits 64 KiB of LDS */
/* Unshifted seeds (crc_sst4k_kernel): U[z] = shift^-z(0xFFFFFFFF), z = 0..16 -- the state that
 * reaches Value()'s starting state 0xFFFFFFFF after z zero bytes, so a block can be hashed
 * front-padded with z zeros (R(0^z || X) from U[z] == R(X) from 0xFFFFFFFF). */
#define PDB_UNSHIFT_OFF (1024u + PDB_NCAT * 1024u)
#define PDB_UNSHIFT_WORDS 64u
/* Record-kernel operators (crc32c_lanespan.h): shifts by 1, 2 and 4 parts -- 132, 264, 528 bytes
 * for its 33-word parts, 108, 216, 432 for the 27-word parts of the 257..512-B class -- by 3
 * parts (396 / 324 B: the per-lane pre-shift of the cross-lane fold), and by 1, 2, 3 parts + 4 B
 * (136, 268, 400 / 112, 220, 328: the pre-shift with the finishing table step folded in), 4 x 256
 * entries each. */
#define PDB_SPANOP_OFF (PDB_UNSHIFT_OFF + PDB_UNSHIFT_WORDS)
#define PDB_SPANOP_N 14
static const unsigned long long kPdbSpanOpDist[PDB_SPANOP_N] = {132, 264, 528, 108, 216, 432, 396, 324,
                                                                136, 268, 400, 112, 220, 328};
/* Device table source: T0..T3 (1024 u32), the catalog (PDB_NCAT * 1024 u32), the unshifted
 * seeds (64 u32, 17 used), the record-kernel operators (PDB_SPANOP_N * 1024 u32). */
#define PDB_TABLE_WORDS (PDB_SPANOP_OFF + PDB_SPANOP_N * 1024u)
