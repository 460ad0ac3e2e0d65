/*
 * pdb_crc32c_diag.h -- BENCH / TEST INFRASTRUCTURE, not the drop-in interface.
 *
 * libpdb_crc32c_diag.so holds what measuring and testing the product needs and the product must
 * not ship: synthetic input generation, the load-pattern kernels behind the roofline and
 * pattern-ceiling numbers, the record kernel's part / clock / work-distribution
 * diagnostics, and a few alternative kernels the parity tests use as independent cross-checks.
 * Variants are selected per call (no global switch) and compute the same CRCs as the product unless
 * their comment in diag_variants.hip says otherwise.  It shares the product's device-side code
 * (pebblesdb_amd/csrc/crc32c_device.h, crc32c_lanespan.h) but not its state: it uploads its own
 * copy of the tables per device.
 */
#ifndef PDB_CRC32C_DIAG_H_
#define PDB_CRC32C_DIAG_H_

#include <stddef.h>
#include <stdint.h>

#include "pdb_crc32c.h"

#ifdef __cplusplus
extern "C" {
#endif

const char* pdb_diag_last_error(void);

/* d_dst[0..nbytes) = bytes [byte_offset, byte_offset + nbytes) of the splitmix64 stream of `seed`
 * (byte k = byte k%8 of splitmix64(seed, k/8); oracle_fill_splitmix is its CPU twin). */
int pdb_diag_fill_splitmix(void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset, void* stream);

/* Streams nbytes from d_base with coalesced 16-B loads, XOR-folded into *d_out. */
int pdb_diag_read_stream(const void* d_base, uint64_t nbytes, uint32_t* d_out, void* stream);
/* The 4-KiB kernel's loads with no CRC work: variant 21 only (1-KiB-contiguous nt instructions,
 * workgroup lock-step); other ids return an error. */
int pdb_diag_read_pattern4k(const void* d_base, uint64_t nblk, int variant, uint32_t* d_out, void* stream);

/* Variants of the batch entry points (same arguments as the product's; ids in diag_variants.hip:
 * fixed 0 / 16, desc 0 / 16 / 161 / 63 / 64 / 67 / 125 / 126 / 127-134 / 180-182, sst 0 / 18 / 72 / 140 / 141 / 142 / 143). */
int pdb_diag_batch_fixed(int variant, const void* d_base, uint64_t stride, uint32_t len, uint64_t nblk,
                         uint32_t flags, uint32_t init, uint32_t* d_out, void* stream);
int pdb_diag_batch_desc(int variant, const void* d_base, const pdb_blk* d_blk, uint64_t nblk, uint32_t flags,
                        uint32_t* d_out, void* stream);
/* seal != 0: pdb_sst_seal_device's contract, else pdb_sst_verify_device's. */
int pdb_diag_sst(int variant, void* d_buf, uint64_t buf_len, const pdb_block_handle* d_h, uint64_t n, int seal,
                 uint8_t* d_ok, uint32_t* d_nbad, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* PDB_CRC32C_DIAG_H_ */
