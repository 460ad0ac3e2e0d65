/*
 * pdb_crc32c_diag.h -- BENCH / TEST INFRASTRUCTURE, not the drop-in interface.
 *
 * libpdb_crc32c_diag.so holds what measuring and A/B-testing the product needs and the product
 * must not ship: synthetic input generation, the load-pattern kernels behind the roofline
 * calibration, and the A/B kernel variants measured against the shipped kernels
 * (profiles/r01_ab_*.json).  Every variant is selected per call (no global switch) and computes
 * the same CRCs as the product unless its comment says otherwise.  It shares the product's
 * device-side code (pebblesdb_amd/csrc/crc32c_device.h) but not its state: it uploads its own
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
/* 4-KiB block load patterns with no CRC work (variant ids: diag_variants.hip, launch_read_pattern4k;
 * 21 = the shipped 4-KiB kernel's exact loads: 1-KiB-contiguous nt instructions, lock-step). */
int pdb_diag_read_pattern4k(const void* d_base, uint64_t nblk, int variant, uint32_t* d_out, void* stream);

/* A/B variants of the batch kernels (same arguments as the product entry points). */
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
