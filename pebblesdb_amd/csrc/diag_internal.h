// diag_internal.h -- launchers of the diagnostics library (diag_variants.hip), bench / test
// infrastructure only (include/pdb_crc32c_diag.h).
#pragma once
#include "crc32c_internal.h"

namespace pdb {

hipError_t launch_fixed_variant(int v, const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                                uint64_t stride, uint32_t len, uint64_t nblk, uint32_t flags, uint32_t init,
                                uint32_t* out, hipStream_t s);
hipError_t launch_desc_variant(int v, const LaunchGeom& g, const uint32_t* d_tables, const uint8_t* base,
                               const pdb_blk* blk, uint64_t nblk, uint32_t flags, uint32_t* out, hipStream_t s);
// sstable hooks: 18 = crc_stream_kernel (32-B pieces), 72 = the seal without trailer parking,
// 140 / 141 = the seal's memory pattern without the hash; other ids = the shipped routing
hipError_t launch_sst_variant(int v, const LaunchGeom& g, const uint32_t* d_tables, uint8_t* buf, uint64_t buf_len,
                              const pdb_block_handle* h, uint64_t n, bool seal, uint8_t* ok, uint32_t* nbad,
                              hipStream_t s);
hipError_t launch_read_stream(const uint8_t* base, uint64_t nbytes, uint32_t* out, hipStream_t s);
hipError_t launch_read_pattern4k(const LaunchGeom& g, const uint8_t* base, uint64_t nblk, int variant, uint32_t* out,
                                 hipStream_t s);
hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset, hipStream_t s);

}  // namespace pdb
