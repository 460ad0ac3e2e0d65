// integration/pdb_crc_route.h -- where the engine hooks send their checksum work.
//
// Default: the GPU, through libpdb_crc32c.so (pdb_sst_seal_host / pdb_sst_verify_host /
// pdb_crc32c_value).  Built with -DPDB_CPU_CRC=1 (integration/build.sh, the *_buffered_cpu A/B
// harnesses ONLY; never in libpdb_crc32c.so): the same batches -- buffered emission in
// pdb_table_builder.cc, read-ahead windows in pdb_table.cc, ReadBlock in pdb_format.cc -- checked
// by the reference's own CPU crc32c (util/crc32c.cc, table_builder.cc:193-200 / format.cc:96-104
// arithmetic) on the calling thread.  That build separates what the I/O batching buys from what the
// GPU CRC buys.
#ifndef PDB_INTEGRATION_CRC_ROUTE_H_
#define PDB_INTEGRATION_CRC_ROUTE_H_

#include <stdint.h>

#include "pdb_crc32c.h"

#if PDB_CPU_CRC
#include <stdlib.h>

#include "util/coding.h"
#include "util/crc32c.h"

namespace pdb_route {
inline const char* Name() { return "cpu"; }
inline const char* LastError() { return "cpu crc"; }
// staging memory for the sealed batches: plain heap memory (no device to copy to)
inline int HostAlloc(uint64_t n, void** out) {
  *out = n ? malloc(static_cast<size_t>(n)) : nullptr;
  return n && !*out ? PDB_ENOMEM : PDB_OK;
}
inline void HostFree(void* p) { free(p); }
// WriteRawBlock's trailer math per handle: [type] is already at contents + size
inline int SstSealHost(void* buf, uint64_t len, const pdb_block_handle* h, uint64_t n) {
  char* b = static_cast<char*>(buf);
  for (uint64_t i = 0; i < n; ++i) {
    if (h[i].offset > len || h[i].size > len - h[i].offset || len - h[i].offset - h[i].size < 5) return PDB_ERANGE;
    char* p = b + h[i].offset;
    const uint32_t crc = leveldb::crc32c::Value(p, static_cast<size_t>(h[i].size) + 1);
    leveldb::EncodeFixed32(p + h[i].size + 1, leveldb::crc32c::Mask(crc));
  }
  return PDB_OK;
}
// ReadBlock's check per handle: ok[i], returns the number of mismatches
inline int64_t SstVerifyHost(const void* buf, uint64_t len, const pdb_block_handle* h, uint64_t n, uint8_t* ok) {
  const char* b = static_cast<const char*>(buf);
  int64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) {
    bool good = h[i].offset <= len && h[i].size <= len - h[i].offset && len - h[i].offset - h[i].size >= 5;
    if (good) {
      const char* p = b + h[i].offset;
      good = leveldb::crc32c::Unmask(leveldb::DecodeFixed32(p + h[i].size + 1)) ==
             leveldb::crc32c::Value(p, static_cast<size_t>(h[i].size) + 1);
    }
    if (ok) ok[i] = good ? 1 : 0;
    bad += good ? 0 : 1;
  }
  return bad;
}
inline uint32_t Value(const void* p, uint64_t n) {
  return leveldb::crc32c::Value(static_cast<const char*>(p), static_cast<size_t>(n));
}
inline uint32_t Unmask(uint32_t m) { return leveldb::crc32c::Unmask(m); }
}  // namespace pdb_route

#else

namespace pdb_route {
inline const char* Name() { return "gpu"; }
inline const char* LastError() { return pdb_last_error(); }
// staging memory for the sealed batches: page-locked, so each batch reaches the device by DMA
inline int HostAlloc(uint64_t n, void** out) { return pdb_host_alloc(n, out); }
inline void HostFree(void* p) { (void)pdb_host_free(p); }
inline int SstSealHost(void* buf, uint64_t len, const pdb_block_handle* h, uint64_t n) {
  return pdb_sst_seal_host(buf, len, h, n);
}
inline int64_t SstVerifyHost(const void* buf, uint64_t len, const pdb_block_handle* h, uint64_t n, uint8_t* ok) {
  return pdb_sst_verify_host(buf, len, h, n, ok);
}
inline uint32_t Value(const void* p, uint64_t n) { return pdb_crc32c_value(p, n); }
inline uint32_t Unmask(uint32_t m) { return pdb_crc32c_unmask(m); }
}  // namespace pdb_route

#endif
#endif  // PDB_INTEGRATION_CRC_ROUTE_H_
