// pebblesdb_amd/crc32c.h -- drop-in replacement for PebblesDB's src/util/crc32c.h.
//
// Same namespace, names and contract as the reference header (util/crc32c.h:11-45):
//   leveldb::crc32c::Extend(init_crc, data, n)   (util/crc32c.h:17)
//   leveldb::crc32c::Value(data, n)              (util/crc32c.h:20-22)
//   leveldb::crc32c::kMaskDelta / Mask / Unmask  (util/crc32c.h:24-40)
// A build that swaps `#include "util/crc32c.h"` for this header (or installs it under that name)
// links util/crc32c.cc out and libpdb_crc32c.so in; every call site (table_builder.cc:197-199,
// format.cc:97-98, log_writer.cc:121, log_reader.cc:237-238, db_bench.cc:1120) is unchanged.
//
// Header-only over the C-ABI (include/pdb_crc32c.h): no C++ types cross the library boundary.
// Extend/Value compute on the GPU (one host batch of one block); callers with many blocks should
// use the batch entry points (see pebblesdb_amd/table_blocks.h) -- that is where the GPU pays.
#ifndef PEBBLESDB_AMD_CRC32C_H_
#define PEBBLESDB_AMD_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#include "../pdb_crc32c.h"

namespace leveldb {
namespace crc32c {

// Return the crc32c of concat(A, data[0,n-1]) where init_crc is the crc32c of some string A.
inline uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  return pdb_crc32c_extend(init_crc, data, n);
}

// Return the crc32c of data[0,n-1]
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

static const uint32_t kMaskDelta = 0xa282ead8ul;

// Return a masked representation of crc (rotate right by 15 bits and add a constant).
inline uint32_t Mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }

// Return the crc whose masked representation is masked_crc.
inline uint32_t Unmask(uint32_t masked_crc) {
  uint32_t rot = masked_crc - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

}  // namespace crc32c
}  // namespace leveldb

#endif  // PEBBLESDB_AMD_CRC32C_H_
