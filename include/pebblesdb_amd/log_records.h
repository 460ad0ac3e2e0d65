// pebblesdb_amd/log_records.h -- batched WAL / MANIFEST record checksums for C++ engines
// (the C++ counterpart of pebblesdb_amd/log.py).
//
// The reference log format (src/db/log_format.h:14-30): 32-KiB blocks; a physical record is
// [masked crc LE32][length LE16][type][payload] and never straddles a block; a block tail shorter
// than the 7-byte header is zero-filled (log_writer.cc:90-97).  The CRC covers type || payload,
// which are contiguous in the file (log_writer.cc:111-121, log_reader.cc:235-249).
//
// ParsePhysicalRecords walks a log image like log::Reader::ReadPhysicalRecord
// (log_reader.cc:185-260) without checking CRCs; VerifyLog then checks every record with ONE
// pdb_crc32c_verify_host call (recovery, repair, MANIFEST replay) instead of one crc32c::Value per
// record.  Header-only, C++11, links against libpdb_crc32c.so.
#ifndef PEBBLESDB_AMD_LOG_RECORDS_H_
#define PEBBLESDB_AMD_LOG_RECORDS_H_

#include <stdint.h>

#include <vector>

#include "pdb_crc32c.h"

namespace pdb {
namespace log {

static const uint64_t kBlockSize = 32768;  // log_format.h:27
static const uint64_t kHeaderSize = 7;     // log_format.h:30: checksum (4), length (2), type (1)
enum RecordType { kZeroType = 0, kFullType = 1, kFirstType = 2, kMiddleType = 3, kLastType = 4 };

struct PhysicalRecord {
  uint64_t offset;  // header offset in the file
  uint32_t length;  // payload bytes
  uint8_t type;
  uint32_t stored;  // masked crc from the header
  uint64_t payload_offset() const { return offset + kHeaderSize; }
};

// Walk the blocks: zero-filled block tails and preallocated zero records are skipped; a record
// whose length runs past its block or the image ends the walk (a truncated tail, which the
// reference reader reports as kEof / a dropped fragment).  Returns the number of bytes walked.
inline uint64_t ParsePhysicalRecords(const char* image, uint64_t n, std::vector<PhysicalRecord>* out) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(image);
  out->clear();
  uint64_t pos = 0;
  while (pos < n) {
    const uint64_t left_in_block = kBlockSize - (pos % kBlockSize);
    if (left_in_block < kHeaderSize) {  // trailer
      pos += left_in_block;
      continue;
    }
    if (pos + kHeaderSize > n) break;
    const uint32_t stored = static_cast<uint32_t>(p[pos]) | (static_cast<uint32_t>(p[pos + 1]) << 8) |
                            (static_cast<uint32_t>(p[pos + 2]) << 16) | (static_cast<uint32_t>(p[pos + 3]) << 24);
    const uint32_t length = static_cast<uint32_t>(p[pos + 4]) | (static_cast<uint32_t>(p[pos + 5]) << 8);
    const uint8_t type = p[pos + 6];
    if (type == kZeroType && length == 0) {  // preallocated region (log_reader.cc:226-233)
      pos += left_in_block;
      continue;
    }
    const uint64_t end = pos + kHeaderSize + length;
    if (end > n || end > pos - (pos % kBlockSize) + kBlockSize) break;
    PhysicalRecord r;
    r.offset = pos;
    r.length = length;
    r.type = type;
    r.stored = stored;
    out->push_back(r);
    pos = end;
  }
  return pos < n ? pos : n;
}

// ok[i] = 1 iff record i's stored CRC == Mask(crc32c(type || payload)).  Returns the number of
// mismatching records (each one log::Reader drops with "checksum mismatch") or a negative PDB_E*.
inline int64_t VerifyRecords(const char* image, uint64_t n, const std::vector<PhysicalRecord>& recs,
                             std::vector<uint8_t>* ok) {
  ok->assign(recs.size(), 0);
  if (recs.empty()) return 0;
  std::vector<pdb_blk> blk(recs.size());
  std::vector<uint32_t> expected(recs.size());
  for (size_t i = 0; i < recs.size(); ++i) {
    blk[i].off = recs[i].offset + 6;  // the type byte, then the payload
    blk[i].len = 1 + recs[i].length;
    blk[i].init = 0;
    expected[i] = recs[i].stored;
  }
  return pdb_crc32c_verify_host(image, n, blk.data(), blk.size(), PDB_CRC_MASK_OUTPUT, expected.data(),
                                ok->data());
}

inline int64_t VerifyLog(const char* image, uint64_t n, std::vector<PhysicalRecord>* recs,
                         std::vector<uint8_t>* ok) {
  ParsePhysicalRecords(image, n, recs);
  return VerifyRecords(image, n, *recs, ok);
}

inline const char* ChecksumMismatchMessage() { return "checksum mismatch"; }  // log_reader.cc:246

}  // namespace log
}  // namespace pdb

#endif  // PEBBLESDB_AMD_LOG_RECORDS_H_
