// pebblesdb_amd/log_records.h -- batched WAL / MANIFEST record checksums for C++ engines
// (the C++ counterpart of pebblesdb_amd/log.py).
//
// The reference log format (src/db/log_format.h:14-30): 32-KiB blocks; a physical record is
// [masked crc LE32][length LE16][type][payload] and never straddles a block; a block tail shorter
// than the 7-byte header is zero-filled (log_writer.cc:90-97).  The CRC covers type || payload,
// which are contiguous in the file (log_writer.cc:111-121, log_reader.cc:235-249).
//
// WalkLog walks a log image like log::Reader::ReadPhysicalRecord (log_reader.cc:181-263) without
// checking CRCs; VerifyLog / ReplayLog then check every record with ONE pdb_crc32c_verify_host
// call (recovery, repair, MANIFEST replay) instead of one crc32c::Value per record, and ReplayLog
// reproduces log::Reader::ReadRecord's output (records + corruption reports) exactly.
// Header-only, C++11, links against libpdb_crc32c.so.
#ifndef PEBBLESDB_AMD_LOG_RECORDS_H_
#define PEBBLESDB_AMD_LOG_RECORDS_H_

#include <stdint.h>

#include <string>
#include <vector>

#include "pdb_crc32c.h"

namespace pdb {
namespace log {

static const uint64_t kBlockSize = 32768;  // log_format.h:27
static const uint64_t kHeaderSize = 7;     // log_format.h:30: checksum (4), length (2), type (1)
enum RecordType { kZeroType = 0, kFullType = 1, kFirstType = 2, kMiddleType = 3, kLastType = 4 };
// log::Reader's extra return values kEof / kBadRecord (log_reader.h:78-84): a record whose type byte
// holds one of them (CRC valid) takes that path in ReadRecord
static const uint8_t kEofValue = 5, kBadRecordValue = 6;

struct PhysicalRecord {
  uint64_t offset;  // header offset in the file
  uint32_t length;  // payload bytes
  uint8_t type;
  uint32_t stored;  // masked crc from the header
  uint64_t payload_offset() const { return offset + kHeaderSize; }
  uint64_t block() const { return offset / kBlockSize; }
};

// One physical item log::Reader::ReadPhysicalRecord (log_reader.cc:181-263) meets: a record, or
// the rest of a block it drops without a CRC check -- a record whose length runs past a full
// block ("bad record length", log_reader.cc:214-220) or a zero-filled preallocated region (type 0,
// length 0, dropped silently, log_reader.cc:227-233).
struct LogItem {
  enum Kind { kRecord = 0, kBadLength = 1, kZeroRegion = 2 };
  Kind kind;
  PhysicalRecord rec;   // kRecord: the record; otherwise rec.offset = where the drop starts
  uint64_t drop_bytes;  // bytes to the end of the block (drops; for a record, from its header)
};

// The walk trusts every length (CRCs are checked afterwards, in one batch).  The file is read in
// 32-KiB blocks and only the last, short block is "eof": a record running past it, or a truncated
// header there, ends the walk without a report (a writer that died mid-record).  A block tail
// shorter than a header is skipped (the writer's zero trailer, log_writer.cc:67-76).
inline void WalkLog(const char* image, uint64_t n, std::vector<LogItem>* out) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(image);
  out->clear();
  for (uint64_t bstart = 0; bstart < n; bstart += kBlockSize) {
    const uint64_t bend = bstart + kBlockSize < n ? bstart + kBlockSize : n;
    const bool eof = bend - bstart < kBlockSize;
    uint64_t pos = bstart;
    while (bend - pos >= kHeaderSize) {
      LogItem it;
      it.rec.offset = pos;
      it.rec.length = static_cast<uint32_t>(p[pos + 4]) | (static_cast<uint32_t>(p[pos + 5]) << 8);
      it.rec.type = p[pos + 6];
      it.rec.stored = static_cast<uint32_t>(p[pos]) | (static_cast<uint32_t>(p[pos + 1]) << 8) |
                      (static_cast<uint32_t>(p[pos + 2]) << 16) | (static_cast<uint32_t>(p[pos + 3]) << 24);
      it.drop_bytes = bend - pos;
      if (kHeaderSize + it.rec.length > bend - pos) {
        if (eof) return;  // kEof
        it.kind = LogItem::kBadLength;
        out->push_back(it);
        break;
      }
      if (it.rec.type == kZeroType && it.rec.length == 0) {
        it.kind = LogItem::kZeroRegion;
        out->push_back(it);
        break;
      }
      it.kind = LogItem::kRecord;
      out->push_back(it);
      pos += kHeaderSize + it.rec.length;
    }
    if (eof) return;  // a short tail in the last block is a truncated header
  }
}

// Every physical record of the walk, without checking CRCs.  Returns the bytes walked.
inline uint64_t ParsePhysicalRecords(const char* image, uint64_t n, std::vector<PhysicalRecord>* out) {
  std::vector<LogItem> items;
  WalkLog(image, n, &items);
  out->clear();
  uint64_t walked = 0;
  for (const LogItem& it : items) {
    if (it.kind == LogItem::kRecord) {
      out->push_back(it.rec);
      walked = it.rec.offset + kHeaderSize + it.rec.length;
    } else {
      walked = it.rec.offset + it.drop_bytes;
    }
  }
  return walked;
}

// ok[i] = 1 iff record i's stored CRC == Mask(crc32c(type || payload)), every record in ONE
// pdb_crc32c_verify_host call.  Returns the number of mismatching records or a negative PDB_E*.
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

inline const char* ChecksumMismatchMessage() { return "checksum mismatch"; }  // log_reader.cc:246

struct LogicalRecord {
  uint64_t offset;   // log::Reader::LastRecordOffset() after the record
  std::string data;  // the payload (fragments joined)
};

struct CorruptionReport {
  uint64_t bytes;      // what the Reporter is told
  std::string reason;  // "Corruption: <message>" (Status::ToString)
  uint64_t before;     // logical records delivered before it: the reader reports it from inside the
                       // ReadRecord call that returns record `before` (or the final, failing call)
};

// What log::Reader::ReadRecord (log_reader.cc:59-164; checksums on, initial offset 0) delivers from
// the image: the logical records and the corruption reports.  ok[] are the batched CRC verdicts
// of the walk's records (in walk order).  A record failing its check drops the rest of its block --
// the reader no longer trusts the length -- so records walked after it in that block are
// discarded, never replayed (log_reader.cc:240-247).  Pinned by tests/golden/log/corruptions.json.
inline void ReplayItems(const char* image, uint64_t n, const std::vector<LogItem>& items, const std::vector<uint8_t>& ok,
                        std::vector<LogicalRecord>* out, std::vector<CorruptionReport>* reports) {
  out->clear();
  reports->clear();
  std::string scratch;
  bool in_frag = false;
  uint64_t prospective = 0, pos = 0, dead_block = UINT64_MAX;
  size_t ri = 0;  // index of the next record verdict
  auto report = [&](uint64_t bytes, const std::string& why) {
    reports->push_back(CorruptionReport{bytes, "Corruption: " + why, static_cast<uint64_t>(out->size())});
  };
  auto bad_record = [&]() {  // kBadRecord in ReadRecord (log_reader.cc:143-149)
    if (in_frag) {
      report(scratch.size(), "error in middle of record");
      in_frag = false;
      scratch.clear();
    }
  };
  for (const LogItem& it : items) {
    const bool is_rec = it.kind == LogItem::kRecord;
    const bool good = is_rec ? (ri < ok.size() && ok[ri] != 0) : false;
    if (is_rec) ++ri;
    const uint64_t blk = it.rec.offset / kBlockSize;
    if (blk == dead_block) continue;
    const uint64_t bend = it.rec.offset + it.drop_bytes;
    if (!is_rec) {
      if (it.kind == LogItem::kBadLength) report(it.drop_bytes, "bad record length");
      bad_record();
      pos = bend;
      continue;
    }
    const uint64_t phys = pos;
    if (!good) {
      report(it.drop_bytes, ChecksumMismatchMessage());
      dead_block = blk;
      bad_record();
      pos = bend;
      continue;
    }
    const PhysicalRecord& r = it.rec;
    pos = r.offset + kHeaderSize + r.length;
    const char* frag = image + r.payload_offset();
    switch (r.type) {
      case kFullType:
        if (in_frag && !scratch.empty()) report(scratch.size(), "partial record without end(1)");
        out->push_back(LogicalRecord{phys, std::string(frag, r.length)});
        scratch.clear();
        in_frag = false;
        break;
      case kFirstType:
        if (in_frag && !scratch.empty()) report(scratch.size(), "partial record without end(2)");
        prospective = phys;
        scratch.assign(frag, r.length);
        in_frag = true;
        break;
      case kMiddleType:
        if (!in_frag) report(r.length, "missing start of fragmented record(1)");
        else scratch.append(frag, r.length);
        break;
      case kLastType:
        if (!in_frag) {
          report(r.length, "missing start of fragmented record(2)");
        } else {
          scratch.append(frag, r.length);
          out->push_back(LogicalRecord{prospective, scratch});
          scratch.clear();
          in_frag = false;
        }
        break;
      case kEofValue:  // ReadRecord returns false: the reader stops here (log_reader.cc:133-141)
        return;
      case kBadRecordValue:  // log_reader.cc:143-149
        bad_record();
        break;
      default: {
        // header[6] is a char read into an unsigned int (log_reader.cc:212): 0x80.. print as 42949671xx
        const unsigned t = static_cast<unsigned>(static_cast<int>(static_cast<signed char>(r.type)));
        report(r.length + (in_frag ? scratch.size() : 0), "unknown record type " + std::to_string(t));
        in_frag = false;
        scratch.clear();
        break;
      }
    }
  }
  (void)n;
}

// Walk + ONE batched CRC check + replay.  Returns the number of corruption reports (>= 0) or a
// negative PDB_E* code.
inline int64_t ReplayLog(const char* image, uint64_t n, std::vector<LogicalRecord>* out,
                         std::vector<CorruptionReport>* reports) {
  std::vector<LogItem> items;
  WalkLog(image, n, &items);
  std::vector<PhysicalRecord> recs;
  for (const LogItem& it : items)
    if (it.kind == LogItem::kRecord) recs.push_back(it.rec);
  std::vector<uint8_t> ok;
  const int64_t rc = VerifyRecords(image, n, recs, &ok);
  if (rc < 0) return rc;
  ReplayItems(image, n, items, ok, out, reports);
  return static_cast<int64_t>(reports->size());
}

// Recovery / repair / MANIFEST check: every record of the log in one GPU batch.  ok[i] per walked
// record.  Returns the number of reports the reference reader's CRC and length checks make --
// "checksum mismatch" for the first failing record of a block (the rest of that block is never
// read) plus "bad record length" drops -- or a negative PDB_E* code.  Fragment-assembly reports
// (records missing their start / end) are ReplayLog's.
inline int64_t VerifyLog(const char* image, uint64_t n, std::vector<PhysicalRecord>* recs, std::vector<uint8_t>* ok) {
  std::vector<LogItem> items;
  WalkLog(image, n, &items);
  recs->clear();
  for (const LogItem& it : items)
    if (it.kind == LogItem::kRecord) recs->push_back(it.rec);
  const int64_t rc = VerifyRecords(image, n, *recs, ok);
  if (rc < 0) return rc;
  int64_t reports = 0;
  uint64_t dead_block = UINT64_MAX;
  size_t ri = 0;
  for (const LogItem& it : items) {
    const uint64_t blk = it.rec.offset / kBlockSize;
    const bool good = it.kind == LogItem::kRecord ? (*ok)[ri++] != 0 : true;
    if (blk == dead_block) continue;
    if (it.kind == LogItem::kBadLength) ++reports;
    if (!good) {
      ++reports;
      dead_block = blk;
    }
  }
  return reports;
}

// Group-commit form of log::Writer (log_writer.cc:28-131): AddRecord fragments and lays out records
// exactly as the reference writer does (block trailers included), with CRC placeholders; Seal()
// writes every physical record's Mask(crc32c(type || payload)) from ONE pdb_crc32c_batch_host call.
class BatchWriter {
 public:
  // dest_length: the log file's current length (the writer's block offset starts there, log_writer.cc:16-26)
  explicit BatchWriter(uint64_t dest_length = 0) : base_(dest_length) {}

  void AddRecord(const char* data, size_t n) {
    size_t left = n;
    bool begin = true;
    do {  // a zero-length record still emits one header (log_writer.cc:63-99)
      uint64_t block_offset = (base_ + buf_.size()) % kBlockSize;
      const uint64_t leftover = kBlockSize - block_offset;
      if (leftover < kHeaderSize) {
        buf_.append(static_cast<size_t>(leftover), '\0');  // trailer (log_writer.cc:67-76)
        block_offset = 0;
      }
      const size_t avail = static_cast<size_t>(kBlockSize - block_offset - kHeaderSize);
      const size_t frag = left < avail ? left : avail;
      const bool end = left == frag;
      const uint8_t type = begin && end ? kFullType : (begin ? kFirstType : (end ? kLastType : kMiddleType));
      hdr_.push_back(buf_.size());
      len_.push_back(static_cast<uint32_t>(frag));
      const char h[7] = {0, 0, 0, 0, static_cast<char>(frag & 0xff), static_cast<char>(frag >> 8),
                         static_cast<char>(type)};
      buf_.append(h, 7);
      buf_.append(data, frag);
      data += frag;
      left -= frag;
      begin = false;
    } while (left > 0);
  }

  // Returns 0 or a negative PDB_E* code; bytes() then holds what Writer::AddRecord would have written.
  int Seal() {
    if (hdr_.empty()) return 0;
    std::vector<pdb_blk> blk(hdr_.size());
    for (size_t i = 0; i < hdr_.size(); ++i) {
      blk[i].off = hdr_[i] + 6;
      blk[i].len = 1 + len_[i];
      blk[i].init = 0;
    }
    std::vector<uint32_t> crc(hdr_.size());
    const int rc = pdb_crc32c_batch_host(buf_.data(), buf_.size(), blk.data(), blk.size(), PDB_CRC_MASK_OUTPUT,
                                         crc.data());
    if (rc) return rc;
    for (size_t i = 0; i < hdr_.size(); ++i)
      for (int k = 0; k < 4; ++k) buf_[hdr_[i] + k] = static_cast<char>((crc[i] >> (8 * k)) & 0xff);
    return 0;
  }

  const std::string& bytes() const { return buf_; }
  size_t num_physical_records() const { return hdr_.size(); }

 private:
  uint64_t base_;
  std::string buf_;
  std::vector<uint64_t> hdr_;
  std::vector<uint32_t> len_;
};

}  // namespace log
}  // namespace pdb

#endif  // PEBBLESDB_AMD_LOG_RECORDS_H_
