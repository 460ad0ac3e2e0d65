// integration/pdb_log_reader.cc -- drop-in for the reference's db/log_reader.cc (the class declared
// in db/log_reader.h, unchanged): log::Reader with every physical record's CRC checked in ONE GPU
// batch per file instead of one crc32c::Value per record (db/log_reader.cc:235-249).  Linked into the
// GPU engine builds (integration/build.sh) for the readers of the WAL (DBImpl::RecoverLogFile,
// db/db_impl.cc:516-600), the MANIFEST (VersionSet::Recover, db/version_set.cc:2450) and repair.
//
// How: the first ReadPhysicalRecord reads the rest of the file (from the block SkipToInitialBlock
// chose) into memory, walks it the way ReadPhysicalRecord does without checking CRCs
// (pdb::log::WalkLog), and verifies every physical record it meets with one pdb_crc32c_verify_host
// call (pdb::log::VerifyRecords).  From then on ReadRecord / ReadPhysicalRecord run the reference's
// own state machine over 32-KiB slices of that image -- the same buffer_, eof_,
// end_of_buffer_offset_ and report arithmetic, so records, LastRecordOffset() and every corruption
// report are exactly the reference's (tests/test_log.py: the 43 corrupted logs) -- and the checksum
// test is a lookup of the batch's verdict for the record at that offset.  The records the reader
// visits are a subset of the walk's (after a bad CRC the reader drops the rest of the block, the walk
// goes on in it; the next block starts at the same offset in both), so every lookup hits; a record the
// walk missed would be checked on its own (pdb_crc32c_value).  A failed batch (no device) aborts, as
// the scalar shim does: the reference's reader cannot fail.
//
// The reader's extra state lives behind backing_store_ (the header's member layout is the
// reference's; its block buffer is the image here).
#include "db/log_reader.h"

#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "pebblesdb/env.h"
#include "pebblesdb_amd/log_records.h"
#include "util/coding.h"

namespace leveldb {
namespace log {

namespace {

struct Batched {
  bool loaded = false;
  std::string image;          // the file from `base` to its end (or to a failed read)
  uint64_t base = 0;          // file offset of image[0] (a block boundary)
  uint64_t next = 0;          // image offset of the next 32-KiB "read"
  bool read_failed = false;   // a Read of the file failed at image offset `failed_at`
  uint64_t failed_at = 0;
  Status read_status;
  std::vector<uint64_t> rec;  // physical records of the walk (image offsets), ascending
  std::vector<uint8_t> ok;    // and the batch's CRC verdicts
  size_t cursor = 0;          // lookup position (the reader visits records in ascending order)
  uint64_t batch_records = 0; // records checked by the batch / on their own (diagnostics)
  uint64_t single_records = 0;
};

inline Batched* state(char* p) { return reinterpret_cast<Batched*>(p); }

}  // namespace

Reader::Reporter::~Reporter() {}

Reader::Reader(SequentialFile* file, Reporter* reporter, bool checksum, uint64_t initial_offset)
    : file_(file),
      reporter_(reporter),
      checksum_(checksum),
      backing_store_(reinterpret_cast<char*>(new Batched)),
      buffer_(),
      eof_(false),
      last_record_offset_(0),
      end_of_buffer_offset_(0),
      initial_offset_(initial_offset) {}

Reader::~Reader() { delete state(backing_store_); }

bool Reader::SkipToInitialBlock() {  // log_reader.cc:35-57, and the image starts at that block
  size_t offset_in_block = initial_offset_ % kBlockSize;
  uint64_t block_start_location = initial_offset_ - offset_in_block;
  if (offset_in_block > kBlockSize - 6) {  // don't search a block if we'd be in the trailer
    offset_in_block = 0;
    block_start_location += kBlockSize;
  }
  end_of_buffer_offset_ = block_start_location;
  Batched* b = state(backing_store_);
  if (!b->loaded) b->base = block_start_location;
  if (block_start_location > 0) {
    Status skip_status = file_->Skip(block_start_location);
    if (!skip_status.ok()) {
      ReportDrop(block_start_location, skip_status);
      return false;
    }
  }
  return true;
}

bool Reader::ReadRecord(Slice* record, std::string* scratch) {  // log_reader.cc:59-157, unchanged
  if (last_record_offset_ < initial_offset_) {
    if (!SkipToInitialBlock()) {
      return false;
    }
  }
  scratch->clear();
  record->clear();
  bool in_fragmented_record = false;
  uint64_t prospective_record_offset = 0;
  Slice fragment;
  while (true) {
    uint64_t physical_record_offset = end_of_buffer_offset_ - buffer_.size();
    const unsigned int record_type = ReadPhysicalRecord(&fragment);
    switch (record_type) {
      case kFullType:
        if (in_fragmented_record) {
          if (scratch->empty()) {
            in_fragmented_record = false;
          } else {
            ReportCorruption(scratch->size(), "partial record without end(1)");
          }
        }
        prospective_record_offset = physical_record_offset;
        scratch->clear();
        *record = fragment;
        last_record_offset_ = prospective_record_offset;
        return true;
      case kFirstType:
        if (in_fragmented_record) {
          if (scratch->empty()) {
            in_fragmented_record = false;
          } else {
            ReportCorruption(scratch->size(), "partial record without end(2)");
          }
        }
        prospective_record_offset = physical_record_offset;
        scratch->assign(fragment.data(), fragment.size());
        in_fragmented_record = true;
        break;
      case kMiddleType:
        if (!in_fragmented_record) {
          ReportCorruption(fragment.size(), "missing start of fragmented record(1)");
        } else {
          scratch->append(fragment.data(), fragment.size());
        }
        break;
      case kLastType:
        if (!in_fragmented_record) {
          ReportCorruption(fragment.size(), "missing start of fragmented record(2)");
        } else {
          scratch->append(fragment.data(), fragment.size());
          *record = Slice(*scratch);
          last_record_offset_ = prospective_record_offset;
          return true;
        }
        break;
      case kEof:
        if (in_fragmented_record) {
          scratch->clear();
        }
        return false;
      case kBadRecord:
        if (in_fragmented_record) {
          ReportCorruption(scratch->size(), "error in middle of record");
          in_fragmented_record = false;
          scratch->clear();
        }
        break;
      default: {
        char buf[40];
        snprintf(buf, sizeof(buf), "unknown record type %u", record_type);
        ReportCorruption((fragment.size() + (in_fragmented_record ? scratch->size() : 0)), buf);
        in_fragmented_record = false;
        scratch->clear();
        break;
      }
    }
  }
  return false;
}

uint64_t Reader::LastRecordOffset() { return last_record_offset_; }

void Reader::ReportCorruption(size_t bytes, const char* reason) { ReportDrop(bytes, Status::Corruption(reason)); }

void Reader::ReportDrop(size_t bytes, const Status& reason) {
  if (reporter_ != NULL && end_of_buffer_offset_ - buffer_.size() - bytes >= initial_offset_) {
    reporter_->Corruption(bytes, reason);
  }
}

namespace {

// The rest of the file into the image (1-MiB reads), then -- with checksums on -- the walk and its one
// verify batch.
void Load(SequentialFile* file, bool checksum, Batched* b) {
  b->loaded = true;
  std::vector<char> scratch(1 << 20);
  for (;;) {
    Slice got;
    Status s = file->Read(scratch.size(), &got, scratch.data());
    if (!s.ok()) {
      b->read_failed = true;
      b->failed_at = b->image.size();
      b->read_status = s;
      break;
    }
    b->image.append(got.data(), got.size());
    if (got.size() < scratch.size()) break;  // end of file (SequentialFile::Read: short only at EOF)
  }
  if (!checksum) return;
  std::vector<pdb::log::PhysicalRecord> recs;
  pdb::log::ParsePhysicalRecords(b->image.data(), b->image.size(), &recs);
  const int64_t bad = pdb::log::VerifyRecords(b->image.data(), b->image.size(), recs, &b->ok);
  if (bad < 0) {
    fprintf(stderr, "log::Reader: device CRC batch failed (%lld): %s\n", static_cast<long long>(bad), pdb_last_error());
    abort();
  }
  b->rec.resize(recs.size());
  for (size_t i = 0; i < recs.size(); ++i) b->rec[i] = recs[i].offset;
  b->batch_records = recs.size();
}

// The next "file_->Read(kBlockSize)" from the image; a failed read of the file fails the read of the
// block holding the failure point.
Status NextBlock(Batched* b, Slice* out) {
  if (b->read_failed && b->next + kBlockSize > b->failed_at) {
    *out = Slice();
    return b->read_status;
  }
  const uint64_t n = b->image.size() - (b->next < b->image.size() ? b->next : b->image.size());
  const uint64_t take = n < kBlockSize ? n : kBlockSize;
  *out = Slice(b->image.data() + b->next, take);
  b->next += take;
  return Status::OK();
}

// The batch's verdict for the record whose header is at image offset `off`.
bool RecordOk(Batched* b, uint64_t off, const char* header, uint32_t length) {
  while (b->cursor < b->rec.size() && b->rec[b->cursor] < off) ++b->cursor;
  if (b->cursor < b->rec.size() && b->rec[b->cursor] == off) return b->ok[b->cursor] != 0;
  // not met by the walk (never expected): checked on its own, as the reference would
  ++b->single_records;
  return pdb_crc32c_unmask(DecodeFixed32(header)) == pdb_crc32c_value(header + 6, 1 + length);
}

}  // namespace

unsigned int Reader::ReadPhysicalRecord(Slice* result) {  // log_reader.cc:181-263 over the image
  Batched* b = state(backing_store_);
  if (!b->loaded) Load(file_, checksum_, b);
  while (true) {
    if (buffer_.size() < kHeaderSize) {
      if (!eof_) {
        // Last read was a full read, so this is a trailer to skip
        buffer_.clear();
        Status status = NextBlock(b, &buffer_);
        end_of_buffer_offset_ += buffer_.size();
        if (!status.ok()) {
          buffer_.clear();
          ReportDrop(kBlockSize, status);
          eof_ = true;
          return kEof;
        } else if (buffer_.size() < kBlockSize) {
          eof_ = true;
        }
        continue;
      } else {
        // a truncated header at the end of the file: EOF, not a corruption
        buffer_.clear();
        return kEof;
      }
    }
    const char* header = buffer_.data();
    const uint32_t a = static_cast<uint32_t>(header[4]) & 0xff;
    const uint32_t c = static_cast<uint32_t>(header[5]) & 0xff;
    const unsigned int type = header[6];
    const uint32_t length = a | (c << 8);
    if (kHeaderSize + length > buffer_.size()) {
      size_t drop_size = buffer_.size();
      buffer_.clear();
      if (!eof_) {
        ReportCorruption(drop_size, "bad record length");
        return kBadRecord;
      }
      return kEof;  // the writer died in the middle of the record
    }
    if (type == kZeroType && length == 0) {
      buffer_.clear();  // a preallocated zero region: skipped without a report
      return kBadRecord;
    }
    if (checksum_ && !RecordOk(b, static_cast<uint64_t>(header - b->image.data()), header, length)) {
      // drop the rest of the buffer: "length" itself may be corrupt
      size_t drop_size = buffer_.size();
      buffer_.clear();
      ReportCorruption(drop_size, "checksum mismatch");
      return kBadRecord;
    }
    buffer_.remove_prefix(kHeaderSize + length);
    // Skip physical record that started before initial_offset_
    if (end_of_buffer_offset_ - buffer_.size() - kHeaderSize - length < initial_offset_) {
      result->clear();
      return kBadRecord;
    }
    *result = Slice(header + kHeaderSize, length);
    return type;
  }
}

}  // namespace log
}  // namespace leveldb
