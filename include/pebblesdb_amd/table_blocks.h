// pebblesdb_amd/table_blocks.h -- batched sstable block emit/verify hooks over the C-ABI.
//
// The reference computes one trailer per block, synchronously, inside
// TableBuilder::WriteRawBlock (table/table_builder.cc:187-205):
//     handle = {offset, n}; Append(contents); trailer = [type][Mask(crc(contents||type))];
//     Append(trailer); offset += n + kBlockTrailerSize
// and checks one block per ReadBlock (table/format.cc:66-104):
//     if verify_checksums && Unmask(DecodeFixed32(data+n+1)) != Value(data, n+1)
//         -> Status::Corruption("block checksum mismatch")
// Here the same byte layout is produced / checked for MANY blocks per call:
//   * BlockTrailerBatch buffers finished blocks (the "buffered emission" SURVEY §7 asks for,
//     because WritableFile only has Append: include/pebblesdb/env.h:292-299), seals every
//     trailer with one pdb_sst_seal_host call, and hands back the exact bytes WriteRawBlock
//     would have appended, plus the BlockHandles.
//   * VerifyBlocks checks every handle of a table image in one pdb_sst_verify_host call -- the
//     batch form of ReadBlock's check used by scans, paranoid compaction and leveldb-verify.
// Header-only; errors surface as the C-ABI's negative codes (no CPU fallback).
#ifndef PEBBLESDB_AMD_TABLE_BLOCKS_H_
#define PEBBLESDB_AMD_TABLE_BLOCKS_H_

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "../pdb_crc32c.h"

namespace pdb {

static const size_t kBlockTrailerSize = 5;  // table/format.h:87: 1-byte type + 32-bit crc

struct BlockHandle {  // table/format.h:22-45 (offset, size of the contents)
  uint64_t offset;
  uint64_t size;
};

// Accumulates blocks in sstable order starting at file offset `base_offset`.
class BlockTrailerBatch {
 public:
  explicit BlockTrailerBatch(uint64_t base_offset = 0) : base_(base_offset) {}

  // Equivalent of WriteRawBlock's bookkeeping: returns the handle the reference would set.
  BlockHandle Add(const char* contents, size_t n, unsigned char type) {
    BlockHandle h{base_ + buf_.size(), n};
    rel_.push_back(pdb_block_handle{buf_.size(), n});
    buf_.append(contents, n);
    buf_.push_back(static_cast<char>(type));
    buf_.append(4, '\0');  // masked crc, filled by Seal()
    return h;
  }

  // Computes every trailer on the GPU.  Returns 0 or a negative PDB_E* code.
  int Seal() {
    if (rel_.empty()) return PDB_OK;
    return pdb_sst_seal_host(&buf_[0], buf_.size(), rel_.data(), rel_.size());
  }

  // The bytes WriteRawBlock would have appended for all blocks so far (valid after Seal()).
  const std::string& bytes() const { return buf_; }
  uint64_t next_offset() const { return base_ + buf_.size(); }
  size_t num_blocks() const { return rel_.size(); }

  void Clear(uint64_t new_base) {
    base_ = new_base;
    buf_.clear();
    rel_.clear();
  }

 private:
  uint64_t base_;
  std::string buf_;
  std::vector<pdb_block_handle> rel_;
};

// Batch ReadBlock check over a table image (or any span holding the blocks and trailers).
// Returns the number of blocks whose checksum mismatches (each one is what ReadBlock reports as
// Corruption("block checksum mismatch")), or a negative PDB_E* code.
inline int64_t VerifyBlocks(const char* image, uint64_t image_len, const BlockHandle* handles,
                            size_t n, std::vector<uint8_t>* ok = nullptr) {
  std::vector<pdb_block_handle> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = pdb_block_handle{handles[i].offset, handles[i].size};
  std::vector<uint8_t> local;
  std::vector<uint8_t>& flags = ok ? *ok : local;
  flags.assign(n, 0);
  return pdb_sst_verify_host(image, image_len, h.data(), n, flags.data());
}

inline const char* ChecksumMismatchMessage() { return "block checksum mismatch"; }  // format.cc:101

}  // namespace pdb

#endif  // PEBBLESDB_AMD_TABLE_BLOCKS_H_
