// integration/pdb_table_builder.cc -- drop-in for the reference's table/table_builder.cc whose
// block trailers are computed on the MI355X in batches (buffered emission).
//
// The reference (table/table_builder.cc:187-205) writes every block synchronously:
//     Append(contents); trailer = [type][Mask(Extend(Value(contents), type))]; Append(trailer)
// one CRC per block on the building thread (the memtable-flush or compaction thread).  Here
// WriteRawBlock only STAGES the block -- contents, type byte, a 4-byte placeholder -- and hands out
// the handle it will have (offsets are known without the CRC), and every kSealBytes of staged
// blocks, and at Finish(), ONE pdb_sst_seal_host call computes all their trailers on the GPU
// (H2D of the staged span, crc_sst4k_kernel, 4 B per block back) before ONE Append of the whole
// span.  The file receives byte for byte what the reference writes (tests: the reference-written
// golden tables are reproduced exactly), just in fewer, larger appends.
//
// Interface: the reference's own include/pebblesdb/table_builder.h (class TableBuilder, private
// Rep); behaviour of Add/Flush/Finish/Abandon/status/NumEntries/FileSize is the reference's
// (table_builder.cc:71-280) with two visible differences, both inherent to buffered emission:
//   * WritableFile::Append/Flush are called once per sealed batch, not per block, so after Flush()
//     a block may still be staged in memory (Finish() always writes everything; Abandon() drops it);
//   * a device error surfaces as Status::IOError("pdb_sst_seal_host", <message>) from the call that
//     sealed (Add, Flush or Finish), never as a wrong trailer (there is no CPU fallback).
// Batch size: PDB_SEAL_BATCH_BYTES (default 16 MiB of staged blocks; a table ends its last batch
// early).  The batches are staged in page-locked, device-mapped memory from the checksum library
// (pdb_host_alloc, pdb_crc_route.h), so each seal runs zero-copy: the kernel reads the blocks and
// writes the trailers through the mapping, one launch, no DMA (the in-engine
// copy-inclusive seal rate; 16-MiB batches 29 013 vs 24 769 MiB/s for 4 MiB, fillrandom 10 M 5.27 vs
// 5.40 us/op, profiles/r05/engine/; with a table's index and filter blocks hashed by span launches
// beside the seal kernel, 35 777 MiB/s and 5.25 us/op, profiles/r05/c5b/).  PDB_SEAL_ASYNC=1 seals a
// full batch asynchronously (one std::async task per batch) while the builder stages the next one;
// the next seal, Finish() or Abandon() first waits for it and appends its bytes, so the file still
// receives the batches in order and the GPU seal overlaps block building.
// Default off: measured at C5 1M it does not help (fillrandom 4.12 / 4.15 vs 3.23 us/op
// synchronous, profiles/r02_c5_seal_async/) -- the seals of concurrent builders serialise on the
// device and the compaction thread is not waiting on them.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <future>
#include <string>
#include <vector>

#include "pdb_crc32c.h"
#include "pdb_crc_route.h"
#include "pdb_hooks.h"
#include "pebblesdb/comparator.h"
#include "pebblesdb/env.h"
#include "pebblesdb/filter_policy.h"
#include "pebblesdb/options.h"
#include "pebblesdb/table_builder.h"
#include "table/block_builder.h"
#include "table/filter_block.h"
#include "table/format.h"
#include "util/coding.h"

namespace leveldb {

namespace {
size_t SealBatchBytes() {
  static const size_t v = [] {
    const char* e = getenv("PDB_SEAL_BATCH_BYTES");
    const long long x = e ? atoll(e) : 0;
    return x > 0 ? static_cast<size_t>(x) : static_cast<size_t>(16u << 20);
  }();
  return v;
}
// A growable byte buffer in the route's staging memory (page-locked on the GPU route).  Growth
// copies; the builder keeps two of them (staged, in flight) for its whole life, so after the first
// batches no allocation happens.
class StageBuf {
 public:
  StageBuf() = default;
  StageBuf(const StageBuf&) = delete;
  StageBuf& operator=(const StageBuf&) = delete;
  ~StageBuf() { pdb_route::HostFree(p_); }
  char* data() { return p_; }
  size_t size() const { return n_; }
  void clear() { n_ = 0; }
  // false: the staging memory could not grow
  bool append(const char* d, size_t k) {
    if (n_ + k > cap_ && !grow(n_ + k)) return false;
    memcpy(p_ + n_, d, k);
    n_ += k;
    return true;
  }
  void swap(StageBuf& o) {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    std::swap(cap_, o.cap_);
  }

 private:
  bool grow(size_t need);
  char* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

bool SealAsync() {
  static const bool v = [] {
    const char* e = getenv("PDB_SEAL_ASYNC");
    return e && e[0] == '1';
  }();
  return v;
}
bool StageBuf::grow(size_t need) {
  // a batch ends just past SealBatchBytes(); one block can be larger
  const size_t cap = std::max(need, std::max(2 * cap_, SealBatchBytes() + (SealBatchBytes() >> 2)));
  void* q = nullptr;
  if (pdb_route::HostAlloc(cap, &q) != 0 || !q) return false;
  if (n_) memcpy(q, p_, n_);
  pdb_route::HostFree(p_);
  p_ = static_cast<char*>(q);
  cap_ = cap;
  return true;
}
}  // namespace

struct TableBuilder::Rep {
  Options options;
  Options index_block_options;  // restart interval 1: every index key is a restart point
  WritableFile* file;
  uint64_t offset;  // file offset of the next block: staged blocks included
  Status status;
  BlockBuilder data_block;
  BlockBuilder index_block;
  std::string last_key;
  int64_t num_entries;
  bool closed;
  FilterBlockBuilder* filter_block;
  // The index entry of a finished data block is written when the next block's first key is seen,
  // so its separator can be short (table_builder.cc:33-41).
  bool pending_index_entry;
  BlockHandle pending_handle;
  std::string compressed_output;
  // buffered emission: blocks in file order, each [contents][type][crc placeholder]
  StageBuf staged;
  std::vector<pdb_block_handle> staged_handles;  // relative to staged
  // the previous batch, being sealed on the GPU by an async task (its bytes follow in the file)
  StageBuf inflight;
  std::vector<pdb_block_handle> inflight_handles;
  std::future<int> inflight_rc;
  uint64_t inflight_ns = 0;
  bool has_inflight = false;

  Rep(const Options& opt, WritableFile* f)
      : options(opt),
        index_block_options(opt),
        file(f),
        offset(0),
        data_block(&options),
        index_block(&index_block_options),
        num_entries(0),
        closed(false),
        filter_block(opt.filter_policy == NULL ? NULL : new FilterBlockBuilder(opt.filter_policy)),
        pending_index_entry(false) {
    index_block_options.block_restart_interval = 1;
  }

  // Wait for the batch in flight, then append its bytes.
  void WaitInflight() {
    if (!has_inflight) return;
    const int rc = inflight_rc.get();
    pdb_hooks::AddSeal(inflight_handles.size(), inflight.size(), inflight_ns);
    if (rc != 0) {
      if (status.ok()) status = Status::IOError("pdb_sst_seal_host", pdb_route::LastError());
    } else if (status.ok()) {
      status = file->Append(Slice(inflight.data(), inflight.size()));
      if (status.ok()) status = file->Flush();
    }
    inflight.clear();
    inflight_handles.clear();
    has_inflight = false;
  }

  // Hand the staged batch to the GPU without waiting (the previous one is appended first).
  void SealStagedAsync() {
    if (staged_handles.empty()) return;
    WaitInflight();
    if (!status.ok() || !SealAsync()) {
      SealStaged();
      return;
    }
    inflight.swap(staged);
    inflight_handles.swap(staged_handles);
    staged.clear();
    staged_handles.clear();
    inflight_rc = std::async(std::launch::async, [this] {
      pdb_hooks::SealBegin();
      const uint64_t t0 = pdb_hooks::NowNs();
      const int rc = pdb_route::SstSealHost(inflight.data(), inflight.size(), inflight_handles.data(), inflight_handles.size());
      inflight_ns = pdb_hooks::NowNs() - t0;
      pdb_hooks::SealEnd();
      return rc;
    });
    has_inflight = true;
  }

  // Seal every staged trailer in one GPU batch, then append the span to the file (after the
  // batch in flight, if any).
  void SealStaged() {
    WaitInflight();
    if (staged_handles.empty()) return;
    if (status.ok()) {
      pdb_hooks::SealBegin();
      const uint64_t t0 = pdb_hooks::NowNs();
      const int rc = pdb_route::SstSealHost(staged.data(), staged.size(), staged_handles.data(), staged_handles.size());
      pdb_hooks::AddSeal(staged_handles.size(), staged.size(), pdb_hooks::NowNs() - t0);
      pdb_hooks::SealEnd();
      if (rc != 0) {
        status = Status::IOError("pdb_sst_seal_host", pdb_route::LastError());
      } else {
        status = file->Append(Slice(staged.data(), staged.size()));
        if (status.ok()) status = file->Flush();
      }
    }
    staged.clear();
    staged_handles.clear();
  }
};

TableBuilder::TableBuilder(const Options& options, WritableFile* file) : rep_(new Rep(options, file)) {
  if (rep_->filter_block != NULL) rep_->filter_block->StartBlock(0);
}

TableBuilder::~TableBuilder() {
  assert(rep_->closed);  // Finish() or Abandon() first
  delete rep_->filter_block;
  delete rep_;
}

Status TableBuilder::ChangeOptions(const Options& options) {
  if (options.comparator != rep_->options.comparator)
    return Status::InvalidArgument("changing comparator while building table");
  // the BlockBuilders hold pointers to these, so they see the new options too
  rep_->options = options;
  rep_->index_block_options = options;
  rep_->index_block_options.block_restart_interval = 1;
  return Status::OK();
}

void TableBuilder::Add(const Slice& key, const Slice& value) {
  Rep* r = rep_;
  assert(!r->closed);
  if (!ok()) return;
  if (r->pending_index_entry) {  // first key of a new data block: index the previous one
    assert(r->data_block.empty());
    r->options.comparator->FindShortestSeparator(&r->last_key, key);
    std::string enc;
    r->pending_handle.EncodeTo(&enc);
    r->index_block.Add(r->last_key, Slice(enc));
    r->pending_index_entry = false;
  }
  if (r->filter_block != NULL) r->filter_block->AddKey(key);
  r->last_key.assign(key.data(), key.size());
  ++r->num_entries;
  r->data_block.Add(key, value);
  if (r->data_block.CurrentSizeEstimate() >= r->options.block_size) Flush();
}

void TableBuilder::Flush() {
  Rep* r = rep_;
  assert(!r->closed);
  if (!ok() || r->data_block.empty()) return;
  assert(!r->pending_index_entry);
  WriteBlock(&r->data_block, &r->pending_handle);
  if (ok()) r->pending_index_entry = true;
  if (r->filter_block != NULL) r->filter_block->StartBlock(r->offset);
}

void TableBuilder::WriteBlock(BlockBuilder* block, BlockHandle* handle) {
  // on disk: contents, 1-byte compression type, 4-byte masked crc (table/format.h:86-87)
  assert(ok());
  Rep* r = rep_;
  const Slice raw = block->Finish();
  Slice contents = raw;
  CompressionType type = r->options.compression;
  if (type == kSnappyCompression) {  // Snappy stays delegated to the port layer (out of scope)
    std::string* c = &r->compressed_output;
    if (port::Snappy_Compress(raw.data(), raw.size(), c) && c->size() < raw.size() - raw.size() / 8u) {
      contents = *c;
    } else {  // not available, or saves less than 12.5 %: store it uncompressed
      type = kNoCompression;
    }
  } else if (type != kNoCompression) {
    abort();
  }
  WriteRawBlock(contents, type, handle);
  r->compressed_output.clear();
  block->Reset();
}

void TableBuilder::WriteRawBlock(const Slice& contents, CompressionType type, BlockHandle* handle) {
  Rep* r = rep_;
  handle->set_offset(r->offset);
  handle->set_size(contents.size());
  const uint64_t rel = r->staged.size();
  const char trailer[kBlockTrailerSize] = {static_cast<char>(type), 0, 0, 0, 0};  // crc: sealed in batch
  if (!r->staged.append(contents.data(), contents.size()) || !r->staged.append(trailer, kBlockTrailerSize)) {
    r->status = Status::IOError("pdb_host_alloc", "staging memory for the sealed batch");
    return;
  }
  r->staged_handles.push_back(pdb_block_handle{rel, contents.size()});
  r->offset += contents.size() + kBlockTrailerSize;
  if (r->staged.size() >= SealBatchBytes()) r->SealStagedAsync();
}

Status TableBuilder::status() const { return rep_->status; }

Status TableBuilder::Finish() {
  Rep* r = rep_;
  Flush();
  assert(!r->closed);
  r->closed = true;
  BlockHandle filter_handle, metaindex_handle, index_handle;
  if (ok() && r->filter_block != NULL) WriteRawBlock(r->filter_block->Finish(), kNoCompression, &filter_handle);
  if (ok()) {  // metaindex: "filter.<policy name>" -> the filter block
    BlockBuilder meta_index(&r->options);
    if (r->filter_block != NULL) {
      std::string enc;
      filter_handle.EncodeTo(&enc);
      meta_index.Add("filter." + std::string(r->options.filter_policy->Name()), enc);
    }
    WriteBlock(&meta_index, &metaindex_handle);
  }
  if (ok()) {
    if (r->pending_index_entry) {  // the last data block's index entry
      r->options.comparator->FindShortSuccessor(&r->last_key);
      std::string enc;
      r->pending_handle.EncodeTo(&enc);
      r->index_block.Add(r->last_key, Slice(enc));
      r->pending_index_entry = false;
    }
    WriteBlock(&r->index_block, &index_handle);
  }
  r->SealStaged();  // every trailer of the table's last batch, then its bytes
  if (ok()) {
    Footer footer;
    footer.set_metaindex_handle(metaindex_handle);
    footer.set_index_handle(index_handle);
    std::string enc;
    footer.EncodeTo(&enc);
    r->status = r->file->Append(enc);
    if (r->status.ok()) r->offset += enc.size();
  }
  return r->status;
}

void TableBuilder::Abandon() {
  Rep* r = rep_;
  assert(!r->closed);
  r->closed = true;
  if (r->has_inflight) (void)r->inflight_rc.get();  // never written: the caller discards the file
  r->has_inflight = false;
  r->inflight.clear();
  r->inflight_handles.clear();
  r->staged.clear();
  r->staged_handles.clear();
}

uint64_t TableBuilder::NumEntries() const { return rep_->num_entries; }

uint64_t TableBuilder::FileSize() const { return rep_->offset; }

}  // namespace leveldb
