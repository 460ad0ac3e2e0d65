// integration/pdb_table.cc -- drop-in for the reference's table/table.cc (the sstable reader:
// Table::Open, the two-level iterator's block function, Get's lookup, ApproximateOffsetOf;
// declarations include/pebblesdb/table.h) with a VERIFIED READ-AHEAD for scans.
//
// with ReadOptions::verify_checksums, a scan over a table (an iterator, and every
// compaction input when Options::paranoid_checks is set: version_set.cc:2907-2910) reads its data
// blocks one ReadBlock at a time (table.cc:193-259 -> format.cc:66-104), i.e. one checksum -- here
// one PCIe round trip to the GPU -- per ~4-KiB block.  This reader keeps the table's data-block
// handles (decoded from the index block it already holds) and, when an iterator asks for a block,
// reads it and the data blocks after it -- 16 KiB, then x4 per window while the iterator reads on in
// order, up to 1 MiB -- with ONE file read and checks all their trailers with ONE
// pdb_sst_verify_host batch; the following block reads are served from that window.  Semantics are ReadBlock's: the bytes a block is built from are exactly the bytes
// whose checksum was checked, and a block whose check failed returns Corruption("block checksum
// mismatch") when, and only when, it is read.  Point reads (Get) and reads without
// verify_checksums take the reference path (ReadBlock; with verify on, pdb_format.cc's GPU check).
// A device failure aborts, as the reference's crc32c::Value() cannot fail either.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "pdb_crc32c.h"
#include "pdb_crc_route.h"
#include "pdb_hooks.h"
#include "pebblesdb/cache.h"
#include "pebblesdb/comparator.h"
#include "pebblesdb/env.h"
#include "pebblesdb/filter_policy.h"
#include "pebblesdb/options.h"
#include "pebblesdb/table.h"
#include "port/port.h"
#include "table/block.h"
#include "table/filter_block.h"
#include "table/format.h"
#include "table/two_level_iterator.h"
#include "util/coding.h"
#include "util/mutexlock.h"

namespace leveldb {
namespace {

// Read-ahead windows of an iterator: 16 KiB of data blocks at its first block, then x4 per window
// while it keeps reading on in order, up to 1 MiB (a Seek followed by a few Next()s costs one small
// batch; a scan settles at 1-MiB batches).  Point reads (Get) never read ahead.
constexpr uint64_t kFirstWindow = 16u << 10;
constexpr int kMaxGrow = 3;  // 16 KiB << 2 * 3 = 1 MiB
thread_local int t_point_read = 0;  // > 0 inside Table::InternalGet

// The read-ahead state of one table (shared by every reader of it, so under a mutex).
class ScanWindow {
 public:
  // The block at `h` for a reader with verify_checksums on: from the window, by a new window, or
  // (not a scan) by ReadBlock.
  Status Read(RandomAccessFile* file, const Block* index, const Comparator* cmp, const ReadOptions& opt,
              const BlockHandle& h, BlockContents* out) {
    if (t_point_read == 0) {
      MutexLock l(&mu_);
      if (!decoded_) Decode(index, cmp);
      const int64_t i = Find(h);
      const bool in_order = i >= 0 && i == last_ + 1;
      last_ = i;
      if (i >= 0 && i >= lo_ && i < hi_) return Serve(i, out);
      grow_ = in_order ? std::min(grow_ + 1, kMaxGrow) : 0;
      if (i >= 0 && Fill(file, i, kFirstWindow << (2 * grow_))) return Serve(i, out);
    }
    return ReadBlock(file, opt, h, out);
  }

 private:
  void Decode(const Block* index, const Comparator* cmp) {
    Iterator* it = const_cast<Block*>(index)->NewIterator(cmp);
    for (it->SeekToFirst(); it->Valid(); it->Next()) {
      Slice v = it->value();
      BlockHandle bh;
      if (!bh.DecodeFrom(&v).ok()) break;  // a damaged index: scans fall back to ReadBlock past it
      blocks_.push_back(pdb_block_handle{bh.offset(), bh.size()});
    }
    delete it;
    decoded_ = true;
  }
  int64_t Find(const BlockHandle& h) const {
    auto p = std::lower_bound(blocks_.begin(), blocks_.end(), h.offset(),
                              [](const pdb_block_handle& b, uint64_t off) { return b.offset < off; });
    if (p == blocks_.end() || p->offset != h.offset() || p->size != h.size()) return -1;
    return p - blocks_.begin();
  }
  // Blocks i.. that lie back to back in the file, up to `window` bytes (at least one): one read,
  // one GPU check.  False (no window) if the read comes back short or fails -- ReadBlock then
  // reports it for the block asked for.
  bool Fill(RandomAccessFile* file, int64_t i, uint64_t window) {
    const uint64_t base = blocks_[i].offset;
    uint64_t end = base;
    int64_t j = i;
    while (j < static_cast<int64_t>(blocks_.size()) && blocks_[j].offset == end &&
           (j == i || blocks_[j].offset + blocks_[j].size + kBlockTrailerSize - base <= window)) {
      end = blocks_[j].offset + blocks_[j].size + kBlockTrailerSize;
      ++j;
    }
    const uint64_t t0 = pdb_hooks::NowNs();
    buf_.resize(end - base);
    Slice got;
    lo_ = hi_ = 0;
    if (!file->Read(base, end - base, &got, &buf_[0]).ok() || got.size() != end - base) return false;
    std::vector<pdb_block_handle> rel(blocks_.begin() + i, blocks_.begin() + j);
    for (auto& b : rel) b.offset -= base;
    ok_.assign(rel.size(), 0);
    const int64_t bad = pdb_route::SstVerifyHost(got.data(), got.size(), rel.data(), rel.size(), ok_.data());
    if (bad < 0) {
      fprintf(stderr, "pdb_table: GPU block check failed: %s\n", pdb_route::LastError());
      abort();
    }
    data_ = got.data();  // buf_, or the file's own (mmap) memory
    base_ = base;
    lo_ = i;
    hi_ = j;
    pdb_hooks::AddScan(static_cast<uint64_t>(j - i), end - base, pdb_hooks::NowNs() - t0, static_cast<uint64_t>(bad));
    return true;
  }
  Status Serve(int64_t i, BlockContents* out) {
    if (!ok_[i - lo_]) return Status::Corruption("block checksum mismatch");
    return pdb_hooks::BlockFromChecked(data_ + (blocks_[i].offset - base_), blocks_[i].size, nullptr, false, out);
  }

  port::Mutex mu_;
  bool decoded_ = false;
  std::vector<pdb_block_handle> blocks_;  // data blocks, index order = file order
  int64_t last_ = -2;                     // index of the block read last (any iterator)
  int grow_ = 0;                          // windows read in order so far (size 16 KiB << 2 grow_)
  std::string buf_;
  const char* data_ = nullptr;
  uint64_t base_ = 0;
  int64_t lo_ = 0, hi_ = 0;  // the window: blocks [lo_, hi_)
  std::vector<uint8_t> ok_;
};

void DeleteOwnedBlock(void* arg, void*) { delete reinterpret_cast<Block*>(arg); }
void DeleteCachedBlock(const Slice&, void* value) { delete reinterpret_cast<Block*>(value); }
void ReleaseCachedBlock(void* cache, void* handle) {
  reinterpret_cast<Cache*>(cache)->Release(reinterpret_cast<Cache::Handle*>(handle));
}

}  // namespace

struct Table::Rep {
  ~Rep() {
    delete filter;
    delete[] filter_data;
    delete index_block;
  }
  Options options;
  Status status;
  RandomAccessFile* file = nullptr;
  uint64_t cache_id = 0;
  FilterBlockReader* filter = nullptr;
  const char* filter_data = nullptr;  // owned when the filter block was heap-allocated
  BlockHandle metaindex_handle;
  Block* index_block = nullptr;
  ScanWindow scan;
};

Status Table::Open(const Options& options, RandomAccessFile* file, uint64_t size, Table** table, Timer* /*timer*/) {
  *table = nullptr;
  if (size < Footer::kEncodedLength) return Status::InvalidArgument("file is too short to be an sstable");
  char space[Footer::kEncodedLength];
  Slice in;
  Status s = file->Read(size - Footer::kEncodedLength, Footer::kEncodedLength, &in, space);
  if (!s.ok()) return s;
  Footer footer;
  s = footer.DecodeFrom(&in);
  if (!s.ok()) return s;
  BlockContents index;
  s = ReadBlock(file, ReadOptions(), footer.index_handle(), &index);  // (verify off, as table.cc:97)
  if (!s.ok()) return s;
  Rep* rep = new Rep;
  rep->options = options;
  rep->file = file;
  rep->metaindex_handle = footer.metaindex_handle();
  rep->index_block = new Block(index);
  rep->cache_id = options.block_cache != nullptr ? options.block_cache->NewId() : 0;
  *table = new Table(rep);
  (*table)->ReadMeta(footer);
  return Status::OK();
}

// The filter named by the metaindex, if the options have a policy; errors are not fatal (the
// table works without it).
void Table::ReadMeta(const Footer& footer) {
  if (rep_->options.filter_policy == nullptr) return;
  BlockContents contents;
  if (!ReadBlock(rep_->file, ReadOptions(), footer.metaindex_handle(), &contents).ok()) return;
  Block meta(contents);
  Iterator* it = meta.NewIterator(BytewiseComparator());
  const std::string name = std::string("filter.") + rep_->options.filter_policy->Name();
  it->Seek(name);
  if (it->Valid() && it->key() == Slice(name)) ReadFilter(it->value());
  delete it;
}

void Table::ReadFilter(const Slice& filter_handle_value) {
  Slice v = filter_handle_value;
  BlockHandle h;
  if (!h.DecodeFrom(&v).ok()) return;
  BlockContents block;
  if (!ReadBlock(rep_->file, ReadOptions(), h, &block).ok()) return;
  if (block.heap_allocated) rep_->filter_data = block.data.data();
  rep_->filter = new FilterBlockReader(rep_->options.filter_policy, block.data);
}

Table::~Table() { delete rep_; }

Iterator* Table::BlockReader(void* arg, const ReadOptions& options, const Slice& index_value) {
  (void)(rand() % NUM_SEEK_THREADS);  // the reference draws a seek-timer slot per call (table.cc:196)
  Table* table = reinterpret_cast<Table*>(arg);
  Rep* r = table->rep_;
  Cache* cache = r->options.block_cache;
  BlockHandle handle;
  Slice in = index_value;
  Status s = handle.DecodeFrom(&in);  // trailing bytes after the handle are allowed
  Block* block = nullptr;
  Cache::Handle* cached = nullptr;
  if (s.ok()) {
    char key_space[16];
    const Slice key(key_space, sizeof(key_space));
    if (cache != nullptr) {
      EncodeFixed64(key_space, r->cache_id);
      EncodeFixed64(key_space + 8, handle.offset());
      cached = cache->Lookup(key);
      if (cached != nullptr) block = reinterpret_cast<Block*>(cache->Value(cached));
    }
    if (block == nullptr) {
      BlockContents contents;
      s = options.verify_checksums
              ? r->scan.Read(r->file, r->index_block, r->options.comparator, options, handle, &contents)
              : ReadBlock(r->file, options, handle, &contents);
      if (s.ok()) {
        block = new Block(contents);
        if (cache != nullptr && contents.cachable && options.fill_cache)
          cached = cache->Insert(key, block, block->size(), &DeleteCachedBlock);
      }
    }
  }
  if (block == nullptr) return NewErrorIterator(s);
  Iterator* it = block->NewIterator(r->options.comparator);
  if (cached == nullptr)
    it->RegisterCleanup(&DeleteOwnedBlock, block, nullptr);
  else
    it->RegisterCleanup(&ReleaseCachedBlock, cache, cached);
  return it;
}

Iterator* Table::NewIterator(const ReadOptions& options) const {
  return NewTwoLevelIterator(rep_->index_block->NewIterator(rep_->options.comparator), &Table::BlockReader,
                             const_cast<Table*>(this), options);
}

Status Table::InternalGet(const ReadOptions& options, const Slice& k, void* arg,
                          void (*saver)(void*, const Slice&, const Slice&), Timer* /*timer*/) {
  Iterator* index = rep_->index_block->NewIterator(rep_->options.comparator);
  index->Seek(k);
  Status s;
  if (index->Valid()) {
    Slice hv = index->value();
    BlockHandle h;
#ifdef FILE_LEVEL_FILTER
    const bool skip = false;  // the file-level filter was consulted by the caller
#else
    const bool skip = rep_->filter != nullptr && h.DecodeFrom(&hv).ok() && !rep_->filter->KeyMayMatch(h.offset(), k);
#endif
    if (!skip) {
      ++t_point_read;  // one block for one key: the ReadBlock path, never a window
      Iterator* bi = BlockReader(this, options, index->value());
      --t_point_read;
      bi->Seek(k);
      if (bi->Valid()) (*saver)(arg, bi->key(), bi->value());
      s = bi->status();
      delete bi;
    }
  }
  if (s.ok()) s = index->status();
  delete index;
  return s;
}

// The offset of the data block that would hold `key`; past the last key (or an undecodable handle),
// the metaindex's offset -- near the end of the file.
uint64_t Table::ApproximateOffsetOf(const Slice& key) const {
  Iterator* index = rep_->index_block->NewIterator(rep_->options.comparator);
  index->Seek(key);
  uint64_t off = rep_->metaindex_handle.offset();
  if (index->Valid()) {
    Slice v = index->value();
    BlockHandle h;
    if (h.DecodeFrom(&v).ok()) off = h.offset();
  }
  delete index;
  return off;
}

}  // namespace leveldb
