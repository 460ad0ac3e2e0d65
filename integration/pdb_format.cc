// integration/pdb_format.cc -- drop-in for the reference's table/format.cc with the ReadBlock
// checksum check on the MI355X.
//
// Replaces, in a PebblesDB build that compiles this file instead of src/table/format.cc:
//   BlockHandle::EncodeTo / DecodeFrom   (format.cc:15-30; two varint64s)
//   Footer::EncodeTo / DecodeFrom        (format.cc:32-64; handles, padding, magic)
//   ReadBlock                            (format.cc:66-148)
// Declarations are the reference's own (table/format.h:22-101); behaviour and Status messages are
// the reference's: "truncated block read", "block checksum mismatch", "bad block type",
// "corrupted compressed block contents", "bad block handle", "not an sstable (bad magic number)".
// The one change: with ReadOptions::verify_checksums the CRC of contents || type is computed by
// libpdb_crc32c.so (pdb_crc32c_value: one request to the persistent scalar service), never on the
// CPU.  A device failure aborts inside the library (the reference's Value() cannot fail either).
#include <string.h>
#include <time.h>

#include <atomic>
#include <mutex>

#include "pdb_crc32c.h"
#include "pdb_crc_route.h"
#include "pdb_hooks.h"
#include "pebblesdb/env.h"
#include "pebblesdb/options.h"
#include "port/port.h"
#include "table/format.h"
#include "util/coding.h"

namespace pdb_hooks {
namespace {
constexpr int kCounters = 29;
std::atomic<uint64_t> g_counters[kCounters];
std::mutex g_seal_mu;
int g_seal_active = 0;
uint64_t g_seal_t0 = 0;
}
uint64_t NowNs() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
}
void AddSeal(uint64_t blocks, uint64_t bytes, uint64_t ns) {
  g_counters[0].fetch_add(1, std::memory_order_relaxed);
  g_counters[1].fetch_add(blocks, std::memory_order_relaxed);
  g_counters[2].fetch_add(bytes, std::memory_order_relaxed);
  g_counters[3].fetch_add(ns, std::memory_order_relaxed);
  const uint64_t mib = bytes >> 20;
  const int b = mib < 1 ? 0 : (mib < 4 ? 1 : (mib < 8 ? 2 : (mib < 15 ? 3 : 4)));
  g_counters[14 + b].fetch_add(1, std::memory_order_relaxed);
  g_counters[19 + b].fetch_add(bytes, std::memory_order_relaxed);
  g_counters[24 + b].fetch_add(ns, std::memory_order_relaxed);
}
void SealBegin() {
  std::lock_guard<std::mutex> lk(g_seal_mu);
  if (g_seal_active++ == 0) g_seal_t0 = NowNs();
  if (static_cast<uint64_t>(g_seal_active) > g_counters[13].load(std::memory_order_relaxed))
    g_counters[13].store(static_cast<uint64_t>(g_seal_active), std::memory_order_relaxed);
}
void SealEnd() {
  std::lock_guard<std::mutex> lk(g_seal_mu);
  if (--g_seal_active == 0) g_counters[12].fetch_add(NowNs() - g_seal_t0, std::memory_order_relaxed);
}
void AddScan(uint64_t blocks, uint64_t bytes, uint64_t ns, uint64_t bad) {
  g_counters[8].fetch_add(1, std::memory_order_relaxed);
  g_counters[9].fetch_add(blocks, std::memory_order_relaxed);
  g_counters[10].fetch_add(bytes, std::memory_order_relaxed);
  g_counters[11].fetch_add(ns, std::memory_order_relaxed);
  if (bad) g_counters[7].fetch_add(bad, std::memory_order_relaxed);
}
void AddVerify(uint64_t bytes, uint64_t ns, bool failed) {
  g_counters[4].fetch_add(1, std::memory_order_relaxed);
  g_counters[5].fetch_add(bytes, std::memory_order_relaxed);
  g_counters[6].fetch_add(ns, std::memory_order_relaxed);
  if (failed) g_counters[7].fetch_add(1, std::memory_order_relaxed);
}
}  // namespace pdb_hooks

extern "C" void pdb_hook_stats_get(pdb_hook_stats* out) {
  uint64_t* v = reinterpret_cast<uint64_t*>(out);
  for (int i = 0; i < pdb_hooks::kCounters; ++i) v[i] = pdb_hooks::g_counters[i].load(std::memory_order_relaxed);
}

extern "C" void pdb_hook_stats_reset(void) {
  for (int i = 0; i < pdb_hooks::kCounters; ++i) pdb_hooks::g_counters[i].store(0, std::memory_order_relaxed);
}

namespace leveldb {

void BlockHandle::EncodeTo(std::string* dst) const {
  assert(offset_ != ~static_cast<uint64_t>(0) && size_ != ~static_cast<uint64_t>(0));  // both set
  PutVarint64(dst, offset_);
  PutVarint64(dst, size_);
}

Status BlockHandle::DecodeFrom(Slice* input) {
  if (!GetVarint64(input, &offset_) || !GetVarint64(input, &size_)) return Status::Corruption("bad block handle");
  return Status::OK();
}

void Footer::EncodeTo(std::string* dst) const {
  const size_t start = dst->size();
  metaindex_handle_.EncodeTo(dst);
  index_handle_.EncodeTo(dst);
  dst->resize(start + 2 * BlockHandle::kMaxEncodedLength);  // zero padding up to the magic number
  PutFixed32(dst, static_cast<uint32_t>(kTableMagicNumber));
  PutFixed32(dst, static_cast<uint32_t>(kTableMagicNumber >> 32));
  assert(dst->size() == start + kEncodedLength);
}

Status Footer::DecodeFrom(Slice* input) {
  const char* magic = input->data() + kEncodedLength - 8;
  const uint64_t m = static_cast<uint64_t>(DecodeFixed32(magic)) |
                     (static_cast<uint64_t>(DecodeFixed32(magic + 4)) << 32);
  if (m != kTableMagicNumber) return Status::InvalidArgument("not an sstable (bad magic number)");
  Status s = metaindex_handle_.DecodeFrom(input);
  if (s.ok()) s = index_handle_.DecodeFrom(input);
  if (s.ok()) {  // skip the padding: the input continues after the magic number
    const char* end = magic + 8;
    *input = Slice(end, input->data() + input->size() - end);
  }
  return s;
}

Status ReadBlock(RandomAccessFile* file, const ReadOptions& options, const BlockHandle& handle,
                 BlockContents* result) {
  *result = BlockContents();
  const size_t n = static_cast<size_t>(handle.size());
  char* buf = new char[n + kBlockTrailerSize];
  Slice got;
  Status s = file->Read(handle.offset(), n + kBlockTrailerSize, &got, buf);
  if (!s.ok()) {
    delete[] buf;
    return s;
  }
  if (got.size() != n + kBlockTrailerSize) {
    delete[] buf;
    return Status::Corruption("truncated block read");
  }
  const char* data = got.data();  // the file may hand back its own memory (mmap reads)
  if (options.verify_checksums) {
    // trailer = [type][Mask(crc32c(contents || type))]: one GPU request over n + 1 bytes
    const uint64_t t0 = pdb_hooks::NowNs();
    const uint32_t actual = pdb_route::Value(data, n + 1);
    const bool bad = pdb_route::Unmask(DecodeFixed32(data + n + 1)) != actual;
    pdb_hooks::AddVerify(n + 1, pdb_hooks::NowNs() - t0, bad);
    if (bad) {
      delete[] buf;
      return Status::Corruption("block checksum mismatch");
    }
  }
  if (data == buf) return pdb_hooks::BlockFromChecked(data, n, buf, true, result);
  delete[] buf;
  return pdb_hooks::BlockFromChecked(data, n, nullptr, true, result);
}

}  // namespace leveldb

namespace pdb_hooks {
// ReadBlock's type dispatch (format.cc:106-145) for data = [contents n B][type] whose checksum has
// been dealt with.  owned: the heap buffer data sits in (taken over; freed on every path), else
// nullptr with stable = true (the file's own memory, live while it is open: handed out uncachable)
// or stable = false (a transient buffer: the contents are copied).
leveldb::Status BlockFromChecked(const char* data, size_t n, char* owned, bool stable, leveldb::BlockContents* result) {
  using leveldb::Slice;
  using leveldb::Status;
  switch (data[n]) {
    case leveldb::kNoCompression:
      if (owned != nullptr) {
        result->data = Slice(owned, n);
        result->heap_allocated = true;
        result->cachable = true;
      } else if (stable) {
        result->data = Slice(data, n);
        result->heap_allocated = false;
        result->cachable = false;
      } else {
        char* copy = new char[n];
        memcpy(copy, data, n);
        result->data = Slice(copy, n);
        result->heap_allocated = true;
        result->cachable = true;
      }
      return Status::OK();
    case leveldb::kSnappyCompression: {  // Snappy stays delegated to the port layer (out of scope)
      size_t ulen = 0;
      if (!leveldb::port::Snappy_GetUncompressedLength(data, n, &ulen)) {
        delete[] owned;
        return Status::Corruption("corrupted compressed block contents");
      }
      char* ubuf = new char[ulen];
      const bool ok = leveldb::port::Snappy_Uncompress(data, n, ubuf);
      delete[] owned;
      if (!ok) {
        delete[] ubuf;
        return Status::Corruption("corrupted compressed block contents");
      }
      result->data = Slice(ubuf, ulen);
      result->heap_allocated = true;
      result->cachable = true;
      return Status::OK();
    }
    default:
      delete[] owned;
      return Status::Corruption("bad block type");
  }
}
}  // namespace pdb_hooks
