// tests/cpp/table_blocks_test.cc -- C++ consumer of the drop-in headers, written the way the
// reference's own tests are (util/crc32c_test.cc, table/table_test.cc): the LevelDB-compatible
// leveldb::crc32c API on known answers, then a buffered WriteRawBlock round trip and the
// ReadBlock checksum check (including a corrupted block).  Built by tests/test_cpp_consumer.py
// with g++ against include/ and pebblesdb_amd/_lib/libpdb_crc32c.so.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "pebblesdb_amd/crc32c.h"
#include "pebblesdb_amd/log_records.h"
#include "pebblesdb_amd/table_blocks.h"

static int failures = 0;
#define EXPECT(cond)                                               \
  do {                                                             \
    if (!(cond)) {                                                 \
      fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

using namespace leveldb;

static void StandardResults() {  // util/crc32c_test.cc:13-48
  char buf[32];
  memset(buf, 0, sizeof(buf));
  EXPECT(0x8a9136aa == crc32c::Value(buf, sizeof(buf)));
  memset(buf, 0xff, sizeof(buf));
  EXPECT(0x62a8ab43 == crc32c::Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = i;
  EXPECT(0x46dd794e == crc32c::Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = 31 - i;
  EXPECT(0x113fdb5c == crc32c::Value(buf, sizeof(buf)));
  unsigned char data[48] = {0x01, 0xc0, 0, 0, 0, 0, 0, 0, 0,    0,    0, 0, 0,    0, 0, 0,
                            0x14, 0,    0, 0, 0, 0, 4, 0, 0,    0,    0, 0x14, 0, 0, 0, 0x18,
                            0x28, 0,    0, 0, 0, 0, 0, 0, 0x02, 0,    0, 0, 0,    0, 0, 0};
  EXPECT(0xd9963a56 == crc32c::Value(reinterpret_cast<char*>(data), sizeof(data)));
}

static void LargeBuffer() {  // util/crc32c_test.cc:50-60
  std::string tmp(4096, 'A');
  EXPECT(0x3c36f666 == crc32c::Value(tmp.data(), 64));
  EXPECT(0xf6607a92 == crc32c::Value(tmp.data(), 1024));
  EXPECT(0xa9bc21ef == crc32c::Value(tmp.data(), 1111));
  EXPECT(0x88ddb66b == crc32c::Value(tmp.data(), 2048));
  EXPECT(0x057251e9 == crc32c::Value(tmp.data(), 4096));
}

static void ExtendAndMask() {  // util/crc32c_test.cc:62-77
  EXPECT(crc32c::Value("a", 1) != crc32c::Value("foo", 3));
  EXPECT(crc32c::Value("hello world", 11) == crc32c::Extend(crc32c::Value("hello ", 6), "world", 5));
  uint32_t crc = crc32c::Value("foo", 3);
  EXPECT(crc != crc32c::Mask(crc));
  EXPECT(crc != crc32c::Mask(crc32c::Mask(crc)));
  EXPECT(crc == crc32c::Unmask(crc32c::Mask(crc)));
  EXPECT(crc == crc32c::Unmask(crc32c::Unmask(crc32c::Mask(crc32c::Mask(crc)))));
}

static void TrailerRoundTrip() {
  // Blocks of the sizes a real table has: ~4 KiB data blocks, a tiny metaindex, a large index.
  std::vector<std::string> blocks;
  unsigned x = 301;
  size_t sizes[] = {4171, 4175, 4096, 0, 51, 17, 213 * 1024 + 3, 4091};
  for (size_t n : sizes) {
    std::string b(n, '\0');
    for (size_t i = 0; i < n; ++i) {
      x = x * 1103515245u + 12345u;
      b[i] = static_cast<char>(x >> 16);
    }
    blocks.push_back(b);
  }
  pdb::BlockTrailerBatch batch(1000);
  std::vector<pdb::BlockHandle> hs;
  uint64_t expect_off = 1000;
  for (size_t i = 0; i < blocks.size(); ++i) {
    pdb::BlockHandle h = batch.Add(blocks[i].data(), blocks[i].size(), i % 2);
    EXPECT(h.offset == expect_off && h.size == blocks[i].size());  // WriteRawBlock's handle
    expect_off += blocks[i].size() + pdb::kBlockTrailerSize;
    hs.push_back(pdb::BlockHandle{h.offset - 1000, h.size});
  }
  EXPECT(batch.Seal() == 0);
  const std::string& img = batch.bytes();
  // Each trailer equals what WriteRawBlock computes with the scalar API (table_builder.cc:196-199)
  for (size_t i = 0; i < blocks.size(); ++i) {
    const char* p = img.data() + hs[i].offset;
    char type = static_cast<char>(i % 2);
    uint32_t crc = crc32c::Value(blocks[i].data(), blocks[i].size());
    crc = crc32c::Extend(crc, &type, 1);
    uint32_t stored;
    memcpy(&stored, p + hs[i].size + 1, 4);
    EXPECT(p[hs[i].size] == type);
    EXPECT(stored == crc32c::Mask(crc));
    EXPECT(crc32c::Unmask(stored) == crc32c::Value(p, hs[i].size + 1));  // ReadBlock's check
  }
  std::vector<uint8_t> ok;
  EXPECT(pdb::VerifyBlocks(img.data(), img.size(), hs.data(), hs.size(), &ok) == 0);
  // Corrupt one byte of block 6 -> exactly that block reports "block checksum mismatch".
  std::string bad = img;
  bad[hs[6].offset + 12345] ^= 0x01;
  EXPECT(pdb::VerifyBlocks(bad.data(), bad.size(), hs.data(), hs.size(), &ok) == 1);
  for (size_t i = 0; i < hs.size(); ++i) EXPECT(ok[i] == (i == 6 ? 0 : 1));
  // A corrupted trailer byte is detected too.
  bad = img;
  bad[hs[2].offset + hs[2].size + 2] ^= 0x80;
  EXPECT(pdb::VerifyBlocks(bad.data(), bad.size(), hs.data(), hs.size(), &ok) == 1 && ok[2] == 0);
}

// The reference-written tables of tests/golden/sst (built by the reference's own TableBuilder):
// VerifyTable walks footer -> index -> metaindex like Table::Open and checks every block in one
// batch; a flipped byte in a data block, the index block or a trailer fails exactly one block.
static std::string ReadFile(const std::string& path) {
  std::string s;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return s;
  char buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, k);
  fclose(f);
  return s;
}

static void VerifyReferenceTables(const std::string& dir) {
  const char* names[] = {"small_bloom.sst", "bigvals.sst", "tinyblocks.sst", "empty.sst"};
  for (const char* nm : names) {
    const std::string img = ReadFile(dir + "/" + nm);
    EXPECT(!img.empty());
    if (img.empty()) continue;
    pdb::TableLayout t;
    std::vector<uint8_t> ok;
    std::string err;
    EXPECT(pdb::VerifyTable(img.data(), img.size(), &t, &ok, &err) == 0);
    EXPECT(err.empty());
    const std::vector<pdb::BlockHandle> all = t.All();
    EXPECT(ok.size() == all.size() && all.size() >= 2);
    // ...and the same blocks through the device hook in one batch
    for (size_t k = 0; k + 2 < all.size() && k < 3; ++k) {
      std::string bad = img;
      bad[all[k].offset + all[k].size / 2] ^= 0x04;
      EXPECT(pdb::VerifyTable(bad.data(), bad.size(), nullptr, &ok, nullptr) == 1 && ok[k] == 0);
    }
    std::string bad = img;  // the stored trailer of the index block: checked before it is parsed
    bad[t.index.offset + t.index.size + 3] ^= 0x10;
    EXPECT(pdb::VerifyTable(bad.data(), bad.size(), nullptr, &ok, &err) == -1000 && err == "block checksum mismatch");
    bad = img;  // a corrupted index entry: the same verdict, never a parse error or garbage handles
    bad[t.index.offset + 1] ^= 0x7f;
    EXPECT(pdb::VerifyTable(bad.data(), bad.size(), nullptr, &ok, &err) == -1000 && err == "block checksum mismatch");
    bad = img;  // ...and the metaindex block
    bad[t.metaindex.offset + t.metaindex.size + 1] ^= 0x01;
    EXPECT(pdb::VerifyTable(bad.data(), bad.size(), nullptr, &ok, &err) == -1000 && err == "block checksum mismatch");
    bad = img;  // a broken magic number is structural corruption, not a checksum count
    bad[bad.size() - 1] ^= 0x01;
    EXPECT(pdb::VerifyTable(bad.data(), bad.size(), nullptr, &ok, &err) == -1000 &&
           err == "not an sstable (bad magic number)");
  }
}

// The reference-written logs of tests/golden/log (the reference's own log::Writer): every
// physical record verified in one batch; the logical record count (Full + Last) matches the
// manifest; a flipped payload byte or stored-CRC byte fails exactly that record.
static void VerifyReferenceLogs(const std::string& dir) {
  struct { const char* name; size_t logical; } logs[] = {{"wal_mixed.log", 15}, {"manifest_small.log", 300}};
  for (const auto& lg : logs) {
    const std::string img = ReadFile(dir + "/" + lg.name);
    EXPECT(!img.empty());
    if (img.empty()) continue;
    std::vector<pdb::log::PhysicalRecord> recs;
    std::vector<uint8_t> ok;
    EXPECT(pdb::log::VerifyLog(img.data(), img.size(), &recs, &ok) == 0);
    size_t logical = 0;
    for (const auto& r : recs) logical += r.type == pdb::log::kFullType || r.type == pdb::log::kLastType;
    EXPECT(logical == lg.logical && ok.size() == recs.size());
    // round trip: logical records (the log::Reader replay) -> the group-commit writer -> one
    // sealing batch == the file
    std::vector<pdb::log::LogicalRecord> payloads;
    std::vector<pdb::log::CorruptionReport> reports;
    EXPECT(pdb::log::ReplayLog(img.data(), img.size(), &payloads, &reports) == 0 && payloads.size() == lg.logical);
    pdb::log::BatchWriter w;
    for (const auto& pl : payloads) w.AddRecord(pl.data.data(), pl.data.size());
    EXPECT(w.num_physical_records() == recs.size() && w.Seal() == 0 && w.bytes() == img);
    for (size_t k = 0; k < recs.size(); k += (recs.size() + 4) / 5) {
      std::string bad = img;
      if (recs[k].length) {
        bad[recs[k].payload_offset() + recs[k].length / 2] ^= 0x20;
        EXPECT(pdb::log::VerifyLog(bad.data(), bad.size(), &recs, &ok) == 1 && ok[k] == 0);
      }
      bad = img;
      bad[recs[k].offset + 2] ^= 0x01;  // the stored crc
      EXPECT(pdb::log::VerifyLog(bad.data(), bad.size(), &recs, &ok) == 1 && ok[k] == 0);
    }
  }
}

// --replay <log>...: print what pdb::log::ReplayLog delivers (records: [LastRecordOffset, length,
// FNV-1a-64], reports: [bytes, reason]) in oracle/ref_logreader's JSON format, so the Python test
// compares it with the reference reader's output on the corrupted logs (corruptions.json).
static uint64_t Fnv1a64(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

static int Replay(const char* path) {
  const std::string img = ReadFile(path);
  std::vector<pdb::log::LogicalRecord> recs;
  std::vector<pdb::log::CorruptionReport> reports;
  if (pdb::log::ReplayLog(img.data(), img.size(), &recs, &reports) < 0) return 1;
  printf("{\"records\":[");
  for (size_t i = 0; i < recs.size(); ++i)
    printf("%s[%llu,%zu,\"%016llx\"]", i ? "," : "", (unsigned long long)recs[i].offset, recs[i].data.size(),
           (unsigned long long)Fnv1a64(recs[i].data));
  printf("],\"reports\":[");
  for (size_t i = 0; i < reports.size(); ++i)
    printf("%s[%llu,\"%s\"]", i ? "," : "", (unsigned long long)reports[i].bytes, reports[i].reason.c_str());
  printf("]}\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && std::string(argv[1]) == "--replay") {  // one JSON line per log file
    if (pdb_crc32c_init(0) != 0) return 2;
    for (int a = 2; a < argc; ++a)
      if (Replay(argv[a])) return 1;
    return 0;
  }
  if (pdb_crc32c_init(0) != 0) {
    fprintf(stderr, "no device: %s\n", pdb_last_error());
    return 2;
  }
  StandardResults();
  LargeBuffer();
  ExtendAndMask();
  TrailerRoundTrip();
  if (argc > 1) VerifyReferenceTables(argv[1]);
  if (argc > 2) VerifyReferenceLogs(argv[2]);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("table_blocks_test: PASS\n");
  return 0;
}
