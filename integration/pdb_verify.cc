// integration/pdb_verify.cc -- the reference's `leveldb-verify` (src/leveldb-verify.cc) with every
// checksum checked in ONE GPU batch per file (batched read verify for
// leveldb-verify), built against the engine compiled from the reference sources in place.
//
// For each file on the command line, by its name (db/filename.h ParseFileName):
//   * table (.sst / .ldb): Table::Open as the reference tool does it, then every data block the
//     tool's verified iterator reads (the index block's handles) is checked in ONE
//     pdb_sst_verify_host call, and the reference tool's walk follows -- every key parsed as an
//     internal key and looked up again through a second iterator (leveldb-verify.cc:142-168) --
//     with per-block checksums off when every block passed, on when one failed (so the engine's
//     ReadBlock, checked on the GPU by pdb_format.cc, reports each bad block where the reference
//     does).  Index, metaindex and filter blocks are not checked: the reference tool never checks
//     them (table.cc:97-133 reads the index with default ReadOptions, the others not at all);
//   * log / MANIFEST: pdb::ReplayLog checks every physical record in one batch and replays the
//     logical records with the reference log::Reader's drop / report rules; each record is then
//     decoded the way the reference tool does (a WriteBatch iterated / a VersionEdit decoded), each
//     corruption report printed where the reference reader prints it (before the record whose
//     ReadRecord call found it).
// Output and exit status follow the reference tool: problems go to stdout / stderr in its words
// ("corruption: N bytes; ...", "iterator error: Corruption: block checksum mismatch", ...), the
// exit status is 1 when a file could not be handled.  --timing prints each phase's wall time.
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "db/dbformat.h"
#include "db/filename.h"
#include "db/version_edit.h"
#include "db/write_batch_internal.h"
#include "pebblesdb/env.h"
#include "pebblesdb/iterator.h"
#include "pebblesdb/options.h"
#include "pebblesdb/table.h"
#include "pebblesdb/write_batch.h"
#include "pebblesdb_amd/log_records.h"
#include "pebblesdb_amd/table_blocks.h"
#include "util/logging.h"

namespace {

using Clock = std::chrono::steady_clock;
bool g_timing = false;
double g_crc_s = 0, g_walk_s = 0, g_read_s = 0;
uint64_t g_bytes = 0, g_blocks = 0, g_records = 0;

double Since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

bool ReadWhole(leveldb::Env* env, const std::string& fname, std::string* out) {
  const auto t0 = Clock::now();
  leveldb::Status s = leveldb::ReadFileToString(env, fname, out);
  g_read_s += Since(t0);
  if (!s.ok()) {
    fprintf(stderr, "%s\n", s.ToString().c_str());
    return false;
  }
  g_bytes += out->size();
  return true;
}

// WriteBatch items are only walked (the reference tool prints nothing per item either)
struct NullHandler : public leveldb::WriteBatch::Handler {
  void Put(const leveldb::Slice&, const leveldb::Slice&) override {}
  void Delete(const leveldb::Slice&) override {}
  void HandleGuard(const leveldb::Slice&, unsigned) override {}
};

bool VerifyLogFile(leveldb::Env* env, const std::string& fname, bool descriptor) {
  std::string img;
  if (!ReadWhole(env, fname, &img)) return false;
  std::vector<pdb::log::LogicalRecord> recs;
  std::vector<pdb::log::CorruptionReport> reports;
  auto t0 = Clock::now();
  const int64_t rc = pdb::log::ReplayLog(img.data(), img.size(), &recs, &reports);
  g_crc_s += Since(t0);
  if (rc < 0) {
    fprintf(stderr, "%s: device error %lld: %s\n", fname.c_str(), static_cast<long long>(rc), pdb_last_error());
    return false;
  }
  // reports are printed where the reference reader prints them: from inside the ReadRecord call
  // that returns record r.before, i.e. before that record's own output
  t0 = Clock::now();
  g_records += recs.size();
  size_t next_report = 0;
  auto flush_reports = [&](uint64_t upto) {
    for (; next_report < reports.size() && reports[next_report].before <= upto; ++next_report)
      printf("corruption: %d bytes; %s\n", static_cast<int>(reports[next_report].bytes),
             reports[next_report].reason.c_str());
  };
  for (size_t i = 0; i < recs.size(); ++i) {
    flush_reports(i);
    const leveldb::Slice rec(recs[i].data);
    if (descriptor) {
      leveldb::VersionEdit edit;
      leveldb::Status s = edit.DecodeFrom(rec);
      if (!s.ok()) fprintf(stderr, "%s\n", s.ToString().c_str());
    } else if (rec.size() < 12) {
      printf("log record length %d is too small\n", static_cast<int>(rec.size()));
    } else {
      leveldb::WriteBatch batch;
      leveldb::WriteBatchInternal::SetContents(&batch, rec);
      NullHandler h;
      leveldb::Status s = batch.Iterate(&h);
      if (!s.ok()) fprintf(stderr, "error: %s\n", s.ToString().c_str());
    }
  }
  flush_reports(UINT64_MAX);
  g_walk_s += Since(t0);
  return true;
}

bool VerifyTableFile(leveldb::Env* env, const std::string& fname) {
  std::string img;
  if (!ReadWhole(env, fname, &img)) return false;
  // Table::Open exactly as the reference tool: footer + index block, unchecked (ReadOptions())
  auto t0 = Clock::now();
  leveldb::RandomAccessFile* file = nullptr;
  leveldb::Table* table = nullptr;
  leveldb::Status s = env->NewRandomAccessFile(fname, &file);
  if (s.ok()) s = leveldb::Table::Open(leveldb::Options(), file, img.size(), &table, nullptr);
  if (!s.ok()) {
    fprintf(stderr, "%s\n", s.ToString().c_str());
    delete table;
    delete file;
    return false;
  }
  g_walk_s += Since(t0);
  // every data block the tool's verified iterator would read, checked in ONE GPU batch
  t0 = Clock::now();
  std::vector<pdb::BlockHandle> data;
  std::vector<uint8_t> ok;
  std::string err;
  int64_t bad = 1;  // an index the walk cannot parse: let the engine's own reads report it
  if (pdb::ReadDataHandles(img.data(), img.size(), &data, &err)) {
    bad = pdb::VerifyBlocks(img.data(), img.size(), data.data(), data.size(), &ok);
    if (bad < 0) {
      fprintf(stderr, "%s: device error %lld: %s\n", fname.c_str(), static_cast<long long>(bad), pdb_last_error());
      delete table;
      delete file;
      return false;
    }
    g_blocks += data.size();
  }
  g_crc_s += Since(t0);
  // The reference tool's walk (leveldb-verify.cc:142-168), statement for statement.  Clean table:
  // per-block checksums off, every one was just checked.  A damaged one: checksums on, so the
  // engine's own ReadBlock (pdb_format.cc: the check on the GPU) reports each bad block exactly
  // where the reference's iterator does -- skipped blocks, "bad iteration" per later key, the final
  // "iterator error".
  t0 = Clock::now();
  leveldb::ReadOptions ro;
  ro.verify_checksums = bad != 0;
  leveldb::Iterator* iter = table->NewIterator(ro);
  leveldb::Iterator* verify = table->NewIterator(ro);
  for (iter->SeekToFirst(); iter->Valid(); iter->Next()) {
    if (!iter->status().ok()) fprintf(stderr, "bad iteration %s\n", iter->status().ToString().c_str());
    leveldb::ParsedInternalKey key;
    if (!leveldb::ParseInternalKey(iter->key(), &key))
      fprintf(stderr, "badkey '%s' => '%s'\n", leveldb::EscapeString(iter->key()).c_str(),
              leveldb::EscapeString(iter->value()).c_str());
    verify->SeekToFirst();
    if (!verify->status().ok()) fprintf(stderr, "bad iteration %s\n", verify->status().ToString().c_str());
    verify->Seek(key.user_key);
    if (!verify->status().ok()) fprintf(stderr, "bad iteration %s\n", verify->status().ToString().c_str());
  }
  s = iter->status();
  if (!s.ok()) fprintf(stderr, "iterator error: %s\n", s.ToString().c_str());
  delete iter;
  delete verify;
  delete table;
  delete file;
  g_walk_s += Since(t0);
  return true;
}

bool VerifyFile(leveldb::Env* env, const std::string& fname) {
  const size_t slash = fname.rfind('/');
  const std::string base = slash == std::string::npos ? fname : fname.substr(slash + 1);
  uint64_t number;
  leveldb::FileType type;
  if (!leveldb::ParseFileName(base, &number, &type)) {
    fprintf(stderr, "%s: unknown file type\n", fname.c_str());
    return false;
  }
  if (type == leveldb::kLogFile) return VerifyLogFile(env, fname, false);
  if (type == leveldb::kDescriptorFile) return VerifyLogFile(env, fname, true);
  if (type == leveldb::kTableFile) return VerifyTableFile(env, fname);
  fprintf(stderr, "%s: not a dump-able file type\n", fname.c_str());
  return false;
}

}  // namespace

int main(int argc, char** argv) {
  leveldb::Env* env = leveldb::Env::Default();
  bool ok = true;
  const auto t0 = Clock::now();
  for (int i = 1; i < argc; ++i) {
    if (strcmp(argv[i], "--timing") == 0) {
      g_timing = true;
      continue;
    }
    ok &= VerifyFile(env, argv[i]);
  }
  if (g_timing)
    fprintf(stderr,
            "{\"tool\": \"pdb_verify\", \"files\": %d, \"bytes\": %llu, \"blocks\": %llu, \"records\": %llu, "
            "\"read_s\": %.4f, \"gpu_crc_s\": %.4f, \"walk_s\": %.4f, \"total_s\": %.4f}\n",
            argc - 1 - (g_timing ? 1 : 0), static_cast<unsigned long long>(g_bytes),
            static_cast<unsigned long long>(g_blocks), static_cast<unsigned long long>(g_records), g_read_s, g_crc_s,
            g_walk_s, Since(t0));
  return ok ? 0 : 1;
}
