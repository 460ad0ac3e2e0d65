// oracle/ref_logwriter.cc -- TEST INFRASTRUCTURE ONLY.
//
// Writes a WAL/MANIFEST-format log with the REFERENCE's own log::Writer (db/log_writer.cc,
// compiled in place from /root/reference by oracle/build_ref.sh), reads it back with the
// reference's log::Reader (checksum = true: log_reader.cc:235-249), and prints a JSON line.
// tests/golden/gen_golden.py uses it to produce tests/golden/log/*.log, which pin the batched
// log verifier / group-commit writer (pebblesdb_amd/log.py).
//
// usage: ref_logwriter <out_file> <seed> <len0> <len1> ...   (one logical record per length)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "db/log_reader.h"
#include "db/log_writer.h"
#include "pebblesdb/env.h"

namespace {

class MemConcurrentFile : public leveldb::ConcurrentWritableFile {
 public:
  std::string data;
  leveldb::Status WriteAt(uint64_t off, const leveldb::Slice& s) {
    if (data.size() < off + s.size()) data.resize(off + s.size(), '\0');
    memcpy(&data[off], s.data(), s.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Append(const leveldb::Slice& s) { return WriteAt(data.size(), s); }
  leveldb::Status Close() { return leveldb::Status::OK(); }
  leveldb::Status Flush() { return leveldb::Status::OK(); }
  leveldb::Status Sync() { return leveldb::Status::OK(); }
};

class MemSeqFile : public leveldb::SequentialFile {
 public:
  explicit MemSeqFile(const std::string& d) : d_(d), pos_(0) {}
  leveldb::Status Read(size_t n, leveldb::Slice* r, char* scratch) {
    if (pos_ + n > d_.size()) n = d_.size() - pos_;
    memcpy(scratch, d_.data() + pos_, n);
    *r = leveldb::Slice(scratch, n);
    pos_ += n;
    return leveldb::Status::OK();
  }
  leveldb::Status Skip(uint64_t n) {
    pos_ = pos_ + n > d_.size() ? d_.size() : pos_ + n;
    return leveldb::Status::OK();
  }

 private:
  const std::string& d_;
  size_t pos_;
};

struct CountingReporter : public leveldb::log::Reader::Reporter {
  size_t dropped = 0;
  void Corruption(size_t bytes, const leveldb::Status&) { dropped += bytes; }
};

uint64_t splitmix(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s out_file seed len...\n", argv[0]);
    return 2;
  }
  const uint64_t seed = strtoull(argv[2], 0, 10);
  std::vector<std::string> recs;
  for (int a = 3; a < argc; ++a) {
    const long n = atol(argv[a]);
    std::string r(n, '\0');
    for (long j = 0; j < n; ++j) r[j] = static_cast<char>(splitmix(seed + a, j / 8) >> (8 * (j % 8)));
    recs.push_back(r);
  }
  MemConcurrentFile f;
  {
    leveldb::log::Writer w(&f);
    for (const std::string& r : recs) {
      leveldb::Status s = w.AddRecord(leveldb::Slice(r));
      if (!s.ok()) return 1;
    }
  }
  FILE* out = fopen(argv[1], "wb");
  if (!out || fwrite(f.data.data(), 1, f.data.size(), out) != f.data.size()) return 1;
  fclose(out);
  // read back with checksums on
  MemSeqFile src(f.data);
  CountingReporter rep;
  leveldb::log::Reader rd(&src, &rep, true, 0);
  leveldb::Slice rec;
  std::string scratch;
  size_t n = 0;
  bool same = true;
  while (rd.ReadRecord(&rec, &scratch)) {
    if (n >= recs.size() || rec.ToString() != recs[n]) same = false;
    ++n;
  }
  const bool ok = same && n == recs.size() && rep.dropped == 0;
  printf("{\"bytes\":%zu,\"records\":%zu,\"reference_verify_ok\":%s}\n", f.data.size(), n,
         ok ? "true" : "false");
  return ok ? 0 : 1;
}
