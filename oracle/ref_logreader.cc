// oracle/ref_logreader.cc -- TEST INFRASTRUCTURE ONLY.
//
// Reads a log image with the REFERENCE's own log::Reader (db/log_reader.cc, compiled in place
// from /root/reference by oracle/build_ref.sh; checksum = true, initial_offset 0) and prints what
// it delivers as one JSON line: every logical record (LastRecordOffset, length, FNV-1a-64 of the
// bytes) and every corruption report (bytes, reason).  tests/golden/gen_golden.py runs it on
// deliberately corrupted copies of the golden logs (tests/golden/log/corruptions.json), which pin
// the batched verifier's replay of log::Reader (log_reader.cc:59-263) in pebblesdb_amd/log.py and
// include/pebblesdb_amd/log_records.h.
//
// usage: ref_logreader <log_file>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "db/log_reader.h"
#include "pebblesdb/env.h"

namespace {

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

struct ListReporter : public leveldb::log::Reader::Reporter {
  std::vector<std::pair<size_t, std::string> > reports;
  void Corruption(size_t bytes, const leveldb::Status& s) { reports.push_back(std::make_pair(bytes, s.ToString())); }
};

uint64_t fnv1a64(const char* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) {
    h ^= static_cast<unsigned char>(p[i]);
    h *= 1099511628211ull;
  }
  return h;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s log_file\n", argv[0]);
    return 2;
  }
  std::string data;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  char buf[1 << 16];
  size_t got;
  while ((got = fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, got);
  fclose(f);
  MemSeqFile src(data);
  ListReporter rep;
  leveldb::log::Reader rd(&src, &rep, true, 0);
  leveldb::Slice rec;
  std::string scratch;
  printf("{\"records\":[");
  bool first = true;
  while (rd.ReadRecord(&rec, &scratch)) {
    printf("%s[%llu,%zu,\"%016llx\"]", first ? "" : ",", (unsigned long long)rd.LastRecordOffset(), rec.size(),
           (unsigned long long)fnv1a64(rec.data(), rec.size()));
    first = false;
  }
  printf("],\"reports\":[");
  for (size_t i = 0; i < rep.reports.size(); ++i)
    printf("%s[%zu,\"%s\"]", i ? "," : "", rep.reports[i].first, rep.reports[i].second.c_str());
  printf("]}\n");
  return 0;
}
