// oracle/ref_sstwriter.cc -- TEST INFRASTRUCTURE ONLY.
//
// Writes small sstables with the REFERENCE's own TableBuilder (table/table_builder.cc, compiled
// in place from /root/reference by oracle/build_ref.sh; nothing copied), re-opens each with the
// reference's Table::Open + an iterator with ReadOptions::verify_checksums = true (every block
// through ReadBlock's checksum check, table/format.cc:96-104), and prints one JSON line per
// table.  tests/golden/gen_golden.py runs it to produce tests/golden/sst/*.sst -- the fixtures
// that pin the batched sstable walker + verify path (pebblesdb_amd/table.py).
//
// usage: ref_sstwriter <out_dir> <name> <nkeys> <value_size> <seed> <block_size> <bloom_bits>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "pebblesdb/env.h"
#include "pebblesdb/filter_policy.h"
#include "pebblesdb/iterator.h"
#include "pebblesdb/options.h"
#include "pebblesdb/table.h"
#include "pebblesdb/table_builder.h"

namespace {

class MemSink : public leveldb::WritableFile {
 public:
  std::string data;
  leveldb::Status Append(const leveldb::Slice& s) {
    data.append(s.data(), s.size());
    return leveldb::Status::OK();
  }
  leveldb::Status Close() { return leveldb::Status::OK(); }
  leveldb::Status Flush() { return leveldb::Status::OK(); }
  leveldb::Status Sync() { return leveldb::Status::OK(); }
};

class MemSource : public leveldb::RandomAccessFile {
 public:
  explicit MemSource(const std::string& d) : data_(d) {}
  leveldb::Status Read(uint64_t off, size_t n, leveldb::Slice* r, char*) const {
    if (off > data_.size()) return leveldb::Status::InvalidArgument("offset past end");
    if (off + n > data_.size()) n = data_.size() - off;
    *r = leveldb::Slice(data_.data() + off, n);
    return leveldb::Status::OK();
  }

 private:
  const std::string& data_;
};

uint64_t splitmix(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 8) {
    fprintf(stderr, "usage: %s out_dir name nkeys value_size seed block_size bloom_bits\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1], name = argv[2];
  const long nkeys = atol(argv[3]), vsize = atol(argv[4]);
  const uint64_t seed = strtoull(argv[5], 0, 10);
  const int block_size = atoi(argv[6]), bloom = atoi(argv[7]);

  leveldb::Options opt;
  opt.block_size = block_size;
  opt.compression = leveldb::kNoCompression;
  const leveldb::FilterPolicy* fp = bloom > 0 ? leveldb::NewBloomFilterPolicy(bloom) : NULL;
  opt.filter_policy = fp;

  MemSink sink;
  leveldb::TableBuilder tb(opt, &sink);
  char key[32];
  std::string val;
  for (long i = 0; i < nkeys; ++i) {
    snprintf(key, sizeof(key), "key%016ld", i);
    val.resize(vsize);
    for (long j = 0; j < vsize; ++j) val[j] = static_cast<char>(splitmix(seed, i * 131 + j / 8) >> (8 * (j % 8)));
    tb.Add(leveldb::Slice(key), leveldb::Slice(val));
  }
  leveldb::Status s = tb.Finish();
  if (!s.ok()) {
    fprintf(stderr, "Finish: %s\n", s.ToString().c_str());
    return 1;
  }
  const std::string path = dir + "/" + name + ".sst";
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || fwrite(sink.data.data(), 1, sink.data.size(), f) != sink.data.size()) return 1;
  fclose(f);

  // Read it back through the reference reader with checksum verification on.
  MemSource src(sink.data);
  leveldb::Table* t = NULL;
  s = leveldb::Table::Open(opt, &src, sink.data.size(), &t, NULL);
  if (!s.ok()) {
    fprintf(stderr, "Open: %s\n", s.ToString().c_str());
    return 1;
  }
  leveldb::ReadOptions ro;
  ro.verify_checksums = true;
  leveldb::Iterator* it = t->NewIterator(ro);
  long n = 0;
  for (it->SeekToFirst(); it->Valid(); it->Next()) ++n;
  const bool ok = it->status().ok() && n == nkeys;
  printf("{\"name\":\"%s\",\"file\":\"%s.sst\",\"bytes\":%zu,\"entries\":%ld,\"block_size\":%d,"
         "\"bloom_bits\":%d,\"reference_verify_ok\":%s}\n",
         name.c_str(), name.c_str(), sink.data.size(), n, block_size, bloom, ok ? "true" : "false");
  delete it;
  delete t;
  delete fp;
  return ok ? 0 : 1;
}
