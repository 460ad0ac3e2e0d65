// integration/pdb_tablegen.cc -- write one real sstable with the REFERENCE engine's own TableBuilder
// (table/table_builder.cc, compiled in place by integration/build.sh and linked as shipped: its
// trailers are the reference's CPU CRC32C), for bench.py --workload sst_tables.  The table holds
// `nkeys` keys "key%016ld" with `value_size`-byte pseudo-random values, kNoCompression, a bloom filter
// of `bloom_bits` bits per key, `block_size`-byte data blocks: data blocks of ~4.1 KiB followed by
// the filter, metaindex and index blocks TableBuilder::Finish writes (table_builder.cc:211-266) --
// at 1 M keys of 1 KiB values, a ~7 MiB index block and a ~3 MiB filter block.
//   usage: pdb_tablegen <out.sst> <nkeys> <value_size> <seed> [block_size=4096] [bloom_bits=10]
// Prints one JSON line: the file's bytes and entries.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "pebblesdb/env.h"
#include "pebblesdb/filter_policy.h"
#include "pebblesdb/options.h"
#include "pebblesdb/table_builder.h"

namespace {

uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s out.sst nkeys value_size seed [block_size] [bloom_bits]\n", argv[0]);
    return 2;
  }
  const std::string path = argv[1];
  const long nkeys = atol(argv[2]), vsize = atol(argv[3]);
  const uint64_t seed = strtoull(argv[4], nullptr, 10);
  const int block_size = argc > 5 ? atoi(argv[5]) : 4096, bloom = argc > 6 ? atoi(argv[6]) : 10;
  leveldb::Options opt;
  opt.block_size = block_size;
  opt.compression = leveldb::kNoCompression;
  const leveldb::FilterPolicy* fp = bloom > 0 ? leveldb::NewBloomFilterPolicy(bloom) : nullptr;
  opt.filter_policy = fp;
  leveldb::WritableFile* file = nullptr;
  leveldb::Status s = leveldb::Env::Default()->NewWritableFile(path, &file);
  if (!s.ok()) {
    fprintf(stderr, "%s\n", s.ToString().c_str());
    return 1;
  }
  leveldb::TableBuilder* tb = new leveldb::TableBuilder(opt, file);
  char key[32];
  std::string val(static_cast<size_t>(vsize), '\0');
  for (long i = 0; i < nkeys; ++i) {
    snprintf(key, sizeof(key), "key%016ld", i);
    for (long j = 0; j < vsize; j += 8) {
      const uint64_t w = mix64(seed + 0x9E3779B97F4A7C15ull * static_cast<uint64_t>(i * 4096 + j / 8 + 1));
      for (long b = 0; b < 8 && j + b < vsize; ++b) val[j + b] = static_cast<char>(w >> (8 * b));
    }
    tb->Add(leveldb::Slice(key), leveldb::Slice(val));
  }
  s = tb->Finish();
  const uint64_t bytes = tb->FileSize();
  delete tb;
  if (s.ok()) s = file->Sync();
  if (s.ok()) s = file->Close();
  delete file;
  delete fp;
  if (!s.ok()) {
    fprintf(stderr, "%s\n", s.ToString().c_str());
    return 1;
  }
  printf("{\"file\": \"%s\", \"bytes\": %llu, \"entries\": %ld, \"block_size\": %d, \"bloom_bits\": %d}\n",
         path.c_str(), static_cast<unsigned long long>(bytes), nkeys, block_size, bloom);
  return 0;
}
