// integration/pdb_table_scan.cc -- scan one sstable with ReadOptions::verify_checksums through the
// engine's table reader and print what a reader sees: entries returned, a hash of every key and
// value, and the iterator's final status.  Built twice by integration/build.sh: table_scan_ref over
// the reference's own table.cc + format.cc (CPU checks), table_scan_gpu over pdb_table.cc +
// pdb_format.cc (scan read-ahead windows checked on the GPU).  tests/test_integration.py runs both on
// clean and damaged tables: the outputs must be identical.
//   usage: table_scan <file.sst> [reps]
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "pebblesdb/env.h"
#include "pebblesdb/iterator.h"
#include "pebblesdb/options.h"
#include "pebblesdb/table.h"
#if PDB_HOOKS
#include "pdb_hooks.h"
#endif

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s file.sst [reps]\n", argv[0]);
    return 2;
  }
  const std::string path = argv[1];
  const int reps = argc > 2 ? atoi(argv[2]) : 1;
  leveldb::Env* env = leveldb::Env::Default();
  uint64_t size = 0;
  leveldb::RandomAccessFile* file = nullptr;
  leveldb::Status s = env->GetFileSize(path, &size);
  if (s.ok()) s = env->NewRandomAccessFile(path, &file);
  leveldb::Table* table = nullptr;
  if (s.ok()) s = leveldb::Table::Open(leveldb::Options(), file, size, &table, nullptr);
  if (!s.ok()) {
    printf("{\"open\": \"%s\"}\n", s.ToString().c_str());
    delete file;
    return 1;
  }
  leveldb::ReadOptions ro;
  ro.verify_checksums = true;
  long n = 0;
  uint64_t h = 1469598103934665603ull;  // FNV-1a over key, value, key, value, ...
  std::string status;
  for (int r = 0; r < reps; ++r) {
    leveldb::Iterator* it = table->NewIterator(ro);
    n = 0;
    h = 1469598103934665603ull;
    for (it->SeekToFirst(); it->Valid(); it->Next()) {
      ++n;
      for (const leveldb::Slice& x : {it->key(), it->value()}) {
        for (size_t i = 0; i < x.size(); ++i) h = (h ^ static_cast<uint8_t>(x[i])) * 1099511628211ull;
        h = (h ^ 0xFF) * 1099511628211ull;
      }
    }
    status = it->status().ToString();
    delete it;
  }
  printf("{\"entries\": %ld, \"hash\": \"%016llx\", \"status\": \"%s\"", n, static_cast<unsigned long long>(h),
         status.c_str());
#if PDB_HOOKS
  pdb_hook_stats st;
  pdb_hook_stats_get(&st);
  printf(", \"scan_batches\": %llu, \"scan_blocks\": %llu, \"verify_calls\": %llu",
         static_cast<unsigned long long>(st.scan_batches), static_cast<unsigned long long>(st.scan_blocks),
         static_cast<unsigned long long>(st.verify_calls));
#endif
  printf("}\n");
  delete table;
  delete file;
  return 0;
}
