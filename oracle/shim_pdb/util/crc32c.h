// oracle/shim_pdb/util/crc32c.h -- include-path shim, TEST/DEMO INFRASTRUCTURE ONLY.
// Placed ahead of the reference's src/ on the include path by oracle/build_ref_dbbench.sh, so that
// every `#include "util/crc32c.h"` in the UNMODIFIED reference sources (table/format.cc:11,
// table/table_builder.cc:16, db/log_writer.cc:10, db/log_reader.cc:10, db/db_bench.cc:27) binds
// leveldb::crc32c to libpdb_crc32c.so instead of util/crc32c.cc (which that build leaves out).
#include "pebblesdb_amd/crc32c.h"
