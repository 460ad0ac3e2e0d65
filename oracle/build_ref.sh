#!/usr/bin/env bash
# oracle/build_ref.sh -- TEST INFRASTRUCTURE ONLY.
# Compiles the reference's own util/crc32c.cc (in place under /root/reference,
# never copied) plus oracle/ref_shim.cc into oracle/_ref/libpdbref.so.
# The -D flags are what the reference's port/port_posix.h needs on Linux
# (SURVEY.md §8(c) "Standalone" recipe).  Output goes ONLY to oracle/_ref/.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF="${PDB_REFERENCE_ROOT:-/root/reference}/src"
if [ ! -f "$REF/util/crc32c.cc" ]; then
  echo "build_ref.sh: reference not present at $REF; skipping oracle/_ref" >&2
  exit 0
fi
mkdir -p "$HERE/_ref"
g++ -O3 -std=c++11 -fPIC -shared \
  -DLEVELDB_PLATFORM_POSIX -DHAVE_FFLUSH_UNLOCKED -DHAVE_FREAD_UNLOCKED \
  -DHAVE_FWRITE_UNLOCKED -DHAVE_FDATASYNC -DHAVE_DECL_FDATASYNC=1 \
  -I"$REF" -I"$REF/include" \
  -o "$HERE/_ref/libpdbref.so" "$HERE/ref_shim.cc" "$REF/util/crc32c.cc" -lpthread
echo "built $HERE/_ref/libpdbref.so"

# The reference's own sstable writer/reader (table/*, util/*, port/*) + oracle/ref_sstwriter.cc
# -> oracle/_ref/ref_sstwriter, used only to generate tests/golden/sst fixtures.
SRCS="table/table_builder.cc table/block_builder.cc table/filter_block.cc table/format.cc
      table/block.cc table/table.cc table/iterator.cc table/two_level_iterator.cc
      util/coding.cc util/crc32c.cc util/comparator.cc util/options.cc util/env.cc
      util/env_posix.cc util/status.cc util/logging.cc util/hash.cc util/bloom.cc
      util/filter_policy.cc util/arena.cc util/atomic.cc util/cache.cc port/port_posix.cc"
ABS=""
for f in $SRCS; do ABS="$ABS $REF/$f"; done
g++ -O2 -std=c++11 -w \
  -DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DHAVE_FFLUSH_UNLOCKED -DHAVE_FREAD_UNLOCKED \
  -DHAVE_FWRITE_UNLOCKED -DHAVE_FDATASYNC -DHAVE_DECL_FDATASYNC=1 \
  -I"$REF" -I"$REF/include" -o "$HERE/_ref/ref_sstwriter" "$HERE/ref_sstwriter.cc" $ABS -lpthread
echo "built $HERE/_ref/ref_sstwriter"

# The reference's own WAL/MANIFEST log writer/reader + oracle/ref_logwriter.cc
# -> oracle/_ref/ref_logwriter, used only to generate tests/golden/log fixtures.
LSRCS="db/log_writer.cc db/log_reader.cc util/coding.cc util/crc32c.cc util/env.cc util/env_posix.cc
       util/status.cc util/logging.cc util/atomic.cc port/port_posix.cc"
LABS=""
for f in $LSRCS; do LABS="$LABS $REF/$f"; done
g++ -O2 -std=c++11 -w \
  -DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DHAVE_FFLUSH_UNLOCKED -DHAVE_FREAD_UNLOCKED \
  -DHAVE_FWRITE_UNLOCKED -DHAVE_FDATASYNC -DHAVE_DECL_FDATASYNC=1 \
  -I"$REF" -I"$REF/include" -o "$HERE/_ref/ref_logwriter" "$HERE/ref_logwriter.cc" $LABS -lpthread
echo "built $HERE/_ref/ref_logwriter"

# The reference's own log::Reader on an arbitrary (corrupted) log image + oracle/ref_logreader.cc
# -> oracle/_ref/ref_logreader, used only to generate tests/golden/log/corruptions.json.
g++ -O2 -std=c++11 -w \
  -DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DHAVE_FFLUSH_UNLOCKED -DHAVE_FREAD_UNLOCKED \
  -DHAVE_FWRITE_UNLOCKED -DHAVE_FDATASYNC -DHAVE_DECL_FDATASYNC=1 \
  -I"$REF" -I"$REF/include" -o "$HERE/_ref/ref_logreader" "$HERE/ref_logreader.cc" $LABS -lpthread
echo "built $HERE/_ref/ref_logreader"
