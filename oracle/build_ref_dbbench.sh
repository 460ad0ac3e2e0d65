#!/usr/bin/env bash
# oracle/build_ref_dbbench.sh -- TEST/DEMO INFRASTRUCTURE ONLY (BASELINE configs 1 and 5).
# Compiles the reference's own db_bench from its sources IN PLACE under /root/reference (never
# copied, never modified, not its build system) twice, outputs ONLY to oracle/_ref/:
#   db_bench_ref  -- as shipped, util/crc32c.cc linked in (config 1: the CPU baseline)
#   db_bench_pdb  -- same sources minus util/crc32c.cc, with oracle/shim_pdb ahead on the include
#                    path so `#include "util/crc32c.h"` resolves to include/pebblesdb_amd/crc32c.h,
#                    linked against pebblesdb_amd/_lib/libpdb_crc32c.so (config 5's hook: every
#                    Extend/Value call site runs on the MI355X, no call site edited).
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(dirname "$HERE")"
REF="${PDB_REFERENCE_ROOT:-/root/reference}/src"
if [ ! -f "$REF/db/db_bench.cc" ]; then
  echo "build_ref_dbbench.sh: reference not present at $REF; skipping" >&2
  exit 0
fi
mkdir -p "$HERE/_ref/obj_ref" "$HERE/_ref/obj_pdb"
CORE="db/builder.cc db/db_impl.cc db/db_iter.cc db/dbformat.cc db/filename.cc db/log_reader.cc
      db/log_writer.cc db/memtable.cc db/murmurhash3.cc db/repair.cc db/replay_iterator.cc
      db/table_cache.cc db/version_edit.cc db/version_set.cc db/write_batch.cc db/c.cc
      table/block.cc table/block_builder.cc table/filter_block.cc table/format.cc table/iterator.cc
      table/merger.cc table/table.cc table/table_builder.cc table/two_level_iterator.cc
      util/arena.cc util/atomic.cc util/bloom.cc util/cache.cc util/coding.cc util/comparator.cc
      util/env.cc util/env_posix.cc util/filter_policy.cc util/hash.cc util/histogram.cc
      util/logging.cc util/options.cc util/status.cc util/testharness.cc util/testutil.cc
      port/port_posix.cc db/db_bench.cc"
DEFS="-DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DHAVE_FFLUSH_UNLOCKED -DHAVE_FREAD_UNLOCKED"
DEFS="$DEFS -DHAVE_FWRITE_UNLOCKED -DHAVE_FDATASYNC -DHAVE_DECL_FDATASYNC=1 -DNDEBUG"
CXX="g++ -O2 -std=c++11 -w -pthread"
JOBS="${PDB_BUILD_JOBS:-8}"

compile() {  # $1 = obj dir, $2.. = extra flags; objects compiled in parallel
  local od="$1"; shift
  local f
  for f in $CORE; do
    echo "$f"
  done | xargs -P "$JOBS" -I{} sh -c \
    "o=\"$od/\$(echo {} | tr / _).o\"; [ \"\$o\" -nt \"$REF/{}\" ] || $CXX $DEFS $* -c \"$REF/{}\" -o \"\$o\""
}

# config 1: the reference as shipped
compile "$HERE/_ref/obj_ref" "-I$REF -I$REF/include"
$CXX -c "$REF/util/crc32c.cc" $DEFS -I"$REF" -I"$REF/include" -o "$HERE/_ref/obj_ref/util_crc32c.cc.o"
$CXX -o "$HERE/_ref/db_bench_ref" "$HERE"/_ref/obj_ref/*.o
echo "built $HERE/_ref/db_bench_ref"

# config 5: util/crc32c.h -> pebblesdb_amd/crc32c.h (GPU), util/crc32c.cc left out
LIB="$ROOT/pebblesdb_amd/_lib/libpdb_crc32c.so"
if [ ! -f "$LIB" ]; then
  echo "build_ref_dbbench.sh: $LIB missing (python -m pebblesdb_amd.build); skipping db_bench_pdb" >&2
  exit 0
fi
compile "$HERE/_ref/obj_pdb" "-I$HERE/shim_pdb -I$ROOT/include -I$REF -I$REF/include"
$CXX -o "$HERE/_ref/db_bench_pdb" "$HERE"/_ref/obj_pdb/*.o -L"$ROOT/pebblesdb_amd/_lib" -lpdb_crc32c \
  -Wl,-rpath,'$ORIGIN/../../pebblesdb_amd/_lib'
echo "built $HERE/_ref/db_bench_pdb"
