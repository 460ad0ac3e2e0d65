#!/usr/bin/env bash
# integration/build_sanitize.sh <thread|address|debug> -- the two CPU-only engine harnesses of
# integration/build.sh (pdb_dbbench_cpu: the engine as shipped; pdb_dbbench_buffered_cpu: this repo's
# table hooks with the reference CRC, no GPU library) compiled with a sanitizer, frame pointers and no
# sibling-call optimisation, so a fault's stack names every caller (the teardown
# abort); `debug`: the same flags with no sanitizer (to run under gdb at full speed).  Sources compiled IN PLACE from /root/reference (never copied or modified); outputs only
# under integration/_build_san_<kind>/ (git-ignored, CPU diagnostics: never run on the GPU box).
set -euo pipefail
KIND="${1:-thread}"
case "$KIND" in thread|address|debug) ;; *) echo "usage: $0 thread|address|debug" >&2; exit 2 ;; esac
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(dirname "$HERE")"
REF="${PDB_REFERENCE_ROOT:-/root/reference}/src"
[ -f "$REF/db/db_impl.cc" ] || { echo "reference not present at $REF" >&2; exit 1; }
B="$HERE/_build_san_$KIND"
mkdir -p "$B/obj_ref" "$B/obj_hooks"
ENGINE="db/builder.cc db/db_impl.cc db/db_iter.cc db/dbformat.cc db/filename.cc db/log_reader.cc
        db/log_writer.cc db/memtable.cc db/murmurhash3.cc db/repair.cc db/replay_iterator.cc
        db/table_cache.cc db/version_edit.cc db/version_set.cc db/write_batch.cc db/c.cc
        table/block.cc table/block_builder.cc table/filter_block.cc table/iterator.cc
        table/merger.cc table/two_level_iterator.cc
        util/arena.cc util/atomic.cc util/bloom.cc util/cache.cc util/coding.cc util/comparator.cc
        util/env.cc util/env_posix.cc util/filter_policy.cc util/hash.cc util/histogram.cc
        util/logging.cc util/options.cc util/status.cc util/testutil.cc port/port_posix.cc"
TABLE_REF="table/table_builder.cc table/format.cc table/table.cc"
DEFS="-DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DHAVE_FFLUSH_UNLOCKED -DHAVE_FREAD_UNLOCKED"
DEFS="$DEFS -DHAVE_FWRITE_UNLOCKED -DHAVE_FDATASYNC -DHAVE_DECL_FDATASYNC=1 -DNDEBUG"
SAN="-fno-omit-frame-pointer -fno-optimize-sibling-calls -g"
[ "$KIND" = debug ] || SAN="-fsanitize=$KIND $SAN"
CXX="g++ -O1 -std=c++11 -w -pthread $SAN"
JOBS="${PDB_BUILD_JOBS:-8}"
for f in $ENGINE $TABLE_REF util/crc32c.cc; do echo "$f"; done | xargs -P "$JOBS" -I{} sh -c \
  "o=\"$B/obj_ref/\$(echo {} | tr / _).o\"; [ \"\$o\" -nt \"$REF/{}\" ] || $CXX $DEFS -I$REF -I$REF/include -c \"$REF/{}\" -o \"\$o\""
HOOKI="-I$ROOT/include -I$HERE -I$REF -I$REF/include"
for f in pdb_table_builder pdb_format pdb_table; do
  $CXX $DEFS $HOOKI -DPDB_CPU_CRC=1 -c "$HERE/$f.cc" -o "$B/obj_hooks/$f.o"
done
$CXX $DEFS $HOOKI -DPDB_HOOKS=0 -c "$HERE/pdb_dbbench.cc" -o "$B/obj_hooks/dbbench_cpu.o"
$CXX $DEFS $HOOKI -DPDB_HOOKS=1 -DPDB_CPU_CRC=1 -c "$HERE/pdb_dbbench.cc" -o "$B/obj_hooks/dbbench_hooks.o"
objs() { local od="$1" f; shift; for f in $*; do printf '%s ' "$od/$(echo "$f" | tr / _).o"; done; }
$CXX -o "$B/pdb_dbbench_cpu" "$B/obj_hooks/dbbench_cpu.o" $(objs "$B/obj_ref" $ENGINE $TABLE_REF util/crc32c.cc)
$CXX -o "$B/pdb_dbbench_buffered_cpu" "$B/obj_hooks/dbbench_hooks.o" "$B/obj_hooks/pdb_table_builder.o" \
  "$B/obj_hooks/pdb_format.o" "$B/obj_hooks/pdb_table.o" $(objs "$B/obj_ref" $ENGINE util/crc32c.cc)
echo "built $B/{pdb_dbbench_cpu,pdb_dbbench_buffered_cpu} ($SAN)"
