#!/usr/bin/env bash
# integration/build.sh -- BASELINE configs 1 and 5 end to end: the PebblesDB engine compiled from
# the reference's own sources IN PLACE under /root/reference (never copied, never modified, not
# its build system) with this repo's table hooks, plus the db_bench-equivalent harness.
# Outputs ONLY to integration/_build/ (git-ignored; travels to the GPU box):
#   pdb_dbbench_cpu        reference engine as shipped (table_builder.cc, format.cc, crc32c.cc)
#   pdb_dbbench_gpu_table  table/table_builder.cc + table/format.cc replaced by pdb_table_builder.cc
#                          + pdb_format.cc (batched GPU trailer seals, GPU ReadBlock verify); the
#                          WAL / MANIFEST keep the reference CRC (util/crc32c.cc); table/table.cc
#                          replaced by pdb_table.cc (scans with verify_checksums: ~1-MiB read-ahead
#                          windows checked in one pdb_sst_verify_host batch)
#   pdb_dbbench_gpu_table_noscan  as gpu_table over the reference's own table.cc (A/B: no read-ahead)
#   (gpu_table and gpu_all read the WAL / MANIFEST at recovery through integration/pdb_log_reader.cc:
#    one GPU verify batch per log file instead of db/log_reader.cc's CRC per record)
#   logreader_gpu          oracle/ref_logreader.cc's harness over pdb_log_reader.cc (corrupted-log parity)
#   pdb_dbbench_gpu_all    as gpu_table, and util/crc32c.h -> include/pebblesdb_amd/crc32c.h for every
#                          other call site (log_writer/log_reader records on the scalar GPU service)
#   pdb_dbbench_buffered_cpu  as gpu_table (buffered emission, read-ahead windows) with every CRC on
#                          the CPU (-DPDB_CPU_CRC=1, integration/pdb_crc_route.h): the attribution A/B
#   sstwriter_gpu          oracle/ref_sstwriter.cc over the GPU hooks (golden-table parity test)
#   leveldb_verify_ref     the reference's own src/leveldb-verify.cc over the engine as shipped
#   pdb_verify_gpu         integration/pdb_verify.cc: the same tool with every checksum of a file
#                          checked in one GPU batch (data blocks / pdb::log::ReplayLog), over the
#                          engine with pdb_format.cc (a damaged table's walk checks on the GPU too)
#   pdb_tablegen          integration/pdb_tablegen.cc: one real sstable (data, filter, metaindex, index
#                          blocks) from the reference TableBuilder as shipped (bench.py sst_tables)
#   table_scan_ref / _gpu  integration/pdb_table_scan.cc: one verified scan of a table through the
#                          reference's table reader / pdb_table.cc (parity of what a reader sees)
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(dirname "$HERE")"
REF="${PDB_REFERENCE_ROOT:-/root/reference}/src"
if [ ! -f "$REF/db/db_impl.cc" ]; then
  echo "integration/build.sh: reference not present at $REF; skipping (prebuilt binaries are used)" >&2
  exit 0
fi
LIB="$ROOT/pebblesdb_amd/_lib/libpdb_crc32c.so"
[ -f "$LIB" ] || { echo "integration/build.sh: $LIB missing (python -m pebblesdb_amd.build)" >&2; exit 1; }
B="$HERE/_build"
mkdir -p "$B/obj_ref" "$B/obj_shim" "$B/obj_hooks"
ENGINE="db/builder.cc db/db_impl.cc db/db_iter.cc db/dbformat.cc db/filename.cc db/log_reader.cc
        db/log_writer.cc db/memtable.cc db/murmurhash3.cc db/repair.cc db/replay_iterator.cc
        db/table_cache.cc db/version_edit.cc db/version_set.cc db/write_batch.cc db/c.cc
        table/block.cc table/block_builder.cc table/filter_block.cc table/iterator.cc
        table/merger.cc table/two_level_iterator.cc
        util/arena.cc util/atomic.cc util/bloom.cc util/cache.cc util/coding.cc util/comparator.cc
        util/env.cc util/env_posix.cc util/filter_policy.cc util/hash.cc util/histogram.cc
        util/logging.cc util/options.cc util/status.cc util/testutil.cc port/port_posix.cc"
TABLE_REF="table/table_builder.cc table/format.cc table/table.cc"
# the engine without db/log_reader.cc (the GPU builds link integration/pdb_log_reader.cc instead)
ENGINE_NOLOG="$(echo $ENGINE | tr ' ' '\n' | grep -v '^db/log_reader.cc$' | tr '\n' ' ')"
DEFS="-DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DHAVE_FFLUSH_UNLOCKED -DHAVE_FREAD_UNLOCKED"
DEFS="$DEFS -DHAVE_FWRITE_UNLOCKED -DHAVE_FDATASYNC -DHAVE_DECL_FDATASYNC=1 -DNDEBUG"
CXX="g++ -O2 -std=c++11 -w -pthread"
JOBS="${PDB_BUILD_JOBS:-8}"

compile() {  # $1 = obj dir, $2 = source list, $3.. = include flags (sources under $REF)
  local od="$1" srcs="$2"; shift 2
  for f in $srcs; do echo "$f"; done | xargs -P "$JOBS" -I{} sh -c \
    "o=\"$od/\$(echo {} | tr / _).o\"; [ \"\$o\" -nt \"$REF/{}\" ] || $CXX $DEFS $* -c \"$REF/{}\" -o \"\$o\""
}
objs() {  # object paths of a source list in an obj dir
  local od="$1" f; shift
  for f in $*; do printf '%s ' "$od/$(echo "$f" | tr / _).o"; done
}

# reference engine as shipped, and the same sources with util/crc32c.h bound to the GPU
compile "$B/obj_ref" "$ENGINE $TABLE_REF util/crc32c.cc leveldb-verify.cc" "-I$REF -I$REF/include"
compile "$B/obj_shim" "$ENGINE" "-I$ROOT/oracle/shim_pdb -I$ROOT/include -I$REF -I$REF/include"
# the hooks and the harness (our sources)
HOOKI="-I$ROOT/include -I$HERE -I$REF -I$REF/include"
mkdir -p "$B/obj_hooks_cpu"
for f in pdb_table_builder pdb_format pdb_table; do
  [ "$B/obj_hooks/$f.o" -nt "$HERE/$f.cc" ] && [ "$B/obj_hooks/$f.o" -nt "$HERE/pdb_hooks.h" ] &&
    [ "$B/obj_hooks/$f.o" -nt "$HERE/pdb_crc_route.h" ] || $CXX $DEFS $HOOKI -c "$HERE/$f.cc" -o "$B/obj_hooks/$f.o"
  # attribution A/B: the same hooks (buffered emission, read-ahead windows) with the CPU CRC
  [ "$B/obj_hooks_cpu/$f.o" -nt "$HERE/$f.cc" ] && [ "$B/obj_hooks_cpu/$f.o" -nt "$HERE/pdb_hooks.h" ] &&
    [ "$B/obj_hooks_cpu/$f.o" -nt "$HERE/pdb_crc_route.h" ] ||
    $CXX $DEFS $HOOKI -DPDB_CPU_CRC=1 -c "$HERE/$f.cc" -o "$B/obj_hooks_cpu/$f.o"
done
$CXX $DEFS $HOOKI -DPDB_HOOKS=0 -c "$HERE/pdb_dbbench.cc" -o "$B/obj_hooks/dbbench_cpu.o"
$CXX $DEFS $HOOKI -DPDB_HOOKS=1 -c "$HERE/pdb_dbbench.cc" -o "$B/obj_hooks/dbbench_hooks.o"
$CXX $DEFS $HOOKI -c "$ROOT/oracle/ref_sstwriter.cc" -o "$B/obj_hooks/sstwriter.o"
$CXX $DEFS $HOOKI -c "$HERE/pdb_verify.cc" -o "$B/obj_hooks/pdb_verify.o"
$CXX $DEFS $HOOKI -c "$HERE/pdb_tablegen.cc" -o "$B/obj_hooks/pdb_tablegen.o"
$CXX $DEFS $HOOKI -c "$HERE/pdb_log_reader.cc" -o "$B/obj_hooks/pdb_log_reader.o"
$CXX $DEFS $HOOKI -c "$ROOT/oracle/ref_logreader.cc" -o "$B/obj_hooks/logreader.o"
$CXX $DEFS $HOOKI -DPDB_HOOKS=0 -c "$HERE/pdb_table_scan.cc" -o "$B/obj_hooks/table_scan_ref.o"
$CXX $DEFS $HOOKI -DPDB_HOOKS=1 -c "$HERE/pdb_table_scan.cc" -o "$B/obj_hooks/table_scan_gpu.o"

RPATH="-Wl,-rpath,\$ORIGIN/../../pebblesdb_amd/_lib"
GPU="-L$ROOT/pebblesdb_amd/_lib -lpdb_crc32c $RPATH"
HOOKS="$B/obj_hooks/pdb_table_builder.o $B/obj_hooks/pdb_format.o $B/obj_hooks/pdb_table.o"
# (A/B: the same hooks over the reference's own table reader, i.e. without the scan read-ahead)
HOOKS_NOSCAN="$B/obj_hooks/pdb_table_builder.o $B/obj_hooks/pdb_format.o $B/obj_ref/table_table.cc.o"
$CXX -o "$B/pdb_dbbench_cpu" "$B/obj_hooks/dbbench_cpu.o" $(objs "$B/obj_ref" $ENGINE $TABLE_REF util/crc32c.cc)
# (the WAL / MANIFEST readers of recovery: one GPU batch per log file, integration/pdb_log_reader.cc)
LOGRD="$B/obj_hooks/pdb_log_reader.o"
$CXX -o "$B/pdb_dbbench_gpu_table" "$B/obj_hooks/dbbench_hooks.o" $HOOKS $LOGRD \
  $(objs "$B/obj_ref" $ENGINE_NOLOG util/crc32c.cc) $GPU
$CXX -o "$B/pdb_dbbench_gpu_table_noscan" "$B/obj_hooks/dbbench_hooks.o" $HOOKS_NOSCAN \
  $(objs "$B/obj_ref" $ENGINE util/crc32c.cc) $GPU
$CXX -o "$B/pdb_dbbench_gpu_all" "$B/obj_hooks/dbbench_hooks.o" $HOOKS $LOGRD $(objs "$B/obj_shim" $ENGINE_NOLOG) $GPU
# the engine's log::Reader (pdb_log_reader.cc) under the reference reader's harness: the corrupted-log
# fixtures through the engine path (tests/test_log.py)
$CXX -o "$B/logreader_gpu" "$B/obj_hooks/logreader.o" $LOGRD $(objs "$B/obj_ref" $ENGINE_NOLOG $TABLE_REF util/crc32c.cc) $GPU
# attribution A/B: buffered emission + read-ahead windows, every CRC on the CPU
# (the reference's crc32c.cc); no GPU library linked
HOOKS_CPU="$B/obj_hooks_cpu/pdb_table_builder.o $B/obj_hooks_cpu/pdb_format.o $B/obj_hooks_cpu/pdb_table.o"
$CXX -o "$B/pdb_dbbench_buffered_cpu" "$B/obj_hooks/dbbench_hooks.o" $HOOKS_CPU $(objs "$B/obj_ref" $ENGINE util/crc32c.cc)
$CXX -o "$B/sstwriter_gpu" "$B/obj_hooks/sstwriter.o" $HOOKS $(objs "$B/obj_ref" $ENGINE util/crc32c.cc) $GPU
$CXX -o "$B/leveldb_verify_ref" $(objs "$B/obj_ref" leveldb-verify.cc $ENGINE $TABLE_REF util/crc32c.cc)
$CXX -o "$B/pdb_verify_gpu" "$B/obj_hooks/pdb_verify.o" "$B/obj_hooks/pdb_format.o" \
  $(objs "$B/obj_ref" $ENGINE table/table_builder.cc table/table.cc util/crc32c.cc) $GPU
# real tables for bench.py --workload sst_tables: the reference TableBuilder as shipped (CPU CRC)
$CXX -o "$B/pdb_tablegen" "$B/obj_hooks/pdb_tablegen.o" $(objs "$B/obj_ref" $ENGINE $TABLE_REF util/crc32c.cc)
$CXX -o "$B/table_scan_ref" "$B/obj_hooks/table_scan_ref.o" $(objs "$B/obj_ref" $ENGINE $TABLE_REF util/crc32c.cc)
$CXX -o "$B/table_scan_gpu" "$B/obj_hooks/table_scan_gpu.o" $HOOKS $(objs "$B/obj_ref" $ENGINE util/crc32c.cc) $GPU
echo "built $B/{logreader_gpu,pdb_tablegen,table_scan_ref,table_scan_gpu,pdb_dbbench_cpu,pdb_dbbench_gpu_table,pdb_dbbench_gpu_table_noscan,pdb_dbbench_gpu_all,pdb_dbbench_buffered_cpu,sstwriter_gpu,leveldb_verify_ref,pdb_verify_gpu}"
