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
