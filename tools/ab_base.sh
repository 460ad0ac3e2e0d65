#!/usr/bin/env bash
# tools/ab_base.sh <git-rev | WORKTREE> <name> -- build the diagnostics library of an earlier revision's
# sources (or of the working tree as it is now)
# as pebblesdb_amd/_lib/ab/libpdb_crc32c_diag_<name>.so, for in-process A/B against the working tree
# (tools/ab_span.py variant tokens "<name>/<id>").  Run here, on the CPU, before the GPU call.
set -euo pipefail
rev=$1 name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
if [ "$rev" = WORKTREE ]; then
  mkdir -p "$tmp/pebblesdb_amd" && cp -r "$root/pebblesdb_amd/csrc" "$tmp/pebblesdb_amd/" && cp -r "$root/include" "$tmp/"
else
  git -C "$root" archive "$rev" pebblesdb_amd/csrc include | tar -x -C "$tmp"
fi
mkdir -p "$root/pebblesdb_amd/_lib/ab"
objs=() pids=()
for s in diag_variants.hip diag_capi.cpp crc32c_kernels.hip crc32c_tables.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -I"$tmp/include" \
    -c "$tmp/pebblesdb_amd/csrc/$s" -o "$tmp/$s.o" &
  pids+=($!) objs+=("$tmp/$s.o")
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--version-script="$tmp/pebblesdb_amd/csrc/pdb_exports.map" \
  -o "$root/pebblesdb_amd/_lib/ab/libpdb_crc32c_diag_$name.so" "${objs[@]}"
echo "built pebblesdb_amd/_lib/ab/libpdb_crc32c_diag_$name.so from $rev"
