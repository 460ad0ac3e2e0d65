#!/usr/bin/env bash
# tools/long_lane_trace.sh <tag> [lib ...] -- the device route of tools/long_block_cost.py under rocprofv3
# --kernel-trace: every dispatch's duration, so the long-block lane's cost splits into the batch kernel,
# the piece kernel, the combine kernel and the gaps between them (tools/long_lane_split.py).  With
# library names, once per ab/<lib>.so (the in-tree library restored after).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="gpurun_out/$1"
mkdir -p "$OUT"
one() {  # one <label>
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/trace_$1" -- python3 tools/long_block_cost.py --device-only \
    > "$OUT/run_$1.log" 2>&1 || { echo "rc=$? ($1)"; tail -5 "$OUT/run_$1.log"; return 1; }
  python3 tools/long_lane_split.py "$OUT/trace_$1" > "$OUT/split_$1.json" && echo "== $1" && cat "$OUT/split_$1.json"
}
if [ $# -le 1 ]; then one cur; exit $?; fi
shift
cp pebblesdb_amd/_lib/libpdb_crc32c.so "$OUT/orig.so"
rc=0
for lib in "$@"; do
  cp "ab/$lib.so" pebblesdb_amd/_lib/libpdb_crc32c.so
  one "$lib" || { rc=1; break; }
done
cp "$OUT/orig.so" pebblesdb_amd/_lib/libpdb_crc32c.so
exit $rc
