#!/usr/bin/env bash
# tools/ab_lane.sh <tag> <lib...> -- A/B of product-library builds on the sst_* and c3 bench lines
# (run on the GPU box): each library in ab/ is copied over pebblesdb_amd/_lib/libpdb_crc32c.so in
# turn (the box's scratch copy of the tree), in the order given and then in reverse, and every
# workload's 50-step line is written to gpurun_out/<tag>/<lib>_<n>_<workload>.json.
set -uo pipefail
TAG="$1"; shift
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
cp pebblesdb_amd/_lib/libpdb_crc32c.so "$OUT/orig.so"
ORDER=("$@")
for ((i=$#-1; i>=0; i--)); do ORDER+=("${@:i+1:1}"); done
n=0
for lib in "${ORDER[@]}"; do
  n=$((n+1))
  cp "ab/$lib.so" pebblesdb_amd/_lib/libpdb_crc32c.so
  for w in ${AB_WORKLOADS:-sst_seal sst_verify sst_crc c3}; do
    extra=""; [ "$w" = sst_tables ] && extra="--tables-dir /tmp/pdb_tables_ab"  # (made once, reused)
    timeout -k 10 240 python bench.py --workload "$w" --steps 50 --no-cpu-baseline --no-ceiling --settle 100 $extra \
      > "$OUT/${lib}_${n}_$w.json" 2> "$OUT/${lib}_${n}_$w.err" || { echo "FAIL $lib $w"; exit 1; }
    python - "$OUT/${lib}_${n}_$w.json" "$lib" "$w" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["value"], d["roofline"]["frac"], (d.get("steady_state") or {}).get("frac"), flush=True)
PY
  done
done
cp "$OUT/orig.so" pebblesdb_amd/_lib/libpdb_crc32c.so
