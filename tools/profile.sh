#!/usr/bin/env bash
# tools/profile.sh <tag> [workload] -- rocprofv3 evidence for the roofline (run on the GPU box).
#  pass 1: --kernel-trace --stats (per-kernel durations)
#  pass 2: --pmc FETCH_SIZE        (own pass: FETCH_SIZE needs 3 TCC slots)
#  pass 3: --pmc WRITE_SIZE
# then tools/pmc_traffic.py summarises into gpurun_out/<tag>_pmc_traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-prof}"
WL="${2:-c2}"
OUT="gpurun_out/${TAG}"
mkdir -p "$OUT"
ARGS="bench.py --workload $WL --no-cpu-baseline --no-copy-inclusive --no-c4-shard --diag"
if [ "$WL" = sst_tables ]; then
  # the tables are written once, before and outside the profiled runs (CPU only: pdb_tablegen)
  TD=/tmp/pdb_tables_prof
  timeout -k 10 300 python3 -c "import bench; bench.real_tables(4, 1000000, 1024, 401, '$TD')" || exit 1
  ARGS="$ARGS --tables-dir $TD"
fi
run() {  # run <name> <rocprof args...>
  local name=$1; shift
  echo "== $name"
  timeout -k 10 420 rocprofv3 "$@" -f csv -d "$OUT/$name" -- python3 $ARGS > "$OUT/${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/${name}.log"
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
python3 tools/pmc_traffic.py "$OUT" "$WL" > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
