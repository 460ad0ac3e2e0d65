#!/usr/bin/env bash
# tools/counters_l2.sh <tag> [workloads...] -- L1->L2 request counters per workload (one --pmc pass
# each, no traces): how many times the lane-per-record kernels fetch each 128-B line from L2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-l2}"; shift || true
OUT="gpurun_out/${TAG}"
mkdir -p "$OUT"
for wl in "${@:-wal400 wal100 c2}"; do
  echo "== $wl"
  timeout -s KILL 120 rocprofv3 --pmc ${PMC:-TCP_TCC_READ_REQ_sum TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum} -f csv -d "$OUT/$wl" -- \
    python3 bench.py --workload "$wl" --steps 10 --warmup 3 --no-cpu-baseline --no-copy-inclusive > "$OUT/$wl.log" 2>&1
  rc=$?; echo "rc=$rc"; tail -2 "$OUT/$wl.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
