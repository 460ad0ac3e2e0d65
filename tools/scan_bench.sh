#!/usr/bin/env bash
# tools/scan_bench.sh -- SURVEY §8(f) row 1 in the engine: verified scans and paranoid compactions
# with the table reader's read-ahead windows (integration/pdb_table.cc) against the engine as shipped
# (CPU checks) and the GPU hooks over the reference's table reader (one GPU round trip per block).
#   usage: tools/scan_bench.sh TAG NUM [FILL] [PARANOID]
#   FILL: the benchmark that writes the scanned database (fillrandom; fillseq at 10 M: the CPU
#   build dumped core in teardown right after a 10 M fillrandom with no read phase, compactions
#   still backed up); PARANOID=0 skips step 3.
#   1. one database (fillrandom, 1 KiB values) written by the CPU build;
#   2. readseq --verify_checksums=1 over it: cpu, gpu_table_noscan, gpu_table (each twice, after an
#      untimed pass that warms the page cache);
#   3. fillrandom --paranoid_checks=1 (every compaction input block verified, version_set.cc:2909)
#      on a fresh database per build; the GPU builds' databases re-checked by tools/verify_db_dir.py.
# Each step runs under its own time limit; a crash or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-scan}"
NUM="${2:-1000000}"
FILL="${3:-fillrandom}"
PARANOID="${4:-1}"
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
DBROOT="${PDB_DB_ROOT:-/tmp}/pdb_scan_$$"
mkdir -p "$DBROOT"
trap 'rm -rf "$DBROOT"' EXIT
B=integration/_build
step() {  # name timeout cmd...
  local name="$1" to="$2"; shift 2
  echo "[scan] $name: $*" | tee -a "$OUT/steps.txt"
  local t0=$(date +%s%N) rc=0
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1 || rc=$?
  echo "[scan] $name rc=$rc wall_ms=$(( ($(date +%s%N) - t0) / 1000000 ))" | tee -a "$OUT/steps.txt"
  grep -a "micros/op" "$OUT/$name.log" | tee -a "$OUT/steps.txt" || true
  if [ $rc -ne 0 ]; then echo "[scan] stopping after rc=$rc" | tee -a "$OUT/steps.txt"; exit $rc; fi
}
db="$DBROOT/db"
step fill_cpu 900 $B/pdb_dbbench_cpu --benchmarks="$FILL" --num="$NUM" --value_size=1024 --db="$db"
step warm 600 $B/pdb_dbbench_cpu --use_existing_db=1 --benchmarks=readseq --num="$NUM" --verify_checksums=0 --db="$db"
for r in 1 2; do
  for v in cpu gpu_table_noscan gpu_table; do
    step "readseq_${v}_$r" 600 $B/pdb_dbbench_$v --use_existing_db=1 --benchmarks=readseq --num="$NUM" \
      --verify_checksums=1 --db="$db"
  done
done
rm -rf "$db"
[ "$PARANOID" = 1 ] || { echo "[scan] done" | tee -a "$OUT/steps.txt"; exit 0; }
for v in cpu gpu_table_noscan gpu_table; do
  d="$DBROOT/p_$v"
  step "paranoid_fill_$v" 1100 $B/pdb_dbbench_$v --benchmarks=fillrandom --num="$NUM" --value_size=1024 \
    --paranoid_checks=1 --db="$d"
  case "$v" in gpu_*) step "paranoid_fill_${v}_verify" 600 python3 tools/verify_db_dir.py --gpu "$d" ;; esac
  rm -rf "$d"
done
echo "[scan] done" | tee -a "$OUT/steps.txt"
