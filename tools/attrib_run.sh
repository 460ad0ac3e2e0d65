#!/usr/bin/env bash
# tools/attrib_run.sh TAG NUM "variant ..." -- what the GPU CRC itself buys in the engine
# (DESIGN.md §6.1d).  For every engine build (integration/build.sh):
#   cpu           the reference engine as shipped (per-block WriteRawBlock + file->Flush, CPU CRC)
#   buffered_cpu  the GPU build's batching -- buffered emission, verified read-ahead windows -- with
#                 every CRC on the CPU (integration/pdb_crc_route.h, -DPDB_CPU_CRC=1)
#   gpu_table     the same batching with the CRCs on the GPU (pdb_sst_seal_host / verify_host /
#                 the scalar service)
#   ref           the reference's own db_bench (fillrandom only: it has no --verify_checksums)
# run on a fresh database: fillrandom NUM, two verified readseq passes, and verified readrandom
# with --threads 1 / 4 / 16 (R reads per thread).  The teardown time (delete db) is logged.
# Each step runs under its own limit; a crash or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-attrib}"
NUM="${2:-1000000}"
VARIANTS="${3:-cpu buffered_cpu gpu_table}"
R="${PDB_READS:-200000}"
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
DBROOT="${PDB_DB_ROOT:-/tmp}/pdb_attrib_$$"
mkdir -p "$DBROOT"
trap 'rm -rf "$DBROOT"' EXIT
df -h "$DBROOT" | tail -1 | tee "$OUT/disk.txt"
step() {  # name timeout cmd...
  local name="$1" to="$2"; shift 2
  echo "[attrib] $name: $*" | tee -a "$OUT/steps.txt"
  local t0=$(date +%s%N) rc=0
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1 || rc=$?
  echo "[attrib] $name rc=$rc wall_ms=$(( ($(date +%s%N) - t0) / 1000000 ))" | tee -a "$OUT/steps.txt"
  grep -a "micros/op\|teardown" "$OUT/$name.log" | tee -a "$OUT/steps.txt" || true
  local lines=0
  lines=$(grep -ac '^{"bench"' "$OUT/$name.log") || true
  grep -a '^{"bench"' "$OUT/$name.log" >> "$OUT/bench_lines.jsonl" || true
  # a fault after every benchmark of the step reported (the engine's shutdown race)
  # is logged with its backtrace and the next step reopens the database (WAL recovery); a step that
  # did not finish its benchmarks, or a time limit, stops the script
  if [ $rc -ne 0 ] && { [ "$lines" -eq 0 ] || [ $rc -eq 124 ] || [ $rc -eq 137 ]; }; then
    echo "[attrib] stopping after rc=$rc" | tee -a "$OUT/steps.txt"; exit $rc
  fi
  if [ $rc -ne 0 ]; then
    echo "[attrib] $name: rc=$rc after its benchmarks reported (teardown); backtrace:" | tee -a "$OUT/steps.txt"
    grep -a -A 24 "fatal signal" "$OUT/$name.log" >> "$OUT/steps.txt" || true
  fi
}
for v in $VARIANTS; do
  db="$DBROOT/$v"
  if [ "$v" = ref ]; then
    step "${v}_fill" 600 oracle/_ref/db_bench_ref --benchmarks=fillrandom --num="$NUM" --value_size=1024 --db="$db"
  else
    exe="integration/_build/pdb_dbbench_$v"
    step "${v}_fill" 600 "$exe" --benchmarks=fillrandom --num="$NUM" --value_size=1024 --db="$db"
    step "${v}_readseq" 300 "$exe" --use_existing_db=1 --benchmarks=readseq,readseq --num="$NUM" --value_size=1024 \
      --verify_checksums=1 --db="$db"
    for t in 1 4 16; do
      step "${v}_readrandom_t$t" 300 "$exe" --use_existing_db=1 --benchmarks=readrandom --num="$NUM" --reads="$R" \
        --threads="$t" --value_size=1024 --verify_checksums=1 --db="$db"
    done
  fi
  rm -rf "$db"
done
echo "[attrib] done" | tee -a "$OUT/steps.txt"
