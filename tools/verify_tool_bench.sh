#!/usr/bin/env bash
# tools/verify_tool_bench.sh TAG NUM -- SURVEY §8(f) row 1 in the engine: the reference's own
# leveldb-verify (integration/_build/leveldb_verify_ref) against pdb_verify_gpu (every checksum of a
# file in one GPU batch) over every file of a database written by the reference engine
# (pdb_dbbench_cpu fillrandom, NUM x 1 KiB values), wall times side by side; then both over a copy
# with one byte flipped in a data block of every table (both must report the mismatch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-vtool}"
NUM="${2:-1000000}"
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
B=integration/_build
DB="${PDB_DB_ROOT:-/tmp}/pdb_vtool_$$"
trap 'rm -rf "$DB" "$DB.bad" "$DB.err"' EXIT
ms() { echo $(( ($(date +%s%N) - $1) / 1000000 )); }
t=$(date +%s%N)
timeout -k 10 600 $B/pdb_dbbench_cpu --benchmarks=fillrandom --num="$NUM" --value_size=1024 --db="$DB" > "$OUT/fill.log" 2>&1 || { echo "fill failed"; exit 1; }
echo "[vtool] fill ${NUM} ms=$(ms $t)" | tee "$OUT/steps.txt"
FILES=$(ls "$DB" | grep -E '\.(sst|ldb|log)$|^MANIFEST' | sed "s#^#$DB/#")
echo "[vtool] files=$(echo $FILES | wc -w) bytes=$(du -sb "$DB" | cut -f1)" | tee -a "$OUT/steps.txt"
for tool in leveldb_verify_ref pdb_verify_gpu; do
  extra=""; [ $tool = pdb_verify_gpu ] && extra="--timing"
  t=$(date +%s%N)
  timeout -k 10 900 $B/$tool $extra $FILES > "$OUT/$tool.out" 2> "$OUT/$tool.err"; rc=$?
  echo "[vtool] $tool rc=$rc ms=$(ms $t) stdout_lines=$(wc -l < "$OUT/$tool.out") stderr_lines=$(wc -l < "$OUT/$tool.err")" | tee -a "$OUT/steps.txt"
  [ $rc -ge 124 ] && exit $rc
done
grep -h '"tool"' "$OUT/pdb_verify_gpu.err" | tee -a "$OUT/steps.txt"
# damaged copy: one byte inside the first data block of every table
cp -r "$DB" "$DB.bad"
python3 - "$DB.bad" <<'PY'
import os, sys
d = sys.argv[1]
for f in os.listdir(d):
    if f.endswith((".sst", ".ldb")):
        p = os.path.join(d, f)
        b = bytearray(open(p, "rb").read()); b[100] ^= 1; open(p, "wb").write(bytes(b))
PY
BAD=$(ls "$DB.bad" | grep -E '\.(sst|ldb)$' | sed "s#^#$DB.bad/#")
NT=$(echo $BAD | wc -w)
for tool in leveldb_verify_ref pdb_verify_gpu; do
  # (the reference prints a line per key on a damaged table: millions -- keep counts and a sample)
  timeout -k 10 900 $B/$tool $BAD > /dev/null 2> "$DB.err"; rc=$?
  n=$(grep -c "block checksum mismatch" "$DB.err" || true)
  head -5 "$DB.err" > "$OUT/$tool.bad.err.head"; rm -f "$DB.err"
  echo "[vtool] damaged tables=$NT $tool rc=$rc mismatch_report_lines=$n (the reference reports every key's failed Seek, pdb_verify one line per table)" | tee -a "$OUT/steps.txt"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
