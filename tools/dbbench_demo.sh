#!/usr/bin/env bash
# tools/dbbench_demo.sh -- BASELINE configs 1 and 5 on the GPU box: the reference's own db_bench,
# built in place by oracle/build_ref_dbbench.sh, as shipped (db_bench_ref, CPU CRC32C) and with
# util/crc32c.h bound to libpdb_crc32c.so (db_bench_pdb, every Extend/Value on the MI355X).
# Afterwards every CRC in each database directory is re-checked by the oracle (and, for the GPU
# build, by the batched GPU verifiers), and each binary reopens the other's database (WAL
# recovery runs log::Reader with checksums on).  Outputs under gpurun_out/dbbench/.
#   usage: tools/dbbench_demo.sh [NUM_CONFIG1] [NUM_CONFIG5]
set -euo pipefail
cd "$(dirname "$0")/.."
N1="${1:-1000000}"
N5="${2:-1000000}"
OUT=gpurun_out/dbbench
mkdir -p "$OUT"
T="$(mktemp -d /tmp/pdb_dbbench.XXXXXX)"
trap 'rm -rf "$T"' EXIT
REF=oracle/_ref/db_bench_ref
PDB=oracle/_ref/db_bench_pdb
step() {  # name timeout cmd...
  local name="$1" to="$2"; shift 2
  echo "[dbbench] $name: $*" | tee -a "$OUT/steps.txt"
  local t0=$(date +%s%N) rc=0
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1 || rc=$?
  echo "[dbbench] $name rc=$rc wall_ms=$(( ($(date +%s%N) - t0) / 1000000 ))" | tee -a "$OUT/steps.txt"
  grep -a "micros/op" "$OUT/$name.log" | sed 's/.*\(fill\|read\|crc\)/\1/' | tee -a "$OUT/steps.txt" || true
  return $rc
}
: > "$OUT/steps.txt"
# config 1: fillseq 1M x 1 KiB, CPU reference vs GPU hook; crc32c microbench (4 KiB per call)
step c1_ref 600 $REF --benchmarks=fillseq,crc32c --num="$N1" --value_size=1024 --db="$T/c1_ref"
step c1_ref_verify 300 python3 tools/verify_db_dir.py "$T/c1_ref"
step c1_pdb 900 $PDB --benchmarks=fillseq,crc32c --num="$N1" --value_size=1024 --db="$T/c1_pdb"
step c1_pdb_verify 300 python3 tools/verify_db_dir.py --gpu "$T/c1_pdb"
# cross-open: each binary recovers (WAL CRC checks) and reads the other's database
step c1_ref_reads_pdb 600 $REF --benchmarks=readseq --use_existing_db=1 --num="$N1" --db="$T/c1_pdb"
step c1_pdb_reads_ref 600 $PDB --benchmarks=readseq --use_existing_db=1 --num="$N1" --db="$T/c1_ref"
rm -rf "$T/c1_ref" "$T/c1_pdb"
# config 5 (scaled --num): fillrandom,readrandom with the GPU hook vs the CPU reference
step c5_ref 900 $REF --benchmarks=fillrandom,readrandom --num="$N5" --value_size=1024 --db="$T/c5_ref"
step c5_pdb 1200 $PDB --benchmarks=fillrandom,readrandom --num="$N5" --value_size=1024 --db="$T/c5_pdb"
step c5_pdb_verify 300 python3 tools/verify_db_dir.py --gpu "$T/c5_pdb"
echo "[dbbench] done"
