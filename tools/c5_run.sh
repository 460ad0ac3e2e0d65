#!/usr/bin/env bash
# tools/c5_run.sh -- BASELINE configs 1 and 5 on the GPU box with the db_bench-equivalent harness
# (integration/pdb_dbbench.cc) over the engine variants built by integration/build.sh, next to the
# reference's own db_bench (oracle/_ref/db_bench_ref).  Every database a GPU build writes is
# re-checked by the oracle and the batched GPU verifiers (tools/verify_db_dir.py).
#   usage: tools/c5_run.sh TAG NUM "variant ..." [BENCHMARKS] [VERIFY]
#   variants: ref (reference db_bench as shipped), cpu, gpu_table, gpu_all
# Each step runs under its own time limit; a crash or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-c5}"
NUM="${2:-1000000}"
VARIANTS="${3:-ref cpu gpu_table gpu_all}"
BENCHES="${4:-fillrandom,readrandom}"
VERIFY="${5:-1}"
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
DBROOT="${PDB_DB_ROOT:-/tmp}/pdb_c5_$$"
mkdir -p "$DBROOT"
trap 'rm -rf "$DBROOT"' EXIT
df -h "$DBROOT" | tail -1 | tee "$OUT/disk.txt"
step() {  # name timeout cmd...
  local name="$1" to="$2"; shift 2
  echo "[c5] $name: $*" | tee -a "$OUT/steps.txt"
  local t0=$(date +%s%N) rc=0
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1 || rc=$?
  echo "[c5] $name rc=$rc wall_ms=$(( ($(date +%s%N) - t0) / 1000000 ))" | tee -a "$OUT/steps.txt"
  grep -a "micros/op" "$OUT/$name.log" | sed 's/.*\(fill\|read\)/\1/' | tee -a "$OUT/steps.txt" || true
  if [ $rc -ne 0 ]; then echo "[c5] stopping after rc=$rc" | tee -a "$OUT/steps.txt"; exit $rc; fi
}
for v in $VARIANTS; do
  db="$DBROOT/$v"
  if [ "$v" = ref ]; then
    step "${v}" 1100 oracle/_ref/db_bench_ref --benchmarks="$BENCHES" --num="$NUM" --value_size=1024 --db="$db"
  else
    step "${v}" 1100 "integration/_build/pdb_dbbench_$v" --benchmarks="$BENCHES" --num="$NUM" --value_size=1024 \
      --verify_checksums="$VERIFY" --db="$db"
    case "$v" in gpu_*) step "${v}_verify" 600 python3 tools/verify_db_dir.py --gpu "$db" ;; esac
  fi
  rm -rf "$db"
done
echo "[c5] done" | tee -a "$OUT/steps.txt"
