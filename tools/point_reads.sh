#!/usr/bin/env bash
# tools/point_reads.sh <tag> -- verified point reads (readrandom --verify_checksums=1) against thread
# count, with the host CPU each read costs (pdb_dbbench's cpu_us_per_op: getrusage user + system over
# the benchmark / reads), for the CPU build and for the GPU build with each library in ab/ (run on the
# GPU box).  One 2 M x 1 KiB database written once by the CPU build (the same on-disk format).
set -uo pipefail
TAG="$1"; shift
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
B=integration/_build
DB=/tmp/pdb_point_reads
cp pebblesdb_amd/_lib/libpdb_crc32c.so "$OUT/orig.so"
# what the scalar wait sees as this process's CPUs (server_call: the affinity mask, capped by the quota)
echo "{\"affinity_cpus\": $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))'), \"cpu_max\": \"$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)\"}"
timeout -k 10 300 $B/pdb_dbbench_cpu --benchmarks=fillrandom --num=2000000 --value_size=1024 --db=$DB \
  > "$OUT/fill.log" 2>&1 || { echo "FAIL fill"; exit 1; }
echo "fill done"
run() {  # $1 = label, $2 = exe, $3 = threads
  timeout -k 10 300 "$2" --benchmarks=readrandom --use_existing_db=1 --verify_checksums=1 --threads="$3" \
    --reads=100000 --num=2000000 --db=$DB > "$OUT/$1_t$3.log" 2>&1 || { echo "FAIL $1 $3"; exit 1; }
  python3 - "$OUT/$1_t$3.log" "$1" "$3" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"bench": "readrandom"')][-1]
print(json.dumps({"build": sys.argv[2], "threads": int(sys.argv[3]), "ops_per_s": d["ops_per_s"],
                  "cpu_us_per_op": d["cpu_us_per_op"], "micros_per_op": d["micros_per_op"]}), flush=True)
PY
}
run warm $B/pdb_dbbench_cpu 8   # page cache warm before anything is recorded
for t in 1 8 16 24 32; do run cpu $B/pdb_dbbench_cpu $t; done
for lib in "$@"; do
  cp "ab/$lib.so" pebblesdb_amd/_lib/libpdb_crc32c.so
  for t in 1 8 16 24 32; do run "gpu_$lib" $B/pdb_dbbench_gpu_table $t; done
done
for t in 8 16; do run cpu_again $B/pdb_dbbench_cpu $t; done
cp "$OUT/orig.so" pebblesdb_amd/_lib/libpdb_crc32c.so
