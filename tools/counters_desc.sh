#!/usr/bin/env bash
# tools/counters_desc.sh <tag> <workload> [variant] [kernel] -- SQ counters of a descriptor-path
# kernel (default crc_stream16_kernel under variant 16; `0 crc_sst1k_kernel` for the WAL's sized
# kernel) on a tools/ab_desc.py workload, one --pmc pass per counter set.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-cntd}"
WL="${2:-wal}"
VAR="${3:-16}"
KERN="${4:-crc_stream16_kernel}"
OUT="gpurun_out/${TAG}"
mkdir -p "$OUT"
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set -f csv -d "$OUT/p$i" -- python3 tools/ab_desc.py "$VAR" "$WL" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 - "$OUT" "$KERN" <<'PY'
import csv, glob, sys, statistics, collections
out, kern = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(agg.items()):
    print(f"{c:24s} {statistics.median(v):.4g}")
PY
