#!/usr/bin/env bash
# tools/counters.sh <tag> -- SQ/GRBM counters for the fast CRC kernel and the load-pattern
# kernel (own passes, --pmc only; never combined with sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-cnt}"
OUT="gpurun_out/${TAG}"
mkdir -p "$OUT"
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set -f csv -d "$OUT/p$i" -- python3 tools/ab_fast.py 0 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; [ $rc -ge 124 ] && exit $rc; fi
  timeout -k 10 300 rocprofv3 --pmc $set -f csv -d "$OUT/q$i" -- python3 tools/ab_pattern.py 8 2 > "$OUT/q$i.log" 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/q$i.log"; [ $rc -ge 124 ] && exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "crc_fast4k" in k: kk = "crc"
        elif "read_pattern4k" in k: kk = "pattern"
        else: continue
        agg[(kk, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:8s} {c:24s} {statistics.median(v):.4g}")
PY
