#!/usr/bin/env bash
# tools/counters_c2.sh <tag> -- SQ counters of the C2 kernel on the lane-quarter table image
# (crc_pack4k_kernel, diagnostics variant 0) beside the round-1 kernel on the 32-replica image
# (crc_pack4k_ab_kernel, variant 99), in one process per pass (tools/ab_fast.py 0,99): LDS
# instructions, bank-conflict cycles, LDS / VALU activity.  Own --pmc passes, no traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-cntc2}"
OUT="gpurun_out/${TAG}"
mkdir -p "$OUT"
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -s KILL 240 rocprofv3 --pmc $set -f csv -d "$OUT/p$i" -- python3 tools/ab_fast.py 0,99 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, statistics, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "crc_pack4k_ab_kernel" in k: kk = "round1_32replica"
        elif "crc_pack4k_kernel" in k: kk = "lane_quarter"
        else: continue
        agg[(kk, r["Counter_Name"])].append(float(r["Counter_Value"]))
res = collections.defaultdict(dict)
for (k, c), v in sorted(agg.items()):
    res[k][c] = statistics.median(v)
for k, d in res.items():  # per 4-KiB block (1 M blocks per launch)
    d["lds_insts_per_block"] = d.get("SQ_INSTS_LDS", 0) / (1 << 20)
    d["valu_insts_per_block"] = d.get("SQ_INSTS_VALU", 0) / (1 << 20)
    d["bank_conflict_cycles_per_block"] = d.get("SQ_LDS_BANK_CONFLICT", 0) / (1 << 20)
print(json.dumps(res, indent=1))
PY
