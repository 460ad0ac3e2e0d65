#!/usr/bin/env bash
# tools/counters_span.sh <tag> [workloads...] -- SQ / LDS / TA counters of the WAL record kernel
# (crc_lanespan_kernel) under bench.py --workload <wl>, one --pmc pass per counter set, no traces;
# prints the per-dispatch medians per workload as JSON (the last line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${1:-span}"; shift || true
OUT="gpurun_out/${TAG}"
mkdir -p "$OUT"
SETS=("GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
      "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
      "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCC_REQ_sum")
for wl in "${@:-wal100 wal400}"; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    echo "== $wl pass $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set -f csv -d "$OUT/$wl/p$i" -- \
      python3 bench.py --workload "$wl" --steps 10 --warmup 3 --no-cpu-baseline --no-copy-inclusive > "$OUT/$wl.p$i.log" 2>&1
    rc=$?; echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 "$OUT/$wl.p$i.log"; exit $rc; fi
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, statistics, sys, collections
out = sys.argv[1]
res = {}
for wdir in sorted(glob.glob(out + "/*/")):
    wl = os.path.basename(wdir.rstrip("/"))
    agg = collections.defaultdict(list)
    for f in glob.glob(wdir + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "lanespan" not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[wl] = {c: statistics.median(v) for c, v in sorted(agg.items())}
print(json.dumps(res))
PY
