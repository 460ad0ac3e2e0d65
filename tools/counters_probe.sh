#!/usr/bin/env bash
# tools/counters_probe.sh <tag> <workload> <variant...> -- SQ / LDS counters of the record kernel
# (crc_lanespan_kernel, any mode) for diagnostics variants of tools/span_probe.py, one --pmc pass
# per counter set, no traces; the last line is JSON {variant: {counter: per-dispatch median}}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="$1"; WL="$2"; shift 2
OUT="gpurun_out/${TAG}"
mkdir -p "$OUT"
SETS=("GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
      "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD")
for v in "$@"; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -f csv -d "$OUT/v$v/p$i" -- python3 tools/span_probe.py "$v" "$WL" 10 > "$OUT/v$v.p$i.log" 2>&1
    rc=$?; echo "v$v pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 "$OUT/v$v.p$i.log"; exit $rc; fi
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, statistics, sys, collections
out = sys.argv[1]
res = {}
for vdir in sorted(glob.glob(out + "/v*/")):
    v = os.path.basename(vdir.rstrip("/"))
    agg = collections.defaultdict(list)
    for f in glob.glob(vdir + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "lanespan" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[v] = {c: statistics.median(x) for c, x in sorted(agg.items())}
print(json.dumps(res))
PY
