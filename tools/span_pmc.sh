#!/usr/bin/env bash
# tools/span_pmc.sh <tag> <variants> <workloads> -- SQ LDS counters per record-kernel MODE under
# tools/ab_span.py (one --pmc pass per workload; per-launch means in millions, grouped by the kernel's
# MODE template argument; PMC="<counters>" overrides the default set).  Prints one JSON object (the
# last line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="$1"; VARS="$2"; WLS="$3"
OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
for wl in ${WLS//,/ }; do
  timeout -s KILL 300 rocprofv3 --pmc ${PMC:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE} \
    -f csv -d "$OUT/$wl" -- python3 tools/ab_span.py "$VARS" "$wl" 1 > "$OUT/$wl.log" 2>&1
  rc=$?; echo "$wl rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$wl.log"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, re, sys, collections
out = sys.argv[1]; res = {}
for wdir in sorted(glob.glob(out + "/*/")):
    wl = os.path.basename(wdir.rstrip("/"))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(wdir + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "lanespan" not in k: continue
            m = re.search(r"Sink, (\d+)u, (\d+),", k)
            key = "MODE%s_%s" % (m.group(2), m.group(1)) if m else k[:60]
            agg[key][(r["Counter_Name"], r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
    res[wl] = {}
    for key, d in agg.items():
        per = collections.defaultdict(list)
        for (c, _), v in d.items(): per[c].append(sum(v))
        res[wl][key] = {c: round(sum(v) / len(v) / 1e6, 3) for c, v in sorted(per.items())}
        res[wl][key]["launches"] = len(next(iter(per.values())))
print(json.dumps(res))
PY
