#!/usr/bin/env python3
"""Summarise tools/profile.sh output: per-kernel average duration (kernel-trace) and HBM bytes
per launch from FETCH_SIZE / WRITE_SIZE (rocprofv3 PMC, KB units).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports 1/2 of the bytes of a wide
16-B/lane streaming read.  We calibrate the factor on the diag kernel read_pattern4k, which
issues exactly the fast path's loads over a known byte count, and apply it to the CRC kernel.
"""
import csv
import glob
import json
import os
import statistics
import sys

out_dir, workload = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "c2")
KERNELS = {"c2": "crc_pack4k_kernel", "sstable": "crc_sst4k_kernel", "c3": "crc_stream16_kernel",
           "wal": "crc_lanespan_kernel", "wal100": "crc_lanespan_kernel", "wal400": "crc_lanespan_kernel",
           "wal1000": "crc_lanespan_kernel", "sst_verify": "crc_sst4k_kernel", "sst_seal": "crc_sst4k_kernel",
           "sst_crc": "crc_sst4k_kernel", "sst_tables": "crc_sst4k_kernel"}
target = KERNELS[workload]
# the launches that follow the batch kernel on the same stream (the long-block lane), reported beside it
LANE = ("crc_longpiece_kernel", "long_combine_kernel", "crc_longlane_kernel") if workload == "sst_tables" else ()


def rows(pattern):
    for f in glob.glob(os.path.join(out_dir, pattern), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def kname(r):
    return r.get("Kernel_Name") or r.get("KernelName") or r.get("Name") or ""


def durations(sub):
    d = []
    for r in rows("trace/**/*kernel_trace.csv"):
        if sub in kname(r):
            d.append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    return [x for _, x in sorted(d)]  # launch order, ns -> ms


def counter(name, sub):
    v = []
    for r in rows(f"pmc_*/**/*counter_collection.csv"):
        if r.get("Counter_Name") == name and sub in kname(r):
            v.append(float(r["Counter_Value"]))
    return v


res = {}
dur = durations(target)
fetch = counter("FETCH_SIZE", target)
write = counter("WRITE_SIZE", target)
cal_fetch = counter("FETCH_SIZE", "read_pattern4k_kernel")
# known bytes for the calibration kernel: the whole buffer (bench allocs it; read from its log)
known = None
steps = None
bench_avg = None
try:
    with open(os.path.join(out_dir, "trace.log")) as fh:
        for ln in fh:
            if ln.startswith("{"):
                line = json.loads(ln)
                known = line["config"]["bytes_per_gpu"]
                steps = line["steps"]
                bench_avg = line["roofline"]["kernel_avg_ms"]
except (OSError, ValueError, KeyError):
    pass
factor = 2.0
if cal_fetch and known:
    factor = known / (statistics.median(cal_fetch) * 1024.0)
entry = {
    "kernel": target,
    "launches_traced": len(dur),
    "avg_ms": round(statistics.mean(dur), 4) if dur else None,
    "median_ms": round(statistics.median(dur), 4) if dur else None,
    # the bench's timed region = the last `steps` launches (warmup launches come first)
    "timed_launches": steps,
    "avg_ms_timed_launches": round(statistics.mean(dur[-steps:]), 4) if dur and steps else None,
    "bench_hip_event_avg_ms": bench_avg,
    "fetch_size_kb_median": statistics.median(fetch) if fetch else None,
    "write_size_kb_median": statistics.median(write) if write else None,
    "fetch_correction_factor": round(factor, 4),
    "fetch_calibration": "read_pattern4k_kernel (same loads, known bytes)" if cal_fetch and known else
                         "MI355X_MICROARCH.md §HBM x2",
}
if fetch and write:
    entry["hbm_bytes_per_launch"] = int(statistics.median(fetch) * 1024 * factor + statistics.median(write) * 1024)
for k in LANE:  # (the combine kernel exists only in builds before the fused piece kernel)
    d, f, w = durations(k), counter("FETCH_SIZE", k), counter("WRITE_SIZE", k)
    if d:
        entry[k] = {"launches_traced": len(d), "avg_ms_timed_launches": round(statistics.mean(d[-steps:]), 4) if steps else None,
                    "hbm_bytes_per_launch": int(statistics.median(f) * 1024 * factor + statistics.median(w) * 1024) if f and w else None}
lane = [entry[k] for k in LANE if k in entry]
if lane and all(x["hbm_bytes_per_launch"] is not None for x in lane) and "hbm_bytes_per_launch" in entry:
    entry["hbm_bytes_per_call"] = entry["hbm_bytes_per_launch"] + sum(x["hbm_bytes_per_launch"] for x in lane)
res[workload] = entry
print(json.dumps(res, indent=1))
