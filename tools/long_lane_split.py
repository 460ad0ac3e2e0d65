#!/usr/bin/env python3
"""tools/long_lane_split.py <trace dir> -- split tools/long_block_cost.py --device-only's kernel trace
(rocprofv3 --kernel-trace -f csv) into the long-block lane's parts.  Every device call is two or
three dispatches on one stream: the batch kernel (crc_sst4k_kernel), the piece kernel
(crc_longpiece_kernel; crc_longlane_kernel, which also folds the records, since round 6's fused
lane) and, before the fused lane, the combine kernel; the script walks them in dispatch order (5 long-block sizes x seal / verify / crc x 55 calls)
and prints, per size and entry, the median duration of each kernel, the gaps between them and the
call-to-call cadence, in microseconds."""
import csv
import glob
import json
import statistics
import sys

SIZES = (0, 64, 400, 1300, 4096)
OPS = ("seal", "verify", "crc")
CALLS = 55


def main():
    files = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                kind = ("batch" if "crc_sst4k_kernel" in name else "piece" if ("crc_longpiece_kernel" in name or "crc_longlane_kernel" in name)
                        else "combine" if "long_combine_kernel" in name else None)
                if kind:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    rows.sort()
    # a call = its batch kernel and what follows it up to the next batch kernel: the piece kernel and
    # (before the fused form) the combine kernel
    calls = []
    for r in rows:
        if r[2] == "batch":
            calls.append([r])
        else:
            calls[-1].append(r)
    assert all([k for _, _, k in c] in (["batch", "piece", "combine"], ["batch", "piece"]) for c in calls), \
        "unexpected dispatch order"
    calls = [c if len(c) == 3 else c + [(c[1][1], c[1][1], "combine")] for c in calls]  # (fused: a 0-us combine)
    assert len(calls) == len(SIZES) * len(OPS) * CALLS, len(calls)
    out = []
    for si, kib in enumerate(SIZES):
        for oi, op in enumerate(OPS):
            base = (si * len(OPS) + oi) * CALLS
            timed = calls[base + 5:base + CALLS]
            med = lambda f: round(statistics.median(f(c) for c in timed) / 1e3, 2)  # noqa: E731
            cadence = [timed[i + 1][0][0] - timed[i][0][0] for i in range(len(timed) - 1)]
            out.append({"long_block_KiB": kib, "entry": op, "batch_us": med(lambda c: c[0][1] - c[0][0]),
                        "gap1_us": med(lambda c: c[1][0] - c[0][1]), "piece_us": med(lambda c: c[1][1] - c[1][0]),
                        "gap2_us": med(lambda c: c[2][0] - c[1][1]), "combine_us": med(lambda c: c[2][1] - c[2][0]),
                        "call_us": med(lambda c: c[2][1] - c[0][0]),
                        "cadence_us": round(statistics.median(cadence) / 1e3, 2)})
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
