#!/usr/bin/env python3
"""tools/seal_stamps.py <stamps.csv> [...] -- phases of the zero-copy host seals recorded with
PDB_SEAL_STAMPS=<path> (crc32c_capi.cpp host_sst_mapped), by batch size: time to take a context,
to launch, from launch to the end of the synchronisation, and the kernel's own time (events);
the kernel's GB/s over the batch bytes."""
import sys

import numpy as np

EDGES = [0, 1 << 20, 4 << 20, 8 << 20, 15 << 20, 1 << 40]
LABELS = ["<1 MiB", "1-4 MiB", "4-8 MiB", "8-15 MiB", ">=15 MiB"]


def main():
    for path in sys.argv[1:]:
        a = np.genfromtxt(path, delimiter=",", names=True)
        a = np.atleast_1d(a)
        print(f"== {path}: {len(a)} calls")
        lock = (a["locked_ns"] - a["entry_ns"]) / 1e3
        launch = (a["launched_ns"] - a["locked_ns"]) / 1e3
        sync = (a["synced_ns"] - a["launched_ns"]) / 1e3
        kern = a["kernel_ms"] * 1e3
        for lo, hi, lab in zip(EDGES[:-1], EDGES[1:], LABELS):
            m = (a["bytes"] >= lo) & (a["bytes"] < hi)
            if not m.any():
                continue
            mb = a["bytes"][m].mean() / 2**20
            print(f"  {lab:9s} calls {m.sum():5d}  mean {mb:6.2f} MiB  lock {lock[m].mean():7.1f} us  launch "
                  f"{launch[m].mean():6.1f}  launch->synced {sync[m].mean():7.1f} (p50 {np.median(sync[m]):7.1f})  kernel "
                  f"{kern[m].mean():7.1f} (p50 {np.median(kern[m]):7.1f})  kernel GB/s {a['bytes'][m].sum() / (kern[m].sum() * 1e-6) / 1e9:5.1f}")


if __name__ == "__main__":
    main()
