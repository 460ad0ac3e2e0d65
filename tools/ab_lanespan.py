#!/usr/bin/env python3
"""Interleaved A/B: the LDS-staged record kernel (variant 0, the shipped routing) against the
round-1 direct-load lane-per-record kernels (diagnostics variants 60 / 61 / 62) on log images of
131-B (db_bench --value_size=100), 431-B (400) and 700-B / 1000-B records (bench.wal_layout), each
~1-2 GiB, device-resident.  GB/s of algorithmic bytes (record bytes + 16-B descriptor + 4-B CRC).
Variants 63 / 64 time the record kernel's loads + staging alone and its hash alone (diagnostic
modes, results undefined).  Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import wal_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402

CASES = [("wal100", 131, 1 << 30, crc32c.SIZE_256, 60), ("wal400", 431, 2 << 30, crc32c.SIZE_512, 61),
         ("wal700", 700, 2 << 30, crc32c.SIZE_1023, 62), ("wal1000", 1000, 2 << 30, crc32c.SIZE_1023, 62)]


# further exact variants to time beside the shipped kernel (AB_EXTRA="68,..."; 68 = 16 waves x 6 KiB,
# one item in flight)
EXTRA = tuple(int(x) for x in os.environ.get("AB_EXTRA", "").split(",") if x)


def timeit(fn, reps=5):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    crc32c.init_device(0)
    res = {}
    for name, payload, nbytes, hint, old in CASES:
        if only and name not in only:
            continue
        offs, lens = wal_layout(nbytes, payload)
        total = int(offs[-1] + lens[-1]) + 64
        d = torch.empty(total, dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d, payload)
        d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens))
        out = torch.empty(len(offs), dtype=torch.int32, device="cuda")
        algo = int(lens.sum()) + 20 * len(lens)
        ref = diag.batch_desc(old, d, d_blk, flags=hint).cpu().numpy()
        for v in (0,) + EXTRA:
            got = diag.batch_desc(v, d, d_blk, flags=hint).cpu().numpy()
            assert (ref == got).all(), (name, v)
        for _ in range(20):  # warm: power management settles
            diag.batch_desc(0, d, d_blk, flags=hint, out=out)
        # 63 / 64 / 67: the record kernel's loads alone / hash alone / bookkeeping alone
        t = {0: [], old: [], 63: [], 64: [], 67: []}
        t.update({v: [] for v in EXTRA})
        for _ in range(5):
            for v in t:
                t[v].append(timeit(lambda: diag.batch_desc(v, d, d_blk, flags=hint, out=out)))
        res[name] = {str(v): {"ms": round(float(np.median(x)), 4), "GB/s": round(algo / (np.median(x) * 1e-3) / 1e9, 1),
                              "frac_8TBs": round(algo / (np.median(x) * 1e-3) / 8e12, 4)} for v, x in t.items()}
        res[name]["records"] = len(offs)
        del d, d_blk, out
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
