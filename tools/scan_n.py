#!/usr/bin/env python3
"""Fit t(n) = a + b*n for the 4-KiB CRC kernel and the matching load-pattern kernel: separates
per-launch overhead (table staging, first HBM round trip, tail) from the per-block cost."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd._native import check, lib  # noqa: E402

variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
ns = [4096, 16384, 65536, 262144, 524288, 1 << 20]
crc32c.init_device(0)

d = torch.empty((1 << 20) * 4096, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 301)
out = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
o = torch.zeros(1, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        f()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


res = {"crc": {}, "pattern": {}, "empty_launch": None}
for n in ns:
    res["crc"][n] = timeit(lambda: diag.batch_fixed(variant, d, 4096, 4096, n, out=out))
    res["pattern"][n] = timeit(lambda: diag.read_pattern4k(d, n, 8, o, s))
for k in ("crc", "pattern"):
    x = np.array(ns, dtype=float)
    y = np.array([res[k][n] for n in ns])
    b, a = np.polyfit(x[2:], y[2:], 1)
    res[k + "_fit"] = {"a_ms": round(a, 4), "per_block_ns": round(b * 1e6, 4),
                       "asymptotic_GB/s": round(4096 / (b * 1e6), 1)}
print(json.dumps(res, indent=1))
