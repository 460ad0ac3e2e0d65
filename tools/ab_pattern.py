#!/usr/bin/env python3
"""Interleaved A/B of the 4-KiB load-pattern calibration kernels (pdb_diag_read_pattern4k)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd._native import check, lib  # noqa: E402

variants = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,5,6,7").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nblk = 1 << 20
crc32c.init_device(0)
d = torch.empty(nblk * 4096, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 301)
o = torch.zeros(1, dtype=torch.int32, device="cuda")
# warm the GPU first: a cold GPU runs its first ~40 launches slower while clocks / power settle
# (DESIGN.md §6), which would bias whichever variant is timed first
for _ in range(60):
    diag.read_pattern4k(d, nblk, variants[0], o)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
times = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        f = lambda: diag.read_pattern4k(d, nblk, v, o, s)
        f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 10)
print(json.dumps({v: {"median_ms": round(float(np.median(t)), 4),
                      "GB/s": round(nblk * 4096 / (np.median(t) * 1e-3) / 1e9, 1)}
                  for v, t in times.items()}, indent=1))
