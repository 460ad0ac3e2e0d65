#!/usr/bin/env python3
"""Interleaved A/B of fixed-stride generic-path variants on the sstable layout (4097 B under the
CRC at stride 4101, unaligned) and on 4-KiB blocks at a 4-B-aligned base."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import diag  # noqa: E402
from pebblesdb_amd._native import lib  # noqa: E402

variants = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,8").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nblk = 1 << 20
crc32c.init_device(0)
d = torch.empty(nblk * 4101 + 64, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 301)
out = torch.empty(nblk, dtype=torch.int32, device="cuda")
cases = {"sstable_4097_s4101": (d, 4101, 4097), "4k_base+4": (d[4:], 4096, 4096)}
s = torch.cuda.current_stream()
res = {}
# warm the GPU first: a cold GPU runs its first ~40 launches slower
for _ in range(60):
    diag.batch_fixed(0, d, 4101, 4097, nblk, out=out)
torch.cuda.synchronize()
for name, (base, stride, L) in cases.items():
    ref = None
    for v in variants:
        diag.batch_fixed(v, base, stride, L, nblk, out=out)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), (name, v)
    times = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            diag.batch_fixed(v, base, stride, L, nblk, out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                diag.batch_fixed(v, base, stride, L, nblk, out=out)
            e1.record(s)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    res[name] = {v: {"median_ms": round(float(np.median(t)), 4),
                     "GB/s": round(nblk * (L + 4) / (np.median(t) * 1e-3) / 1e9, 1)} for v, t in times.items()}
print(json.dumps(res, indent=1))
