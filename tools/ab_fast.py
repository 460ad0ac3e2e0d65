#!/usr/bin/env python3
"""A/B the 4-KiB fast-path variants interleaved in ONE process (cdna guide §5.4 rule 24).

variant ids (per-call variant (pdb_diag_batch_*)): 0 = shipped default; others per launch_fixed's switch.
Each variant's output is checked bit-exact against variant 0 before timing.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import diag  # noqa: E402
from pebblesdb_amd._native import lib  # noqa: E402

variants = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,5").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nblk = 1 << 20
crc32c.init_device(0)
d = torch.empty(nblk * 4096, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 301)
out = torch.empty(nblk, dtype=torch.int32, device="cuda")
ref = None
for v in variants:
    diag.batch_fixed(v, d, 4096, 4096, nblk, out=out)
    torch.cuda.synchronize()
    o = out.clone()
    if ref is None:
        ref = o
    assert torch.equal(o, ref), f"variant {v} differs from variant {variants[0]}"
# warm the GPU first: a cold GPU runs its first ~40 launches slower while clocks / power settle
# (DESIGN.md §6), which would bias whichever variant is timed first
for _ in range(60):
    diag.batch_fixed(0, d, 4096, 4096, nblk, out=out)
torch.cuda.synchronize()
times = {v: [] for v in variants}
s = torch.cuda.current_stream()
for r in range(rounds):
    for v in variants:
        diag.batch_fixed(v, d, 4096, 4096, nblk, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            diag.batch_fixed(v, d, 4096, 4096, nblk, out=out)
        e1.record(s)
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 10)
res = {}
for v in variants:
    t = np.array(times[v])
    res[v] = {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
              "GB/s_median": round(nblk * 4100 / (np.median(t) * 1e-3) / 1e9, 1)}
print(json.dumps(res, indent=1))
