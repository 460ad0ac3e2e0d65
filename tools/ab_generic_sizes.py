#!/usr/bin/env python3
"""Interleaved A/B of fixed-stride stream-kernel variants at given block lengths (stride = length
+ 4, unaligned): argv[1] = variants (e.g. 15,17), argv[2] = lengths.  Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import diag  # noqa: E402
from pebblesdb_amd._native import lib  # noqa: E402

variants = [int(x) for x in sys.argv[1].split(",")]
lens = [int(x) for x in sys.argv[2].split(",")]
total = 4 << 30
crc32c.init_device(0)
d = torch.empty(total + (1 << 20), dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 7)
for _ in range(20):
    diag.batch_fixed(0, d, 4096, 4096, total // 4096)
res = {}
for L in lens:
    stride = L + 4
    n = total // stride
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ref = None
    times = {v: [] for v in variants}
    for v in variants:
        diag.batch_fixed(v, d, stride, L, n, out=out)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), (L, v)
    for _ in range(4):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                diag.batch_fixed(v, d, stride, L, n, out=out)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 3)
    res[L] = {v: round(n * L / (np.median(t) * 1e-3) / 1e9, 1) for v, t in times.items()}
print(json.dumps(res, indent=1))
