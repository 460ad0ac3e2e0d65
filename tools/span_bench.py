#!/usr/bin/env python3
"""Throughput of ONE long device-resident span through pdb_crc32c_extend_device (parallel
segments + device tree combine), vs the 4-KiB batch path on the same bytes."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd._native import check, lib  # noqa: E402

crc32c.init_device(0)
res = {}
s = torch.cuda.current_stream()
for gib in (1, 4, 16):
    n = gib << 30
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 9)
    words = int(lib().pdb_crc32c_extend_scratch_words(n))
    scratch = torch.empty(words, dtype=torch.int32, device="cuda")
    out = torch.empty(1, dtype=torch.int32, device="cuda")
    f = lambda: check(lib().pdb_crc32c_extend_device(0, d.data_ptr(), n, scratch.data_ptr(), words, out.data_ptr(),
                                                     s.cuda_stream))
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        f()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    res[f"{gib}GiB"] = {"ms": round(ms, 3), "GiB/s": round(gib / (ms * 1e-3), 1), "GB/s": round(n / (ms * 1e-3) / 1e9, 1)}
    del d, scratch
    torch.cuda.empty_cache()
print(json.dumps(res, indent=1))
