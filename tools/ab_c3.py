#!/usr/bin/env python3
"""Interleaved A/B of the descriptor path on BASELINE config 3 (Zipf 1-64 KiB, 16 GiB):
variant 0 = shipped (workgroup-local dynamic blocks), 8 = static strided assignment."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import zipf_kib_sizes  # noqa: E402
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import diag  # noqa: E402
from pebblesdb_amd._native import lib  # noqa: E402

variants = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,8").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
total_target = 16 << 30
crc32c.init_device(0)
sizes = zipf_kib_sizes(int(total_target / (13.5 * 1024) * 1.1) + 16, 301)
n = int(np.searchsorted(np.cumsum(sizes), total_target, side="right"))
sizes = sizes[:n]
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
total = int(sizes.sum())
d = torch.empty(total, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 303)
blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, sizes))
out = torch.empty(n, dtype=torch.int32, device="cuda")
ref = None
for v in variants:
    diag.batch_desc(v, d, blk, out=out)
    torch.cuda.synchronize()
    if ref is None:
        ref = out.clone()
    assert torch.equal(out, ref), v
# warm the GPU first: a cold GPU runs its first ~40 launches slower while clocks / power settle
# (DESIGN.md §6), which would bias whichever variant is timed first
for _ in range(15):
    diag.batch_desc(0, d, blk, out=out)
torch.cuda.synchronize()
s = torch.cuda.current_stream()
times = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            diag.batch_desc(v, d, blk, out=out)
        e1.record(s)
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 3)
algo = total + 20 * n
print(json.dumps({v: {"median_ms": round(float(np.median(t)), 4),
                      "GB/s": round(algo / (np.median(t) * 1e-3) / 1e9, 1)} for v, t in times.items()}, indent=1))
