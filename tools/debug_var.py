#!/usr/bin/env python3
"""tools/debug_var.py -- the record kernel's per-record lanes (mixed sizes) on small WAL layouts:
failing records against the oracle, with the item geometry of their batch (diagnostics variant 126:
first record, records, lane, lanes, mode per record)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from bench import wal_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402

crc32c.init_device(0)
ora = oracle.Oracle()
for payload, hint in ((300, crc32c.SIZE_512), (1000, crc32c.SIZE_1023), (131, crc32c.SIZE_256)):
    offs, lens = wal_layout(1 << 20, payload)
    base = oracle.splitmix_bytes(int(offs[-1] + lens[-1]) + 64, payload)
    blk = crc32c.make_blocks(offs, lens)
    d_base, d_blk = torch.from_numpy(base).cuda(), crc32c.blocks_to_device(blk)
    exp = ora.batch(base, blk, flags=0, nthreads=8)
    got = diag.batch_desc(0, d_base, d_blk, flags=hint).cpu().numpy().view(np.uint32)
    geo = diag.batch_desc(126, d_base, d_blk, flags=hint).cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != exp)[0]
    print(f"payload {payload}: {bad.size} bad of {len(exp)}; first {bad[:12].tolist()}")
    for b in sorted(set((bad[:6] >> 6).tolist())):
        print(f"  batch {b}: lens {lens[64 * b:64 * b + 64].tolist()}")
        rows = []
        for r in range(64):
            g = int(geo[64 * b + r])
            rows.append((r, g >> 24, (g >> 16) & 255, (g >> 8) & 255, (g >> 4) & 15, g & 15, int(64 * b + r) in set(bad.tolist())))
        print("   ", rows)
