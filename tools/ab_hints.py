#!/usr/bin/env python3
"""tools/ab_hints.py -- the product routing (diagnostics variant 0) under different size hints on
the same log images, interleaved, both orders (results checked equal): which class and whether the
mixed-size hint pays for records of 1..256 B of varied sizes (the <= 256-B class has no per-record
lanes; the 257..512-B class with PDB_CRC_SIZE_MIXED gives a record ceil(words / 27) lanes)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import wal_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402

H = {"256": crc32c.SIZE_256, "512": crc32c.SIZE_512, "512m": crc32c.SIZE_512 | crc32c.SIZE_MIXED,
     "1023m": crc32c.SIZE_1023 | crc32c.SIZE_MIXED}
WL = {"rand32_256": (32, 256), "rand1_256": (1, 256), "rand100_256": (100, 256), "rand1_200": (1, 200),
      "wal100": 131}
crc32c.init_device(0)
for wl, payload in WL.items():
    if isinstance(payload, tuple):
        rng = np.random.default_rng(7)
        lens = rng.integers(payload[0], payload[1], size=int((1 << 30) / (sum(payload) / 2 + 7)))
        offs = np.concatenate([[0], np.cumsum(lens + 7)[:-1]]) + 6
    else:
        offs, lens = wal_layout(1 << 30, payload)
    d = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 11)
    d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens))
    out = torch.empty(len(offs), dtype=torch.int32, device="cuda")
    hints = ["256", "512", "512m"]
    ref = diag.batch_desc(0, d, d_blk, flags=H["256"]).cpu().numpy()
    for h in hints:
        assert (diag.batch_desc(0, d, d_blk, flags=H[h]).cpu().numpy() == ref).all(), (wl, h)
    for h in hints:
        for _ in range(100):
            diag.batch_desc(0, d, d_blk, flags=H[h], out=out)
    torch.cuda.synchronize()
    t = {h: [] for h in hints}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(6):
        for h in (hints if r % 2 == 0 else hints[::-1]):
            e0.record()
            for _ in range(20):
                diag.batch_desc(0, d, d_blk, flags=H[h], out=out)
            e1.record()
            torch.cuda.synchronize()
            t[h].append(e0.elapsed_time(e1) / 20)
    algo = int(lens.sum()) + 20 * len(lens)
    print(json.dumps({"workload": wl, **{h: round(algo / (float(np.mean(v)) * 1e-3) / 8e12, 4) for h, v in t.items()}}),
          flush=True)
    del d, d_blk, out
    torch.cuda.empty_cache()
