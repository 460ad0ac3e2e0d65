#!/usr/bin/env python3
"""Seal-write pricing, seals only (tools/ab_sst.py interleaves verifies, whose kernels differ per
variant): the in-place seal (variant 0) against the same kernel writing each trailer into a shadow
image as 4 B (94), its aligned 32-B (95), 64-B (96) or 128-B window (93); and the in-place seal with
parked trailers, written 1 / 2 / 4 / 8 / 16 groups after their hash (88-92; each checked to
reproduce variant 0's sealed image); scatter passes alone (85 into the shadow, 86 into the image,
87 after a compact-CRC pass into the shadow); 80-84 = 85 / 87 / 93 / 94 / 96 into one of three
shadows in turn (the written lines are no longer in the MALL from the launch before).  Each variant: 30 warm
launches, then 20 timed with one event pair; the variant order is run forward and reversed, twice.
Prints one JSON object: GB/s of algorithmic bytes per (pass, variant)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c, diag  # noqa: E402
from pebblesdb_amd import table as T  # noqa: E402

VARIANTS = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,94,95,96").split(",")]
nblk = 1 << 20
crc32c.init_device(0)
rng = np.random.Generator(np.random.PCG64(301))
sizes = rng.integers(4166, 4175, size=nblk).astype(np.int64)
offs = np.concatenate([[0], np.cumsum(sizes + 5)[:-1]])
total = int(offs[-1] + sizes[-1] + 5)
data = torch.empty(total, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(data, 301)
data[torch.from_numpy(offs + sizes).cuda()] = 0
h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
h["offset"], h["size"] = offs, sizes
d_h = T.handles_to_device(h)
sp = int(torch.cuda.current_stream().cuda_stream)
algo = int((sizes + 1).sum()) + nblk * 20


def seal(v):
    diag.lib().pdb_diag_sst(v, data.data_ptr(), total, d_h.data_ptr(), nblk, 1, None, None, sp)


seal(0)
ref = data.clone()  # the in-place seal's image
tpos = torch.from_numpy((offs + sizes + 1)[:, None] + np.arange(4)[None, :]).reshape(-1).cuda()
for v in VARIANTS:  # allocate the shadow image up front; in-place variants must reproduce the seal
    data[tpos] = 0
    seal(v)
    torch.cuda.synchronize()
    if not (80 <= v <= 87 or 93 <= v <= 96 or v == 33 or 140 <= v <= 151):
        assert torch.equal(data, ref), f"variant {v}: sealed image differs"
    data.copy_(ref)
torch.cuda.synchronize()
res = {}
for p, order in enumerate([VARIANTS, VARIANTS[::-1], VARIANTS, VARIANTS[::-1]]):
    for v in order:
        for _ in range(30):
            seal(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            seal(v)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res.setdefault(str(v), []).append(round(algo / (ms * 1e-3) / 1e9, 1))
print(json.dumps(res), flush=True)
