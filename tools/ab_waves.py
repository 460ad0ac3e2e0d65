#!/usr/bin/env python3
"""tools/ab_waves.py -- 16 vs 12 waves for the sstable-sized kernel's other forms: the fixed-stride
sstable layout (4096 B + type at stride 4101; diagnostics batch_fixed 0 vs 130) and the compact
trailer words (pdb_sst_crc_device; pdb_diag_sst 131 = 16 waves vs 132 = 12 waves) on bench.py's
images.  Interleaved, both orders, 6 rounds of 20 launches after 100 warm ones; results checked
equal.  Prints one JSON object (GB/s of algorithmic bytes).  (Run before the product switched to 12
waves: "fixed16" is batch_fixed variant 0 only in that run; since then variant 0 is the 12-wave kernel.)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import sst_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402
from pebblesdb_amd import table as T  # noqa: E402

crc32c.init_device(0)
nblk = 1 << 20
res = {}
# fixed-stride sstable layout
L, stride = 4097, 4101
data = torch.empty(nblk * stride, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(data, 301)
o0 = diag.batch_fixed(0, data, stride, L, nblk)
o1 = diag.batch_fixed(130, data, stride, L, nblk)
assert torch.equal(o0, o1)
algo = nblk * (L + 4)
fns = {"fixed16": lambda: diag.batch_fixed(0, data, stride, L, nblk, out=o0),
       "fixed12": lambda: diag.batch_fixed(130, data, stride, L, nblk, out=o1)}


def run(fns, algo):
    for f in fns.values():
        for _ in range(100):
            f()
    t = {k: [] for k in fns}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(6):
        for k in (list(fns) if r % 2 == 0 else list(fns)[::-1]):
            e0.record()
            for _ in range(20):
                fns[k]()
            e1.record()
            torch.cuda.synchronize()
            t[k].append(e0.elapsed_time(e1) / 20)
    return {k: round(algo / (float(np.mean(v)) * 1e-3) / 1e9, 1) for k, v in t.items()}


res.update(run(fns, algo))
del data
torch.cuda.empty_cache()
# compact trailer words on the sst image
sizes, offs, total = sst_layout(nblk, 301)
img = torch.empty(total, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(img, 301)
img[torch.from_numpy(offs + sizes).cuda()] = 0
h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
h["offset"], h["size"] = offs, sizes
d_h = T.handles_to_device(h)
c16 = torch.zeros(nblk, dtype=torch.int32, device="cuda")
c12 = torch.zeros(nblk, dtype=torch.int32, device="cuda")
diag.sst(131, img, d_h, seal=True, ok=c16)
diag.sst(132, img, d_h, seal=True, ok=c12)
assert torch.equal(c16, c12)
algo = int((sizes + 1).sum()) + nblk * 20
res.update(run({"crc16": lambda: diag.sst(131, img, d_h, seal=True, ok=c16),
                "crc12": lambda: diag.sst(132, img, d_h, seal=True, ok=c12)}, algo))
print(json.dumps(res), flush=True)
