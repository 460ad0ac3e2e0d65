#!/usr/bin/env python3
"""Throughput of the any-length stream kernels vs block length (fixed stride = length + 4, so
every block starts at a different byte phase): where do rounds, heads and extra chains cost?
Also the sstable seal hook with every block the same size.  Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import table as T  # noqa: E402

lens = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                         "1024,1056,2048,4064,4096,4097,4104,4111,4128,4160,4167,4175,4200,4352,5000,6144,8192").split(",")]
total = 4 << 30
crc32c.init_device(0)
d = torch.empty(total + (1 << 20), dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 7)
res = {}


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for _ in range(20):  # warm the GPU
    diag.batch_fixed(0, d, 4096, 4096, total // 4096)
for L in lens:
    for stride in (L + 4, (L + 15) // 16 * 16):
        n = total // stride
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        ms = timeit(lambda: diag.batch_fixed(0, d, stride, L, n, out=out))
        res[f"fixed L={L} stride={stride}"] = round(n * L / (ms * 1e-3) / 1e9, 1)
    # sstable hook, every block `L - 1` contents + type
    n = total // (L + 4)
    h = np.zeros(n, dtype=crc32c.HANDLE_DTYPE)
    h["offset"] = np.arange(n, dtype=np.uint64) * (L + 4)
    h["size"] = L - 1
    d_h = T.handles_to_device(h)
    ms = timeit(lambda: T.seal_device(d, d_h))
    res[f"seal L={L}"] = round(n * L / (ms * 1e-3) / 1e9, 1)
print(json.dumps(res, indent=1))
