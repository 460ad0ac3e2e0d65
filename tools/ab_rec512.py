#!/usr/bin/env python3
"""A/B for the record classes (variants 55/56: the next batch's window issued before hashing the
current one).  The 257..512-B record class: crc_lanerec17_kernel (hint "512"; 4 chains, variant 54 the
two-chain 9 + 8-group version) against the descriptor
path with hints ignored (variant 40: the generic stream kernel) and against the <= 256-B kernel
(hint "256", whose whole-wave slow path these records take).  Records packed back to back (any
alignment), ~2 GiB per case; GB/s = (record bytes + 16-B descriptor + 4-B result) / kernel time.
Also the fixed-stride entry at 431 B.  Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import diag  # noqa: E402
_HINT_FLAGS = {None: 0, '1k': 0x4, '4k': 0x8, '256': 0x10, '512': 0x20, '1023': 0x40}
from pebblesdb_amd._native import lib  # noqa: E402

crc32c.init_device(0)
total = 2 << 30
d = torch.empty(total + (1 << 20), dtype=torch.uint8, device="cuda")
diag.fill_splitmix(d, 11)


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


rng = np.random.Generator(np.random.PCG64(5))
cases = {
    "uniform_257_512": rng.integers(257, 513, size=total // 385),
    "fixed_431": np.full(total // 431, 431),
    "uniform_1_512": rng.integers(1, 513, size=total // 257),
    "fixed_512": np.full(total // 512, 512),
    "small_fixed_131": np.full(total // 262, 131),
    "small_uniform_1_256": rng.integers(1, 257, size=total // 258),
    "big_fixed_700": np.full(total // 700, 700),
    "big_uniform_513_1024": rng.integers(513, 1025, size=total // 770),
}
res = {}
only = os.environ.get("AB_CASES")
for name, sizes in cases.items():
    if only and not any(name.startswith(o) for o in only.split(",")):
        continue
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]) + 3
    d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, sizes))
    out = torch.empty(len(sizes), dtype=torch.int32, device="cuda")
    nbytes = int(sizes.sum()) + 20 * len(sizes)
    row = {}
    ref = None
    tags = ((("lanerec9", "256", 0), ("lanerec9_prefetch512", "256", 55), ("quadrec5", "256", 57))
            if name.startswith("small") else
            (("generic", None, 40), ("lanerec33", "1023", 0), 
             ("lanerec17_slow", "512", 0))
            if name.startswith("big") else
            (("lanerec17", "512", 0), ("lanerec17_2chains", "512", 54), ("lanerec17_prefetch256", "512", 56),
             ("quadrec9", "512", 58),
             ("generic", None, 40), ("lanerec9_slow", "256", 0)))
    for tag, hint, var in tags:
        ms = timeit(lambda: diag.batch_desc(var, d, d_blk, out=out, flags=_HINT_FLAGS[hint]))
        got = out.cpu().numpy().copy()
        ref = got if ref is None else ref
        row[tag] = {"ms": round(ms, 4), "GB/s": round(nbytes / ms / 1e6, 1), "same": bool((got == ref).all())}
    res[name] = row
    del d_blk, out
L, n = 431, total // 431
ms = timeit(lambda: diag.batch_fixed(0, d[3:], L, L, n))
res["fixed_stride_431"] = {"ms": round(ms, 4), "GB/s": round((n * L + 4 * n) / ms / 1e6, 1)}
print(json.dumps(res))
