#!/usr/bin/env python3
"""Cold-start transient per C2 kernel variant (the power manager's dip).

For each variant: let the GPU idle `--idle` s, then time `--n` back-to-back C2 launches (1M x 4 KiB)
with per-launch HIP events; report the mean over launches 5..25 (what `bench.py --warmup 5
--steps 20` times), over the last 20 (steady) and the worst launch.  Variants run in two passes,
the second in reverse order, so drift on the box does not favour one of them.  Variant 0 is the
shipped routing; -1 is the load-only pattern kernel (no CRC work).  Prints one JSON object.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c, diag  # noqa: E402

NBLK = 1 << 20


def timed(fn, n):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,-1,19,24,25")
    ap.add_argument("--idle", type=float, default=2.5)
    ap.add_argument("--n", type=int, default=80)
    a = ap.parse_args()
    crc32c.init_device(0)
    d = torch.empty(NBLK * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 301)
    out = torch.empty(NBLK, dtype=torch.int32, device="cuda")
    o = torch.zeros(1, dtype=torch.int32, device="cuda")
    vs = [int(x) for x in a.variants.split(",")]
    ref = None
    for v in vs:  # parity of every CRC variant against the shipped one (untimed)
        if v < 0:
            continue
        diag.batch_fixed(v, d, 4096, 4096, NBLK, out=out)
        torch.cuda.synchronize()
        x = out.cpu().numpy().copy()
        if ref is None:
            ref = x
        assert np.array_equal(x, ref), f"variant {v} differs"
    res = {}
    for order in (vs, vs[::-1]):
        for v in order:
            time.sleep(a.idle)
            fn = (lambda: diag.read_pattern4k(d, NBLK, 21, o)) if v < 0 else \
                (lambda v=v: diag.batch_fixed(v, d, 4096, 4096, NBLK, out=out))
            t = np.array(timed(fn, a.n))
            res.setdefault(str(v), []).append({"w5_25": round(float(t[5:25].mean()), 4),
                                               "last20": round(float(t[-20:].mean()), 4),
                                               "max": round(float(t.max()), 4),
                                               "first12": [round(float(x), 3) for x in t[:12]]})
            print(v, res[str(v)][-1], flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
