#!/usr/bin/env python3
"""tools/ab_pattern.py [variants] [rounds] -- the 4-KiB kernel's loads with no hash (pdb_diag_read_pattern4k):
variant 21 (the C2 kernel's static, grid-interleaved block assignment) against 23 (64-block chunks
from device-wide per-XCD queues), interleaved after ~200 warm launches, both orders, on C2's 4 GiB.
Prints one JSON line: mean / min ms per launch and GB/s (4096 B read per block)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c, diag  # noqa: E402


def main():
    variants = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "21,23").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    nblk = 1 << 20
    crc32c.init_device(0)
    d = torch.empty(nblk * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 301)
    o = torch.zeros(1, dtype=torch.int32, device="cuda")
    ref = None
    for v in variants:  # every variant reads every byte: the XOR of all loads must agree
        o.zero_()
        diag.read_pattern4k(d, nblk, v, o)
        x = int(o.item())
        assert ref is None or x == ref, (v, x, ref)
        ref = x
    for _ in range(200):
        diag.read_pattern4k(d, nblk, variants[0], o)
    torch.cuda.synchronize()
    t = {v: [] for v in variants}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            for _ in range(3):
                diag.read_pattern4k(d, nblk, v, o)
            e0.record()
            for _ in range(20):
                diag.read_pattern4k(d, nblk, v, o)
            e1.record()
            torch.cuda.synchronize()
            t[v].append(e0.elapsed_time(e1) / 20)
    res = {}
    for v in variants:
        ms = float(np.mean(t[v]))
        res[str(v)] = {"ms": round(ms, 4), "ms_min": round(float(np.min(t[v])), 4),
                       "GB/s": round(nblk * 4096 / (ms * 1e-3) / 1e9, 1), "frac": round(nblk * 4096 / (ms * 1e-3) / 8e12, 4)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
