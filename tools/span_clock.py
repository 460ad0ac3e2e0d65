#!/usr/bin/env python3
"""tools/span_clock.py [workloads] [rounds] -- the record kernel's shader clock, product vs its parts.

Diagnostics variants 180 / 181 / 182 are the shipped crc_lanespan_kernel, its loads + LDS staging
alone, and its hash alone (MODE 40 / 41 / 42), each wave stamping [start, end] in s_memrealtime
(100 MHz) and s_memtime (shader clock).  After ~200 warm launches of the product, the three are
launched round-robin; per launch: the kernel span (first wave start -> last wave end), the mean
per-wave clock (s_memtime ticks / s_memrealtime time over the wave's life) and the tail (the last
wave end minus the median wave end).  Tells whether the product is slower than max(loads, hash)
because the clock drops when both run (power) or for another reason at the same clock."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import wal_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402

WL = {"wal100": (131, 1 << 30, crc32c.SIZE_256), "wal400": (431, 2 << 30, crc32c.SIZE_512),
      "wal1000": (1000, 2 << 30, crc32c.SIZE_1023), "wal": (1055, 4 << 30, crc32c.SIZE_1K)}
NAMES = {180: "product", 181: "loads_only", 182: "hash_only"}


def one(v, d, d_blk, hint, out, n):
    out.zero_()
    diag.batch_desc(v, d, d_blk, flags=hint, out=out)
    torch.cuda.synchronize()
    st = out[((n + 1) & ~1):].cpu().numpy().view(np.uint64).reshape(-1, 4)
    st = st[st[:, 1] > 0].astype(np.float64)
    t0, t1, c0, c1 = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
    life = (t1 - t0) * 10e-9  # s
    mhz = (c1 - c0) / np.maximum(life, 1e-9) / 1e6
    span_ms = (t1.max() - t0.min()) * 10e-6
    end = (t1 - t0.min()) * 10e-6  # ms after the first wave start
    nw = len(st) // 256 if len(st) % 256 == 0 else 0  # waves per workgroup (one workgroup per CU)
    wg_end = end.reshape(256, nw).max(axis=1) if nw else end
    xcd = [float(np.mean(wg_end[x::8])) for x in range(8)] if nw else []
    return {"span_ms": span_ms, "end_mean_ms": float(np.mean(end)), "end_p50_ms": float(np.median(end)),
            "end_p90_ms": float(np.percentile(end, 90)), "wg_end_p10_ms": float(np.percentile(wg_end, 10)),
            "wg_end_p50_ms": float(np.median(wg_end)), "xcd_wg_end_min_ms": min(xcd) if xcd else 0.0,
            "xcd_wg_end_max_ms": max(xcd) if xcd else 0.0,
            "mhz_mean": float(np.mean(mhz)), "mhz_p10": float(np.percentile(mhz, 10)),
            "tail_ms": float((t1.max() - np.median(t1)) * 10e-6), "start_ramp_ms": float((np.median(t0) - t0.min()) * 10e-6),
            "waves": int(len(st))}


def main():
    wls = sys.argv[1].split(",") if len(sys.argv) > 1 else ["wal1000", "wal100"]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    crc32c.init_device(0)
    for wl in wls:
        payload, nbytes, hint = WL[wl]
        offs, lens = wal_layout(nbytes, payload)
        d = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d, payload)
        d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens))
        n = len(offs)
        out = torch.zeros(((n + 1) & ~1) + 2 * 4 * 8192, dtype=torch.int32, device="cuda")
        ref = diag.batch_desc(0, d, d_blk, flags=hint).cpu().numpy()
        got = diag.batch_desc(180, d, d_blk, flags=hint, out=out)[:n].cpu().numpy()
        assert (got == ref).all(), "variant 180 CRCs differ from the product"
        for _ in range(200):
            diag.batch_desc(0, d, d_blk, flags=hint)
        torch.cuda.synchronize()
        acc = {v: [] for v in NAMES}
        for r in range(rounds):
            for v in (list(NAMES) if r % 2 == 0 else list(NAMES)[::-1]):
                for _ in range(3):
                    diag.batch_desc(v, d, d_blk, flags=hint, out=out)
                acc[v].append(one(v, d, d_blk, hint, out, n))
        res = {"workload": wl, "records": n}
        for v, name in NAMES.items():
            res[name] = {k: round(float(np.mean([x[k] for x in acc[v]])), 4) for k in acc[v][0]}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
