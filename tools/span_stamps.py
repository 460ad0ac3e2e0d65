#!/usr/bin/env python3
"""tools/span_stamps.py [workload ...] -- where the record kernel's time goes between waves.

Runs diagnostics variants 110 / 112 (the shipped crc_lanespan_kernel / the round-2 static batch
assignment, + per-wave s_memrealtime stamps: start, end, items hashed, batches opened) on bench.py's
WAL layouts and prints, per workload, one JSON line: interleaved HIP-event timings of the product
(variant 0) and the static form (111), and for both stamped forms the kernel span from the first
wave start to the last wave end, the mean wave lifetime as a fraction of that span (the 'resident'
share: what the SQ counters' SQ_WAVE_CYCLES / GRBM ratio shows), the start ramp and the end tail
(percentiles of wave start / end offsets), and the spread of work per wave.  Every variant's CRCs
are checked against the product's."""
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
TICK_NS = 10.0  # s_memrealtime: 100 MHz


def run(wl: str, reps: int = 20) -> dict:
    payload, nbytes, hint = WL[wl]
    offs, lens = wal_layout(nbytes, payload)
    d = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, payload)
    d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens))
    n = len(offs)
    nst = 4 * 8192  # 4 words x up to 8192 waves
    out = torch.zeros(((n + 1) & ~1) + 2 * nst, dtype=torch.int32, device="cuda")
    ref = diag.batch_desc(0, d, d_blk, flags=hint)
    refh = ref.cpu().numpy()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {}
    scratch = torch.zeros_like(ref)
    for v in (0, 111, 0, 111, 0, 111):  # product (workgroup counter) vs the round-2 static assignment
        for _ in range(5):
            diag.batch_desc(v, d, d_blk, flags=hint, out=scratch)
        ev[0].record()
        for _ in range(reps):
            diag.batch_desc(v, d, d_blk, flags=hint, out=scratch)
        ev[1].record()
        torch.cuda.synchronize()
        times.setdefault(v, []).append(round(ev[0].elapsed_time(ev[1]) / reps, 4))
        assert (scratch.cpu().numpy() == refh).all(), f"variant {v} CRCs differ from the product"
    res = {"workload": wl, "records": n, "kernel_ms_events": {"v0_dyn": times[0], "v111_static": times[111]}}
    for v, name in ((110, "dyn"), (112, "static")):
        out.zero_()
        for _ in range(3):
            diag.batch_desc(v, d, d_blk, flags=hint, out=out)
        torch.cuda.synchronize()
        assert (out[:n].cpu().numpy() == refh).all(), f"variant {v} CRCs differ from the product"
        st = out[((n + 1) & ~1):].cpu().numpy().view(np.uint64).reshape(-1, 4)
        st = st[st[:, 1] > 0].astype(np.float64)
        t0, t1 = st[:, 0].min(), st[:, 1].max()
        span = t1 - t0
        life = st[:, 1] - st[:, 0]
        pct = lambda a, q: round(float(np.percentile(a, q)) * TICK_NS / 1e3, 2)  # noqa: E731  (us)
        res[name] = {
            "waves": int(len(st)),
            "span_us": round(span * TICK_NS / 1e3, 2),
            "resident_frac": round(float(life.mean() / span), 4),
            "start_offset_us_p50_p90_max": [pct(st[:, 0] - t0, 50), pct(st[:, 0] - t0, 90), pct(st[:, 0] - t0, 100)],
            "end_offset_us_min_p10_p50": [pct(st[:, 1] - t0, 0), pct(st[:, 1] - t0, 10), pct(st[:, 1] - t0, 50)],
            "items_per_wave_min_mean_max": [int(st[:, 2].min()), round(float(st[:, 2].mean()), 2), int(st[:, 2].max())],
            "batches_per_wave_min_max": [int(st[:, 3].min()), int(st[:, 3].max())],
            "us_per_item_mean": round(float((life / np.maximum(st[:, 2], 1)).mean()) * TICK_NS / 1e3, 3),
        }
    return res


def main():
    crc32c.init_device(0)
    for wl in (sys.argv[1:] or ["wal100", "wal400", "wal1000", "wal"]):
        print(json.dumps(run(wl)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
