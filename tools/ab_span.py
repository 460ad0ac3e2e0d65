#!/usr/bin/env python3
"""tools/ab_span.py <variants> [workloads] [rounds] -- interleaved A/B of record-kernel variants.

Variants (comma list, diagnostics ids of pebblesdb_amd.diag.batch_desc; 0 = the shipped routing;
"<name>/<id>" = id in pebblesdb_amd/_lib/ab/libpdb_crc32c_diag_<name>.so, an earlier revision built
by tools/ab_base.sh, loaded beside the working tree's library) are timed round-robin on bench.py's WAL layouts (wal100 / wal400 / wal1000 / wal), after ~200 warm
launches (the power manager's cold transient), `rounds` rounds of 20 launches each,
the order reversed every other round.  Exact variants are checked against variant 0; pricing
variants (wrong CRCs by design: 113-117) are not.  GB/s = algorithmic bytes (record bytes + 16-B
descriptor + 4-B CRC) / mean launch time.  Prints one JSON line per workload."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import wal_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402

WL = {"wal100": (131, 1 << 30, crc32c.SIZE_256), "wal400": (431, 2 << 30, crc32c.SIZE_512),
      "wal700": (700, 2 << 30, crc32c.SIZE_1023), "wal1000": (1000, 2 << 30, crc32c.SIZE_1023),
      "wal": (1055, 4 << 30, crc32c.SIZE_1K),
      # records of random sizes (uniform in [lo, hi) B incl. the type byte, 7-B headers between)
      "rand300_500": ((300, 500), 2 << 30, crc32c.SIZE_512 | crc32c.SIZE_MIXED),
      "rand64_1000": ((64, 1000), 2 << 30, crc32c.SIZE_1023 | crc32c.SIZE_MIXED),
      "rand32_256": ((32, 256), 1 << 30, crc32c.SIZE_256), "rand1_512": ((1, 512), 2 << 30, crc32c.SIZE_512 | crc32c.SIZE_MIXED),
      "rand1000_1152": ((1000, 1152), 4 << 30, crc32c.SIZE_1K),
      "wal419": (419, 2 << 30, crc32c.SIZE_512), "wal463": (463, 2 << 30, crc32c.SIZE_512),
      "wal443": (443, 2 << 30, crc32c.SIZE_512), "wal800": (800, 2 << 30, crc32c.SIZE_1023),
      "wal900": (900, 2 << 30, crc32c.SIZE_1023)}


def layout(payload, nbytes):
    if isinstance(payload, tuple):
        rng = np.random.default_rng(7)
        lens = rng.integers(payload[0], payload[1], size=int(nbytes / (sum(payload) / 2 + 7)))
        offs = np.concatenate([[0], np.cumsum(lens + 7)[:-1]]) + 6
        return offs.astype(np.int64), lens.astype(np.int64)
    return wal_layout(nbytes, payload)
PRICING = {63, 64, 67, 113, 114, 115, 116, 117, 127, 128, 129, 130, 131, 132}
_ALT = {}


def run(tok, d, d_blk, hint, out):
    """One launch of variant token `tok` (an id, or "<name>/<id>" from an A/B library)."""
    if "/" not in str(tok):
        return diag.batch_desc(int(tok), d, d_blk, flags=hint, out=out)
    name, v = tok.split("/")
    if name not in _ALT:
        import ctypes
        L = ctypes.CDLL(os.path.join(os.path.dirname(diag.DIAG_LIB), "ab", f"libpdb_crc32c_diag_{name}.so"))
        res, args = diag.SIGNATURES["pdb_diag_batch_desc"]
        L.pdb_diag_batch_desc.restype, L.pdb_diag_batch_desc.argtypes = res, args
        _ALT[name] = L
    n = d_blk.numel() * d_blk.element_size() // 16
    diag.check(_ALT[name].pdb_diag_batch_desc(int(v), diag._ptr(d), diag._ptr(d_blk), n, hint, diag._ptr(out),
                                              diag._stream(None)))
    return out


def main():
    variants = sys.argv[1].split(",")
    wls = sys.argv[2].split(",") if len(sys.argv) > 2 else ["wal100", "wal400", "wal1000", "wal"]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    crc32c.init_device(0)
    for wl in wls:
        payload, nbytes, hint = WL[wl]
        offs, lens = layout(payload, nbytes)
        d = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d, payload if isinstance(payload, int) else 7 * payload[0] + payload[1])
        d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens))
        out = torch.empty(len(offs), dtype=torch.int32, device="cuda")
        algo = int(lens.sum()) + 20 * len(lens)
        ref = diag.batch_desc(0, d, d_blk, flags=hint).cpu().numpy()
        for v in variants:
            if int(v.split("/")[-1]) not in PRICING:
                got = run(v, d, d_blk, hint, out).cpu().numpy()
                assert (got == ref).all(), (wl, v, int(np.count_nonzero(got != ref)))
        for _ in range(200):
            run(variants[0], d, d_blk, hint, out)
        torch.cuda.synchronize()
        t = {v: [] for v in variants}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(rounds):
            for v in (variants if r % 2 == 0 else variants[::-1]):
                for _ in range(3):
                    run(v, d, d_blk, hint, out)
                e0.record()
                for _ in range(20):
                    run(v, d, d_blk, hint, out)
                e1.record()
                torch.cuda.synchronize()
                t[v].append(e0.elapsed_time(e1) / 20)
        res = {"workload": wl, "records": len(offs), "algo_bytes": algo}
        for v in variants:
            ms = float(np.mean(t[v]))
            res[v] = {"ms": round(ms, 4), "ms_min": round(float(np.min(t[v])), 4),
                           "GB/s": round(algo / (ms * 1e-3) / 1e9, 1), "frac": round(algo / (ms * 1e-3) / 8e12, 4)}
        print(json.dumps(res), flush=True)
        del d, d_blk, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
