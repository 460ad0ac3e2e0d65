#!/usr/bin/env python3
"""tools/seal_gaps.py -- the zero-copy seal (pdb_sst_seal_host on pdb_host_alloc memory) of 0.6 /
4 / 16-MiB sstable batches after 0..500 ms of idle GPU, 10 calls per gap: does the GPU's idle state
explain the engine's slow small seals?  Run with PDB_SEAL_STAMPS=<csv> for the kernels' own times
(tools/seal_stamps.py); prints one JSON line per batch size with the mean call time per gap."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import sst_layout  # noqa: E402
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd._native import check, lib  # noqa: E402


def main():
    crc32c.init_device(0)
    gaps = [0, 1, 5, 20, 50, 100, 200, 500]
    for kib in (600, 4096, 16384):
        nblk = max(1, (kib << 10) // 4175)
        sizes, offs, total = sst_layout(nblk, 77 + kib)
        img = np.random.default_rng(kib).integers(0, 256, size=total, dtype=np.uint8)
        img[offs + sizes] = 0
        h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
        h["offset"], h["size"] = offs, sizes
        p = ctypes.c_void_p()
        check(lib().pdb_host_alloc(total, ctypes.byref(p)))
        pin = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p.value))
        pin[:] = img
        res = {"batch_KiB": kib, "bytes": total}
        for g in gaps:
            ts = []
            for _ in range(10):
                time.sleep(g * 1e-3)
                t0 = time.perf_counter()
                check(lib().pdb_sst_seal_host(p.value, total, h.ctypes.data, nblk))
                ts.append(time.perf_counter() - t0)
            res[f"gap{g}ms_us"] = round(float(np.mean(ts)) * 1e6, 1)
        print(json.dumps(res), flush=True)
        check(lib().pdb_host_free(p))


if __name__ == "__main__":
    main()
