#!/usr/bin/env python3
"""tools/long_block_cost.py -- what one long block (an index / filter block: 64 KiB .. 4 MiB) costs a
host seal / verify batch: pdb_sst_seal_host and pdb_sst_verify_host on 16 MiB of 4-KiB blocks with and
without one long block, from pageable memory (the DMA route) and from pdb_host_alloc memory
(zero-copy).  One JSON line per route and long-block size: microseconds per call."""
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


def per_call(fn, reps=30):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    crc32c.init_device(0)
    nblk = (16 << 20) // 4175
    for long_kib in (0, 64, 400, 1300, 4096):
        sizes, offs, total = sst_layout(nblk, 5)
        sizes = sizes.copy()
        if long_kib:
            sizes[nblk // 2] = long_kib << 10
            offs = np.concatenate([[0], np.cumsum(sizes + 5)[:-1]]).astype(np.int64)
            total = int(offs[-1] + sizes[-1] + 5)
        img = np.random.default_rng(long_kib).integers(0, 256, size=total, dtype=np.uint8)
        img[offs + sizes] = 0
        h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
        h["offset"], h["size"] = offs, sizes
        p = ctypes.c_void_p()
        check(lib().pdb_host_alloc(total, ctypes.byref(p)))
        pin = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p.value))
        pin[:] = img
        page = img.copy()
        ok = np.zeros(nblk, dtype=np.uint8)
        for route, ptr in (("pageable", page.ctypes.data), ("pinned", p.value)):
            seal = per_call(lambda: check(lib().pdb_sst_seal_host(ptr, total, h.ctypes.data, nblk)))
            ver = per_call(lambda: lib().pdb_sst_verify_host(ptr, total, h.ctypes.data, nblk, ok.ctypes.data))
            assert ok.all(), route
            print(json.dumps({"route": route, "long_block_KiB": long_kib, "bytes": total, "seal_us": round(seal, 1),
                              "verify_us": round(ver, 1)}), flush=True)
        assert (page == pin).all()
        check(lib().pdb_host_free(p))


if __name__ == "__main__":
    main()
