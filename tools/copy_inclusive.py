#!/usr/bin/env python3
"""Copy-inclusive rates: sstable blocks that start and end in host memory (BASELINE.json north
star: "the rate including H2D/D2H copies is also measured").  1 GiB of the C2 blocks and of the
sstable layout, through the host entry points (H2D + kernel + D2H on the library's stream):

  batch_host pageable / pinned  pdb_crc32c_batch_host: CRCs of 4-KiB blocks into a host array
  seal_host                     pdb_sst_seal_host: trailers of an sstable image (4 B per block back)
  verify_host                   pdb_sst_verify_host: ReadBlock's check over every handle
  h2d pageable / pinned         torch copy of the same bytes only (the PCIe ceiling)

Every CRC is checked against the oracle on a sample.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402  (checker only)
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import diag  # noqa: E402
from pebblesdb_amd._native import lib  # noqa: E402

GIB = float(1 << 30)
NBLK = 1 << 18


def timed(fn, reps=5):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def main():
    crc32c.init_device(0)
    o = oracle.Oracle()
    res = {"metric": "copy-inclusive GiB/s (host-resident blocks)", "blocks": NBLK}
    # C2 blocks, pageable and pinned
    d = torch.empty(NBLK * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 301)
    page = d.cpu().numpy()
    pin_t = torch.empty(NBLK * 4096, dtype=torch.uint8, pin_memory=True)
    pin_t.copy_(d)
    pin = pin_t.numpy()
    blk = crc32c.make_blocks(np.arange(NBLK) * 4096, np.full(NBLK, 4096))
    exp = o.batch(page[: 4096 * 4096], blk[:4096])
    for name, host in (("batch_host_pageable", page), ("batch_host_pinned", pin)):
        got = crc32c.batch_host(host, blk)
        assert (got[:4096] == exp).all(), name
        dt = timed(lambda: crc32c.batch_host(host, blk))
        res[name] = round(NBLK * 4096 / dt / GIB, 2)
    for name, src in (("h2d_pageable", torch.from_numpy(page)), ("h2d_pinned", pin_t)):
        def cp():
            d.copy_(src, non_blocking=False)
            torch.cuda.synchronize()
        res[name] = round(NBLK * 4096 / timed(cp) / GIB, 2)
    # sstable image: contents 4096 B + type byte + 4-B trailer, stride 4101
    L, stride = 4096, 4101
    img_d = torch.empty(NBLK * stride, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(img_d, 302)
    img = img_d.cpu().numpy().copy()
    img[L::stride] = 0  # type byte kNoCompression
    h = np.zeros(NBLK, dtype=[("offset", "<u8"), ("size", "<u8")])
    h["offset"] = np.arange(NBLK, dtype=np.uint64) * stride
    h["size"] = L

    def seal():
        return lib().pdb_sst_seal_host(img.ctypes.data, img.size, h.ctypes.data, NBLK)

    assert seal() == 0
    chk = o.batch(img[: 64 * stride], crc32c.make_blocks(np.arange(64) * stride, np.full(64, L + 1)), flags=1)
    tr = img[: 64 * stride].reshape(64, stride)[:, L + 1 : L + 5].copy().view("<u4").reshape(-1)
    assert (tr == chk).all(), "sealed trailers differ from the oracle"
    res["seal_host"] = round(NBLK * (L + 1) / timed(seal) / GIB, 2)
    ok = np.zeros(NBLK, dtype=np.uint8)

    def verify():
        return lib().pdb_sst_verify_host(img.ctypes.data, img.size, h.ctypes.data, NBLK, ok.ctypes.data)

    assert verify() == 0 and ok.all()
    res["verify_host"] = round(NBLK * (L + 1) / timed(verify) / GIB, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
