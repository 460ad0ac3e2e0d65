#!/usr/bin/env python3
"""tools/long_block_cost.py -- what one long block (an index / filter block: 64 KiB .. 4 MiB) costs a
seal / verify batch of 16 MiB of 4-KiB blocks, with and without one long block:
  * host routes: pdb_sst_seal_host / pdb_sst_verify_host from pageable memory (the DMA route) and from
    pdb_host_alloc memory (zero-copy), wall-clock microseconds per call;
  * device route: pdb_sst_seal_device / _verify_device / _crc_device on the image in HBM (the
    long-block lane), kernel-side microseconds per call from HIP events around 50 back-to-back calls.
One JSON line per route and long-block size; the device lines also give the cost per MiB of the
batch relative to the batch without the long block.  --device-only skips the host routes (for a kernel
trace of the device route: tools/long_lane_trace.sh)."""
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
    import torch

    torch.cuda.set_device(0)  # torch's HIP initialisation first (the device route uses its tensors)
    crc32c.init_device(0)
    rows = []
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
        routes = () if "--device-only" in sys.argv else (("pageable", page.ctypes.data), ("pinned", p.value))
        for route, ptr in routes:
            seal = per_call(lambda: check(lib().pdb_sst_seal_host(ptr, total, h.ctypes.data, nblk)))
            ver = per_call(lambda: lib().pdb_sst_verify_host(ptr, total, h.ctypes.data, nblk, ok.ctypes.data))
            assert ok.all(), route
            print(json.dumps({"route": route, "long_block_KiB": long_kib, "bytes": total, "seal_us": round(seal, 1),
                              "verify_us": round(ver, 1)}), flush=True)
        assert (page == pin).all()
        check(lib().pdb_host_free(p))
        rows.append(device_route(page, h, total, nblk, long_kib))  # (the sealed image)
    base = rows[0]
    for r in rows:
        for k in ("seal_us", "verify_us", "crc_us"):
            r[k + "_per_MiB_vs_none"] = round((r[k] / (r["bytes"] / 2**20)) / (base[k] / (base["bytes"] / 2**20)), 3)
        print(json.dumps(r), flush=True)


def device_route(img, h, total, nblk, long_kib, reps=50):
    import torch

    from pebblesdb_amd import table as T

    d = torch.from_numpy(img).cuda()
    d_h = T.handles_to_device(h)
    ok = torch.empty(nblk, dtype=torch.uint8, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.empty(nblk, dtype=torch.int32, device="cuda")
    sp = int(torch.cuda.current_stream().cuda_stream)
    calls = {
        "seal_us": lambda: check(lib().pdb_sst_seal_device(d.data_ptr(), total, d_h.data_ptr(), nblk, sp)),
        "verify_us": lambda: check(lib().pdb_sst_verify_device(d.data_ptr(), total, d_h.data_ptr(), nblk, ok.data_ptr(),
                                                               nbad.data_ptr(), sp)),
        "crc_us": lambda: check(lib().pdb_sst_crc_device(d.data_ptr(), total, d_h.data_ptr(), nblk, out.data_ptr(), sp)),
    }
    row = {"route": "device", "long_block_KiB": long_kib, "bytes": total}
    for k, fn in calls.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        row[k] = round(s.elapsed_time(e) / reps * 1e3, 1)
    assert ok.cpu().numpy().all() and int(nbad.item()) == 0
    return row


if __name__ == "__main__":
    main()
