#!/usr/bin/env python3
"""tools/seal_batches.py [MiB,...] -- the engine's seal call (pdb_sst_seal_host) on sstable batches of
4 / 16 / 32 MiB (the TableBuilder's PDB_SEAL_BATCH_BYTES), against the bare H2D copy of the same
bytes, from page-locked staging (pdb_host_alloc, what integration/pdb_table_builder.cc stages in) and
from pageable memory; and the zero-copy form: the device seal kernel run directly on the page-locked
batch through its device mapping (hipHostGetDevicePointer), the trailers written in place across
PCIe, no DMA.  Also the conditions of the engine's seals: the batch freshly written by the CPU,
8 batches in rotation, a new allocation per batch, 1 / 5 / 20 ms of idle GPU between seals.  argv[2]:
run on that NUMA node's CPUs.  Every form's image must equal the host seal's.  One JSON line per
batch size.  argv[3] (e.g. "0,2,4,8"): the seal of the pinned batch again with that many host
threads copying 256-MiB arrays in the background (the engine's compaction and page-cache traffic as
host-memory load)."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import sst_layout  # noqa: E402
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd._native import check, lib  # noqa: E402

GIB = float(1 << 30)
hip = ctypes.CDLL("libamdhip64.so")


def pinned(nbytes: int):
    p = ctypes.c_void_p()
    check(lib().pdb_host_alloc(nbytes, ctypes.byref(p)))
    return p.value, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))


def dev_ptr(host_ptr: int) -> int:
    d = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(host_ptr), 0)
    if rc != 0:
        raise RuntimeError(f"hipHostGetDevicePointer rc={rc}")
    return d.value


def per_call(fn, reps: int) -> float:
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def node_cpus(node: int):
    out = set()
    for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def copy_load_rates(total: int, p_img: int, h, nblk: int, counts):
    """Seals of one pinned batch while `n` host threads copy 256-MiB arrays (numpy releases the GIL)."""
    import threading
    out = {}
    for n in counts:
        stop = threading.Event()
        copied = [0] * n

        def worker(i):
            a = np.ones(256 << 20, dtype=np.uint8)
            b = np.empty_like(a)
            while not stop.is_set():
                np.copyto(b, a)
                copied[i] += a.nbytes
        ths = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
        for t in ths:
            t.start()
        time.sleep(0.5 if n else 0.0)
        c0, t0 = sum(copied), time.perf_counter()
        reps = 200
        for _ in range(reps):
            check(lib().pdb_sst_seal_host(p_img, total, h.ctypes.data, nblk))
        dt = time.perf_counter() - t0
        c1 = sum(copied)
        stop.set()
        for t in ths:
            t.join()
        out[n] = {"seal_GiB_s": round(total * reps / dt / GIB, 2), "host_copy_GiB_s": round((c1 - c0) / dt / GIB, 1)}
    return out


def main():
    sizes_mib = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,16,32").split(",")]
    node = int(sys.argv[2]) if len(sys.argv) > 2 else -1  # run (and page-lock) on this NUMA node's CPUs
    if node >= 0:
        os.sched_setaffinity(0, node_cpus(node) & os.sched_getaffinity(0) or node_cpus(node))
    crc32c.init_device(0)
    bus = torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0), "pci_bus_id") else -1
    stream = torch.cuda.Stream()
    sp = int(stream.cuda_stream)
    for mib in sizes_mib:
        nblk = max(1, (mib << 20) // 4175)
        sizes, offs, total = sst_layout(nblk, 401 + mib)
        rng = np.random.Generator(np.random.PCG64(mib))
        img = rng.integers(0, 256, size=total, dtype=np.uint8)
        img[offs + sizes] = 0  # kNoCompression type bytes
        h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
        h["offset"], h["size"] = offs, sizes
        ref = img.copy()
        check(lib().pdb_sst_seal_host(ref.ctypes.data, total, h.ctypes.data, nblk))
        p_img, pin = pinned(total)
        p_h, pin_h = pinned(h.nbytes)
        pin_h[:] = h.view(np.uint8)
        res = {"batch_MiB": mib, "blocks": nblk, "bytes": total, "cpu_node": node, "gpu_pci_bus": bus}
        reps = max(20, 2000 // mib)

        def host_seal(arr):
            return lambda: check(lib().pdb_sst_seal_host(arr.ctypes.data, total, h.ctypes.data, nblk))

        for name, arr in (("seal_host_pinned", pin), ("seal_host_pageable", img.copy())):
            arr[:] = img
            dt = per_call(host_seal(arr), reps)
            assert (arr == ref).all(), name
            res[name] = {"us_per_call": round(dt * 1e6, 1), "GiB_s": round(total / dt / GIB, 2)}
        # zero-copy: the seal kernel reads the batch and writes its trailers through the mapping
        d_img, d_h = dev_ptr(p_img), dev_ptr(p_h)
        pin[:] = img

        def zero_copy():
            check(lib().pdb_sst_seal_device(ctypes.c_void_p(d_img), total, ctypes.c_void_p(d_h), nblk, ctypes.c_void_p(sp)))
            stream.synchronize()

        dt = per_call(zero_copy, reps)
        assert (pin == ref).all(), "zero-copy seal differs from the host seal"
        res["seal_zero_copy"] = {"us_per_call": round(dt * 1e6, 1), "GiB_s": round(total / dt / GIB, 2)}
        # the engine's case: the batch was just written by the CPU (its lines dirty in the CPU caches)
        tot = 0.0
        for _ in range(reps):
            pin[:] = img
            t0 = time.perf_counter()
            zero_copy()
            tot += time.perf_counter() - t0
        assert (pin == ref).all()
        res["seal_zero_copy_fresh"] = {"us_per_call": round(tot / reps * 1e6, 1), "GiB_s": round(total * reps / tot / GIB, 2)}
        tot = 0.0
        for _ in range(reps):
            pin[:] = img
            t0 = time.perf_counter()
            check(lib().pdb_sst_seal_host(pin.ctypes.data, total, h.ctypes.data, nblk))
            tot += time.perf_counter() - t0
        res["seal_host_pinned_fresh"] = {"us_per_call": round(tot / reps * 1e6, 1), "GiB_s": round(total * reps / tot / GIB, 2)}
        # rotating over 8 page-locked batches (a builder per table, the allocations kept for reuse)
        bufs = [pinned(total) for _ in range(8)]
        for _, b_ in bufs:
            b_[:] = img
        tot = 0.0
        for k in range(reps):
            p_, b_ = bufs[k % 8]
            b_[:] = img
            t0 = time.perf_counter()
            check(lib().pdb_sst_seal_host(p_, total, h.ctypes.data, nblk))
            tot += time.perf_counter() - t0
        res["seal_host_pinned_rot8"] = {"us_per_call": round(tot / reps * 1e6, 1), "GiB_s": round(total * reps / tot / GIB, 2)}
        # the engine's cadence: one seal every few milliseconds, the GPU idle in between
        for gap_ms in (1, 5, 20):
            tot = 0.0
            for k in range(min(reps, 40)):
                time.sleep(gap_ms * 1e-3)
                t0 = time.perf_counter()
                check(lib().pdb_sst_seal_host(p_img, total, h.ctypes.data, nblk))
                tot += time.perf_counter() - t0
            res[f"seal_host_pinned_gap{gap_ms}ms"] = {"us_per_call": round(tot / min(reps, 40) * 1e6, 1),
                                                     "GiB_s": round(total * min(reps, 40) / tot / GIB, 2)}
        # a new page-locked allocation per batch
        tot = 0.0
        for k in range(min(reps, 20)):
            p_, b_ = pinned(total + 4096 * (k + 1))  # (never a kept allocation)
            b_[:total] = img
            t0 = time.perf_counter()
            check(lib().pdb_sst_seal_host(p_, total, h.ctypes.data, nblk))
            tot += time.perf_counter() - t0
        res["seal_host_pinned_new"] = {"us_per_call": round(tot / min(reps, 20) * 1e6, 1),
                                       "GiB_s": round(total * min(reps, 20) / tot / GIB, 2)}
        # the bare copy of the same bytes (pinned -> device), the DMA ceiling of the host form
        d = torch.empty(total, dtype=torch.uint8, device="cuda")
        src = torch.from_numpy(pin)

        def h2d():
            with torch.cuda.stream(stream):
                d.copy_(src, non_blocking=True)
            stream.synchronize()

        dt = per_call(h2d, reps)
        res["h2d_pinned"] = {"us_per_call": round(dt * 1e6, 1), "GiB_s": round(total / dt / GIB, 2)}
        if len(sys.argv) > 3:
            res["under_host_copies"] = copy_load_rates(total, p_img, h, nblk, [int(x) for x in sys.argv[3].split(",")])
        print(json.dumps(res), flush=True)
        check(lib().pdb_host_free(ctypes.c_void_p(p_img)))
        check(lib().pdb_host_free(ctypes.c_void_p(p_h)))


if __name__ == "__main__":
    main()
