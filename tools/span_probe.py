#!/usr/bin/env python3
"""tools/span_probe.py <variant> <workload> [reps] -- run one diagnostics variant of the descriptor
path (pebblesdb_amd.diag.batch_desc) on a bench.py WAL layout `reps` times (for rocprofv3 --pmc
passes over the record kernel's modes: tools/counters_probe.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import wal_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402

WL = {"wal100": (131, 1 << 30, crc32c.SIZE_256), "wal400": (431, 2 << 30, crc32c.SIZE_512),
      "wal700": (700, 2 << 30, crc32c.SIZE_1023), "wal1000": (1000, 2 << 30, crc32c.SIZE_1023)}


def main():
    v, wl = int(sys.argv[1]), sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    payload, nbytes, hint = WL[wl]
    crc32c.init_device(0)
    offs, lens = wal_layout(nbytes, payload)
    d = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, payload)
    d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens))
    out = torch.empty(len(offs), dtype=torch.int32, device="cuda")
    for _ in range(reps):
        diag.batch_desc(v, d, d_blk, flags=hint, out=out)
    torch.cuda.synchronize()
    print("ok", v, wl, reps, flush=True)


if __name__ == "__main__":
    main()
