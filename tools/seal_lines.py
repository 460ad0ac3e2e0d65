#!/usr/bin/env python3
"""tools/seal_lines.py [rounds] -- diagnostics: what the in-place seal's trailer stores cost, by how
they are written.  On bench.py's sst_seal image (1 M blocks of 4166-4174 B + type + trailer, HBM),
interleaved rounds of 20 launches each, after ~0.5 s of warm launches:

  seal                pdb_sst_seal_device (the product: hash + 4-B trailer stores, parked)
  140                 seal_pattern_kernel<0>: the seal's loads alone
  141                 + each trailer stored as 4 bytes (the product's store pattern)
  142 / 143           + instead the whole aligned 64-B / 128-B line holding each trailer, 16-B stores

One JSON line per kernel: ms per launch, and GB/s and % of 8 TB/s over the seal's algorithmic bytes
(contents + type + 4-B trailer + 16-B handle per block).  The pattern variants write wrong bytes by
design (the image is not checked)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import sst_layout  # noqa: E402
from pebblesdb_amd import crc32c, diag  # noqa: E402
from pebblesdb_amd import table as T  # noqa: E402
from pebblesdb_amd._native import check, lib  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    crc32c.init_device(0)
    nblk = 1 << 20
    sizes, offs, total = sst_layout(nblk, 301)
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    diag.fill_splitmix(data, 301)
    data[torch.from_numpy(offs + sizes).to(dev)] = 0
    h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d_h = T.handles_to_device(h, dev)
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    algo = int((sizes + 1).sum()) + nblk * (4 + 16)
    runs = {
        "seal": lambda: check(lib().pdb_sst_seal_device(data.data_ptr(), total, d_h.data_ptr(), nblk, sp)),
        "140 loads": lambda: diag.sst(140, data, d_h, seal=True, stream=stream),
        "141 loads + 4-B trailer stores": lambda: diag.sst(141, data, d_h, seal=True, stream=stream),
        "142 loads + 64-B line stores": lambda: diag.sst(142, data, d_h, seal=True, stream=stream),
        "143 loads + 128-B line stores": lambda: diag.sst(143, data, d_h, seal=True, stream=stream),
    }
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for fn in runs.values():
            fn()
        torch.cuda.synchronize()
    ms = {k: [] for k in runs}
    names = list(runs)
    for r in range(rounds):
        for k in (names if r % 2 == 0 else names[::-1]):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(20):
                runs[k]()
            e.record(stream)
            torch.cuda.synchronize()
            ms[k].append(s.elapsed_time(e) / 20)
    for k in names:
        m = float(np.median(ms[k]))
        gbs = algo / (m * 1e-3) / 1e9
        print(json.dumps({"kernel": k, "ms": round(m, 4), "GB/s": round(gbs, 1), "frac": round(gbs / 8000, 4),
                          "ms_all": [round(x, 4) for x in ms[k]]}), flush=True)


if __name__ == "__main__":
    main()
