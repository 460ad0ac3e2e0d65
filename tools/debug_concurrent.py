#!/usr/bin/env python3
"""tools/debug_concurrent.py [rounds] -- record-kernel launches from 4 streams at once (as
tests/test_gpu_parity.py::test_record_batches_on_concurrent_streams), repeated; on a mismatch prints
the bad records grouped into 64-record batches (which units were lost or wrong)."""
import os
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from pebblesdb_amd import crc32c as crc, diag  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    crc.init_device(0)
    rng = np.random.Generator(np.random.PCG64(606))
    lens = rng.integers(300, 1000, size=60000)
    offs = np.concatenate([[6], 6 + np.cumsum(lens + 7)[:-1]])
    d = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 607)
    blk = crc.make_blocks(offs, lens)
    d_blk = crc.blocks_to_device(blk)
    exp = oracle.Oracle().batch(d.cpu().numpy(), blk, nthreads=8)
    torch.cuda.synchronize()
    nbad_total = 0
    for r in range(rounds):
        bad = []

        def run(k):
            st = torch.cuda.Stream()
            outs = [torch.full((len(lens),), -1, dtype=torch.int32, device="cuda") for _ in range(6)]
            torch.cuda.synchronize()
            with torch.cuda.stream(st):
                for o in outs:
                    crc.batch(d, d_blk, out=o, size_hint="1023", stream=st)
            st.synchronize()
            for j, o in enumerate(outs):
                g = o.cpu().numpy().view(np.uint32)
                w = np.nonzero(g != exp)[0]
                if w.size:
                    bad.append((k, j, w, g[w]))

        th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for k, j, w, vals in bad:
            nbad_total += 1
            b = np.unique(w // 64)
            print(f"round {r} thread {k} launch {j}: {w.size} bad records in batches {b[:20].tolist()}; "
                  f"untouched (-1): {int((vals == 0xFFFFFFFF).sum())}; first {w[:8].tolist()}", flush=True)
    print("bad launches:", nbad_total, "of", rounds * 24, flush=True)


if __name__ == "__main__":
    main()
