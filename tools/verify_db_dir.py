"""Check every CRC in a PebblesDB directory: sstable block trailers (table/format.cc:96-98,
format.cc:97-108) and WAL / MANIFEST physical records (log_writer.cc:121, log_reader.cc:237).

Used by tools/dbbench_demo.sh after the reference's own db_bench, rebuilt with util/crc32c.h
bound to libpdb_crc32c.so (oracle/build_ref_dbbench.sh), has written a database through the GPU:
the oracle (CPU, test infrastructure) re-checks every checksum the GPU produced, and with --gpu
the batched GPU verifiers (pebblesdb_amd.table.verify_table / log.verify_log) must agree.
Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import Oracle  # noqa: E402
from pebblesdb_amd import log as L  # noqa: E402
from pebblesdb_amd import table as T  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--gpu", action="store_true", help="also run the batched GPU verifiers")
    a = ap.parse_args()
    orc = Oracle()
    res = {"db": a.db, "tables": 0, "tables_incomplete": 0, "blocks": 0, "blocks_bad_oracle": 0, "logs": 0, "records": 0,
           "records_bad_oracle": 0, "blocks_bad_gpu": None, "records_bad_gpu": None, "bytes": 0}
    if a.gpu:
        from pebblesdb_amd import crc32c

        crc32c.init_device(0)
        res["blocks_bad_gpu"] = res["records_bad_gpu"] = 0
    for name in sorted(os.listdir(a.db)):
        path = os.path.join(a.db, name)
        img = open(path, "rb").read()
        if name.endswith(".sst") or name.endswith(".ldb"):
            try:
                lay = T.table_layout(img, verify_checksums=False)
            except T.Corruption:  # no footer: a table still being written when the process exited
                res["tables_incomplete"] += 1
                continue
            hs = lay.all_handles()
            u8 = np.frombuffer(img, dtype=np.uint8)
            offs = np.array([h.offset for h in hs], dtype=np.int64)
            sizes = np.array([h.size for h in hs], dtype=np.int64)
            tr = offs + sizes + 1
            stored = (u8[tr].astype(np.uint32) | (u8[tr + 1].astype(np.uint32) << 8) |
                      (u8[tr + 2].astype(np.uint32) << 16) | (u8[tr + 3].astype(np.uint32) << 24))
            blk = np.zeros(len(hs), dtype=[("off", "<u8"), ("len", "<u4"), ("init", "<u4")])
            blk["off"], blk["len"] = offs, sizes + 1  # contents || type
            res["blocks_bad_oracle"] += int((orc.batch(u8, blk, flags=1, nthreads=8) != stored).sum())
            if a.gpu:
                res["blocks_bad_gpu"] += int((T.verify_table(img)[1] == 0).sum())
            res["tables"] += 1
            res["blocks"] += len(hs)
        elif name.endswith(".log") or name.startswith("MANIFEST-"):
            recs = L.physical_records(img)
            if recs:
                blk = np.zeros(len(recs), dtype=[("off", "<u8"), ("len", "<u4"), ("init", "<u4")])
                blk["off"] = [r.offset + 6 for r in recs]  # type || payload
                blk["len"] = [1 + r.length for r in recs]
                stored = np.array([r.stored for r in recs], dtype=np.uint32)
                res["records_bad_oracle"] += int((orc.batch(np.frombuffer(img, dtype=np.uint8), blk, flags=1,
                                                            nthreads=8) != stored).sum())
            if a.gpu and recs:
                res["records_bad_gpu"] += int((L.verify_log(img)[1] == 0).sum())
            res["logs"] += 1
            res["records"] += len(recs)
        else:
            continue
        res["bytes"] += len(img)
    print(json.dumps(res), flush=True)
    bad = res["blocks_bad_oracle"] + res["records_bad_oracle"] + (res["blocks_bad_gpu"] or 0) + (
        res["records_bad_gpu"] or 0)
    return 1 if bad or res["blocks"] == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
