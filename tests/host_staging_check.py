"""Child-process check for tests/test_gpu_parity.py::test_host_staging_small_groups_subprocess.

Run with PDB_HOST_CHUNK_BYTES set (the product reads it once per process): the host batch, verify,
seal and sstable-verify entry points must give the reference's answers however small the staging
groups are.  Checked against the golden vectors (generated from the reference's util/crc32c.cc)
and the sstable files the reference's TableBuilder wrote.  Prints "host staging ok".
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
from pebblesdb_amd import crc32c as crc  # noqa: E402
from pebblesdb_amd import table as T  # noqa: E402


def golden_batches():
    with open(os.path.join(HERE, "golden", "crc32c_golden.json")) as f:
        g = json.load(f)
    for b in g["batches"]:
        if b["total_bytes"] > (64 << 20):
            continue
        base = oracle.splitmix_bytes(b["total_bytes"], b["seed"])
        use_init = b["use_init"]
        blk = crc.make_blocks(b["off"], b["len"], b["init"] if use_init else None)
        exp = np.array(b["crc"], dtype=np.uint64).astype(np.uint32)
        got = crc.batch_host(base, blk, use_init=use_init)
        assert (got == exp).all(), b["name"]
        bad = exp.copy()
        flip = np.arange(0, len(bad), 7)
        bad[flip] ^= 1
        ok, nbad = crc.verify_host(base, blk, bad, masked=False, use_init=use_init)
        assert nbad == len(flip) and (ok[flip] == 0).all() and ok.sum() == len(bad) - len(flip), b["name"]


def reference_tables():
    sst = os.path.join(HERE, "golden", "sst")
    with open(os.path.join(sst, "manifest.json")) as f:
        names = [t["file"] for t in json.load(f)["tables"]]
    for name in names:
        with open(os.path.join(sst, name), "rb") as f:
            img = f.read()
        lay = T.table_layout(img, verify_checksums=False)
        hs = sorted(lay.all_handles(), key=lambda h: h.offset)
        w = T.TableBlockWriter()
        for h in hs:
            contents, typ = T.read_block(img, h, verify_checksums=False)
            w.add(contents, typ)
        w.seal()
        assert w.data + img[-T.K_FOOTER_ENCODED_LENGTH:] == img, name
        assert T.verify_blocks(img, hs).all(), name
        bad = bytearray(img)
        victims = list(range(0, len(hs), 3))
        for v in victims:
            bad[hs[v].offset] ^= 0x01
        ok = T.verify_blocks(bytes(bad), hs)
        assert [i for i in range(len(hs)) if not ok[i]] == victims, name


if __name__ == "__main__":
    crc.init_device(0)
    golden_batches()
    reference_tables()
    print("host staging ok (PDB_HOST_CHUNK_BYTES=%s)" % os.environ.get("PDB_HOST_CHUNK_BYTES"))
