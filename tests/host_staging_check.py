"""Child-process check for tests/test_gpu_parity.py::test_host_staging_small_groups_subprocess.

Run with PDB_HOST_CHUNK_BYTES set (the product reads it once per process): the host batch, verify,
seal and sstable-verify entry points must give the reference's answers however small the staging
groups are, long (index / filter sized) blocks included.  Checked against the golden vectors (generated from the reference's util/crc32c.cc)
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


def long_blocks():
    """Index- and filter-sized blocks (16 KiB .. 1.3 MiB) among 4-KiB ones, from pageable memory
    (the DMA route: 0-byte stand-ins in the sst kernel, the blocks by span launches), every trailer
    against the oracle, then verify with corrupted long and short blocks."""
    import ctypes

    from pebblesdb_amd._native import check, lib
    orc = oracle.Oracle()
    rng = np.random.Generator(np.random.PCG64(53))
    sizes = rng.integers(4166, 4175, size=120).tolist()
    for i, z in enumerate([16384, 16383, 70001, 1363149, 4096 * 9]):
        sizes.insert(7 + 23 * i, z)
    sizes = np.array(sizes, dtype=np.int64)
    offs = np.concatenate([[9], 9 + np.cumsum(sizes + 5)[:-1]]).astype(np.int64)
    total = int(offs[-1] + sizes[-1] + 5) + 7
    img = oracle.splitmix_bytes(total, 29).copy()
    img[offs + sizes] = rng.integers(0, 2, size=len(sizes))
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    check(lib().pdb_sst_seal_host(img.ctypes.data, total, h.ctypes.data, len(h)))
    for o, z in zip(offs.tolist(), sizes.tolist()):
        word = int.from_bytes(img[o + z + 1 : o + z + 5].tobytes(), "little")
        assert word == orc.mask(orc.value(img[o : o + z + 1].tobytes())), (o, z)
    ok = np.zeros(len(h), dtype=np.uint8)
    assert lib().pdb_sst_verify_host(img.ctypes.data, total, h.ctypes.data, len(h), ok.ctypes.data) == 0 and ok.all()
    assert lib().pdb_sst_verify_host(img.ctypes.data, total, h.ctypes.data, len(h), None) == 0
    bad = [int(np.flatnonzero(sizes == 1363149)[0]), int(np.flatnonzero(sizes == 16384)[0]), 2]
    img[offs[bad[0]] + 1000000] ^= 0x20
    img[offs[bad[1]] + sizes[bad[1]] + 3] ^= 0x01  # a trailer byte
    img[offs[bad[2]] + 17] ^= 0x02
    ok[:] = 1
    assert lib().pdb_sst_verify_host(img.ctypes.data, total, h.ctypes.data, len(h), ok.ctypes.data) == 3
    assert sorted(np.flatnonzero(ok == 0).tolist()) == sorted(bad)
    assert lib().pdb_sst_verify_host(img.ctypes.data, total, h.ctypes.data, len(h), None) == 3


if __name__ == "__main__":
    crc.init_device(0)
    if "--mask" in sys.argv:  # the striped route (pdb_crc32c_init_mask) over device 0 alone
        from pebblesdb_amd._native import check, lib

        assert check(lib().pdb_crc32c_init_mask(1)) == 1
    golden_batches()
    reference_tables()
    long_blocks()
    print("host staging ok (PDB_HOST_CHUNK_BYTES=%s%s)" % (os.environ.get("PDB_HOST_CHUNK_BYTES"),
                                                         ", device mask 1" if "--mask" in sys.argv else ""))
