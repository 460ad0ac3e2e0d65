"""Real tables through the device hooks (VERDICT r05 "next round" #1): a table written by the
REFERENCE engine's TableBuilder as shipped (integration/_build/pdb_tablegen: reference
table_builder.cc + util/crc32c.cc, CPU trailers), 200 k keys of 1 KiB values with a bloom filter, so
its filter (~0.9 MiB) and index (~1.6 MiB) blocks take the long-block lane.  The device seal's trailer
words must equal the reference's own trailers in the file for every block (data, filter, metaindex,
index), and a device verify of the file must pass -- then flag exactly the blocks a flipped byte hits.
Reference: table/table_builder.cc:187-266, table/format.cc:66-104, table/table.cc:70-170."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLEGEN = os.path.join(ROOT, "integration", "_build", "pdb_tablegen")


def test_reference_table_on_device(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(TABLEGEN):
        pytest.skip("integration/_build/pdb_tablegen not built")
    import bench
    from pebblesdb_amd import crc32c
    from pebblesdb_amd import table as T

    crc32c.init_device(0)
    img, hs, info = bench.real_tables(2, 200000, 1024, 77)
    assert len(info) == 2 and all(t["index_bytes"] > 16384 and t["filter_bytes"] > 16384 for t in info)
    offs, sizes = hs["offset"].astype(np.int64), hs["size"].astype(np.int64)
    t = offs + sizes + 1
    words = (img[t].astype(np.uint32) | (img[t + 1].astype(np.uint32) << 8) | (img[t + 2].astype(np.uint32) << 16) |
             (img[t + 3].astype(np.uint32) << 24))
    d = torch.from_numpy(img).cuda()
    d_h = T.handles_to_device(hs)
    got = T.crc_device(d, d_h).cpu().numpy().view(np.uint32)
    assert (got == words).all(), np.flatnonzero(got != words)[:10]
    ok, nbad = T.verify_device(d, d_h)
    assert ok.cpu().numpy().all() and int(nbad.item()) == 0
    # one byte in the first table's index block, one in the second's filter block, one data block
    big = np.flatnonzero(sizes + 1 >= 16384)
    assert len(big) == 4
    bad = [int(big[1]), int(big[2]), 5]
    for b in bad:
        d[int(offs[b] + sizes[b] // 2)] ^= 0x08
    ok, nbad = T.verify_device(d, d_h)
    assert int(nbad.item()) == 3
    assert sorted(np.flatnonzero(ok.cpu().numpy() == 0).tolist()) == sorted(bad)
    # the same through the in-place device seal: it restores exactly the reference's trailers
    # wherever the contents are the reference's
    d2 = torch.from_numpy(img).cuda()
    d2[torch.from_numpy(t).cuda()] = 0
    T.seal_device(d2, d_h)
    assert (d2.cpu().numpy() == img).all()
