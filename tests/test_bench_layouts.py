"""CPU checks of bench.py's synthetic layouts against the reference formats they stand for.

* ``wal_layout`` (bench.py --workload wal) must put every CRC'd span (type byte + fragment)
  exactly where log::Writer::AddRecord puts it (db/log_writer.cc:39-81): our group-commit
  LogWriter lays records out the same way (its sealed bytes equal logs written by the
  reference's own log::Writer, tests/test_log.py), so its framing is the yardstick here.
* the sst workload's handles tile the image like WriteRawBlock's offsets (offset += n + 5).
"""
import numpy as np

import bench
from pebblesdb_amd import log as L


def test_wal_layout_matches_log_writer_framing():
    w = L.LogWriter()
    for _ in range(3000):  # ~3.2 MB: 97 log blocks, every fragment type and block-tail case
        w.add_record(b"\x01" * 1055)
    exp_off = np.array([h + 6 for h, _ in w._hdrs])
    exp_len = np.array([1 + n for _, n in w._hdrs])
    offs, lens = bench.wal_layout(len(w._buf), 1055)
    k = len(exp_off)
    assert (offs[:k] == exp_off).all() and (lens[:k] == exp_len).all()
    # and records that end exactly 7 bytes short of a block (a zero-length FIRST fragment)
    w2 = L.LogWriter()
    for n in (32768 - 7 - 7, 100, 200):
        w2.add_record(b"\x02" * n)
    assert [n for _, n in w2._hdrs][:2] == [32768 - 14, 0]


def test_sst_handles_tile_like_write_raw_block():
    rng = np.random.Generator(np.random.PCG64(301))
    sizes = rng.integers(4166, 4175, size=1000).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes + 5)[:-1]])
    assert (offs[1:] == offs[:-1] + sizes[:-1] + 5).all()  # table_builder.cc:203-204
