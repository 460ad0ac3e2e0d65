"""pebblesdb_amd -- MI355X-native CRC32C block-checksum path for a PebblesDB/LevelDB-compatible
sstable layer.

The product is the HIP library ``_lib/libpdb_crc32c.so`` behind the C-ABI in
``include/pdb_crc32c.h``; this package is its host-side mirror of the reference interfaces:

* :mod:`pebblesdb_amd.crc32c` -- ``leveldb::crc32c`` (src/util/crc32c.h) + batch entry points
* :mod:`pebblesdb_amd.table`  -- the sstable block emit/verify hooks
  (``TableBuilder::WriteRawBlock``, ``ReadBlock``: src/table/table_builder.cc:187-205,
  src/table/format.cc:66-148), batched
* :mod:`pebblesdb_amd.shard`  -- block-range sharding across ranks (multi-GPU = independent shards)
"""
from ._native import PdbError  # noqa: F401

__version__ = "0.1.0"
