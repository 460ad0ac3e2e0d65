"""sstable block emit/verify hooks, batched, over the MI355X CRC32C kernels.

Mirrors the two reference call sites of the block checksum:

* ``TableBuilder::WriteRawBlock`` (src/table/table_builder.cc:187-205): a block is appended as
  ``[contents n B][type 1 B][Mask(crc32c(contents || type)) LE32]`` and gets the BlockHandle
  ``{offset, n}``; the next block starts at ``offset + n + kBlockTrailerSize``.
* ``ReadBlock`` (src/table/format.cc:66-148): with ``verify_checksums`` it compares
  ``Unmask(DecodeFixed32(data + n + 1))`` with ``Value(data, n + 1)`` and returns
  ``Status::Corruption("block checksum mismatch")``; a short read is
  ``Corruption("truncated block read")``.

Here ``TableBlockWriter`` buffers blocks and seals all trailers with one GPU batch
(``pdb_sst_seal_host``), and ``verify_blocks`` checks many handles in one batch
(``pdb_sst_verify_host``) -- the scan / paranoid-compaction / leveldb-verify form of ReadBlock.
The BlockHandle varint codec and the Footer codec (table/format.cc:15-64, table/format.h:47-79)
are included so real table images can be walked.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._native import check, lib
from .crc32c import HANDLE_DTYPE, _buf

K_BLOCK_TRAILER_SIZE = 5  # table/format.h:87
K_NO_COMPRESSION = 0  # include/pebblesdb/options.h (CompressionType)
K_SNAPPY_COMPRESSION = 1
K_TABLE_MAGIC_NUMBER = 0xDB4775248B80FB57  # table/format.h:84
K_MAX_ENCODED_HANDLE_LENGTH = 10 + 10  # table/format.h:41
K_FOOTER_ENCODED_LENGTH = 2 * K_MAX_ENCODED_HANDLE_LENGTH + 8  # table/format.h:71


class Corruption(Exception):
    """The reference's Status::Corruption (include/pebblesdb/status.h)."""


@dataclass(frozen=True)
class BlockHandle:
    offset: int
    size: int

    def encode(self) -> bytes:  # table/format.cc:15-21 (two varint64s)
        return encode_varint64(self.offset) + encode_varint64(self.size)

    @staticmethod
    def decode(buf: bytes, pos: int = 0) -> tuple["BlockHandle", int]:  # format.cc:23-30
        off, pos = decode_varint64(buf, pos)
        size, pos = decode_varint64(buf, pos)
        return BlockHandle(off, size), pos


def encode_varint64(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def decode_varint64(buf: bytes, pos: int) -> tuple[int, int]:
    result, shift = 0, 0
    while shift <= 63:
        if pos >= len(buf):
            raise Corruption("bad block handle")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
    raise Corruption("bad block handle")


@dataclass(frozen=True)
class Footer:
    """table/format.h:47-79: metaindex handle, index handle, padding, 8-byte magic."""

    metaindex: BlockHandle
    index: BlockHandle

    def encode(self) -> bytes:  # format.cc:32-42
        b = self.metaindex.encode() + self.index.encode()
        b = b + b"\x00" * (2 * K_MAX_ENCODED_HANDLE_LENGTH - len(b))
        m = K_TABLE_MAGIC_NUMBER
        return b + (m & 0xFFFFFFFF).to_bytes(4, "little") + (m >> 32).to_bytes(4, "little")

    @staticmethod
    def decode(buf: bytes) -> "Footer":  # format.cc:44-64
        if len(buf) < K_FOOTER_ENCODED_LENGTH:
            raise Corruption("file is too short to be an sstable")
        buf = buf[-K_FOOTER_ENCODED_LENGTH:]
        lo = int.from_bytes(buf[-8:-4], "little")
        hi = int.from_bytes(buf[-4:], "little")
        if (hi << 32) | lo != K_TABLE_MAGIC_NUMBER:
            raise Corruption("not an sstable (bad magic number)")
        mi, pos = BlockHandle.decode(buf, 0)
        ix, _ = BlockHandle.decode(buf, pos)
        return Footer(mi, ix)


class TableBlockWriter:
    """Buffered WriteRawBlock: ``add`` returns the handle the reference would set; ``seal``
    computes every trailer in one GPU batch; ``data`` is the byte stream to Append."""

    def __init__(self, base_offset: int = 0):
        self.base = base_offset
        self._buf = bytearray()
        self._rel: list[tuple[int, int]] = []
        self._sealed = True

    def add(self, contents: bytes, type_: int = K_NO_COMPRESSION) -> BlockHandle:
        h = BlockHandle(self.base + len(self._buf), len(contents))
        self._rel.append((len(self._buf), len(contents)))
        self._buf += contents
        self._buf.append(type_ & 0xFF)
        self._buf += b"\x00\x00\x00\x00"
        self._sealed = False
        return h

    def seal(self) -> None:
        if not self._rel:
            self._sealed = True
            return
        h = np.array(self._rel, dtype=np.uint64).view(HANDLE_DTYPE).reshape(-1)
        h = np.ascontiguousarray(h)
        arr = np.frombuffer(self._buf, dtype=np.uint8)
        check(lib().pdb_sst_seal_host(arr.ctypes.data, arr.size, h.ctypes.data, len(h)))
        self._sealed = True

    @property
    def data(self) -> bytes:
        if not self._sealed:
            raise RuntimeError("seal() before reading the sealed bytes")
        return bytes(self._buf)

    @property
    def next_offset(self) -> int:
        return self.base + len(self._buf)

    def handles(self) -> list[BlockHandle]:
        return [BlockHandle(self.base + o, n) for o, n in self._rel]


def _handles_array(handles) -> np.ndarray:
    h = np.zeros(len(handles), dtype=HANDLE_DTYPE)
    for i, x in enumerate(handles):
        h[i]["offset"], h[i]["size"] = (x.offset, x.size) if isinstance(x, BlockHandle) else x
    return h


def verify_blocks(image, handles) -> np.ndarray:
    """ok[i] = 1 iff block i's stored trailer matches crc32c(contents||type)."""
    p, n, _keep = _buf(image)
    h = _handles_array(handles)
    for x in h:
        if int(x["offset"]) + int(x["size"]) + K_BLOCK_TRAILER_SIZE > n:
            raise Corruption("truncated block read")
    ok = np.zeros(len(h), dtype=np.uint8)
    rc = lib().pdb_sst_verify_host(p, n, h.ctypes.data, len(h), ok.ctypes.data)
    check(int(rc))
    return ok


def read_block(image, handle: BlockHandle, verify_checksums: bool = True) -> tuple[bytes, int]:
    """ReadBlock (format.cc:66-148) for an in-memory image: returns (contents, type).
    Compression is left to the caller (Snappy is delegated, out of scope)."""
    data = bytes(image[handle.offset : handle.offset + handle.size + K_BLOCK_TRAILER_SIZE])
    if len(data) != handle.size + K_BLOCK_TRAILER_SIZE:
        raise Corruption("truncated block read")
    if verify_checksums and not verify_blocks(data, [BlockHandle(0, handle.size)])[0]:
        raise Corruption("block checksum mismatch")
    return data[: handle.size], data[handle.size]


def read_blocks(image, handles, verify_checksums: bool = True) -> list[tuple[bytes, int]]:
    """Batch ReadBlock: one GPU verify for all handles, then the per-block slices."""
    if verify_checksums:
        ok = verify_blocks(image, handles)
        bad = np.nonzero(ok == 0)[0]
        if bad.size:
            raise Corruption(f"block checksum mismatch (block {int(bad[0])} of {len(handles)})")
    mv = memoryview(bytes(image))
    return [(bytes(mv[h.offset : h.offset + h.size]), mv[h.offset + h.size]) for h in handles]


# ---- whole-table walk: the batched form of leveldb-verify (src/leveldb-verify.cc:120-164) -------


def decode_varint32(buf: bytes, pos: int) -> tuple[int, int]:
    v, pos = decode_varint64(buf, pos)
    if v > 0xFFFFFFFF:
        raise Corruption("bad varint32")
    return v, pos


def block_entries(contents: bytes) -> list[tuple[bytes, bytes]]:
    """Parse a block (table/block_builder.cc: prefix-compressed entries
    [shared][non_shared][value_len][key_delta][value], then uint32 restarts[], uint32 count)."""
    n = len(contents)
    if n < 4:
        raise Corruption("bad block contents")
    num_restarts = int.from_bytes(contents[n - 4 :], "little")
    limit = n - 4 * (num_restarts + 1)
    if limit < 0:
        raise Corruption("bad block contents")
    out, pos, key = [], 0, b""
    while pos < limit:
        shared, pos = decode_varint32(contents, pos)
        non_shared, pos = decode_varint32(contents, pos)
        vlen, pos = decode_varint32(contents, pos)
        if shared > len(key) or pos + non_shared + vlen > limit:
            raise Corruption("bad entry in block")
        key = key[:shared] + contents[pos : pos + non_shared]
        pos += non_shared
        out.append((key, contents[pos : pos + vlen]))
        pos += vlen
    return out


@dataclass
class TableLayout:
    footer: Footer
    data: list  # BlockHandle of every data block, in file order
    meta: dict  # metaindex name -> BlockHandle (e.g. "filter.leveldb.BuiltinBloomFilter")

    def all_handles(self) -> list:
        return list(self.data) + list(self.meta.values()) + [self.footer.metaindex, self.footer.index]


def table_layout(image, verify_checksums: bool = True) -> TableLayout:
    """Footer -> index block -> data-block handles, metaindex block -> meta handles
    (table/table.cc:70-170 Table::Open / ReadMeta).  Index and metaindex are read through
    read_block, i.e. checksum-verified on the GPU when verify_checksums is set."""
    image = bytes(image)
    f = Footer.decode(image)
    idx, _ = read_block(image, f.index, verify_checksums)
    data = [BlockHandle.decode(v)[0] for _, v in block_entries(idx)]
    mi, _ = read_block(image, f.metaindex, verify_checksums)
    meta = {k.decode("latin-1"): BlockHandle.decode(v)[0] for k, v in block_entries(mi)}
    return TableLayout(f, data, meta)


def verify_table(image) -> tuple[TableLayout, np.ndarray]:
    """leveldb-verify for one table image: every block (data, meta, metaindex, index) checked in
    ONE GPU batch.  Returns (layout, ok flags in all_handles() order).  The index and metaindex
    blocks are checked first (one small batch), so a corrupt index is reported as
    Corruption("block checksum mismatch") -- ReadBlock's verdict -- before its entries are parsed."""
    image = bytes(image)
    f = Footer.decode(image)
    if not verify_blocks(image, [f.index, f.metaindex]).all():
        raise Corruption("block checksum mismatch")
    lay = table_layout(image, verify_checksums=False)
    return lay, verify_blocks(image, lay.all_handles())


# ---- device-resident sstable images (pdb_sst_seal_device / pdb_sst_verify_device) -------------
# The same two hooks on an image already in HBM (a compaction output being assembled on the GPU,
# or a table read in bulk): handles are a device tensor of pdb_block_handle {u64 offset; u64
# size} (16 B each); everything is stream-ordered and capturable.
def handles_to_device(handles, device=None):
    """BlockHandles (or (offset, size) pairs, or a HANDLE_DTYPE array) -> uint8 device tensor."""
    import torch

    h = handles if isinstance(handles, np.ndarray) else _handles_array(handles)
    raw = np.ascontiguousarray(h, dtype=HANDLE_DTYPE).view(np.uint8)
    return torch.from_numpy(raw.copy()).to(device or "cuda")


def _dev(t) -> int:
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("expected a contiguous device tensor")
    return int(t.data_ptr())


def _stream(stream) -> int:
    import torch

    return int((stream if stream is not None else torch.cuda.current_stream()).cuda_stream)


def seal_device(d_image, d_handles, stream=None) -> None:
    """WriteRawBlock's trailer for every handle of a device image: Mask(crc32c(contents||type))
    little-endian at offset+size+1 (the type byte at offset+size is input)."""
    n = d_handles.numel() * d_handles.element_size() // 16
    check(lib().pdb_sst_seal_device(_dev(d_image), d_image.numel() * d_image.element_size(), _dev(d_handles), n,
                                    _stream(stream)))


def crc_device(d_image, d_handles, stream=None, out=None):
    """The seal's trailer words without writing them: int32 tensor of Mask(crc32c(contents||type))
    per handle (an engine writes the trailer while it copies blocks out; the in-place seal pays
    for scattered 4-B writes).  Out-of-image handles leave their entry untouched (zero here)."""
    import torch

    n = d_handles.numel() * d_handles.element_size() // 16
    if out is None:
        out = torch.zeros(n, dtype=torch.int32, device=d_image.device)
    check(lib().pdb_sst_crc_device(_dev(d_image), d_image.numel() * d_image.element_size(), _dev(d_handles), n,
                                   _dev(out), _stream(stream)))
    return out


def verify_device(d_image, d_handles, stream=None):
    """ReadBlock's check for every handle of a device image -> (ok uint8 tensor, nbad int32[1])."""
    import torch

    n = d_handles.numel() * d_handles.element_size() // 16
    ok = torch.empty(n, dtype=torch.uint8, device=d_image.device)
    nbad = torch.zeros(1, dtype=torch.int32, device=d_image.device)
    check(lib().pdb_sst_verify_device(_dev(d_image), d_image.numel() * d_image.element_size(), _dev(d_handles), n,
                                      _dev(ok), _dev(nbad), _stream(stream)))
    return ok, nbad
