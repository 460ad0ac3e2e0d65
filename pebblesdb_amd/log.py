"""WAL / MANIFEST record checksums, batched.

The reference log format (src/db/log_format.h, doc/log_format.txt): the file is a sequence of
32 KiB blocks; a physical record is ``[masked crc LE32][length LE16][type][payload]`` and never
straddles a block; a block tail shorter than the 7-byte header is zero-filled.  The writer
(src/db/log_writer.cc:28-131) computes ``Mask(Extend(type_crc[t], payload))`` per physical
record; the reader (src/db/log_reader.cc:235-249) checks
``Unmask(DecodeFixed32(header)) == Value(header + 6, 1 + length)`` -- the CRC covers the type
byte followed by the payload, which are contiguous in the file.

Here every record of a log image is verified with ONE GPU batch (recovery / repair /
MANIFEST replay), and ``LogWriter`` is a group-commit writer: it lays out many records exactly
as ``Writer::AddRecord`` would and seals all their CRCs with one batch.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import crc32c

K_BLOCK_SIZE = 32768  # log_format.h:27
K_HEADER_SIZE = 7  # log_format.h:30: checksum (4), length (2), type (1)
K_ZERO, K_FULL, K_FIRST, K_MIDDLE, K_LAST = 0, 1, 2, 3, 4  # log_format.h:14-24


class LogCorruption(Exception):
    pass


@dataclass(frozen=True)
class PhysicalRecord:
    offset: int  # header offset in the file
    type: int
    length: int
    stored: int  # masked crc from the header

    @property
    def payload_offset(self) -> int:
        return self.offset + K_HEADER_SIZE


def physical_records(image) -> list[PhysicalRecord]:
    """Walk the blocks like log::Reader::ReadPhysicalRecord (log_reader.cc:185-260), without
    checking CRCs: zero-filled block tails and preallocated zero records are skipped; a
    record whose length runs past its block or the file ends the walk (truncated tail)."""
    img = memoryview(bytes(image))
    n = len(img)
    out = []
    pos = 0
    while pos < n:
        left_in_block = K_BLOCK_SIZE - (pos % K_BLOCK_SIZE)
        if left_in_block < K_HEADER_SIZE:
            pos += left_in_block  # trailer (log_writer.cc:90-97)
            continue
        if pos + K_HEADER_SIZE > n:
            break
        stored = int.from_bytes(img[pos : pos + 4], "little")
        length = img[pos + 4] | (img[pos + 5] << 8)
        typ = img[pos + 6]
        if typ == K_ZERO and length == 0:  # preallocated region: skip the rest of the block
            pos += left_in_block
            continue
        end = pos + K_HEADER_SIZE + length
        if end > n or end > pos - (pos % K_BLOCK_SIZE) + K_BLOCK_SIZE:
            break
        out.append(PhysicalRecord(pos, typ, length, stored))
        pos = end
    return out


def verify_log(image, records=None) -> tuple[list[PhysicalRecord], np.ndarray]:
    """(records, ok): ok[i] = 1 iff record i's stored CRC matches crc32c(type || payload);
    all records checked in one GPU batch (pdb_crc32c_batch_host)."""
    recs = physical_records(image) if records is None else records
    if not recs:
        return recs, np.zeros(0, dtype=np.uint8)
    blk = crc32c.make_blocks([r.offset + 6 for r in recs], [1 + r.length for r in recs])
    got = crc32c.batch_host(np.frombuffer(bytes(image), dtype=np.uint8), blk, masked=True)
    stored = np.array([r.stored for r in recs], dtype=np.uint32)
    return recs, (got == stored).astype(np.uint8)


def read_log(image, checksum: bool = True) -> tuple[list[bytes], int]:
    """Logical records (Full, or First Middle* Last) and the bytes dropped as corrupt, in the
    spirit of log::Reader::ReadRecord: a bad physical record is dropped and any partially
    assembled fragment is discarded."""
    img = bytes(image)
    recs, ok = verify_log(img) if checksum else (physical_records(img), None)
    out, dropped = [], 0
    frag = None
    for i, r in enumerate(recs):
        if ok is not None and not ok[i]:
            dropped += K_HEADER_SIZE + r.length
            if frag is not None:
                dropped += len(frag)
                frag = None
            continue
        payload = img[r.payload_offset : r.payload_offset + r.length]
        if r.type == K_FULL:
            if frag is not None:
                dropped += len(frag)
            frag = None
            out.append(payload)
        elif r.type == K_FIRST:
            if frag is not None:
                dropped += len(frag)
            frag = bytearray(payload)
        elif r.type == K_MIDDLE:
            if frag is None:
                dropped += r.length
            else:
                frag += payload
        elif r.type == K_LAST:
            if frag is None:
                dropped += r.length
            else:
                frag += payload
                out.append(bytes(frag))
                frag = None
        else:
            dropped += K_HEADER_SIZE + r.length
    return out, dropped


class LogWriter:
    """Group-commit form of log::Writer (log_writer.cc:28-131): records are fragmented and laid
    out exactly as AddRecord would, with CRC placeholders; ``seal`` computes every physical
    record's Mask(crc32c(type || payload)) in one GPU batch."""

    def __init__(self, offset: int = 0):
        self.base = offset
        self._buf = bytearray()
        self._hdrs: list[tuple[int, int]] = []  # (header offset in _buf, payload length)

    @property
    def offset(self) -> int:
        return self.base + len(self._buf)

    def add_record(self, payload: bytes) -> None:
        left = len(payload)
        ptr = 0
        begin = True
        while True:
            block_offset = self.offset % K_BLOCK_SIZE
            leftover = K_BLOCK_SIZE - block_offset
            if leftover < K_HEADER_SIZE:
                self._buf += b"\x00" * leftover  # trailer (log_writer.cc:90-97)
                block_offset = 0
            avail = K_BLOCK_SIZE - block_offset - K_HEADER_SIZE
            frag = min(left, avail)
            end = left == frag
            typ = K_FULL if begin and end else K_FIRST if begin else K_LAST if end else K_MIDDLE
            self._hdrs.append((len(self._buf), frag))
            self._buf += b"\x00\x00\x00\x00" + bytes((frag & 0xFF, frag >> 8, typ))
            self._buf += payload[ptr : ptr + frag]
            ptr += frag
            left -= frag
            begin = False
            if left <= 0:
                break

    def seal(self) -> bytes:
        if self._hdrs:
            blk = crc32c.make_blocks([h + 6 for h, _ in self._hdrs], [1 + n for _, n in self._hdrs])
            crcs = crc32c.batch_host(np.frombuffer(bytes(self._buf), dtype=np.uint8), blk, masked=True)
            for (h, _), c in zip(self._hdrs, crcs):
                self._buf[h : h + 4] = int(c).to_bytes(4, "little")
        return bytes(self._buf)
