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
# log::Reader's extra return values kEof = kMaxRecordType + 1, kBadRecord = + 2 (log_reader.h:78-84):
# a record whose type byte holds one of them (and a valid CRC) takes that path in ReadRecord
K_EOF_VALUE, K_BADRECORD_VALUE = 5, 6


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

    @property
    def block(self) -> int:
        return self.offset // K_BLOCK_SIZE


@dataclass(frozen=True)
class BlockDrop:
    """The rest of a block that log::Reader drops without a CRC check: a record whose length runs
    past a full block ("bad record length", log_reader.cc:214-220) or a zero-filled preallocated
    region (type 0, length 0: dropped silently, log_reader.cc:227-233)."""
    offset: int
    nbytes: int
    reason: str | None

    @property
    def block(self) -> int:
        return self.offset // K_BLOCK_SIZE


def walk(image) -> list:
    """The physical items log::Reader::ReadPhysicalRecord (log_reader.cc:181-263) meets, trusting
    every length (CRCs are checked afterwards, in one batch): PhysicalRecord or BlockDrop, in file
    order.  The file is read in 32-KiB blocks; only the last, short block sets eof: a record running
    past it, or a truncated header there, ends the walk (a writer that died mid-record: no report).
    A block tail shorter than a header is skipped (the writer's zero trailer)."""
    img = memoryview(bytes(image))
    n = len(img)
    out = []
    for bstart in range(0, n, K_BLOCK_SIZE):
        bend = min(bstart + K_BLOCK_SIZE, n)
        eof = bend - bstart < K_BLOCK_SIZE
        pos = bstart
        while bend - pos >= K_HEADER_SIZE:
            length = img[pos + 4] | (img[pos + 5] << 8)
            typ = img[pos + 6]
            if K_HEADER_SIZE + length > bend - pos:
                if eof:
                    return out  # kEof: the writer died in the middle of this record
                out.append(BlockDrop(pos, bend - pos, "bad record length"))
                break
            if typ == K_ZERO and length == 0:
                out.append(BlockDrop(pos, bend - pos, None))
                break
            out.append(PhysicalRecord(pos, typ, length, int.from_bytes(img[pos : pos + 4], "little")))
            pos += K_HEADER_SIZE + length
        if eof:
            break  # a short tail in the last block is a truncated header: kEof
    return out


def physical_records(image) -> list[PhysicalRecord]:
    """Every physical record of the walk (see walk()), without checking CRCs."""
    return [r for r in walk(image) if isinstance(r, PhysicalRecord)]


def verify_log(image, records=None) -> tuple[list[PhysicalRecord], np.ndarray]:
    """(records, ok): ok[i] = 1 iff record i's stored CRC matches crc32c(type || payload);
    all records checked in one GPU batch (pdb_crc32c_batch_host).  Records the reader would never
    reach (after a bad one in the same block) are checked too; replay_log() discards them."""
    recs = physical_records(image) if records is None else records
    if not recs:
        return recs, np.zeros(0, dtype=np.uint8)
    blk = crc32c.make_blocks([r.offset + 6 for r in recs], [1 + r.length for r in recs])
    got = crc32c.batch_host(np.frombuffer(bytes(image), dtype=np.uint8), blk, masked=True)
    stored = np.array([r.stored for r in recs], dtype=np.uint32)
    return recs, (got == stored).astype(np.uint8)


@dataclass
class LogReplay:
    records: list  # (LastRecordOffset, payload bytes) per logical record, in order
    reports: list  # (bytes, "Corruption: <reason>") per Reporter::Corruption call, in order

    @property
    def dropped(self) -> int:
        return sum(b for b, _ in self.reports)


def replay_log(image, checksum: bool = True, ok=None) -> LogReplay:
    """What log::Reader::ReadRecord (log_reader.cc:59-164, checksums on, initial offset 0) delivers
    from `image`: the logical records with their LastRecordOffset and the corruption reports, from
    ONE batched CRC check of every walked record (`ok`, from verify_log when not given).  A record
    failing its check drops the rest of its block -- the reader no longer trusts the length -- so
    the records walked after it in that block are discarded, never replayed (log_reader.cc:240-247).
    Pinned by tests/golden/log/corruptions.json (the reference reader on corrupted logs)."""
    img = bytes(image)
    items = walk(img)
    recs = [it for it in items if isinstance(it, PhysicalRecord)]
    if checksum and ok is None:
        _, ok = verify_log(img, recs)
    good = {}
    if checksum:
        for r, k in zip(recs, ok):
            good[r.offset] = bool(k)
    out, reports = [], []
    scratch, in_frag = b"", False
    prospective = 0
    pos = 0  # reader position before the next physical read (end_of_buffer_offset_ - buffer_.size())
    dead_block = -1

    def bad_record():  # kBadRecord in ReadRecord (log_reader.cc:143-149)
        nonlocal scratch, in_frag
        if in_frag:
            reports.append((len(scratch), "Corruption: error in middle of record"))
            in_frag, scratch = False, b""

    for it in items:
        if it.block == dead_block:
            continue
        bend = min((it.block + 1) * K_BLOCK_SIZE, len(img))
        if isinstance(it, BlockDrop):
            if it.reason:
                reports.append((it.nbytes, "Corruption: " + it.reason))
            bad_record()
            pos = bend
            continue
        phys_off = pos
        if checksum and not good[it.offset]:
            reports.append((bend - it.offset, "Corruption: checksum mismatch"))
            dead_block = it.block
            bad_record()
            pos = bend
            continue
        pos = it.offset + K_HEADER_SIZE + it.length
        frag = img[it.payload_offset : it.payload_offset + it.length]
        t = it.type
        if t == K_FULL:
            if in_frag and scratch:
                reports.append((len(scratch), "Corruption: partial record without end(1)"))
            out.append((phys_off, frag))
            scratch, in_frag = b"", False
        elif t == K_FIRST:
            if in_frag and scratch:
                reports.append((len(scratch), "Corruption: partial record without end(2)"))
            prospective = phys_off
            scratch, in_frag = frag, True
        elif t == K_MIDDLE:
            if not in_frag:
                reports.append((len(frag), "Corruption: missing start of fragmented record(1)"))
            else:
                scratch += frag
        elif t == K_LAST:
            if not in_frag:
                reports.append((len(frag), "Corruption: missing start of fragmented record(2)"))
            else:
                out.append((prospective, scratch + frag))
                scratch, in_frag = b"", False
        elif t == K_EOF_VALUE:  # a valid record whose type byte is kEof: ReadRecord returns false (stop)
            break
        elif t == K_BADRECORD_VALUE:  # ... or kBadRecord: 'error in middle of record' if mid-fragment
            bad_record()
        else:  # header[6] is a (signed) char read into an unsigned int: 0x80.. print as 42949671xx
            tu = t | 0xFFFFFF00 if t >= 0x80 else t
            reports.append((len(frag) + (len(scratch) if in_frag else 0), f"Corruption: unknown record type {tu}"))
            scratch, in_frag = b"", False
    return LogReplay(out, reports)


def read_log(image, checksum: bool = True) -> tuple[list[bytes], int]:
    """Logical records and the bytes the reader reports as dropped (log::Reader::ReadRecord)."""
    r = replay_log(image, checksum)
    return [p for _, p in r.records], r.dropped


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
