"""LevelDB-compatible CRC32C API over the MI355X kernels.

Mirrors ``leveldb::crc32c`` (reference src/util/crc32c.h:14-40):

    extend(init_crc, data) -> int   # util/crc32c.h:17  (crc of A||data given init_crc = crc(A))
    value(data) -> int              # util/crc32c.h:20-22
    mask(crc) / unmask(masked)      # util/crc32c.h:29-40  (ror 15 + 0xa282ead8)

plus the batch entry points the reference lacks (one call per many independent blocks):

    batch_fixed(d_base, stride, length, nblk)     device-resident fixed-stride blocks
    batch(d_base, d_blocks)                       device-resident descriptor list
    verify(d_base, d_blocks, d_expected)          device-resident verify (ReadBlock's check)
    batch_host(base, blocks)                      host buffers, H2D + kernel + D2H
    verify_host(base, blocks, expected)           host ReadBlock check over many blocks

Every checksum comes from the HIP library; nothing here computes a CRC on the CPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from ._native import PdbError, check, lib

MASK_OUTPUT = 0x1  # PDB_CRC_MASK_OUTPUT
USE_INIT = 0x2  # PDB_CRC_USE_INIT
SIZE_1K = 0x4  # PDB_CRC_SIZE_1K: most blocks 1024..1152 B (WAL records) -- a speed hint only
SIZE_4K = 0x8  # PDB_CRC_SIZE_4K: most blocks 4096..4352 B (sstable data blocks)
SIZE_256 = 0x10  # PDB_CRC_SIZE_256: most blocks 1..256 B (small WAL / MANIFEST records)
SIZE_512 = 0x20  # PDB_CRC_SIZE_512: most blocks 257..512 B (WAL records of ~400-B values)
SIZE_1023 = 0x40  # PDB_CRC_SIZE_1023: most blocks 513..1023 B
SIZE_MIXED = 0x80  # PDB_CRC_SIZE_MIXED: with 512 / 1023, lengths varying within the class (per-record lanes)
_SIZE_HINT = {None: 0, "1k": SIZE_1K, "4k": SIZE_4K, "256": SIZE_256, "512": SIZE_512, "1023": SIZE_1023,
              "512m": SIZE_512 | SIZE_MIXED, "1023m": SIZE_1023 | SIZE_MIXED}
K_MASK_DELTA = 0xA282EAD8  # util/crc32c.h:24

BLK_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("init", "<u4")])  # == pdb_blk (16 B)
HANDLE_DTYPE = np.dtype([("offset", "<u8"), ("size", "<u8")])  # == pdb_block_handle

__all__ = [
    "extend", "value", "mask", "unmask", "batch_fixed", "batch", "verify", "batch_host", "verify_host",
    "make_blocks", "blocks_to_device", "PdbError", "MASK_OUTPUT", "USE_INIT", "BLK_DTYPE",
    "HANDLE_DTYPE", "init_device", "extend_device",
]


def _buf(data):
    """(pointer, nbytes, keepalive) for bytes-like / numpy input on the host."""
    if isinstance(data, (bytes, bytearray)):
        a = np.frombuffer(bytes(data), dtype=np.uint8)
    elif isinstance(data, memoryview):
        a = np.frombuffer(data.tobytes(), dtype=np.uint8)
    else:
        a = np.ascontiguousarray(data)
        if a.dtype != np.uint8:
            a = a.view(np.uint8)
        a = a.reshape(-1)
    return a.ctypes.data, a.size, a


def init_device(device: int = -1) -> None:
    check(lib().pdb_crc32c_init(device))


def extend(init_crc: int, data) -> int:
    """crc32c of A||data where init_crc = crc32c(A)  (util/crc32c.h:17)."""
    p, n, _keep = _buf(data)
    if n and lib().pdb_crc32c_init(-1) < 0:  # surface the error instead of the C abort()
        check(-1)
    return int(lib().pdb_crc32c_extend(init_crc & 0xFFFFFFFF, p, n))


def value(data) -> int:
    """crc32c of data  (util/crc32c.h:20-22)."""
    return extend(0, data)


def mask(crc: int) -> int:
    """util/crc32c.h:29-32 (pure integer op, exported by the library)."""
    return int(lib().pdb_crc32c_mask(crc & 0xFFFFFFFF))


def unmask(masked_crc: int) -> int:
    """util/crc32c.h:35-40."""
    return int(lib().pdb_crc32c_unmask(masked_crc & 0xFFFFFFFF))


def make_blocks(offs, lens, inits=None) -> np.ndarray:
    """Host descriptor array (pdb_blk layout)."""
    offs = np.asarray(offs, dtype=np.uint64).reshape(-1)
    lens = np.asarray(lens, dtype=np.uint64).reshape(-1)
    if offs.shape != lens.shape:
        raise ValueError("offs/lens shape mismatch")
    if lens.size and int(lens.max()) > 0xFFFFFFFF:
        raise ValueError("per-block length must be < 4 GiB (util/crc32c.cc:589 narrows to uint32)")
    b = np.zeros(offs.size, dtype=BLK_DTYPE)
    b["off"] = offs
    b["len"] = lens
    if inits is not None:
        b["init"] = np.asarray(inits, dtype=np.uint64).reshape(-1) & 0xFFFFFFFF
    return b


def _torch():
    import torch

    return torch


def blocks_to_device(blocks: np.ndarray, device=None):
    """Copy a pdb_blk array to the GPU as a uint8 tensor (16 B per block)."""
    torch = _torch()
    raw = np.ascontiguousarray(blocks, dtype=BLK_DTYPE).view(np.uint8)
    return torch.from_numpy(raw.copy()).to(device or "cuda")


def _stream_ptr(stream) -> int:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _dev_ptr(t) -> int:
    if not t.is_cuda:
        raise ValueError("expected a device (cuda) tensor")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return int(t.data_ptr())


def _out_tensor(n: int, like, out):
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=like.device)
    elif out.numel() < n or out.dtype != torch.int32:
        raise ValueError("out must be an int32 tensor with >= nblk elements")
    return out


def batch_fixed(d_base, stride: int, length: int, nblk: int, *, masked: bool = False,
                init: int | None = None, out=None, stream=None):
    """CRC of blocks i at d_base[i*stride : i*stride+length] -> int32 tensor (bit pattern = u32)."""
    if nblk and (nblk - 1) * stride + length > d_base.numel() * d_base.element_size():
        raise ValueError("blocks exceed the base tensor")
    out = _out_tensor(nblk, d_base, out)
    flags = (MASK_OUTPUT if masked else 0) | (USE_INIT if init is not None else 0)
    check(lib().pdb_crc32c_batch_device_fixed(
        _dev_ptr(d_base), stride, length, nblk, flags, (init or 0) & 0xFFFFFFFF,
        _dev_ptr(out), _stream_ptr(stream)))
    return out


def batch(d_base, d_blocks, *, masked: bool = False, use_init: bool = False, out=None, stream=None,
          size_hint: str | None = None):
    """CRC of each descriptor (pdb_blk, 16 B each, device tensor) -> int32 tensor.  size_hint "1k"
    / "4k" selects the sized kernel for batches of mostly WAL-record / sstable-block lengths (the
    device cannot see the lengths before launching; the results do not depend on it)."""
    n = d_blocks.numel() * d_blocks.element_size() // 16
    out = _out_tensor(n, d_base, out)
    flags = (MASK_OUTPUT if masked else 0) | (USE_INIT if use_init else 0) | _SIZE_HINT[size_hint]
    check(lib().pdb_crc32c_batch_device(
        _dev_ptr(d_base), _dev_ptr(d_blocks), n, flags, _dev_ptr(out), _stream_ptr(stream)))
    return out


def verify(d_base, d_blocks, d_expected, *, masked: bool = True, use_init: bool = False,
           stream=None, size_hint: str | None = None):
    """(ok uint8 tensor, nbad int32 tensor[1]) -- ReadBlock's check for many blocks at once."""
    torch = _torch()
    n = d_blocks.numel() * d_blocks.element_size() // 16
    ok = torch.empty(n, dtype=torch.uint8, device=d_base.device)
    nbad = torch.zeros(1, dtype=torch.int32, device=d_base.device)
    flags = (MASK_OUTPUT if masked else 0) | (USE_INIT if use_init else 0) | _SIZE_HINT[size_hint]
    check(lib().pdb_crc32c_verify_device(
        _dev_ptr(d_base), _dev_ptr(d_blocks), n, flags, _dev_ptr(d_expected), _dev_ptr(ok),
        _dev_ptr(nbad), _stream_ptr(stream)))
    return ok, nbad


def batch_host(base, blocks: np.ndarray, *, masked: bool = False, use_init: bool = False) -> np.ndarray:
    """Host buffers in, host CRCs out (copy-inclusive path)."""
    p, n, _keep = _buf(base)
    blocks = np.ascontiguousarray(blocks, dtype=BLK_DTYPE)
    out = np.zeros(len(blocks), dtype=np.uint32)
    flags = (MASK_OUTPUT if masked else 0) | (USE_INIT if use_init else 0)
    check(lib().pdb_crc32c_batch_host(p, n, blocks.ctypes.data, len(blocks), flags, out.ctypes.data))
    return out


def verify_host(base, blocks: np.ndarray, expected, *, masked: bool = True, use_init: bool = False):
    """(ok uint8 array, nbad) for host blocks against host expected CRCs (copy-inclusive
    ReadBlock check, table/format.cc:96-104)."""
    p, n, _keep = _buf(base)
    blocks = np.ascontiguousarray(blocks, dtype=BLK_DTYPE)
    exp = np.ascontiguousarray(expected, dtype=np.uint32)
    if exp.size != len(blocks):
        raise ValueError("one expected CRC per block")
    ok = np.zeros(len(blocks), dtype=np.uint8)
    flags = (MASK_OUTPUT if masked else 0) | (USE_INIT if use_init else 0)
    nbad = lib().pdb_crc32c_verify_host(p, n, blocks.ctypes.data, len(blocks), flags, exp.ctypes.data,
                                        ok.ctypes.data)
    check(int(nbad))
    return ok, int(nbad)


def extend_device(init_crc: int, d_data, nbytes: int | None = None, stream=None) -> int:
    """Extend(init_crc, span) for ONE device-resident span of any length (split into up to 16384
    segments hashed in parallel and folded on the device).  Returns the CRC (synchronises)."""
    torch = _torch()
    n = d_data.numel() * d_data.element_size() if nbytes is None else nbytes
    words = int(lib().pdb_crc32c_extend_scratch_words(n))
    scratch = torch.empty(words, dtype=torch.int32, device=d_data.device)
    out = torch.empty(1, dtype=torch.int32, device=d_data.device)
    check(lib().pdb_crc32c_extend_device(init_crc & 0xFFFFFFFF, _dev_ptr(d_data), n, _dev_ptr(scratch), words,
                                         _dev_ptr(out), _stream_ptr(stream)))
    return int(out.cpu().numpy().view(np.uint32)[0])
