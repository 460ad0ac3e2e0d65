"""ctypes binding of ``_lib/libpdb_crc32c_diag.so`` -- BENCH / TEST INFRASTRUCTURE.

include/pdb_crc32c_diag.h: synthetic input on the device (the splitmix64 stream the oracle also
generates), the load-pattern kernels behind the roofline calibration, and the A/B kernel variants
(selected per call).  The product (``_native`` / ``crc32c``) never loads this library.
"""
from __future__ import annotations

import ctypes
import os
import threading

from .build import DIAG_LIB
from ._native import PdbError

_lock = threading.Lock()
_lib = None
_V, _U32, _U64, _I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int

SIGNATURES = {
    "pdb_diag_last_error": (ctypes.c_char_p, []),
    "pdb_diag_fill_splitmix": (_I, [_V, _U64, _U64, _U64, _V]),
    "pdb_diag_read_stream": (_I, [_V, _U64, _V, _V]),
    "pdb_diag_read_pattern4k": (_I, [_V, _U64, _I, _V, _V]),
    "pdb_diag_batch_fixed": (_I, [_I, _V, _U64, _U32, _U64, _U32, _U32, _V, _V]),
    "pdb_diag_batch_desc": (_I, [_I, _V, _V, _U64, _U32, _V, _V]),
    "pdb_diag_sst": (_I, [_I, _V, _U64, _V, _U64, _I, _V, _V, _V]),
}


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(DIAG_LIB):
                raise ImportError(f"{DIAG_LIB} missing (run `python -m pebblesdb_amd.build`)")
            L = ctypes.CDLL(DIAG_LIB)
            for name, (res, args) in SIGNATURES.items():
                f = getattr(L, name)
                f.restype, f.argtypes = res, args
            _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        msg = lib().pdb_diag_last_error()
        raise PdbError(rc, msg.decode() if msg else "")
    return rc


def _stream(stream) -> int:
    import torch

    return int((stream if stream is not None else torch.cuda.current_stream()).cuda_stream)


def _ptr(t) -> int:
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("expected a contiguous device tensor")
    return int(t.data_ptr())


def fill_splitmix(d_dst, seed: int, byte_offset: int = 0, nbytes: int | None = None, stream=None):
    """Fill a device tensor with the splitmix64 synthetic byte stream (oracle.splitmix_bytes' twin)."""
    nb = d_dst.numel() * d_dst.element_size() if nbytes is None else nbytes
    check(lib().pdb_diag_fill_splitmix(_ptr(d_dst), nb, seed & 0xFFFFFFFFFFFFFFFF, byte_offset, _stream(stream)))
    return d_dst


def read_stream(d_base, nbytes: int, d_out, stream=None) -> None:
    check(lib().pdb_diag_read_stream(_ptr(d_base), nbytes, _ptr(d_out), _stream(stream)))


def read_pattern4k(d_base, nblk: int, variant: int, d_out, stream=None) -> None:
    check(lib().pdb_diag_read_pattern4k(_ptr(d_base), nblk, variant, _ptr(d_out), _stream(stream)))


def batch_fixed(variant: int, d_base, stride: int, length: int, nblk: int, *, masked: bool = False,
                init: int | None = None, out=None, stream=None):
    """A/B variant of crc32c.batch_fixed (variant 0 = the shipped routing)."""
    import torch

    if out is None:
        out = torch.empty(nblk, dtype=torch.int32, device=d_base.device)
    flags = (1 if masked else 0) | (2 if init is not None else 0)
    check(lib().pdb_diag_batch_fixed(variant, _ptr(d_base), stride, length, nblk, flags, (init or 0) & 0xFFFFFFFF,
                                     _ptr(out), _stream(stream)))
    return out


def batch_desc(variant: int, d_base, d_blocks, *, flags: int = 0, out=None, stream=None):
    """A/B variant of crc32c.batch (variant 0 = the shipped routing, size hints in `flags`)."""
    import torch

    n = d_blocks.numel() * d_blocks.element_size() // 16
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=d_base.device)
    check(lib().pdb_diag_batch_desc(variant, _ptr(d_base), _ptr(d_blocks), n, flags, _ptr(out), _stream(stream)))
    return out


def sst(variant: int, d_buf, d_handles, *, seal: bool, ok=None, nbad=None, stream=None) -> None:
    """A/B variant of pdb_sst_seal_device (seal=True) / pdb_sst_verify_device."""
    n = d_handles.numel() * d_handles.element_size() // 16
    nb = d_buf.numel() * d_buf.element_size()
    check(lib().pdb_diag_sst(variant, _ptr(d_buf), nb, _ptr(d_handles), n, 1 if seal else 0,
                             _ptr(ok) if ok is not None else None, _ptr(nbad) if nbad is not None else None,
                             _stream(stream)))
