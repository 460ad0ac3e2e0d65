"""ctypes binding of ``_lib/libpdb_crc32c.so`` (the C-ABI in include/pdb_crc32c.h).

The library is the product: every CRC is computed by its gfx950 kernels.  There is no CPU
fallback -- if the library is missing or no device is usable, calls raise ``PdbError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

from .build import LIB

ABI_VERSION = 2  # include/pdb_crc32c.h PDB_CRC32C_ABI_VERSION this binding is written against

_lock = threading.Lock()
_lib = None


class PdbError(RuntimeError):
    """A negative PDB_E* code from the C-ABI (message from pdb_last_error())."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"pdb_crc32c error {code}: {msg}")
        self.code = code


class pdb_blk(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint32), ("init", ctypes.c_uint32)]


class pdb_block_handle(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("size", ctypes.c_uint64)]


_V = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int

# name -> (restype, argtypes): the complete exported surface of include/pdb_crc32c.h
SIGNATURES = {
    "pdb_crc32c_abi_version": (_I, []),
    "pdb_host_alloc": (_I, [_U64, ctypes.POINTER(ctypes.c_void_p)]),
    "pdb_host_free": (_I, [_V]),
    "pdb_crc32c_init": (_I, [_I]),
    "pdb_crc32c_prepare_stream": (_I, [_V]),
    "pdb_crc32c_init_mask": (_I, [_U64]),
    "pdb_host_stripe_plan": (ctypes.c_int64, [_V, _U64, _U32, _U64, _V, _V, _U64]),
    "pdb_last_error": (ctypes.c_char_p, []),
    "pdb_crc32c_current_device": (_I, []),
    "pdb_crc32c_extend": (_U32, [_U32, _V, ctypes.c_size_t]),
    "pdb_crc32c_value": (_U32, [_V, ctypes.c_size_t]),
    "pdb_crc32c_mask": (_U32, [_U32]),
    "pdb_crc32c_unmask": (_U32, [_U32]),
    "pdb_crc32c_extend_scratch_words": (_U64, [_U64]),
    "pdb_crc32c_extend_device": (_I, [_U32, _V, _U64, _V, _U64, _V, _V]),
    "pdb_crc32c_batch_device_fixed": (_I, [_V, _U64, _U32, _U64, _U32, _U32, _V, _V]),
    "pdb_crc32c_batch_device": (_I, [_V, _V, _U64, _U32, _V, _V]),
    "pdb_crc32c_verify_device": (_I, [_V, _V, _U64, _U32, _V, _V, _V, _V]),
    "pdb_crc32c_batch_host": (_I, [_V, _U64, _V, _U64, _U32, _V]),
    "pdb_crc32c_verify_host": (ctypes.c_int64, [_V, _U64, _V, _U64, _U32, _V, _V]),
    "pdb_sst_seal_device": (_I, [_V, _U64, _V, _U64, _V]),
    "pdb_sst_seal_host": (_I, [_V, _U64, _V, _U64]),
    "pdb_sst_verify_host": (ctypes.c_int64, [_V, _U64, _V, _U64, _V]),
    "pdb_sst_verify_device": (_I, [_V, _U64, _V, _U64, _V, _V, _V]),
    "pdb_sst_crc_device": (_I, [_V, _U64, _V, _U64, _V, _V]),
}


def lib():
    """Load (never build) the in-tree library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB):
            raise ImportError(
                f"pebblesdb_amd HIP library not built: {LIB} missing "
                "(run `python -m pebblesdb_amd.build`); there is no CPU fallback"
            )
        L = ctypes.CDLL(LIB)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.pdb_crc32c_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB}: ABI version {L.pdb_crc32c_abi_version()}, this binding expects {ABI_VERSION} "
                              "(rebuild with `python -m pebblesdb_amd.build`)")
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        msg = lib().pdb_last_error()
        raise PdbError(rc, msg.decode() if msg else "")
    return rc
