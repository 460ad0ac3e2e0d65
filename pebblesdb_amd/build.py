"""Build the in-tree HIP library ``pebblesdb_amd/_lib/libpdb_crc32c.so`` for gfx950.

Run ``python -m pebblesdb_amd.build`` (or ``__graft_entry__.build()``).  hipcc cross-compiles
without a GPU; the .so is git-ignored but travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIBDIR, "libpdb_crc32c.so")
ARCH = "gfx950"

SOURCES = ["crc32c_kernels.hip", "crc32c_server.hip", "crc32c_variants.hip", "crc32c_capi.cpp", "crc32c_tables.cpp"]
HEADERS = ["crc32c_math.h", "crc32c_internal.h", "crc32c_device.h"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the pebblesdb_amd HIP library cannot be built")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "pdb_crc32c.h"))
    deps.append(os.path.join(ROOT, "include", "pebblesdb_amd", "crc32c.h"))
    deps.append(os.path.join(ROOT, "include", "pebblesdb_amd", "table_blocks.h"))
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [
        _hipcc(),
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-Wall",
        "-Wno-unused-function",
        f"-I{os.path.join(ROOT, 'include')}",
        "-o",
        tmp,
    ] + [os.path.join(CSRC, f) for f in SOURCES if os.path.exists(os.path.join(CSRC, f))]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
