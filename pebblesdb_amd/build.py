"""Build the in-tree HIP libraries for gfx950.

    pebblesdb_amd/_lib/libpdb_crc32c.so       the product: the C-ABI of include/pdb_crc32c.h
    pebblesdb_amd/_lib/libpdb_crc32c_diag.so  bench / test infrastructure (include/pdb_crc32c_diag.h):
                                              synthetic input, A/B variants, roofline calibration

Run ``python -m pebblesdb_amd.build`` (or ``__graft_entry__.build()``).  hipcc cross-compiles
without a GPU; the .so files are git-ignored but travel to the GPU box with the repo snapshot.
Each source compiles once to an object (in parallel); both libraries export only ``pdb_*``
symbols (csrc/pdb_exports.map), so the diagnostics library's copy of the shared kernels never
interposes on the product's.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libpdb_crc32c.so")
DIAG_LIB = os.path.join(LIBDIR, "libpdb_crc32c_diag.so")
ARCH = "gfx950"

SOURCES = ["crc32c_kernels.hip", "crc32c_server.hip", "crc32c_capi.cpp", "crc32c_tables.cpp"]
DIAG_SOURCES = ["diag_variants.hip", "diag_capi.cpp", "crc32c_kernels.hip", "crc32c_tables.cpp"]
INCLUDES = ["pdb_crc32c.h", "pdb_crc32c_diag.h"]
EXPORTS = os.path.join(CSRC, "pdb_exports.map")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the pebblesdb_amd HIP library cannot be built")


def _obj(src: str) -> str:
    return os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")


def _deps(obj: str):
    """Every file the object was compiled from, from the compiler's own -MMD record (so a header
    added to an #include chain is tracked without a hand-kept list).  None if there is no record."""
    try:
        with open(obj + ".d") as f:
            text = f.read().replace("\\\n", " ")
    except OSError:
        return None
    _, _, rest = text.partition(":")
    return rest.split()


def _stale(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    deps = _deps(obj)
    if deps is None:
        return True
    t = os.path.getmtime(obj)
    deps = deps + [os.path.join(CSRC, src)]
    return any(not os.path.exists(d) or os.path.getmtime(d) > t for d in deps)


def _compile(src: str, force: bool, verbose: bool) -> str:
    o = _obj(src)
    if not force and not _stale(o, src):
        return o
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
           f"-I{os.path.join(ROOT, 'include')}", "-MMD", "-MF", o + ".d.tmp", "-c", os.path.join(CSRC, src),
           "-o", o + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(o + ".tmp", o)
    os.replace(o + ".d.tmp", o + ".d")
    return o


def _link(target: str, srcs, verbose: bool) -> None:
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", f"-Wl,--version-script={EXPORTS}", "-o",
           target + ".tmp"] + [_obj(s) for s in srcs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(target + ".tmp", target)


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(set(SOURCES) | set(DIAG_SOURCES))
    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "8"))))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda s: _compile(s, force, verbose), srcs))
    for target, lst in ((LIB, SOURCES), (DIAG_LIB, DIAG_SOURCES)):
        if (force or not os.path.exists(target) or os.path.getmtime(EXPORTS) > os.path.getmtime(target)
                or any(os.path.getmtime(_obj(s)) > os.path.getmtime(target) for s in lst)):
            _link(target, lst, verbose)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
