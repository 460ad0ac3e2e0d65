"""CPU: the C-ABI library builds for gfx950, loads, and exports every entry point that
include/pdb_crc32c.h declares; pure integer helpers work; compute entry points fail loudly
(PDB_ENODEV) when no GPU is present -- there is no CPU fallback."""
import ctypes
import os
import re
import subprocess

import pytest

from pebblesdb_amd import _native, build, crc32c

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pdb_crc32c.h")


DIAG_HEADER = os.path.join(ROOT, "include", "pdb_crc32c_diag.h")


def declared_functions(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pdb_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    build.build(verbose=False)
    return _native.lib()


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ("pdb_crc32c_extend", "pdb_crc32c_value", "pdb_crc32c_mask", "pdb_crc32c_unmask",
                 "pdb_crc32c_batch_device", "pdb_crc32c_batch_device_fixed", "pdb_crc32c_batch_host",
                 "pdb_crc32c_verify_device", "pdb_sst_seal_host", "pdb_sst_verify_host"):
        assert must in fns


def test_every_declared_symbol_is_exported(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", build.LIB], text=True)
    exported = set(re.findall(r" T (\w+)$", out, flags=re.M))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    # and the ctypes binding covers exactly the declared surface
    assert sorted(_native.SIGNATURES) == declared_functions()


def test_product_exports_only_the_reference_interface(lib):
    """libpdb_crc32c.so exports exactly include/pdb_crc32c.h (the reference interface plus
    init / last_error): no diagnostics, no variant switch, no internal C++ symbols."""
    out = subprocess.check_output(["nm", "-D", "--defined-only", build.LIB], text=True)
    exported = sorted(set(re.findall(r" [TtWV] (\w+)$", out, flags=re.M)))
    assert exported == declared_functions(), sorted(set(exported) ^ set(declared_functions()))
    assert not [f for f in exported if "diag" in f or "variant" in f]


def test_diag_library_is_separate_and_complete(lib):
    """The bench / test library exports its header's functions only and is never loaded by the
    product modules."""
    from pebblesdb_amd import diag

    out = subprocess.check_output(["nm", "-D", "--defined-only", build.DIAG_LIB], text=True)
    exported = sorted(set(re.findall(r" [TtWV] (\w+)$", out, flags=re.M)))
    assert exported == declared_functions(DIAG_HEADER)
    assert sorted(diag.SIGNATURES) == declared_functions(DIAG_HEADER)
    diag.lib()
    for mod in ("pebblesdb_amd/crc32c.py", "pebblesdb_amd/_native.py", "pebblesdb_amd/table.py",
                "pebblesdb_amd/log.py", "pebblesdb_amd/shard.py"):
        assert "diag" not in open(os.path.join(ROOT, mod)).read().replace("diagnostic", ""), mod


def test_flag_constants_match_the_python_mirror():
    """Every PDB_CRC_* flag in the header has the same value in pebblesdb_amd.crc32c."""
    src = open(HEADER).read()
    flags = {k: int(v, 16) for k, v in re.findall(r"#define PDB_CRC_(\w+) (0x[0-9a-fA-F]+)u", src)}
    assert {"MASK_OUTPUT", "USE_INIT", "SIZE_1K", "SIZE_4K", "SIZE_256", "SIZE_512", "SIZE_1023", "SIZE_MIXED"} <= set(flags)
    for k, v in flags.items():
        assert getattr(crc32c, k) == v, k
    assert len(set(flags.values())) == len(flags)  # distinct bits
    # the mixed-size hint only exists with the two classes that take per-record lane counts
    assert crc32c._SIZE_HINT["512m"] == flags["SIZE_512"] | flags["SIZE_MIXED"]
    assert crc32c._SIZE_HINT["1023m"] == flags["SIZE_1023"] | flags["SIZE_MIXED"]


def test_library_is_gfx950_code(lib):
    """The offload bundle inside the .so carries a gfx950 code object (hipcc cross-compile)."""
    blob = open(build.LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob or b"gfx950" in blob


def test_abi_version_and_pure_helpers(lib):
    assert lib.pdb_crc32c_abi_version() == 2
    assert crc32c.mask(0) == 0xA282EAD8
    for c in (0, 1, 0x8A9136AA, 0xFFFFFFFF, 0x12345678):
        assert crc32c.unmask(crc32c.mask(c)) == c
        assert crc32c.mask(c) == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def test_no_cpu_fallback_without_gpu(lib):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(_native.PdbError) as ei:
        crc32c.value(b"abc")
    assert ei.value.code == -1
    with pytest.raises(_native.PdbError):
        crc32c.batch_host(b"abcd", crc32c.make_blocks([0], [4]))
    buf = ctypes.create_string_buffer(16)
    assert lib.pdb_crc32c_batch_device_fixed(buf, 4, 4, 1, 0, 0, buf, None) == -1
    assert b"no CPU fallback" in lib.pdb_last_error()


def test_argument_validation(lib):
    # empty batches are no-ops, even without a device
    assert lib.pdb_crc32c_batch_host(None, 0, None, 0, 0, None) == 0
    assert lib.pdb_sst_seal_host(None, 0, None, 0) == 0
    assert crc32c.extend(0x1234, b"") == 0x1234  # Extend over nothing is the identity
    with pytest.raises(ValueError):
        crc32c.make_blocks([0], [1 << 32])


def _legacy_groups(offs, lens, chunk):
    """Round 5's single-device grouping (crc32c_capi.cpp host_desc): the plan over one device must
    reproduce it exactly."""
    firsts, g_first, lo, hi, count = [], 0, None, 0, 0
    for i, (o, n) in enumerate(zip(offs, lens)):
        if n:
            blo, bhi = o & ~15, o + n
            nlo, nhi = (blo, bhi) if lo is None else (min(lo, blo), max(hi, bhi))
            if count and lo is not None and nhi - nlo > chunk:
                firsts.append(g_first)
                g_first, lo, hi, count = i, blo, bhi, 0
            else:
                lo, hi = nlo, nhi
        count += 1
    firsts.append(g_first)
    return firsts


def _plan(lib, blk, ndev, chunk):
    import numpy as np

    cap = len(blk) + 8
    first = np.zeros(cap, dtype=np.uint64)
    dev = np.zeros(cap, dtype=np.uint32)
    ng = lib.pdb_host_stripe_plan(blk.ctypes.data, len(blk), ndev, chunk, first.ctypes.data, dev.ctypes.data, cap)
    assert ng > 0
    return first[:ng].astype(np.int64), dev[:ng].astype(np.int64)


def test_stripe_plan(lib):
    """pdb_crc32c_init_mask's striping plan (pure host code, no device): groups are contiguous runs
    covering every block in order, each at most `chunk` bytes of span unless one block is longer;
    device indices are non-decreasing and each device's share of the bytes is within one group of 1/N;
    a batch of < 8 MiB per device uses fewer devices; one device reproduces round 5's grouping."""
    import numpy as np

    rng = np.random.Generator(np.random.PCG64(3))
    lens = rng.integers(1, 70000, size=6000).astype(np.int64)
    lens[::97] = 0  # empty blocks ride along in whatever group they fall in
    lens[1234] = 9 << 20  # longer than a chunk: a group of its own
    offs = np.concatenate([[5], 5 + np.cumsum(lens + 3)[:-1]]).astype(np.int64)
    blk = crc32c.make_blocks(offs, lens)
    total = int(lens.sum())
    chunk = 4 << 20
    for ndev in (1, 2, 3, 8):
        first, dev = _plan(lib, blk, ndev, chunk)
        assert first[0] == 0 and (np.diff(first) > 0).all() and first[-1] < len(blk)
        assert (np.diff(dev) >= 0).all() and dev[0] == 0
        nd = int(dev[-1]) + 1
        assert nd == min(ndev, total // (8 << 20))
        ends = np.append(first[1:], len(blk))
        share = np.zeros(nd)
        for f, e, d in zip(first, ends, dev):
            lo = min(int(o) & ~15 for o, n in zip(offs[f:e], lens[f:e]) if n) if lens[f:e].any() else 0
            hi = max(int(o + n) for o, n in zip(offs[f:e], lens[f:e]) if n) if lens[f:e].any() else 0
            assert hi - lo <= chunk or (e - f == 1) or lens[f:e].max() > chunk
            share[d] += lens[f:e].sum()
        assert np.abs(share - total / nd).max() <= chunk + lens.max()
        if ndev == 1:
            assert first.tolist() == _legacy_groups(offs.tolist(), lens.tolist(), chunk)
    # a small batch stays on one device
    first, dev = _plan(lib, blk[:100], 8, 0)
    assert dev.max() == 0 and len(first) == 1
