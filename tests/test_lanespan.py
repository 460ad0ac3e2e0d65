"""GPU parity of the LDS-staged record kernel (crc_lanespan_kernel, pebblesdb_amd/csrc/
crc32c_lanespan.h) behind the PDB_CRC_SIZE_256 / _512 / _1023 / _1K hints and the 1..1152-B fixed strides:
bit-exact against the oracle on WAL layouts (the reference's record framing, db/log_writer.cc), on
descriptor lists it must cut into smaller groups (spread, unsorted, duplicated, overlapping,
far apart: the staging may only read 16-B lines within 64 B of a record byte), with records outside
the class in the same batches, at batch-boundary counts, and in verify mode.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HINTS = ["256", "512", "1023", "1k"]
CLASS = {"256": 256, "512": 512, "1023": 1023, "1k": 1152}  # the 1K hint: records of 1024..1152 B


@pytest.fixture(scope="module")
def crc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pebblesdb_amd import crc32c

    crc32c.init_device(0)
    return crc32c


def _check(crc, oracle_lib, base, offs, lens, hint, verify=True):
    blk = crc.make_blocks(offs, lens)
    d_base = torch.from_numpy(base).cuda()
    d_blk = crc.blocks_to_device(blk)
    exp = oracle_lib.batch(base, blk, flags=1, nthreads=8)
    got = crc.batch(d_base, d_blk, masked=True, size_hint=hint).cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (hint, bad.size, int(bad[0]), int(lens[bad[0]]), int(offs[bad[0]]))
    if verify:
        wrong = exp.copy()
        flip = np.arange(3, len(exp), 11)
        wrong[flip] ^= 0x100
        ok, nbad = crc.verify(d_base, d_blk, torch.from_numpy(wrong.view(np.int32)).cuda(), size_hint=hint)
        okh = ok.cpu().numpy()
        assert int(nbad.item()) == len(flip) and (okh[flip] == 0).all() and okh.sum() == len(exp) - len(flip)


@pytest.mark.parametrize("payload,hint", [(100, "256"), (131, "256"), (255, "256"), (431, "512"), (300, "512"),
                                          (511, "512"), (600, "1023"), (700, "1023"), (850, "1023"), (1000, "1023"),
                                          (131, "1023"), (1024, "1k"), (1055, "1k"), (1056, "1k"), (1057, "1k"),
                                          (1100, "1k"), (1152, "1k"), (1000, "1k")])
def test_wal_layouts(crc, oracle_lib, payload, hint):
    """Log images as log::Writer lays them out: records + 7-byte headers, fragments at 32-KiB block
    ends, block trailers; the CRC spans are type || payload."""
    import oracle
    from bench import wal_layout

    offs, lens = wal_layout(3 << 20, payload)
    base = oracle.splitmix_bytes(int(offs[-1] + lens[-1]) + 64, payload)
    _check(crc, oracle_lib, base, offs, lens, hint)


@pytest.mark.parametrize("hint", HINTS)
def test_spread_unsorted_and_far_records(crc, oracle_lib, hint):
    """Descriptor lists the span staging must split: gaps of 0..5000 B, a shuffled order, duplicated
    and overlapping records, records 1 MiB apart, records outside the class among them."""
    import oracle

    cls = CLASS[hint]
    rng = np.random.Generator(np.random.PCG64(cls))
    n = 6000
    lens = rng.integers(1, cls + 1, size=n)
    gaps = np.where(rng.random(n) < 0.7, rng.integers(0, 64, size=n), rng.integers(64, 5000, size=n))
    offs = np.concatenate([[5], 5 + np.cumsum(lens + gaps)[:-1]])
    far = rng.random(n) < 0.05  # some records 1 MiB further on
    offs = offs + np.cumsum(far) * (1 << 20)
    perm = rng.permutation(n)
    offs, lens = offs.copy(), lens.copy()
    offs[perm[: n // 4]] = offs[np.sort(perm[: n // 4])]  # a quarter of the list out of order
    lens[perm[: n // 4]] = lens[np.sort(perm[: n // 4])]
    dup = rng.choice(n, size=200, replace=False)
    offs[dup] = offs[(dup + 1) % n]  # duplicates / overlaps of a neighbour
    out = rng.choice(n, size=100, replace=False)
    lens[out] = rng.choice([0, cls + 1, 2000, 70000], size=100)  # outside the class (whole-wave path)
    total = int((offs + lens).max()) + 64
    base = oracle.splitmix_bytes(total, cls + 1)
    _check(crc, oracle_lib, base, offs, lens, hint)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 4095, 4097])
def test_batch_boundaries(crc, oracle_lib, n):
    import oracle

    for hint, L in (("256", 131), ("512", 431), ("1023", 1000), ("1k", 1055), ("1k", 1150)):
        lens = np.full(n, L)
        lens[::7] = L - 3
        offs = np.concatenate([[3], 3 + np.cumsum(lens + 7)[:-1]])
        base = oracle.splitmix_bytes(int(offs[-1] + lens[-1]) + 64, n + L)
        _check(crc, oracle_lib, base, offs, lens, hint, verify=n > 20)


# k (lanes per record) by length (span_pick; words: the record's dwords after its first, ~ length / 4):
# <= 256 B (33-word parts) 1..132 -> 1, 133..256 -> 2; 257..512 B (27-word parts) 257..324 -> 3,
# 325..448 -> 4, 449..512 -> 5; 513..1152 B (33-word parts) ..532 -> 4, ..664 -> 5, ..796 -> 6,
# ..924 -> 7, beyond -> 8 (past 1056 B the head chain runs on alone)
@pytest.mark.parametrize("length", [1, 3, 4, 5, 17, 131, 132, 133, 255, 256, 257, 300, 431, 512, 513, 576, 577, 600,
                                    700, 720, 721, 850, 864, 865, 1000, 1001, 1008, 1009, 1023, 1024, 1055, 1056, 1057,
                                    1100, 1151, 1152])
@pytest.mark.parametrize("shift", [0, 1, 3])
def test_fixed_strides(crc, oracle_lib, length, shift):
    """pdb_crc32c_batch_device_fixed with 1..1152-B blocks (the same kernel, FixedSrc)."""
    from pebblesdb_amd import diag

    nblk = 3001
    for stride in (length, length + 7):
        total = shift + (nblk - 1) * stride + length
        d = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d, stride * 3 + shift)
        view = d[shift : shift + total]
        got = crc.batch_fixed(view, stride, length, nblk, masked=True).cpu().numpy().view(np.uint32)
        blk = crc.make_blocks(np.arange(nblk) * stride, np.full(nblk, length))
        exp = oracle_lib.batch(view.cpu().numpy(), blk, flags=1, nthreads=8)
        assert (got == exp).all(), (length, stride, shift)


@pytest.mark.parametrize("lo,hi,hint", [(1, 257, "256"), (64, 257, "256"), (1, 200, "256"), (120, 216, "512"),
                                        (257, 513, "512m"), (300, 500, "512m"),
                                        (1, 513, "512m"), (64, 1000, "1023m"), (513, 1024, "1023m"), (1, 1024, "1023m"),
                                        (300, 500, "512"), (64, 1000, "1023"), (1024, 1153, "1k"), (1, 1153, "1k")])
def test_mixed_sizes_per_record_lanes(crc, oracle_lib, lo, hi, hint):
    """Logs of records of random sizes, packed with 7-byte headers (a write-heavy WAL with varied
    values): with PDB_CRC_SIZE_MIXED ("512m" / "1023m") a batch's records take their own lane counts
    (ceil(words / part) each, on consecutive lane ranges) -- against the oracle, against the
    batch-uniform-k kernel (diagnostics variant 125), and through the host batch entry, which sets
    the hint itself from the lengths (varied records of 133..216 B: the 512 class, which hashes them
    on two 27-word parts in fewer steps than the 256 class's two 33-word ones)."""
    import oracle
    from pebblesdb_amd import diag

    rng = np.random.Generator(np.random.PCG64(lo * 7 + hi))
    n = 20000
    lens = rng.integers(lo, hi, size=n)
    lens[rng.random(n) < 0.02] = rng.integers(1, 16, size=1)[0]  # a few tiny fragments among them
    offs = np.concatenate([[6], 6 + np.cumsum(lens + 7)[:-1]])
    base = oracle.splitmix_bytes(int(offs[-1] + lens[-1]) + 64, lo + hi)
    _check(crc, oracle_lib, base, offs, lens, hint)
    flags = crc._SIZE_HINT[hint]
    d_base, d_blk = torch.from_numpy(base).cuda(), crc.blocks_to_device(crc.make_blocks(offs, lens))
    a = diag.batch_desc(0, d_base, d_blk, flags=flags).cpu().numpy()
    b = diag.batch_desc(125, d_base, d_blk, flags=flags).cpu().numpy()
    assert (a == b).all()
    blk = crc.make_blocks(offs, lens)
    got = crc.batch_host(base, blk, masked=True).view(np.uint32)
    assert (got == oracle_lib.batch(base, blk, flags=1, nthreads=8)).all()


def test_mixed_geometry_items():
    """The per-record item geometry (diagnostics variant 126: first record, records, lane, lanes per
    record) on a batch of 300-B records with two block-end fragments: records on consecutive lane
    ranges of ceil(words / 27) lanes (words: the record's dwords after its first), at most 64 lanes an item."""
    from pebblesdb_amd import crc32c, diag

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lens = np.full(64 * 40, 431)
    rng = np.random.Generator(np.random.PCG64(5))
    lens[:] = rng.integers(100, 500, size=lens.size)
    offs = np.concatenate([[6], 6 + np.cumsum(lens + 7)[:-1]])
    d = torch.zeros(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens))
    geo = diag.batch_desc(126, d, d_blk, flags=crc32c.SIZE_512 | crc32c.SIZE_MIXED).cpu().numpy().view(np.uint32)
    # the lanes cover a record's dwords after the one holding its first byte (the p-word)
    words = np.maximum(1, ((offs & 3) + lens + 3) // 4 - 1)
    k = np.minimum(5, (words + 26) // 27)
    for b in range(40):
        g = geo[64 * b:64 * b + 64]
        if not (g & 1).all():
            continue  # this batch kept the uniform k
        first, cnt, lane, kl = g >> 24, (g >> 16) & 127, (g >> 8) & 255, (g >> 4) & 15
        assert (kl == k[64 * b:64 * b + 64]).all()
        for r in range(64):
            i0 = int(first[r])
            assert i0 <= r < i0 + int(cnt[r])
            assert lane[r] == int(k[64 * b + i0:64 * b + r].sum()) and lane[r] + kl[r] <= 64


# 125: the batch-uniform lane count only (no per-record lanes for mixed sizes); 133: the cross-lane
# pre-shift's lookups EXEC-masked to the lanes that use them (profiles/r05/ab/ab_slot_lookups_masked.log);
# 134: each part hashed as four chains with three in-part folds (round 5's form, MODE 52; the product hashes
# two chains since round 6)
RECORD_VARIANTS = [125, 133, 134]


@pytest.mark.parametrize("hint", ["256", "512", "512m", "1023", "1023m", "1k"])
def test_record_variants_exact(crc, oracle_lib, hint):
    """The record kernel's diagnostics forms are exact too: spread, unsorted, duplicated and far records with
    records outside the class among them (the slow path), against the oracle."""
    import oracle
    from pebblesdb_amd import diag

    cls = CLASS[hint.rstrip("m")]
    rng = np.random.Generator(np.random.PCG64(cls * 3 + len(hint)))
    n = 3000
    lens = rng.integers(1, cls + 1, size=n)
    gaps = np.where(rng.random(n) < 0.8, 7, rng.integers(0, 3000, size=n))
    offs = np.concatenate([[5], 5 + np.cumsum(lens + gaps)[:-1]])
    out = rng.choice(n, size=40, replace=False)
    lens[out] = rng.choice([0, cls + 1, 2000], size=40)
    base = oracle.splitmix_bytes(int((offs + lens).max()) + 64, cls + 5)
    blk = crc.make_blocks(offs, lens)
    exp = oracle_lib.batch(base, blk, flags=1, nthreads=8)
    d_base, d_blk = torch.from_numpy(base).cuda(), crc.blocks_to_device(blk)
    flags = crc._SIZE_HINT[hint] | 1  # masked output, as crc.batch(masked=True)
    for v in RECORD_VARIANTS:
        got = diag.batch_desc(v, d_base, d_blk, flags=flags).cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (hint, v, bad.size, int(lens[bad[0]]))
