"""GPU parity of crc_sst4k_kernel -- the sstable-sized-block path (4096..4352 CRC bytes: the
block's last 4 KiB hashed with the 4-KiB geometry, the leading 0..256 B of 4 blocks hashed
together as zero-padded pieces from the unshifted seed) and its in-launch slow path for every
other length -- against the oracle, through the C-ABI sstable hooks (table/table_builder.cc:
193-200 seal, table/format.cc:96-104 verify) and the fixed-stride batch entry.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from pebblesdb_amd import diag  # noqa: E402  (synthetic input, A/B variants)

# CRC input length n = contents + type byte; the kernel's fast range is 4096 <= n <= 4352
EDGE_N = [1, 2, 3, 4, 5, 15, 16, 17, 100, 1024, 4080, 4095, 4096, 4097, 4098, 4099, 4100, 4111, 4112,
          4113, 4127, 4128, 4167, 4170, 4175, 4336, 4337, 4351, 4352, 4353, 4354, 4368, 8191, 8192, 8193,
          12288, 12289]


@pytest.fixture(scope="module")
def crc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pebblesdb_amd import crc32c

    crc32c.init_device(0)
    return crc32c


def _image(sizes, seed, gap_max=7):
    """An sstable-like image: [contents][type][trailer] per block, random 0..gap_max-byte gaps."""
    import oracle

    rng = np.random.Generator(np.random.PCG64(seed))
    gaps = rng.integers(0, gap_max + 1, size=len(sizes))
    offs = np.zeros(len(sizes), dtype=np.int64)
    cur = int(rng.integers(0, 4))
    for i, (sz, g) in enumerate(zip(sizes, gaps)):
        offs[i] = cur
        cur += int(sz) + 5 + int(g)
    img = oracle.splitmix_bytes(cur + 16, seed)
    types = rng.integers(0, 2, size=len(sizes)).astype(np.uint8)
    img[offs + np.asarray(sizes)] = types
    return img, offs


def _expected_trailers(oracle_lib, crc, img, offs, sizes):
    blk = crc.make_blocks(offs, np.asarray(sizes) + 1)
    return oracle_lib.batch(img, blk, flags=1, nthreads=8)  # Mask(crc(contents || type))


def _trailers(img, offs, sizes):
    pos = offs + np.asarray(sizes) + 1
    b = np.stack([img[pos + k] for k in range(4)], axis=1).astype(np.uint32)
    return b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16) | (b[:, 3] << 24)


def _seal_verify_roundtrip(crc, oracle_lib, sizes, seed):
    from pebblesdb_amd import table as T

    sizes = np.asarray(sizes, dtype=np.int64)
    img, offs = _image(sizes, seed)
    exp = _expected_trailers(oracle_lib, crc, img, offs, sizes)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d_img = torch.from_numpy(img).cuda()
    d_h = T.handles_to_device(h)
    T.seal_device(d_img, d_h)
    got = _trailers(d_img.cpu().numpy(), offs, sizes)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} bad trailers, first block {bad[0]} size {sizes[bad[0]]}"
    ok, nbad = T.verify_device(d_img, d_h)
    assert int(nbad.item()) == 0 and bool(ok.cpu().numpy().all())
    return d_img, d_h, offs, sizes


def test_edge_lengths_seal_verify(crc, oracle_lib):
    """Every fast-range boundary (E = 0..16 prefix pieces, z = 0..15 pad bytes) and slow lengths on
    both sides, at every start alignment."""
    sizes = np.array([n - 1 for n in EDGE_N for _ in range(8) if n >= 1], dtype=np.int64)
    _seal_verify_roundtrip(crc, oracle_lib, sizes, 11)


def test_db_bench_sized_blocks(crc, oracle_lib):
    """The fast path proper: 4166-4174-B contents (db_bench data blocks), random gaps."""
    rng = np.random.Generator(np.random.PCG64(5))
    _seal_verify_roundtrip(crc, oracle_lib, rng.integers(4166, 4175, size=20000), 12)


@pytest.mark.parametrize("frac_slow", [0.02, 0.5, 1.0])
def test_mixed_fast_and_slow(crc, oracle_lib, frac_slow):
    """Slow blocks (index / metaindex / last data block sizes) interleaved with fast ones, enough
    per wave to overflow the deferred list (64) several times, plus a few 100-200 KB blocks."""
    rng = np.random.Generator(np.random.PCG64(int(frac_slow * 100) + 1))
    n = 30000
    sizes = rng.integers(4095, 4352, size=n)  # fast (contents + 1 in range)
    slow = rng.random(n) < frac_slow
    sizes[slow] = np.where(rng.random(int(slow.sum())) < 0.5, rng.integers(0, 4095, size=int(slow.sum())),
                           rng.integers(4352, 20000, size=int(slow.sum())))
    big = rng.choice(n, size=6, replace=False)
    sizes[big] = rng.integers(100_000, 213_000, size=6)
    _seal_verify_roundtrip(crc, oracle_lib, sizes, 13)


@pytest.mark.parametrize("nblk", [1, 2, 3, 5, 17, 63, 64, 65, 255, 1025])
def test_partial_groups(crc, oracle_lib, nblk):
    rng = np.random.Generator(np.random.PCG64(nblk))
    sizes = rng.integers(4095, 4352, size=nblk)
    if nblk > 3:
        sizes[::3] = rng.integers(1, 9000, size=len(sizes[::3]))
    _seal_verify_roundtrip(crc, oracle_lib, sizes, 100 + nblk)


def test_verify_detects_corruption(crc, oracle_lib):
    """A flipped byte anywhere under the CRC (prefix, body, type byte) or in the stored trailer
    fails exactly that block, on fast and slow blocks alike."""
    from pebblesdb_amd import table as T

    rng = np.random.Generator(np.random.PCG64(21))
    sizes = rng.integers(4095, 4352, size=4000)
    sizes[::7] = rng.integers(1, 30000, size=len(sizes[::7]))
    d_img, d_h, offs, sizes = _seal_verify_roundtrip(crc, oracle_lib, sizes, 22)
    victims = rng.choice(len(sizes), size=300, replace=False)
    img = d_img.cpu().numpy().copy()
    for v in victims:
        where = int(rng.integers(0, int(sizes[v]) + 1 + 4))  # contents, type byte or trailer
        img[offs[v] + where] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ok, nbad = T.verify_device(torch.from_numpy(img).cuda(), d_h)
    okn = ok.cpu().numpy()
    assert int(nbad.item()) == len(victims)
    assert set(np.nonzero(okn == 0)[0].tolist()) == set(int(v) for v in victims)


def test_host_hooks_same_bytes(crc, oracle_lib):
    """pdb_sst_seal_host / pdb_sst_verify_host (host image, staged groups) on the edge lengths."""
    from pebblesdb_amd import table as T

    sizes = np.array([n - 1 for n in EDGE_N for _ in range(3)], dtype=np.int64)
    img, offs = _image(sizes, 31)
    exp = _expected_trailers(oracle_lib, crc, img, offs, sizes)
    hs = [T.BlockHandle(int(o), int(s)) for o, s in zip(offs, sizes)]
    res = T.verify_blocks(img, hs)  # trailers not sealed yet: (almost) all bad
    assert res.sum() < len(sizes)
    from pebblesdb_amd._native import lib

    h = T._handles_array(hs)
    assert lib().pdb_sst_seal_host(img.ctypes.data, img.size, h.ctypes.data, len(h)) == 0
    assert (_trailers(img, offs, sizes) == exp).all()
    assert T.verify_blocks(img, hs).all()


@pytest.mark.parametrize("length", [4096, 4097, 4100, 4111, 4112, 4113, 4170, 4351, 4352])
@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_fixed_stride_sst_range(crc, oracle_lib, length, shift):
    """pdb_crc32c_batch_device_fixed with len in the fast range and any alignment (the sstable
    layout workload takes this kernel); with an Extend seed the generic kernels serve it."""
    nblk = 1000
    for stride in (length, length + 5):
        total = shift + (nblk - 1) * stride + length
        d = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d, 3 + stride + shift)
        view = d[shift : shift + total]
        host = view.cpu().numpy()
        for masked, init in ((False, None), (True, None), (False, 0x12345678)):
            if length == 4096 and stride == 4096 and shift == 0:
                continue  # the aligned 4-KiB kernel's case
            got = crc.batch_fixed(view, stride, length, nblk, masked=masked, init=init).cpu().numpy().view(np.uint32)
            blk = crc.make_blocks(np.arange(nblk) * stride, np.full(nblk, length),
                                  None if init is None else np.full(nblk, init))
            exp = oracle_lib.batch(host, blk, flags=(1 if masked else 0) | (2 if init is not None else 0),
                                   nthreads=8)
            assert (got == exp).all(), (stride, masked, init)


def test_new_path_matches_previous_kernel(crc):
    """Diagnostics variant 72 seals without parking the trailers (each group's written when hashed)
    and 18 routes the hooks through the 32-B-piece any-length kernel: the same trailers as the
    shipped seal."""
    from pebblesdb_amd import table as T

    rng = np.random.Generator(np.random.PCG64(41))
    sizes = rng.integers(4095, 4352, size=5000)
    sizes[::11] = rng.integers(1, 20000, size=len(sizes[::11]))
    img, offs = _image(sizes, 42)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d_h = T.handles_to_device(h)
    outs = []
    for v in (0, 72, 18):
        d = torch.from_numpy(img).cuda()
        if v == 0:
            T.seal_device(d, d_h)
        else:
            diag.sst(v, d, d_h, seal=True)
        outs.append(d.cpu().numpy())
        ok, nbad = T.verify_device(d, d_h)
        assert int(nbad.item()) == 0, v
    assert all((outs[0] == o).all() for o in outs[1:])


@pytest.mark.parametrize("variant", [0])
def test_parked_seal_matches_plain_seal(crc, variant):
    """The shipped seal parks each wave's trailers (ring of 64 groups, 4 per lane) and writes them
    later.  On 1.3 M blocks (> 64 groups per wave, so every ring wraps; index-sized and tiny blocks
    on the slow path mixed in) the sealed image must equal the one written by variant 72 (each
    group's trailers written when hashed)."""
    from pebblesdb_amd import table as T

    rng = np.random.Generator(np.random.PCG64(77))
    n = 1_300_000
    sizes = rng.integers(4166, 4175, size=n).astype(np.int64)
    sizes[::997] = rng.integers(1, 9000, size=len(sizes[::997]))
    offs = np.concatenate([[0], np.cumsum(sizes + 5)[:-1]])
    total = int(offs[-1] + sizes[-1] + 5)
    img = torch.empty(total, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(img, 78)
    img[torch.from_numpy(offs + sizes).cuda()] = 0
    h = np.zeros(n, dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d_h = T.handles_to_device(h)
    ref = img.clone()
    diag.sst(72, ref, d_h, seal=True)
    got = img.clone()
    if variant == 0:
        T.seal_device(got, d_h)
    else:
        diag.sst(variant, got, d_h, seal=True)
    assert torch.equal(got, ref), variant
    ok, nbad = T.verify_device(got, d_h)
    assert int(nbad.item()) == 0


# ---- descriptor batches with a size-class hint: crc_sst1k_kernel / crc_sst4k_kernel<DescSrc> ----
EDGE_1K = [0, 1, 2, 3, 4, 15, 16, 17, 100, 255, 256, 257, 1000, 1023, 1024, 1025, 1026, 1027, 1039, 1040,
           1041, 1055, 1056, 1100, 1136, 1137, 1151, 1152, 1153, 1168, 1264, 1265, 1279, 1280, 1281, 1282, 2048,
           4095, 4096, 4097, 5000, 70000, 288, 289, 400, 431, 480, 511, 512, 513, 544, 700, 1022]


def _desc_case(crc, sizes, seed, gap_max=7):
    import oracle

    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = np.asarray(sizes, dtype=np.int64)
    gaps = rng.integers(0, gap_max + 1, size=len(sizes))
    offs = np.concatenate([[0], np.cumsum(sizes + gaps)[:-1]]) + int(rng.integers(0, 4))
    total = int(offs[-1] + sizes[-1] + 16)
    base = oracle.splitmix_bytes(total, seed)
    return base, crc.make_blocks(offs, sizes)


@pytest.mark.parametrize("hint", ["1k", "4k", "256", "512", "1023"])
def test_size_hint_edge_lengths(crc, oracle_lib, hint):
    """The sized kernels on every fast-range boundary of every class and slow lengths either
    side, each repeated at 8 alignments, masked and unmasked, batch and verify."""
    sizes = [n for n in EDGE_1K + EDGE_N for _ in range(8)]
    base, blk = _desc_case(crc, sizes, 51)
    d_base = torch.from_numpy(base).cuda()
    d_blk = crc.blocks_to_device(blk)
    for masked in (False, True):
        got = crc.batch(d_base, d_blk, masked=masked, size_hint=hint).cpu().numpy().view(np.uint32)
        exp = oracle_lib.batch(base, blk, flags=1 if masked else 0, nthreads=8)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (hint, masked, bad.size, int(blk["len"][bad[0]]))
    exp = oracle_lib.batch(base, blk, flags=1, nthreads=8)
    wrong = exp.copy()
    flip = np.arange(0, len(exp), 5)
    wrong[flip] ^= 0x10
    ok, nbad = crc.verify(d_base, d_blk, torch.from_numpy(wrong.view(np.int32)).cuda(), size_hint=hint)
    assert int(nbad.item()) == len(flip)
    assert (ok.cpu().numpy() == 0).sum() == len(flip) and (ok.cpu().numpy()[flip] == 0).all()


def test_size_hint_wal_layout(crc, oracle_lib):
    """A WAL image (32-KiB log blocks, 1055-B records fragmented at block ends: type || fragment
    under the CRC) through the 1-KiB kernel, fragments on its slow path."""
    import oracle
    from bench import wal_layout

    offs, lens = wal_layout(24 << 20, 1055)
    total = int(offs[-1] + lens[-1] + 16)
    base = oracle.splitmix_bytes(total, 61)
    blk = crc.make_blocks(offs, lens)
    got = crc.batch(torch.from_numpy(base).cuda(), crc.blocks_to_device(blk), size_hint="1k")
    assert (got.cpu().numpy().view(np.uint32) == oracle_lib.batch(base, blk, nthreads=8)).all()


def test_size_hint_ignored_with_extend_seed(crc, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(71))
    sizes = rng.integers(1024, 1281, size=3000)
    base, blk = _desc_case(crc, sizes, 72)
    blk["init"] = rng.integers(0, 1 << 32, size=len(sizes), dtype=np.uint64).astype(np.uint32)
    got = crc.batch(torch.from_numpy(base).cuda(), crc.blocks_to_device(blk), use_init=True, size_hint="1k")
    assert (got.cpu().numpy().view(np.uint32) == oracle_lib.batch(base, blk, flags=2, nthreads=8)).all()


@pytest.mark.parametrize("lo,hi", [(1024, 1153), (4096, 4353), (1, 257), (900, 1400)])
def test_host_batch_picks_size_class(crc, oracle_lib, lo, hi):
    """pdb_crc32c_batch_host / verify_host choose the sized kernel from the host-visible lengths."""
    rng = np.random.Generator(np.random.PCG64(lo))
    sizes = rng.integers(lo, hi, size=6000)
    sizes[::17] = rng.integers(0, 9000, size=len(sizes[::17]))
    base, blk = _desc_case(crc, sizes, lo + 1)
    exp = oracle_lib.batch(base, blk, flags=1, nthreads=8)
    assert (crc.batch_host(base, blk, masked=True) == exp).all()
    ok, nbad = crc.verify_host(base, blk, exp)
    assert nbad == 0 and ok.all()


def test_sized_kernels_match_generic_kernel(crc):
    """Diagnostics variant 16 ignores the size hints (the any-length crc_stream16_kernel for every
    list): the same CRCs as every sized kernel on a mixed batch, for every size hint."""
    rng = np.random.Generator(np.random.PCG64(81))
    sizes = np.concatenate([rng.integers(1024, 1281, size=4000), rng.integers(4096, 4353, size=4000),
                            rng.integers(0, 300, size=4000), rng.integers(0, 20000, size=2000)])
    rng.shuffle(sizes)
    base, blk = _desc_case(crc, sizes, 82)
    d_base, d_blk = torch.from_numpy(base).cuda(), crc.blocks_to_device(blk)
    hints = (crc.SIZE_1K, crc.SIZE_4K, crc.SIZE_256, crc.SIZE_512, crc.SIZE_1023)
    ref = [crc.batch(d_base, d_blk, size_hint=h).cpu().numpy() for h in ("1k", "4k", "256", "512", "1023")]
    for v in (0, 16):
        for a, hint in zip(ref, hints):
            b = diag.batch_desc(v, d_base, d_blk, flags=hint).cpu().numpy()
            assert (a == b).all(), (v, hint)


@pytest.mark.parametrize("variant", [0, 18])
def test_handles_outside_image_are_reported_not_followed(crc, oracle_lib, variant):
    """A corrupt index can hand out any (offset, size): blocks whose contents + 5-byte trailer do
    not fit the image are bad (verify) and untouched (seal) -- ReadBlock's "truncated block read"
    (table/format.cc:84-87) -- and the kernel never reads or writes outside the image.  The tail of
    the image is a guard region the handles must not reach."""
    from pebblesdb_amd import table as T
    from pebblesdb_amd._native import lib

    rng = np.random.Generator(np.random.PCG64(91))
    sizes = rng.integers(4095, 4352, size=600)
    sizes[::9] = rng.integers(0, 9000, size=len(sizes[::9]))
    img, offs = _image(sizes, 92)
    total = int(offs[-1] + sizes[-1] + 5)  # the image proper; img carries 16 more bytes
    exp = _expected_trailers(oracle_lib, crc, img, offs, sizes)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    bad = rng.choice(len(sizes), size=40, replace=False)
    kinds = np.arange(len(bad)) % 4
    h["offset"][bad[kinds == 0]] = total - 4                   # trailer past the end
    h["size"][bad[kinds == 1]] = total                         # contents past the end
    h["offset"][bad[kinds == 2]] = np.uint64(1) << np.uint64(62)  # offset far out
    h["size"][bad[kinds == 3]] = (np.uint64(1) << np.uint64(32)) + np.uint64(10)  # >= 4 GiB
    guard = np.full(1 << 16, 0xA5, dtype=np.uint8)
    d_img = torch.from_numpy(np.concatenate([img[:total], guard])).cuda()
    d_h = T.handles_to_device(h)
    before = d_img.cpu().numpy().copy()
    sp = int(torch.cuda.current_stream().cuda_stream)
    dl = diag.lib()
    if variant == 0:
        assert lib().pdb_sst_seal_device(d_img.data_ptr(), total, d_h.data_ptr(), len(sizes), sp) == 0
    else:
        assert dl.pdb_diag_sst(variant, d_img.data_ptr(), total, d_h.data_ptr(), len(sizes), 1, None, None, sp) == 0
    after = d_img.cpu().numpy()
    good = np.setdiff1d(np.arange(len(sizes)), bad)
    assert (_trailers(after, offs[good], sizes[good]) == exp[good]).all()
    assert (after[total:] == before[total:]).all(), "seal wrote outside the image"
    ok = torch.empty(len(sizes), dtype=torch.uint8, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    if variant == 0:
        assert lib().pdb_sst_verify_device(d_img.data_ptr(), total, d_h.data_ptr(), len(sizes), ok.data_ptr(),
                                           nbad.data_ptr(), sp) == 0
    else:
        assert dl.pdb_diag_sst(variant, d_img.data_ptr(), total, d_h.data_ptr(), len(sizes), 0, ok.data_ptr(),
                               nbad.data_ptr(), sp) == 0
    okn = ok.cpu().numpy()
    assert int(nbad.item()) == len(bad) and (okn[bad] == 0).all() and (okn[good] == 1).all()


def test_sst_crc_device_matches_seal(crc, oracle_lib):
    """pdb_sst_crc_device: the trailer words a seal would write, as a compact array; out-of-image
    handles leave their entry untouched."""
    from pebblesdb_amd import table as T

    rng = np.random.Generator(np.random.PCG64(101))
    sizes = rng.integers(4095, 4352, size=3000)
    sizes[::13] = rng.integers(0, 20000, size=len(sizes[::13]))
    img, offs = _image(sizes, 102)
    exp = _expected_trailers(oracle_lib, crc, img, offs, sizes)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    h["offset"][7] = len(img)  # out of the image
    d_img = torch.from_numpy(img).cuda()
    out = torch.full((len(sizes),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    T.crc_device(d_img, T.handles_to_device(h), out=out)
    got = out.cpu().numpy().view(np.uint32)
    keep = np.arange(len(sizes)) != 7
    assert (got[keep] == exp[keep]).all() and got[7] == 0x5A5A5A5A
    assert (d_img.cpu().numpy() == img).all()  # nothing written into the image


@pytest.mark.parametrize("length", [1, 2, 3, 15, 16, 17, 100, 131, 255, 256, 257, 288, 431, 511, 512, 513, 700, 1023,
                                    1024, 1025,
                                    1056, 1151, 1152])
def test_fixed_stride_small_classes(crc, oracle_lib, length):
    """pdb_crc32c_batch_device_fixed with len in the 1..256, 257..512 and 1024..1152 classes (the record
    kernels) at every alignment and two strides; with an Extend seed the generic kernels."""
    nblk = 2000
    for shift in range(4):
        for stride in (length, length + 5):
            total = shift + (nblk - 1) * stride + length
            d = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
            diag.fill_splitmix(d, 7 * length + stride + shift)
            view = d[shift : shift + total]
            host = view.cpu().numpy()
            for masked, init in ((False, None), (True, None), (False, 0x0BADF00D)):
                got = crc.batch_fixed(view, stride, length, nblk, masked=masked, init=init).cpu().numpy().view(np.uint32)
                blk = crc.make_blocks(np.arange(nblk) * stride, np.full(nblk, length),
                                      None if init is None else np.full(nblk, init))
                exp = oracle_lib.batch(host, blk, flags=(1 if masked else 0) | (2 if init is not None else 0),
                                       nthreads=8)
                assert (got == exp).all(), (shift, stride, masked, init)


@pytest.mark.parametrize("seed", [95, 96])
def test_lane_per_record_1023_kernel(crc, oracle_lib, seed):
    """crc_lanerec33_kernel (the 513..1023-B class, 256-thread workgroups, window in VGPRs + AGPRs):
    30 001 records of 1..1024 B at any alignment, back to back or with gaps, 0- and > 1024-B ones on
    the slow path; batch and verify; the host entry picks the class from the lengths."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = rng.integers(513, 1024, size=30_001)
    sizes[1::4] = rng.integers(1, 1025, size=len(sizes[1::4]))
    sizes[::997] = 0
    sizes[5::1009] = rng.integers(1025, 9000, size=len(sizes[5::1009]))
    base, blk = _desc_case(crc, sizes, seed, gap_max=0 if seed == 95 else 9)
    d_base, d_blk = torch.from_numpy(base).cuda(), crc.blocks_to_device(blk)
    for masked in (False, True):
        got = crc.batch(d_base, d_blk, masked=masked, size_hint="1023").cpu().numpy().view(np.uint32)
        exp = oracle_lib.batch(base, blk, flags=1 if masked else 0, nthreads=8)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (masked, bad.size, int(blk["len"][bad[0]]), int(blk["off"][bad[0]]))
    wrong = exp.copy()
    flip = np.arange(3, len(exp), 7)
    wrong[flip] ^= 0x100
    ok, nbad = crc.verify(d_base, d_blk, torch.from_numpy(wrong.view(np.int32)).cuda(), size_hint="1023")
    okh = ok.cpu().numpy()
    assert int(nbad.item()) == len(flip) and (okh == 0).sum() == len(flip) and (okh[flip] == 0).all()
    assert (np.asarray(crc.batch_host(base, blk, masked=True)).view(np.uint32) == exp).all()


@pytest.mark.parametrize("seed", [93, 94])
def test_lane_per_record_512_kernel(crc, oracle_lib, seed):
    """crc_lanerec17_kernel (the 257..512-B class, 512-thread workgroups): 60 001 records of
    1..512 B at any alignment, back to back or with gaps, a sprinkling of 0- and > 512-B ones on the
    whole-wave slow path; batch and verify; the host entry picks the class from the lengths."""
    from pebblesdb_amd._native import lib

    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = rng.integers(257, 513, size=60_001)
    sizes[1::3] = rng.integers(1, 513, size=len(sizes[1::3]))
    sizes[::997] = 0
    sizes[5::1009] = rng.integers(513, 6000, size=len(sizes[5::1009]))
    base, blk = _desc_case(crc, sizes, seed, gap_max=0 if seed == 93 else 9)
    d_base, d_blk = torch.from_numpy(base).cuda(), crc.blocks_to_device(blk)
    for masked in (False, True):
        got = crc.batch(d_base, d_blk, masked=masked, size_hint="512").cpu().numpy().view(np.uint32)
        exp = oracle_lib.batch(base, blk, flags=1 if masked else 0, nthreads=8)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (masked, bad.size, int(blk["len"][bad[0]]), int(blk["off"][bad[0]]))
    wrong = exp.copy()
    flip = np.arange(3, len(exp), 7)
    wrong[flip] ^= 0x100
    ok, nbad = crc.verify(d_base, d_blk, torch.from_numpy(wrong.view(np.int32)).cuda(), size_hint="512")
    okh = ok.cpu().numpy()
    assert int(nbad.item()) == len(flip) and (okh == 0).sum() == len(flip) and (okh[flip] == 0).all()
    # host-buffer entry: no hint given, the lengths pick the class
    assert (np.asarray(crc.batch_host(base, blk, masked=True)).view(np.uint32) == exp).all()


@pytest.mark.parametrize("seed", [91, 92])
def test_lane_per_record_kernel(crc, oracle_lib, seed):
    """crc_lanerec9_kernel (the <= 256-B class): 100 003 records of 1..256 B at any alignment,
    back to back or with gaps (the first records within 16 B of the base and a sprinkling of 0- and
    > 256-B ones take the whole-wave slow path inside the same launch), batch and verify, fixed
    stride too."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = rng.integers(1, 257, size=100_003)
    sizes[::997] = 0
    sizes[5::1009] = rng.integers(257, 6000, size=len(sizes[5::1009]))
    base, blk = _desc_case(crc, sizes, seed, gap_max=0 if seed == 91 else 9)
    d_base, d_blk = torch.from_numpy(base).cuda(), crc.blocks_to_device(blk)
    for masked in (False, True):
        got = crc.batch(d_base, d_blk, masked=masked, size_hint="256").cpu().numpy().view(np.uint32)
        exp = oracle_lib.batch(base, blk, flags=1 if masked else 0, nthreads=8)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (masked, bad.size, int(blk["len"][bad[0]]), int(blk["off"][bad[0]]))
    wrong = exp.copy()
    flip = np.arange(3, len(exp), 7)
    wrong[flip] ^= 0x100
    ok, nbad = crc.verify(d_base, d_blk, torch.from_numpy(wrong.view(np.int32)).cuda(), size_hint="256")
    okh = ok.cpu().numpy()
    assert int(nbad.item()) == len(flip) and (okh == 0).sum() == len(flip) and (okh[flip] == 0).all()
