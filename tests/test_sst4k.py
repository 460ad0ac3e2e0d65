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
        crc.fill_splitmix(d, 3 + stride + shift)
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
    """Variant 30 routes the hooks through the previous any-length kernel: same trailers."""
    from pebblesdb_amd import table as T
    from pebblesdb_amd._native import lib

    rng = np.random.Generator(np.random.PCG64(41))
    sizes = rng.integers(4095, 4352, size=5000)
    sizes[::11] = rng.integers(1, 20000, size=len(sizes[::11]))
    img, offs = _image(sizes, 42)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d_h = T.handles_to_device(h)
    outs = []
    for v in (0, 30):
        lib().pdb_diag_set_variant(v)
        try:
            d = torch.from_numpy(img).cuda()
            T.seal_device(d, d_h)
            outs.append(d.cpu().numpy())
        finally:
            lib().pdb_diag_set_variant(0)
    assert (outs[0] == outs[1]).all()
