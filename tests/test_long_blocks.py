"""The long-block lane (crc32c_internal.h, VERDICT r05 "next round" #1): device-resident sstable and
descriptor batches hand every block of >= 16 KiB (> 64 KiB without a size hint) to a piece list
hashed on the whole GPU and folded with shift operators, instead of one wave.  Every trailer, CRC,
ok byte and mismatch count below is checked against the oracle (oracle/crc32c_oracle.c, pinned by
tests/golden): 64 KiB / 1.3 MiB / 4 MiB blocks inside 16 MiB of 4-KiB blocks for seal, verify, crc
and descriptor batches (no hint and the 4K hint with the lane; Extend seeds; the WAL-record hints,
which take no lane, exact on the one-wave path), the thresholds +-1, a 40 MiB block (two LDS
chunks in the combine), the scratch overflowing (more long blocks than records), host batches, and
a captured hipGraph on a prepared and on an unprepared stream.

Reference: table/table_builder.cc:211-266 (Finish writes the filter, metaindex and index blocks),
table/format.cc:66-104 (ReadBlock's check), util/crc32c.cc:25-32 (Extend).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LONGS = [16383, 16384, 16385, 65535, 65536, 65537, 4096 * 37 + 3, 1363149, 4 << 20, 20000]


@pytest.fixture(scope="module")
def crc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pebblesdb_amd import crc32c

    crc32c.init_device(0)
    return crc32c


def _image(longs, nsmall, seed, big=0):
    """An sstable-like image: `nsmall` blocks of 4166..4174 B with `longs` spread among them (and one
    `big` block at the end), each followed by a 5-B trailer, odd offsets.  (sizes, offsets, bytes)."""
    import oracle

    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = rng.integers(4166, 4175, size=nsmall).tolist()
    step = max(1, nsmall // (len(longs) + 1))
    for i, z in enumerate(longs):
        sizes.insert(step * (i + 1) + i, z)
    if big:
        sizes.append(big)
    sizes = np.array(sizes, dtype=np.int64)
    offs = np.concatenate([[3], 3 + np.cumsum(sizes + 5)[:-1]]).astype(np.int64)
    total = int(offs[-1] + sizes[-1] + 5) + 7
    img = oracle.splitmix_bytes(total, seed).copy()
    img[offs + sizes] = rng.integers(0, 2, size=len(sizes))  # type bytes (input to the CRC)
    return sizes, offs, img


def _trailers(oracle_lib, img, offs, sizes):
    """Mask(Value(contents || type)) per block, from the oracle (16 threads)."""
    from pebblesdb_amd import crc32c

    crcs = oracle_lib.batch(img, crc32c.make_blocks(offs, sizes + 1), nthreads=16)
    return (((crcs >> np.uint32(15)) | (crcs << np.uint32(17))) + np.uint32(0xA282EAD8)).astype(np.uint32)


def _stored(img, offs, sizes):
    t = offs + sizes + 1
    return (img[t].astype(np.uint32) | (img[t + 1].astype(np.uint32) << 8) | (img[t + 2].astype(np.uint32) << 16) |
            (img[t + 3].astype(np.uint32) << 24))


@pytest.mark.parametrize("big", [0, 40 << 20])
def test_device_sst_long_blocks(crc, oracle_lib, big):
    from pebblesdb_amd import table as T

    sizes, offs, img = _image(LONGS, (16 << 20) // 4170, 11 + (big > 0), big)
    want = _trailers(oracle_lib, img, offs, sizes)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d = torch.from_numpy(img).cuda()
    d_h = T.handles_to_device(h)
    # the trailer words into a compact array
    got = T.crc_device(d, d_h).cpu().numpy().view(np.uint32)
    assert (got == want).all(), np.flatnonzero(got != want)[:10]
    # in-place seal: exactly the trailer bytes change
    T.seal_device(d, d_h)
    sealed = d.cpu().numpy()
    assert (_stored(sealed, offs, sizes) == want).all()
    mask = np.ones(len(img), dtype=bool)
    for k in range(1, 5):
        mask[offs + sizes + k] = False
    assert (sealed[mask] == img[mask]).all()
    # verify: all good, then one flipped byte in long and short blocks of both kinds
    ok, nbad = T.verify_device(d, d_h)
    assert ok.cpu().numpy().all() and int(nbad.item()) == 0
    bad = [int(np.flatnonzero(sizes == 4 << 20)[0]), int(np.flatnonzero(sizes == 16384)[0]), 7,
           int(np.flatnonzero(sizes == 65537)[0])]
    flips = [offs[bad[0]] + (3 << 20), offs[bad[1]] + sizes[bad[1]], offs[7] + 9, offs[bad[3]] + sizes[bad[3]] + 3]
    if big:
        bad.append(len(sizes) - 1)
        flips.append(offs[-1] + 17)  # the 40 MiB block's first piece (the head)
    for f in flips:
        d[int(f)] ^= 0x20
    ok, nbad = T.verify_device(d, d_h)
    assert int(nbad.item()) == len(bad)
    assert sorted(np.flatnonzero(ok.cpu().numpy() == 0).tolist()) == sorted(bad)


@pytest.mark.parametrize("hint", [None, "4k", "256", "1k"])
@pytest.mark.parametrize("use_init", [False, True])
def test_device_desc_long_blocks(crc, oracle_lib, hint, use_init):
    if use_init and hint is not None:
        pytest.skip("hints are ignored with Extend seeds (any-length kernel)")
    rng = np.random.Generator(np.random.PCG64(5))
    small = {None: (1024, 65536), "4k": (4096, 4353), "256": (1, 257), "1k": (1024, 1153)}[hint]
    sizes = rng.integers(small[0], small[1], size=6000).tolist()
    for i, z in enumerate(LONGS + [0, 1, 65535]):
        sizes.insert(300 + 500 * i, z)
    sizes = np.array(sizes, dtype=np.int64)
    offs = np.concatenate([[1], 1 + np.cumsum(sizes + 3)[:-1]]).astype(np.int64)
    import oracle

    img = oracle.splitmix_bytes(int(offs[-1] + sizes[-1] + 16), 17)
    inits = rng.integers(0, 1 << 32, size=len(sizes), dtype=np.uint64) if use_init else None
    blk = crc.make_blocks(offs, sizes, inits)
    want = oracle_lib.batch(img, blk, flags=2 if use_init else 0, nthreads=16)
    d = torch.from_numpy(img).cuda()
    d_blk = crc.blocks_to_device(blk)
    got = crc.batch(d, d_blk, use_init=use_init, size_hint=hint).cpu().numpy().view(np.uint32)
    assert (got == want).all(), np.flatnonzero(got != want)[:10]
    # verify against masked expectations, two of them wrong (one long, one short)
    exp = (((want >> np.uint32(15)) | (want << np.uint32(17))) + np.uint32(0xA282EAD8)).astype(np.uint32)
    wrong = [int(np.flatnonzero(sizes == 1363149)[0]), 11]
    exp[wrong] ^= 1
    ok, nbad = crc.verify(d, d_blk, torch.from_numpy(exp.view(np.int32)).cuda(), use_init=use_init, size_hint=hint)
    assert int(nbad.item()) == 2
    assert sorted(np.flatnonzero(ok.cpu().numpy() == 0).tolist()) == sorted(wrong)


def test_long_lane_overflow(crc, oracle_lib):
    """More long blocks than the lane has records (65536): the rest are hashed by the batch kernel's
    one-wave path in the same launch, and every trailer is still exact."""
    from pebblesdb_amd import table as T

    n = 72000
    rng = np.random.Generator(np.random.PCG64(23))
    sizes = np.where(np.arange(n) % 20 != 7, 16384 + rng.integers(0, 64, size=n), 4170).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes + 5)[:-1]]).astype(np.int64)
    total = int(offs[-1] + sizes[-1] + 5)
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    from pebblesdb_amd import diag

    diag.fill_splitmix(d, 29)
    d[torch.from_numpy(offs + sizes).cuda()] = 0
    h = np.zeros(n, dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d_h = T.handles_to_device(h)
    got = T.crc_device(d, d_h).cpu().numpy().view(np.uint32)
    img = d.cpu().numpy()
    want = _trailers(oracle_lib, img, offs, sizes)
    assert int((sizes >= 16384).sum()) > 65536
    assert (got == want).all(), np.flatnonzero(got != want)[:10]
    # the lane is reset after an overflowing call: the next call is exact too
    got2 = T.crc_device(d[: int(offs[100])], T.handles_to_device(h[:99])).cpu().numpy().view(np.uint32)
    assert (got2 == want[:99]).all()


def test_host_batches_long_blocks(crc, oracle_lib):
    """Host descriptor batches (the context's own lane) and host sstable seals / verifies with long
    blocks, including one of 70 MiB (more than 2^14 pieces: its own span launch on the zero-copy
    route -- ADVICE r05) among smaller long ones, from pageable and from pinned memory."""
    import ctypes

    from pebblesdb_amd._native import check, lib

    sizes, offs, img = _image(LONGS, 2000, 31, big=70 << 20)
    blk = crc.make_blocks(offs, sizes + 1)
    want_crc = oracle_lib.batch(img, blk, nthreads=16)
    got = crc.batch_host(img, blk)
    assert (got == want_crc).all(), np.flatnonzero(got != want_crc)[:10]
    want = _trailers(oracle_lib, img, offs, sizes)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    page = img.copy()
    check(lib().pdb_sst_seal_host(page.ctypes.data, len(page), h.ctypes.data, len(h)))
    assert (_stored(page, offs, sizes) == want).all()
    p = ctypes.c_void_p()
    check(lib().pdb_host_alloc(len(img), ctypes.byref(p)))
    try:
        pin = np.ctypeslib.as_array((ctypes.c_uint8 * len(img)).from_address(p.value))
        pin[:] = img
        check(lib().pdb_sst_seal_host(p.value, len(pin), h.ctypes.data, len(h)))
        assert (pin == page).all()
        ok = np.zeros(len(h), dtype=np.uint8)
        pin[offs[-1] + (69 << 20)] ^= 1
        pin[offs[5] + 2] ^= 1
        assert lib().pdb_sst_verify_host(p.value, len(pin), h.ctypes.data, len(h), ok.ctypes.data) == 2
        assert sorted(np.flatnonzero(ok == 0).tolist()) == [5, len(h) - 1]
    finally:
        check(lib().pdb_host_free(p))


@pytest.mark.parametrize("prepared", [True, False])
def test_graph_capture_long_blocks(crc, oracle_lib, prepared):
    """A device verify captured into a graph: on a prepared stream the lane is in the graph, on a
    stream first seen inside the capture there is no lane (nothing may be allocated while capturing)
    and the one-wave path runs -- the verdicts are the same."""
    from pebblesdb_amd import table as T
    from pebblesdb_amd._native import check, lib

    sizes, offs, img = _image([1363149, 65536, 20000], 3000, 41)
    want = _trailers(oracle_lib, img, offs, sizes)
    t = offs + sizes + 1
    for k in range(4):
        img[t + k] = (want >> np.uint32(8 * k)).astype(np.uint8)
    h = np.zeros(len(sizes), dtype=crc.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    d = torch.from_numpy(img).cuda()
    d_h = T.handles_to_device(h)
    ok = torch.zeros(len(h), dtype=torch.uint8, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    if prepared:
        check(lib().pdb_crc32c_prepare_stream(int(s.cuda_stream)))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        check(lib().pdb_sst_verify_device(int(d.data_ptr()), len(img), int(d_h.data_ptr()), len(h), int(ok.data_ptr()),
                                          int(nbad.data_ptr()), int(s.cuda_stream)))
    g.replay()
    torch.cuda.synchronize()
    assert ok.cpu().numpy().all() and int(nbad.item()) == 0
    d[int(offs[int(np.flatnonzero(sizes == 1363149)[0])]) + 1000] ^= 0x40
    ok.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert int(nbad.item()) == 1
    assert np.flatnonzero(ok.cpu().numpy() == 0).tolist() == [int(np.flatnonzero(sizes == 1363149)[0])]
