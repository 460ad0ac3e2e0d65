"""sstable block hooks (table/table_builder.cc:187-205 WriteRawBlock, table/format.cc:66-148
ReadBlock) through pebblesdb_amd.table.  CPU: the handle/footer codecs.  GPU: trailers vs the
reference-generated golden trailers and vs the oracle, corruption detection."""
import numpy as np
import pytest

from pebblesdb_amd import table as T


def test_varint_handle_roundtrip():
    for off, size in [(0, 0), (1, 127), (128, 16383), (2**35 + 7, 4171), (2**63 - 1, 2**40)]:
        h = T.BlockHandle(off, size)
        enc = h.encode()
        assert len(enc) <= T.K_MAX_ENCODED_HANDLE_LENGTH
        d, pos = T.BlockHandle.decode(enc)
        assert d == h and pos == len(enc)
    with pytest.raises(T.Corruption):
        T.BlockHandle.decode(b"\x80\x80")


def test_footer_roundtrip_and_magic():
    f = T.Footer(T.BlockHandle(123456, 51), T.BlockHandle(123512, 3000))
    enc = f.encode()
    assert len(enc) == T.K_FOOTER_ENCODED_LENGTH == 48
    assert T.Footer.decode(b"junk" + enc) == f
    with pytest.raises(T.Corruption):
        T.Footer.decode(enc[:-1] + b"\x00")
    with pytest.raises(T.Corruption):
        T.Footer.decode(b"short")


gpu = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pebblesdb_amd import crc32c

    crc32c.init_device(0)


@gpu
def test_writer_matches_golden_trailers(dev, golden):
    import oracle

    w = T.TableBlockWriter(base_offset=777)
    handles = []
    for t in golden["trailers"]:
        contents = oracle.splitmix_bytes(t["input"]["len"], t["input"]["seed"]).tobytes()
        h = w.add(contents, t["type"])
        handles.append(h)
    w.seal()
    data = w.data
    off = 777
    for t, h in zip(golden["trailers"], handles):
        assert h.offset == off  # WriteRawBlock's handle bookkeeping
        tr = data[h.offset - 777 + h.size : h.offset - 777 + h.size + 5]
        assert tr.hex() == t["trailer_hex"]
        off += h.size + T.K_BLOCK_TRAILER_SIZE
    assert w.next_offset == off


@gpu
def test_verify_and_read_blocks(dev, oracle_lib):
    import oracle

    rng = np.random.Generator(np.random.PCG64(9))
    sizes = [int(x) for x in rng.integers(0, 9000, size=300)] + [4096, 4171, 213 * 1024]
    w = T.TableBlockWriter()
    hs = [w.add(oracle.splitmix_bytes(n, 1000 + i).tobytes(), i % 2) for i, n in enumerate(sizes)]
    w.seal()
    img = bytearray(w.data)
    # trailers agree with the oracle (table_builder.cc:197-199 with the restatement)
    for h in hs[:50]:
        body = bytes(img[h.offset : h.offset + h.size + 1])
        stored = int.from_bytes(img[h.offset + h.size + 1 : h.offset + h.size + 5], "little")
        assert stored == oracle_lib.mask(oracle_lib.value(body))
    assert T.verify_blocks(img, hs).all()
    blocks = T.read_blocks(img, hs)
    assert blocks[5][0] == oracle.splitmix_bytes(sizes[5], 1005).tobytes() and blocks[5][1] == 1
    # one flipped bit in block 17's contents -> ReadBlock's Corruption("block checksum mismatch")
    bad = bytearray(img)
    bad[hs[17].offset + hs[17].size // 2] ^= 0x04
    ok = T.verify_blocks(bad, hs)
    assert ok.sum() == len(hs) - 1 and ok[17] == 0
    with pytest.raises(T.Corruption, match="block checksum mismatch"):
        T.read_block(bad, hs[17])
    with pytest.raises(T.Corruption, match="block checksum mismatch"):
        T.read_blocks(bad, hs)
    assert T.read_block(bad, hs[17], verify_checksums=False)[0] != blocks[17][0]
    # a flipped type byte is covered by the CRC too (contents || type)
    bad = bytearray(img)
    bad[hs[3].offset + hs[3].size] ^= 0x01
    assert T.verify_blocks(bad, hs)[3] == 0
    # truncated read (format.cc:84-87)
    with pytest.raises(T.Corruption, match="truncated block read"):
        T.read_block(img[: hs[-1].offset + 10], hs[-1])


@gpu
def test_pinned_staging_zero_copy_seal_and_verify(dev, oracle_lib):
    """pdb_sst_seal_host / pdb_sst_verify_host on a buffer from pdb_host_alloc run zero-copy (the
    kernel reads the blocks and writes the trailers through the device mapping): the sealed image is
    byte for byte the pageable path's, the verify's ok bytes and bad count agree, a batch that only
    partly lies in the allocation takes the DMA path, and freed allocations are reused."""
    import ctypes

    import oracle
    from pebblesdb_amd import crc32c
    from pebblesdb_amd._native import check, lib

    rng = np.random.Generator(np.random.PCG64(31))
    sizes = np.concatenate([rng.integers(4166, 4175, size=900), rng.integers(0, 9000, size=60), [0, 1, 70000]])
    offs = np.concatenate([[3], 3 + np.cumsum(sizes + 5)[:-1]]).astype(np.int64)
    total = int(offs[-1] + sizes[-1] + 5) + 11
    img = oracle.splitmix_bytes(total, 77).copy()
    img[offs + sizes] = rng.integers(0, 2, size=len(sizes))  # type bytes
    h = np.zeros(len(sizes), dtype=crc32c.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    ref = img.copy()
    check(lib().pdb_sst_seal_host(ref.ctypes.data, total, h.ctypes.data, len(h)))
    for i in (0, 1, 900, len(h) - 1):  # the pageable path against the oracle
        body = ref[offs[i] : offs[i] + sizes[i] + 1].tobytes()
        assert int.from_bytes(ref[offs[i] + sizes[i] + 1 : offs[i] + sizes[i] + 5].tobytes(), "little") == \
            oracle_lib.mask(oracle_lib.value(body))
    p = ctypes.c_void_p()
    check(lib().pdb_host_alloc(total + 64, ctypes.byref(p)))
    pin = np.ctypeslib.as_array((ctypes.c_uint8 * (total + 64)).from_address(p.value))
    pin[:total] = img
    check(lib().pdb_sst_seal_host(p.value, total, h.ctypes.data, len(h)))
    assert (pin[:total] == ref).all()
    ok = np.zeros(len(h), dtype=np.uint8)
    assert lib().pdb_sst_verify_host(p.value, total, h.ctypes.data, len(h), ok.ctypes.data) == 0 and ok.all()
    pin[offs[5] + 9] ^= 0x10
    pin[offs[-1] + sizes[-1]] ^= 0x01  # a type byte
    ok[:] = 1
    assert lib().pdb_sst_verify_host(p.value, total, h.ctypes.data, len(h), ok.ctypes.data) == 2
    assert ok.sum() == len(h) - 2 and ok[5] == 0 and ok[-1] == 0
    # a span reaching past the allocation is still served (by DMA), with the same answer
    big = np.zeros(total + 4096, dtype=np.uint8)
    big[:total] = pin[:total]
    assert lib().pdb_sst_verify_host(big.ctypes.data, total + 4096, h.ctypes.data, len(h), ok.ctypes.data) == 2
    # a freed allocation comes back for a request of about its size; foreign / double frees are errors
    check(lib().pdb_host_free(p))
    q = ctypes.c_void_p()
    check(lib().pdb_host_alloc(total, ctypes.byref(q)))
    assert q.value == p.value
    check(lib().pdb_host_free(q))
    assert lib().pdb_host_free(q) == -3
    assert lib().pdb_host_free(ctypes.c_void_p(big.ctypes.data)) == -3


@gpu
def test_pinned_staging_long_blocks(dev, oracle_lib):
    """A zero-copy seal / verify batch with index- and filter-sized blocks: blocks of 16 KiB and more
    leave the sst kernel for 4-KiB-segment span launches (crc32c_capi.cpp kLongBlock) and the host
    writes / checks their trailers.  Every trailer is checked against the oracle, including the
    sizes either side of the threshold and a 1.3-MiB block; ok bytes keep the handles' order.  The
    pageable route (DMA; 0-byte stand-ins in the sst kernel) gives the same image and verdicts."""
    import ctypes

    import oracle
    from pebblesdb_amd import crc32c
    from pebblesdb_amd._native import check, lib

    rng = np.random.Generator(np.random.PCG64(47))
    longs = [16383, 16384, 16385, 65535, 65543, 4096 * 37 + 3, 1363149, 20000]
    sizes = rng.integers(4166, 4175, size=300).tolist()
    for i, z in enumerate(longs):  # spread through the batch, the last block long
        sizes.insert(20 + 37 * i, z)
    sizes += [0, 7, 300001]
    sizes = np.array(sizes, dtype=np.int64)
    offs = np.concatenate([[5], 5 + np.cumsum(sizes + 5)[:-1]]).astype(np.int64)
    total = int(offs[-1] + sizes[-1] + 5) + 3
    img = oracle.splitmix_bytes(total, 91).copy()
    img[offs + sizes] = rng.integers(0, 2, size=len(sizes))
    h = np.zeros(len(sizes), dtype=crc32c.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    p = ctypes.c_void_p()
    check(lib().pdb_host_alloc(total, ctypes.byref(p)))
    try:
        pin = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p.value))
        pin[:] = img
        check(lib().pdb_sst_seal_host(p.value, total, h.ctypes.data, len(h)))
        for o, z in zip(offs.tolist(), sizes.tolist()):
            word = int.from_bytes(pin[o + z + 1 : o + z + 5].tobytes(), "little")
            assert word == oracle_lib.mask(oracle_lib.value(pin[o : o + z + 1].tobytes())), (o, z)
        mask = np.ones(total, dtype=bool)
        for o, z in zip(offs.tolist(), sizes.tolist()):
            mask[o + z + 1 : o + z + 5] = False
        assert (pin[mask] == img[mask]).all()  # nothing but the trailers written
        ok = np.zeros(len(h), dtype=np.uint8)
        assert lib().pdb_sst_verify_host(p.value, total, h.ctypes.data, len(h), ok.ctypes.data) == 0 and ok.all()
        bad = [int(np.flatnonzero(sizes == 16384)[0]), int(np.flatnonzero(sizes == 1363149)[0]), 3, len(h) - 1]
        pin[offs[bad[0]] + 16000] ^= 0x04
        pin[offs[bad[1]] + sizes[bad[1]]] ^= 0x01  # a type byte
        pin[offs[bad[2]] + 100] ^= 0x80
        pin[offs[bad[3]] + sizes[bad[3]] + 2] ^= 0x10  # a trailer byte
        ok[:] = 1
        assert lib().pdb_sst_verify_host(p.value, total, h.ctypes.data, len(h), ok.ctypes.data) == 4
        assert sorted(np.flatnonzero(ok == 0).tolist()) == sorted(bad)
        # the same batch from pageable memory (the DMA route: 0-byte stand-ins for the long blocks)
        page = img.copy()
        check(lib().pdb_sst_seal_host(page.ctypes.data, total, h.ctypes.data, len(h)))
        pin[offs[bad[0]] + 16000] ^= 0x04  # (undo the corruptions: the sealed image again)
        pin[offs[bad[1]] + sizes[bad[1]]] ^= 0x01
        pin[offs[bad[2]] + 100] ^= 0x80
        pin[offs[bad[3]] + sizes[bad[3]] + 2] ^= 0x10
        assert (page == pin).all()
        ok[:] = 0
        assert lib().pdb_sst_verify_host(page.ctypes.data, total, h.ctypes.data, len(h), ok.ctypes.data) == 0 and ok.all()
        page[offs[bad[0]] + 16000] ^= 0x04
        page[offs[bad[3]] + sizes[bad[3]] + 2] ^= 0x10
        assert lib().pdb_sst_verify_host(page.ctypes.data, total, h.ctypes.data, len(h), ok.ctypes.data) == 2
        assert sorted(np.flatnonzero(ok == 0).tolist()) == sorted([bad[0], bad[3]])
    finally:
        check(lib().pdb_host_free(p))


@gpu
def test_pinned_staging_block_over_64mib(dev, oracle_lib):
    """a host batch with one block of more than 2^14 pieces of 4 KiB (64 MiB) beside
    smaller long blocks.  Zero-copy, such a block leaves the shared descriptor launch for a span
    launch of its own whose result is remapped into the handles' order (crc32c_capi.cpp
    host_sst_mapped); from pageable memory it goes through the device long-block lane.  Every
    trailer vs the oracle, ok bytes in the handles' order, corruptions of the huge block and of a
    neighbour counted once each, on both routes."""
    import ctypes

    import oracle
    from pebblesdb_amd import crc32c
    from pebblesdb_amd._native import check, lib

    rng = np.random.Generator(np.random.PCG64(53))
    huge = (64 << 20) + 4096 * 3 + 11  # (huge + 1) / 4096 > 2^14 pieces
    sizes = rng.integers(4166, 4175, size=40).tolist()
    sizes[5] = 20000
    sizes[17] = huge
    sizes[18] = 1363149  # a long block right after it: the order remap
    sizes[30] = 65536
    sizes += [0, 9]
    sizes = np.array(sizes, dtype=np.int64)
    offs = np.concatenate([[3], 3 + np.cumsum(sizes + 5)[:-1]]).astype(np.int64)
    total = int(offs[-1] + sizes[-1] + 5) + 1
    img = oracle.splitmix_bytes(total, 97).copy()
    img[offs + sizes] = rng.integers(0, 2, size=len(sizes))
    h = np.zeros(len(sizes), dtype=crc32c.HANDLE_DTYPE)
    h["offset"], h["size"] = offs, sizes
    want = [oracle_lib.mask(oracle_lib.value(img[o : o + z + 1].tobytes())) for o, z in zip(offs.tolist(), sizes.tolist())]
    bad = [17, 18, 2]

    def check_image(buf):
        for i, (o, z) in enumerate(zip(offs.tolist(), sizes.tolist())):
            assert int.from_bytes(buf[o + z + 1 : o + z + 5].tobytes(), "little") == want[i], (i, z)

    def corrupt(buf):
        buf[offs[17] + (40 << 20) + 5] ^= 0x20
        buf[offs[18] + sizes[18] + 3] ^= 0x01  # a trailer byte
        buf[offs[2] + 7] ^= 0x80

    p = ctypes.c_void_p()
    check(lib().pdb_host_alloc(total, ctypes.byref(p)))
    try:
        pin = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p.value))
        pin[:] = img
        check(lib().pdb_sst_seal_host(p.value, total, h.ctypes.data, len(h)))
        check_image(pin)
        ok = np.zeros(len(h), dtype=np.uint8)
        assert lib().pdb_sst_verify_host(p.value, total, h.ctypes.data, len(h), ok.ctypes.data) == 0 and ok.all()
        corrupt(pin)
        assert lib().pdb_sst_verify_host(p.value, total, h.ctypes.data, len(h), ok.ctypes.data) == 3
        assert sorted(np.flatnonzero(ok == 0).tolist()) == sorted(bad)
        page = img.copy()  # pageable: the DMA route and the device long-block lane
        check(lib().pdb_sst_seal_host(page.ctypes.data, total, h.ctypes.data, len(h)))
        check_image(page)
        ok[:] = 0
        assert lib().pdb_sst_verify_host(page.ctypes.data, total, h.ctypes.data, len(h), ok.ctypes.data) == 0 and ok.all()
        corrupt(page)
        assert lib().pdb_sst_verify_host(page.ctypes.data, total, h.ctypes.data, len(h), ok.ctypes.data) == 3
        assert sorted(np.flatnonzero(ok == 0).tolist()) == sorted(bad)
    finally:
        check(lib().pdb_host_free(p))
