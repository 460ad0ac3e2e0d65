"""GPU parity: the HIP C-ABI (pebblesdb_amd/_lib/libpdb_crc32c.so) vs the reference's golden
vectors (tests/golden, generated from the reference's own util/crc32c.cc) and vs the oracle on
the same seeded inputs.  Bit-exact is the only bar (integer work).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from pebblesdb_amd import diag  # noqa: E402  (bench / test infrastructure: synthetic input, A/B variants)


@pytest.fixture(scope="module")
def crc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pebblesdb_amd import crc32c

    crc32c.init_device(0)
    return crc32c


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _materialize(spec):
    import oracle

    k = spec["kind"]
    if k == "fill":
        return np.full(spec["len"], spec["byte"], dtype=np.uint8)
    if k == "iota":
        return (np.arange(spec["len"]) & 0xFF).astype(np.uint8)
    if k == "riota":
        return ((spec["len"] - 1 - np.arange(spec["len"])) & 0xFF).astype(np.uint8)
    if k == "hex":
        return np.frombuffer(bytes.fromhex(spec["hex"]), dtype=np.uint8).copy()
    if k == "ascii":
        return np.frombuffer(spec["text"].encode(), dtype=np.uint8).copy()
    if k == "splitmix":
        return oracle.splitmix_bytes(spec["len"], spec["seed"], spec.get("byte_offset", 0))
    raise ValueError(k)


def test_known_answers_scalar(crc, golden):
    """util/crc32c_test.cc:13-60 vectors + db_bench 'x'x4096 through pdb_crc32c_value."""
    for ka in golden["known_answers"]:
        data = _materialize(ka["input"])
        assert crc.value(data) == ka["crc"], ka["name"]
        assert crc.mask(crc.value(data)) == ka["masked"], ka["name"]


def test_known_answers_batch(crc, golden):
    kas = golden["known_answers"]
    datas = [_materialize(k["input"]) for k in kas]
    offs, cur = [], 0
    for d in datas:
        offs.append(cur)
        cur += len(d) + 3  # ragged alignment between blocks
    base = np.zeros(max(cur, 1), dtype=np.uint8)
    for o, d in zip(offs, datas):
        base[o : o + len(d)] = d
    blk = crc.make_blocks(offs, [len(d) for d in datas])
    d_base = torch.from_numpy(base).cuda()
    got = _u32(crc.batch(d_base, crc.blocks_to_device(blk)))
    assert [int(x) for x in got] == [k["crc"] for k in kas]
    host = crc.batch_host(base, blk, masked=True)
    assert [int(x) for x in host] == [k["masked"] for k in kas]


def test_extend_semantics(crc, golden):
    """util/crc32c_test.cc:66-68 and per-block Extend(init, data)."""
    assert crc.value(b"hello world") == crc.extend(crc.value(b"hello "), b"world")
    for e in golden["extend"]:
        data = _materialize(e["input"])
        assert crc.extend(e["init"], data) == e["crc"]


def test_sweep_offsets_lengths(crc, golden):
    """Every byte alignment 0..15 x every length 0..300 (head/tail/chunk boundaries)."""
    sw = golden["sweep"]
    buf = _materialize(sw["input"])
    offs, lens = np.meshgrid(np.arange(sw["offsets"]), np.arange(sw["max_len"] + 1), indexing="ij")
    blk = crc.make_blocks(offs.reshape(-1), lens.reshape(-1))
    got = _u32(crc.batch(torch.from_numpy(buf).cuda(), crc.blocks_to_device(blk)))
    exp = np.array(sw["crc"], dtype=np.uint64).reshape(-1).astype(np.uint32)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first (off,len)={divmod(int(bad[0]), 301)}"


@pytest.mark.parametrize("name", ["fixed4k", "sstable_layout", "zipf_1_64k", "ragged", "ragged_init", "large"])
def test_golden_batches_device(crc, golden, name):
    b = next(x for x in golden["batches"] if x["name"] == name)
    d_base = torch.empty(b["total_bytes"], dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d_base, b["seed"])
    blk = crc.make_blocks(b["off"], b["len"], b["init"] if b["use_init"] else None)
    d_blk = crc.blocks_to_device(blk)
    got = _u32(crc.batch(d_base, d_blk, use_init=b["use_init"]))
    assert (got == np.array(b["crc"], dtype=np.uint32)).all()
    gotm = _u32(crc.batch(d_base, d_blk, use_init=b["use_init"], masked=True))
    assert (gotm == np.array(b["masked"], dtype=np.uint32)).all()


def test_device_fill_matches_numpy(crc):
    import oracle

    for off in (0, 3, 8, 13):
        n = 4096 + 5
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d, 301, byte_offset=off)
        assert (d.cpu().numpy() == oracle.splitmix_bytes(n, 301, off)).all()


@pytest.mark.parametrize("stride,length,nblk,shift", [
    (4096, 4096, 4099, 0),     # fast path (aligned 4 KiB)
    (4096, 4096, 513, 4),      # 4 KiB, 4-B aligned (generic path)
    (4101, 4097, 777, 0),      # sstable-like: contents+type at stride n+5
    (1000, 999, 1000, 1),      # odd everything
    (65536, 65536, 64, 0),     # 16 rounds per lane
    (64, 64, 5000, 0),         # exactly one chunk per block
    (63, 63, 5000, 2),         # head only
])
def test_fixed_stride_vs_oracle(crc, oracle_lib, stride, length, nblk, shift):
    total = shift + (nblk - 1) * stride + length
    d = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 7 + stride)
    view = d[shift : shift + total]
    for masked, init in ((False, None), (True, None), (False, 0xDEADBEEF)):
        got = _u32(crc.batch_fixed(view, stride, length, nblk, masked=masked, init=init))
        host = view.cpu().numpy()
        blk = crc.make_blocks(np.arange(nblk) * stride, np.full(nblk, length),
                              None if init is None else np.full(nblk, init))
        exp = oracle_lib.batch(host, blk, flags=(1 if masked else 0) | (2 if init is not None else 0),
                               nthreads=8)
        assert (got == exp).all(), (masked, init, int(np.nonzero(got != exp)[0][0]))


def test_verify_detects_single_byte_flip(crc):
    n, L = 2048, 4097
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 99)
    blk = crc.blocks_to_device(crc.make_blocks(np.arange(n) * L, np.full(n, L)))
    exp = crc.batch(d, blk, masked=True)
    ok, nbad = crc.verify(d, blk, exp, masked=True)
    assert int(nbad.item()) == 0 and bool(ok.all())
    victim = 1234
    d[victim * L + 2000] ^= 0x10  # ReadBlock would return Corruption("block checksum mismatch")
    ok, nbad = crc.verify(d, blk, exp, masked=True)
    okh = ok.cpu().numpy()
    assert int(nbad.item()) == 1 and okh[victim] == 0 and okh.sum() == n - 1


def test_full_size_config2_vs_oracle(crc, oracle_lib):
    """BASELINE config 2 at full size: 1M x 4 KiB (4 GiB) device-resident, every CRC checked
    against the oracle (multi-threaded) on the same bytes, plus idempotence of the launch."""
    nblk, L = 1 << 20, 4096
    d = torch.empty(nblk * L, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 301)
    got = _u32(crc.batch_fixed(d, L, L, nblk))
    again = _u32(crc.batch_fixed(d, L, L, nblk))
    assert (got == again).all()
    host = d.cpu().numpy()
    del d
    torch.cuda.empty_cache()
    exp = oracle_lib.batch(host, crc.make_blocks(np.arange(nblk) * L, np.full(nblk, L)), nthreads=16)
    assert (got == exp).all(), int(np.count_nonzero(got != exp))


@pytest.mark.parametrize("nblk", [1, 2, 3, 5, 4095, 4096, 4097, 16383, 16384, 16385, 65539])
def test_fast_path_partial_groups(crc, oracle_lib, nblk):
    """4-KiB fast path (4 blocks per wave-iteration, 64-block result windows): every count
    around the wave / group / window boundaries, with seed and mask flags."""
    d = torch.empty(nblk * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 1000 + nblk)
    host = d.cpu().numpy()
    blk = crc.make_blocks(np.arange(nblk) * 4096, np.full(nblk, 4096), np.full(nblk, 0x1234567))
    got = _u32(crc.batch_fixed(d, 4096, 4096, nblk, masked=True, init=0x1234567))
    exp = oracle_lib.batch(host, blk, flags=3, nthreads=8)
    assert (got == exp).all()


def test_device_entry_points_capture_into_hip_graph(crc, oracle_lib):
    """Device entry points are stream-ordered and allocation-free (include/pdb_crc32c.h): a
    captured hipGraph replays them and recomputes after the input changes."""
    nblk = 4096 + 3
    d = torch.empty(nblk * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 77)
    blk = crc.blocks_to_device(crc.make_blocks(np.arange(nblk) * 4096 + 1, np.full(nblk, 4095)))
    out1 = torch.empty(nblk, dtype=torch.int32, device="cuda")
    out2 = torch.empty(nblk, dtype=torch.int32, device="cuda")
    # the record kernel too (size hint 512: WAL-sized records); captured it runs its workgroup-local
    # distribution, since a graph may be replayed beside any other launch
    roffs, rlens = np.arange(20000) * 431 + 6, np.full(20000, 425)
    rblk = crc.blocks_to_device(crc.make_blocks(roffs, rlens))
    out3 = torch.empty(len(roffs), dtype=torch.int32, device="cuda")
    crc.batch_fixed(d, 4096, 4096, nblk, out=out1)  # warm (per-device state exists before capture)
    crc.batch(d, blk, out=out2)
    crc.batch(d, rblk, out=out3, size_hint="512")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        crc.batch_fixed(d, 4096, 4096, nblk, out=out1)
        crc.batch(d, blk, out=out2)
        crc.batch(d, rblk, out=out3, size_hint="512")
    for seed in (78, 79):
        diag.fill_splitmix(d, seed)
        out1.zero_()
        out2.zero_()
        out3.zero_()
        g.replay()
        crc.batch(d, rblk, out=out3, size_hint="512")  # a direct launch after the replay: both exact
        torch.cuda.synchronize()
        host = d.cpu().numpy()
        e1 = oracle_lib.batch(host, crc.make_blocks(np.arange(nblk) * 4096, np.full(nblk, 4096)), nthreads=8)
        e2 = oracle_lib.batch(host, crc.make_blocks(np.arange(nblk) * 4096 + 1, np.full(nblk, 4095)), nthreads=8)
        e3 = oracle_lib.batch(host, crc.make_blocks(roffs, rlens), nthreads=8)
        assert (_u32(out1) == e1).all() and (_u32(out2) == e2).all() and (_u32(out3) == e3).all()


def test_record_batches_on_concurrent_streams(crc, oracle_lib):
    """Record-kernel launches from several streams at once, each launch many times back to back:
    launches that run side by side share nothing (each workgroup's work counter is in its own LDS),
    so every record is hashed exactly once by every launch."""
    import threading

    rng = np.random.Generator(np.random.PCG64(606))
    lens = rng.integers(300, 1000, size=60000)
    offs = np.concatenate([[6], 6 + np.cumsum(lens + 7)[:-1]])
    d = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 607)
    blk = crc.make_blocks(offs, lens)
    d_blk = crc.blocks_to_device(blk)
    exp = oracle_lib.batch(d.cpu().numpy(), blk, nthreads=8)
    torch.cuda.synchronize()
    errors = []

    def run(k):
        st = torch.cuda.Stream()
        outs = [torch.empty(len(lens), dtype=torch.int32, device="cuda") for _ in range(6)]
        with torch.cuda.stream(st):
            for o in outs:
                crc.batch(d, d_blk, out=o, size_hint="1023", stream=st)
        st.synchronize()
        for o in outs:
            if not (_u32(o) == exp).all():
                errors.append(k)

    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("n", [0, 1, 65535, 65536, 65537, 3 * 65536 + 5, (64 << 20) + 13, (1 << 30) + 7])
def test_long_span_extend_device(crc, oracle_lib, n):
    """One span split into parallel segments + device tree combine."""
    d = torch.empty(max(n, 1) + 3, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 555 + n)
    view = d[3 : 3 + n]  # misaligned start
    init = 0x9E3779B9
    host = view.cpu().numpy()
    assert crc.extend_device(init, view, n) == oracle_lib.extend(init, host)
    assert crc.extend_device(0, view, n) == oracle_lib.value(host)


def test_long_span_past_4gib(crc, oracle_lib):
    """> 2^32 bytes in one Extend: the true CRC32C (the reference narrows the length to uint32,
    util/crc32c.cc:19-23,589, so it has no defined answer there; the oracle keeps size_t)."""
    n = (4 << 30) + 4099
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 4242)
    got = crc.extend_device(0x12345678, d, n)
    host = d.cpu().numpy()
    del d
    torch.cuda.empty_cache()
    assert got == oracle_lib.extend(0x12345678, host)


def test_scalar_extend_long_host_span(crc, oracle_lib):
    """pdb_crc32c_extend on host data >= 8 MiB takes the split path."""
    import oracle

    for n in ((8 << 20) + 3, (40 << 20) + 1):
        data = oracle.splitmix_bytes(n, 777 + n)
        assert crc.extend(0xDEADBEEF, data) == oracle_lib.extend(0xDEADBEEF, data)


@pytest.mark.gpu
def test_scalar_extend_zero_copy_sizes(crc, oracle_lib):
    """pdb_crc32c_extend below 8 MiB (pinned mapped staging, no DMA): one-leaf launches below
    64 KiB (incl. the 4096-B packed kernel), span split above; unaligned source pointers; the
    staging buffer growing between calls; results identical to the oracle."""
    import oracle

    sizes = (1, 7, 63, 4095, 4096, 4097, 32768 + 7, 65535, 65536, 65537, (1 << 20) + 3,
             (8 << 20) - 1, 100, 4096)
    for i, n in enumerate(sizes):
        buf = oracle.splitmix_bytes(n + 5, 31 + i)
        data = buf[i % 5 : i % 5 + n]  # caller pointer at every alignment
        init = (0x9E3779B9 * (i + 1)) & 0xFFFFFFFF
        assert crc.extend(init, data) == oracle_lib.extend(init, data), n
        assert crc.value(data) == oracle_lib.value(data), n


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [16])
def test_stream_variants_exact(crc, golden, oracle_lib, variant):
    """The shipped any-length kernel forced on every list (diagnostics variant 16, whatever the
    sizes would route to): the golden sweep (every alignment x every length 0..300), the golden batches, and unaligned /
    multi-round fixed strides, all against the reference's vectors and the oracle."""
    sw = golden["sweep"]
    buf = _materialize(sw["input"])
    offs, lens = np.meshgrid(np.arange(sw["offsets"]), np.arange(sw["max_len"] + 1), indexing="ij")
    blk = crc.make_blocks(offs.reshape(-1), lens.reshape(-1))
    got = _u32(diag.batch_desc(variant, torch.from_numpy(buf).cuda(), crc.blocks_to_device(blk)))
    exp = np.array(sw["crc"], dtype=np.uint64).reshape(-1).astype(np.uint32)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} sweep mismatches, first (off,len)={divmod(int(bad[0]), 301)}"
    for b in golden["batches"]:
        d_base = torch.empty(b["total_bytes"], dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d_base, b["seed"])
        blk = crc.make_blocks(b["off"], b["len"], b["init"] if b["use_init"] else None)
        flags = crc.MASK_OUTPUT | (crc.USE_INIT if b["use_init"] else 0)
        got = _u32(diag.batch_desc(variant, d_base, crc.blocks_to_device(blk), flags=flags))
        assert (got == np.array(b["masked"], dtype=np.uint32)).all(), b["name"]
    for stride, length, nblk, shift in ((4101, 4097, 777, 0), (1000, 999, 1000, 1), (65536 + 3, 65536 + 3, 40, 2),
                                        (4096, 4096, 513, 4), (63, 63, 500, 2), (12345, 12289, 100, 3)):
        total = shift + (nblk - 1) * stride + length
        d = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
        diag.fill_splitmix(d, 7 + stride)
        view = d[shift : shift + total]
        got = _u32(diag.batch_fixed(variant, view, stride, length, nblk, init=0xDEADBEEF))
        blk = crc.make_blocks(np.arange(nblk) * stride, np.full(nblk, length), np.full(nblk, 0xDEADBEEF))
        exp = oracle_lib.batch(view.cpu().numpy(), blk, flags=2, nthreads=8)
        assert (got == exp).all(), (stride, length, int(np.nonzero(got != exp)[0][0]))


@pytest.mark.gpu
def test_host_batches_grouped_and_verify_host(crc, golden, oracle_lib):
    """pdb_crc32c_batch_host / pdb_crc32c_verify_host over the golden Zipf and ragged batches
    (empty blocks, unaligned offsets, blocks larger than a staging group): CRCs equal the
    reference's, corrupted expected values are counted and flagged exactly.  The same batches laid
    out 300 MiB apart in one host buffer make one call run several 256-MiB staging groups through
    the double-buffered pipeline; tests/host_staging_check.py repeats it all with the group span
    forced down to 8 KiB / 3 MiB (PDB_HOST_CHUNK_BYTES, read once per process, so in a child)."""
    gap = 300 << 20
    parts = [b for b in golden["batches"] if b["total_bytes"] <= (64 << 20)]
    for b in parts:
        base = _materialize({"kind": "splitmix", "len": b["total_bytes"], "seed": b["seed"]})
        use_init = b["use_init"]
        blk = crc.make_blocks(b["off"], b["len"], b["init"] if use_init else None)
        exp = np.array(b["crc"], dtype=np.uint64).astype(np.uint32)
        got = crc.batch_host(base, blk, use_init=use_init)
        assert (got == exp).all(), b["name"]
        ok, nbad = crc.verify_host(base, blk, exp, masked=False, use_init=use_init)
        assert nbad == 0 and ok.all(), b["name"]
        bad = exp.copy()
        flip = np.arange(0, len(bad), 7)
        bad[flip] ^= 1
        ok, nbad = crc.verify_host(base, blk, bad, masked=False, use_init=use_init)
        assert nbad == len(flip), b["name"]
        assert (ok[flip] == 0).all() and ok.sum() == len(bad) - len(flip), b["name"]
    # three copies of two batches, 300 MiB apart: three staging groups in one call
    big = np.zeros(3 * gap, dtype=np.uint8)
    blks, exps = [], []
    for k in range(3):
        for b in parts[:2]:
            o = k * gap + (k + 1) * 1000 + (0 if b is parts[0] else 100 << 20)
            big[o : o + b["total_bytes"]] = _materialize({"kind": "splitmix", "len": b["total_bytes"], "seed": b["seed"]})
            blk = crc.make_blocks(np.asarray(b["off"], dtype=np.int64) + o, b["len"], b["init"] if b["use_init"] else None)
            blks.append(blk)
            exps.append(np.array(b["crc"], dtype=np.uint64).astype(np.uint32))
    assert not any(b["use_init"] for b in parts[:2])
    blk, exp = np.concatenate(blks), np.concatenate(exps)
    assert (crc.batch_host(big, blk) == exp).all()
    ok, nbad = crc.verify_host(big, blk, exp, masked=False)
    assert nbad == 0 and ok.all()


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,mask", [(8192, False), (3 << 20, False), (3 << 20, True)])
def test_host_staging_small_groups_subprocess(crc, chunk, mask):
    """The host batch / seal / verify entry points with the staging group span forced small (most
    groups hold one or two blocks, big blocks their own group), in a child process that sets
    PDB_HOST_CHUNK_BYTES before loading the library (tests/host_staging_check.py); with `mask`, through
    pdb_crc32c_init_mask({0}) -- the striped host route on the one device this box has (the plan over
    more devices: tests/test_capi.py::test_stripe_plan)."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, PDB_HOST_CHUNK_BYTES=str(chunk))
    r = subprocess.run([sys.executable, os.path.join(here, "host_staging_check.py")] + (["--mask"] if mask else []), env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host staging ok" in r.stdout


@pytest.mark.gpu
def test_round_boundaries_all_stream_paths(crc, oracle_lib):
    """Block lengths around every round boundary of the stream kernels -- 4-KiB rounds, the last
    round's extra chain (up to +2 KiB of 32-B pieces / +1 KiB of 16-B pieces), one past it -- at
    every 4-B phase, through the descriptor path (16-B kernel), the unaligned fixed-stride path
    (32-B kernel), the 4-B-aligned fixed-stride path (16-B kernel) and the sstable hooks."""
    import oracle
    from pebblesdb_amd import table as T

    deltas = [-33, -17, -1, 0, 1, 15, 31, 32, 33, 100, 1007, 1023, 1024, 1025, 1040, 1041, 2047, 2048,
              2049, 2080, 2081, 3000]
    lens = sorted({4096 * r + d for r in (0, 1, 2, 3) for d in deltas if 4096 * r + d > 0})
    offs, cur = [], 0
    for i, n in enumerate(lens * 4):
        cur += (i % 4) + 1  # every 4-B phase
        offs.append(cur)
        cur += n
    all_lens = lens * 4
    base = oracle.splitmix_bytes(cur + 64, 999)
    blk = crc.make_blocks(offs, all_lens)
    exp = oracle_lib.batch(base, blk)
    d_base = torch.from_numpy(base).cuda()
    got = _u32(crc.batch(d_base, crc.blocks_to_device(blk)))
    assert (got == exp).all(), [all_lens[i] for i in np.nonzero(got != exp)[0][:5]]
    for n in lens:
        for stride, lo in ((n + 5, 1), (n + (-n) % 4 + 4, 0)):  # unaligned (32-B) / 4-B aligned (16-B)
            nb = 33
            b2 = crc.make_blocks(lo + np.arange(nb) * stride, np.full(nb, n))
            e2 = oracle_lib.batch(base[: lo + nb * stride + 8], b2)
            g2 = _u32(crc.batch_fixed(d_base[lo:], stride, n, nb))
            assert (g2 == e2).all(), (n, stride)
    # sstable hooks: handles of these sizes (contents n-1 + type byte under the CRC)
    img = bytearray(base[: sum(lens) + 5 * len(lens) + 16].tobytes())
    hs, pos = [], 3
    for n in lens:
        hs.append((pos, n - 1))
        img[pos + n - 1] = 0
        pos += n + 4
    d_img = torch.frombuffer(img, dtype=torch.uint8).cuda()
    d_h = T.handles_to_device(hs)
    T.seal_device(d_img, d_h)
    sealed = d_img.cpu().numpy()
    for (o, sz) in hs:
        want = oracle_lib.mask(oracle_lib.value(sealed[o : o + sz + 1]))
        assert int.from_bytes(sealed[o + sz + 1 : o + sz + 5].tobytes(), "little") == want, sz
    ok, nbad = T.verify_device(d_img, d_h)
    assert int(nbad.item()) == 0 and bool(ok.all())


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["packed", "shuffled", "descending", "overlapping", "gaps"])
def test_byte_balanced_ranges_any_list(crc, oracle_lib, order):
    """Descriptor lists without a size hint run crc_stream16_kernel with byte-balanced workgroup
    ranges (bal_bound: boundaries searched by offset, clamped around the count split so they
    always partition the list).  Every block must be hashed exactly as the oracle does whatever the
    list's order -- packed ascending (C3's shape, the balanced case), shuffled, descending,
    overlapping (all blocks share one window) or with gaps -- and as variant 71 (count split)."""
    rng = np.random.Generator(np.random.PCG64(91))
    n = 60000  # > 4 x 256 workgroups: the search windows are non-trivial
    lens = np.minimum(rng.zipf(1.3, size=n), 40).astype(np.int64) * 97 + rng.integers(0, 97, size=n)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    if order == "shuffled":
        p = rng.permutation(n)
        offs, lens = offs[p], lens[p]
    elif order == "descending":
        offs, lens = offs[::-1].copy(), lens[::-1].copy()
    elif order == "overlapping":
        offs = rng.integers(0, 5000, size=n).astype(np.int64)
    elif order == "gaps":
        offs = offs + np.cumsum(rng.integers(0, 3000, size=n))
    total = int((offs + lens).max()) + 16
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 92)
    blk = crc.make_blocks(offs, lens)
    d_blk = crc.blocks_to_device(blk)
    got = _u32(crc.batch(d, d_blk))
    exp = oracle_lib.batch(d.cpu().numpy(), blk, nthreads=8)
    assert (got == exp).all(), int(np.nonzero(got != exp)[0][0])
    assert (_u32(diag.batch_desc(16, d, d_blk)) == exp).all()
