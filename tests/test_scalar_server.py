"""The scalar Extend service (pebblesdb_amd/csrc/crc32c_server.hip): pdb_crc32c_extend on host
bytes <= 64 KiB is answered by a persistent one-workgroup kernel polling a pinned mailbox.

Parity bar: bit-exact against the reference's vectors (tests/golden, generated from the
reference's own util/crc32c.cc) and the oracle, across every alignment/length of the golden
sweep, every size class of the request geometry (head bytes, 4-KiB rounds, 16-KiB load
batches, the 64-KiB cap and the split path above it), and across the server's life cycle:
parked by batch launches, idle exit, lifetime exit, concurrent callers.
"""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def crc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pebblesdb_amd import crc32c

    crc32c.init_device(0)
    return crc32c


def test_golden_sweep_scalar(crc, golden):
    """Every source alignment 0..15 x every length 0..300 (util/crc32c.cc's byte/word paths)."""
    import oracle

    sw = golden["sweep"]
    spec = sw["input"]
    assert spec["kind"] == "splitmix"
    buf = oracle.splitmix_bytes(spec["len"], spec["seed"], spec.get("byte_offset", 0))
    exp = np.array(sw["crc"], dtype=np.uint64).reshape(sw["offsets"], sw["max_len"] + 1)
    bad = []
    for off in range(sw["offsets"]):
        for n in range(sw["max_len"] + 1):
            if crc.value(buf[off : off + n]) != int(exp[off, n]):
                bad.append((off, n))
    assert not bad, f"{len(bad)} mismatches, first (off, len) = {bad[0]}"


def test_known_answers_and_extend(crc, golden):
    assert crc.value(b"x" * 4096) == 0xA46AB21F  # db_bench crc32c (db/db_bench.cc:1112-1129)
    assert crc.value(b"\x00" * 32) == 0x8A9136AA  # util/crc32c_test.cc
    assert crc.value(b"\xff" * 32) == 0x62A8AB43
    import oracle

    for e in golden["extend"]:
        spec = e["input"]
        assert spec["kind"] == "splitmix"
        data = oracle.splitmix_bytes(spec["len"], spec["seed"], spec.get("byte_offset", 0))
        assert crc.extend(e["init"], data) == e["crc"]


@pytest.mark.parametrize(
    "n",
    [1, 15, 16, 17, 1023, 1024, 1041, 4095, 4096, 4097, 4101, 4172, 8191, 16383, 16384, 16385,
     20485, 32768, 32775, 65535, 65536, 65537, 131072 + 9],
)
def test_request_geometry_vs_oracle(crc, oracle_lib, n):
    """Head bytes (n mod 16), partial last rounds, multi-batch requests (> 16 KiB), the 64-KiB
    cap, and sizes just above it (launch path), at unaligned caller pointers."""
    import oracle

    for k in range(3):
        buf = oracle.splitmix_bytes(n + 8, 1000 + n + k)
        data = buf[k * 3 : k * 3 + n]
        init = (0x9E3779B9 * (n + k + 1)) & 0xFFFFFFFF
        assert crc.extend(init, data) == oracle_lib.extend(init, data), (n, k)


def test_server_parked_by_batches(crc, oracle_lib):
    """Scalar calls interleaved with full-grid batch launches (which park the server): every
    answer and every batch stays exact."""
    import oracle

    d = torch.empty(64 * 4096, dtype=torch.uint8, device="cuda")
    __import__('pebblesdb_amd.diag', fromlist=['diag']).fill_splitmix(d, 77)
    host = d.cpu().numpy()
    blk = crc.make_blocks(np.arange(64) * 4096, np.full(64, 4096))
    exp_batch = oracle_lib.batch(host, blk)
    for i in range(20):
        data = oracle.splitmix_bytes(3000 + 37 * i, 500 + i)
        assert crc.value(data) == oracle_lib.value(data)
        got = crc.batch_fixed(d, 4096, 4096, 64).cpu().numpy().view(np.uint32)
        assert (got == exp_batch).all()
        assert crc.extend(i, data[:100]) == oracle_lib.extend(i, data[:100])


def test_server_idle_and_lifetime_exit(crc, oracle_lib):
    """A call after the server's idle exit (20 ms) relaunches it; a stream of calls longer than
    its lifetime (200 ms) crosses at least one relaunch; all answers exact."""
    import oracle

    data = oracle.splitmix_bytes(4101, 9)
    want = oracle_lib.value(data)
    assert crc.value(data) == want
    time.sleep(0.06)
    assert crc.value(data) == want
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < 0.45:
        n = 1 + (i * 613) % 5000
        assert crc.extend(i, data[:n]) == oracle_lib.extend(i, data[:n]), (i, n)
        i += 1
    assert i > 100


def test_concurrent_callers(crc, oracle_lib):
    """Extend is called from the writer, memtable, compaction and reader threads at once
    (db/db_impl.cc:235-239): 4 threads x 300 calls, every answer exact."""
    import oracle

    pool = oracle.splitmix_bytes(70000, 4242)
    errors = []

    def worker(t):
        rng = np.random.default_rng(t)
        for _ in range(300):
            off = int(rng.integers(0, 1000))
            n = int(rng.integers(0, 66000))
            init = int(rng.integers(0, 1 << 32))
            got = crc.extend(init, pool[off : off + n])
            if got != oracle_lib.extend(init, pool[off : off + n]):
                errors.append((t, off, n, init))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:3]


def test_scalar_callers_beside_batch_seals(crc, oracle_lib):
    """The engine's real mix (`pdb_dbbench_gpu_all`): foreground threads call the
    scalar service per WAL record while a compaction thread runs host batches.  Host batches do NOT
    park the server: they run on the CUs it leaves (grid = CUs - 1) from the host-context pool, and
    the server's stream has a hardware queue of its own (greatest priority), so a batch never waits
    behind the persistent kernel (lifetime 200 ms, idle exit 20 ms).  Two scalar threads keep the
    server busy for the whole run; every batch (after one warm-up) must finish far inside the server's
    lifetime, every scalar call too, and every answer is exact."""
    import oracle

    pool = oracle.splitmix_bytes(70000, 777)
    rng = np.random.default_rng(5)
    bsizes = rng.integers(1, 9000, size=3000)
    boffs = np.concatenate([[0], np.cumsum(bsizes)[:-1]])
    bbuf = oracle.splitmix_bytes(int(boffs[-1] + bsizes[-1]), 778)
    blk = crc.make_blocks(boffs, bsizes)
    bexp = oracle_lib.batch(bbuf, blk, flags=0, nthreads=4)
    assert np.array_equal(crc.batch_host(bbuf, blk), bexp)  # warm-up: workspace, code objects
    errors, call_ms, batch_ms = [], [], []
    stop = threading.Event()

    def scalar(t):
        r = np.random.default_rng(t)
        while not stop.is_set():
            off, n, init = int(r.integers(0, 1000)), int(r.integers(0, 1200)), int(r.integers(0, 1 << 32))
            t1 = time.perf_counter()
            got = crc.extend(init, pool[off : off + n])
            call_ms.append((time.perf_counter() - t1) * 1e3)
            if got != oracle_lib.extend(init, pool[off : off + n]):
                errors.append(("scalar", t, off, n))

    th = [threading.Thread(target=scalar, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    time.sleep(0.05)  # the server is up and busy
    try:
        for k in range(12):
            t1 = time.perf_counter()
            ok = np.array_equal(crc.batch_host(bbuf, blk), bexp)
            batch_ms.append((time.perf_counter() - t1) * 1e3)
            if not ok:
                errors.append(("batch", k))
    finally:
        stop.set()
        for x in th:
            x.join()
    assert not errors, errors[:3]
    assert len(call_ms) > 100
    # liveness only (a loaded box may be slow; the latency figures are tools/scalar_latency.py's): a
    # host batch never waits out more than a few of the server's 200-ms lifetimes, no call is stuck
    assert max(batch_ms) < 2000.0, batch_ms
    assert max(call_ms) < 5000.0, max(call_ms)


def test_scalar_slots_shared_by_many_threads(crc, oracle_lib):
    """More calling threads than request slots (64): 80 threads x 25 calls, so slots are shared
    (each slot's mutex serialises its threads); every answer exact, no call stuck."""
    import oracle

    pool = oracle.splitmix_bytes(9000, 4243)
    errors, worst = [], [0.0]

    def worker(t):
        r = np.random.default_rng(100 + t)
        for _ in range(25):
            off, n, init = int(r.integers(0, 500)), int(r.integers(0, 8000)), int(r.integers(0, 1 << 32))
            t1 = time.perf_counter()
            got = crc.extend(init, pool[off : off + n])
            worst[0] = max(worst[0], time.perf_counter() - t1)
            if got != oracle_lib.extend(init, pool[off : off + n]):
                errors.append((t, off, n, init))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(80)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:3]
    assert worst[0] < 30.0, worst[0]  # liveness: no call stuck behind a shared slot
