"""CPU: pin the oracle (C restatement of src/util/crc32c.cc) against the reference's golden
vectors (tests/golden/crc32c_golden.json, produced from the reference's own crc32c.cc), and
check its two formulations (bit-serial definition, slicing-by-8 restatement) agree."""
import numpy as np
import pytest

import oracle
from tests.test_gpu_parity import _materialize  # same input materialisation as the GPU tests


def test_known_answers(oracle_lib, golden):
    for ka in golden["known_answers"]:
        data = _materialize(ka["input"])
        assert oracle_lib.value(data) == ka["crc"], ka["name"]
        assert oracle_lib.extend_bitwise(0, data) == ka["crc"], ka["name"]
        assert oracle_lib.mask(ka["crc"]) == ka["masked"]
        assert oracle_lib.unmask(ka["masked"]) == ka["crc"]
    assert oracle_lib.mask(0) == golden["mask_of_zero"] == 0xA282EAD8


def test_reference_unit_test_properties(oracle_lib):
    """util/crc32c_test.cc:62-77 (Values, Extend, Mask)."""
    assert oracle_lib.value(b"a") != oracle_lib.value(b"foo")
    assert oracle_lib.value(b"hello world") == oracle_lib.extend(oracle_lib.value(b"hello "), b"world")
    c = oracle_lib.value(b"foo")
    assert c != oracle_lib.mask(c) and c != oracle_lib.mask(oracle_lib.mask(c))
    assert oracle_lib.unmask(oracle_lib.mask(c)) == c
    assert oracle_lib.unmask(oracle_lib.unmask(oracle_lib.mask(oracle_lib.mask(c)))) == c


def test_sweep(oracle_lib, golden):
    sw = golden["sweep"]
    buf = _materialize(sw["input"])
    for off in range(sw["offsets"]):
        for n in range(0, sw["max_len"] + 1, 7):
            assert oracle_lib.value(buf[off : off + n]) == sw["crc"][off][n], (off, n)
    # the full grid through the batch entry (alignment handled inside the restatement)
    offs, lens = np.meshgrid(np.arange(sw["offsets"]), np.arange(sw["max_len"] + 1), indexing="ij")
    blk = np.zeros(offs.size, dtype=oracle.BLK_DTYPE)
    blk["off"], blk["len"] = offs.reshape(-1), lens.reshape(-1)
    got = oracle_lib.batch(buf, blk, nthreads=4)
    assert (got == np.array(sw["crc"], dtype=np.uint64).reshape(-1).astype(np.uint32)).all()


def test_extend(oracle_lib, golden):
    for e in golden["extend"]:
        assert oracle_lib.extend(e["init"], _materialize(e["input"])) == e["crc"]


@pytest.mark.parametrize("name", ["fixed4k", "sstable_layout", "zipf_1_64k", "ragged", "ragged_init", "large"])
def test_batches(oracle_lib, golden, name):
    b = next(x for x in golden["batches"] if x["name"] == name)
    data = oracle.splitmix_bytes(b["total_bytes"], b["seed"])
    blk = np.zeros(len(b["off"]), dtype=oracle.BLK_DTYPE)
    blk["off"], blk["len"], blk["init"] = b["off"], b["len"], b["init"]
    f = 2 if b["use_init"] else 0
    assert (oracle_lib.batch(data, blk, flags=f, nthreads=4) == np.array(b["crc"], dtype=np.uint32)).all()
    assert (oracle_lib.batch(data, blk, flags=f | 1, nthreads=4) == np.array(b["masked"], dtype=np.uint32)).all()


def test_trailers(oracle_lib, golden):
    """table/table_builder.cc:187-205: trailer = [type][Mask(crc(contents||type))] LE."""
    for t in golden["trailers"]:
        contents = _materialize(t["input"])
        crc = oracle_lib.extend(oracle_lib.value(contents), bytes([t["type"]]))
        assert crc == t["crc"]
        assert (bytes([t["type"]]) + oracle_lib.mask(crc).to_bytes(4, "little")).hex() == t["trailer_hex"]
        # ReadBlock's check (table/format.cc:96-98): Value(data, n+1) over contents||type
        assert oracle_lib.value(np.concatenate([contents, np.array([t["type"]], np.uint8)])) == crc


def test_bitwise_vs_sliced_random(oracle_lib):
    rng = np.random.Generator(np.random.PCG64(5))
    buf = rng.integers(0, 256, size=70000, dtype=np.uint8)
    for _ in range(200):
        o = int(rng.integers(0, 1000))
        n = int(rng.integers(0, 3000))
        init = int(rng.integers(0, 2**32))
        assert oracle_lib.extend(init, buf[o : o + n]) == oracle_lib.extend_bitwise(init, buf[o : o + n])


def test_splitmix_c_matches_numpy(oracle_lib):
    for off in (0, 1, 7, 8, 4093):
        assert (oracle_lib.fill(5000, 301, off) == oracle.splitmix_bytes(5000, 301, off)).all()


@pytest.mark.skipif(not oracle.reference_available(), reason="oracle/_ref not built (no /root/reference)")
def test_reference_vs_restatement_random():
    """The compiled reference and the restatement agree on random spans, any alignment."""
    ref, o = oracle.Reference(), oracle.Oracle()
    rng = np.random.Generator(np.random.PCG64(6))
    buf = oracle.splitmix_bytes(200000, 77)
    for _ in range(300):
        off = int(rng.integers(0, 100000))
        n = int(rng.integers(0, 70000))
        init = int(rng.integers(0, 2**32))
        assert ref.extend(init, buf[off : off + n]) == o.extend(init, buf[off : off + n])


@pytest.mark.skipif(not oracle.reference_available(), reason="oracle/_ref not built (reference absent)")
def test_reference_dbbench_loop_golden():
    """db_bench's `crc32c` loop (db/db_bench.cc:1112-1129) run on the reference's own code prints
    crc=0xa46ab21f; bench.py's cpu_baseline reports its MiB/s next to the GPU rate."""
    mib_s, c = oracle.Reference().dbbench_crc32c(8 << 20)
    assert c == 0xA46AB21F and mib_s > 0
