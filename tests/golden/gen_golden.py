#!/usr/bin/env python3
"""Generate tests/golden/crc32c_golden.json from the REFERENCE CRC32C.

Run in the build container (where /root/reference exists):
    oracle/build_ref.sh && python tests/golden/gen_golden.py

Every expected value below comes from ``oracle/_ref/libpdbref.so`` -- the reference's
own src/util/crc32c.cc compiled in place -- not from this repo's code.  Inputs are stored
generatively (fill byte / iota / hex / splitmix64 seed), so the fixture is small data.

Sections
  known_answers : the reference's unit-test vectors (util/crc32c_test.cc:13-60), the
                  db_bench crc32c probe (db/db_bench.cc:1112-1129) and SURVEY §8(c) edges
  sweep         : offsets 0..15 x lengths 0..300 over one splitmix buffer (alignment prefix
                  and tail paths of util/crc32c.cc:25-32,600-623)
  extend        : Extend(init, data) with random init (util/crc32c.h:14-17)
  batches       : seeded random block batches {off,len,init} + expected crc and Mask(crc)
  trailers      : sstable block trailers [type][Mask(crc(contents||type))]
                  (table/table_builder.cc:187-205)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "crc32c_golden.json")


def materialize(spec: dict) -> np.ndarray:
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


def zipf_kib_sizes(n: int, seed: int, kmax: int = 64) -> np.ndarray:
    """Block sizes k KiB, k in 1..kmax, p(k) ~ 1/k."""
    rng = np.random.Generator(np.random.PCG64(seed))
    k = np.arange(1, kmax + 1)
    p = (1.0 / k) / np.sum(1.0 / k)
    return (rng.choice(k, size=n, p=p) * 1024).astype(np.int64)


def main() -> None:
    if not oracle.reference_available():
        sys.exit("oracle/_ref/libpdbref.so missing: run oracle/build_ref.sh first")
    ref = oracle.Reference()
    out: dict = {
        "generator": "tests/golden/gen_golden.py via oracle/_ref/libpdbref.so "
        "(reference src/util/crc32c.cc compiled in place)",
        "splitmix64": "byte j = byte (j%8) of splitmix64(seed + (j//8 + 1)*0x9E3779B97F4A7C15), LE",
    }

    # ---- known answers -------------------------------------------------------------------
    iscsi = (
        "01c00000000000000000000000000000"
        "14000000000004000000001400000018"
        "28000000000000000200000000000000"
    )
    ka_specs = [
        ("rfc3720 32x00", {"kind": "fill", "byte": 0, "len": 32}, 0x8A9136AA),
        ("rfc3720 32xff", {"kind": "fill", "byte": 255, "len": 32}, 0x62A8AB43),
        ("rfc3720 0..31", {"kind": "iota", "len": 32}, 0x46DD794E),
        ("rfc3720 31..0", {"kind": "riota", "len": 32}, 0x113FDB5C),
        ("rfc3720 iscsi pdu", {"kind": "hex", "hex": iscsi}, 0xD9963A56),
        ("LargeBuffer A x64", {"kind": "fill", "byte": 0x41, "len": 64}, 0x3C36F666),
        ("LargeBuffer A x1024", {"kind": "fill", "byte": 0x41, "len": 1024}, 0xF6607A92),
        ("LargeBuffer A x1111", {"kind": "fill", "byte": 0x41, "len": 1111}, 0xA9BC21EF),
        ("LargeBuffer A x2048", {"kind": "fill", "byte": 0x41, "len": 2048}, 0x88DDB66B),
        ("LargeBuffer A x4096", {"kind": "fill", "byte": 0x41, "len": 4096}, 0x057251E9),
        ("db_bench crc32c x x4096", {"kind": "fill", "byte": 0x78, "len": 4096}, 0xA46AB21F),
        ("4096 x 00", {"kind": "fill", "byte": 0, "len": 4096}, 0x98F94189),
        ("4097 x 00 (block+type 0)", {"kind": "fill", "byte": 0, "len": 4097}, 0xA8A14AA4),
        ("empty", {"kind": "fill", "byte": 0, "len": 0}, 0x00000000),
        ("a", {"kind": "ascii", "text": "a"}, 0xC1D04330),
        ("hello world", {"kind": "ascii", "text": "hello world"}, None),
        ("foo", {"kind": "ascii", "text": "foo"}, None),
    ]
    kas = []
    for name, spec, published in ka_specs:
        v = ref.value(materialize(spec))
        if published is not None and v != published:
            raise SystemExit(f"reference disagrees with its own known answer {name}: {v:#x}")
        kas.append({"name": name, "input": spec, "crc": v, "masked": ref.mask(v)})
    out["known_answers"] = kas
    out["mask_of_zero"] = ref.mask(0)

    # ---- sweep: every offset 0..15 x length 0..300 over one buffer ------------------------
    sweep_seed = 0x5EED
    buf = oracle.splitmix_bytes(16 + 300 + 64, sweep_seed)
    crcs = []
    for off in range(16):
        row = []
        for n in range(301):
            row.append(ref.value(buf[off : off + n]))
        crcs.append(row)
    out["sweep"] = {
        "input": {"kind": "splitmix", "seed": sweep_seed, "len": len(buf)},
        "offsets": 16,
        "max_len": 300,
        "crc": crcs,
    }

    # ---- extend ---------------------------------------------------------------------------
    rng = np.random.Generator(np.random.PCG64(11))
    ext = []
    for i in range(40):
        n = int(rng.integers(0, 9000))
        init = int(rng.integers(0, 2**32))
        spec = {"kind": "splitmix", "seed": 1000 + i, "len": n}
        ext.append({"init": init, "input": spec, "crc": ref.extend(init, materialize(spec))})
    out["extend"] = ext

    # ---- batches --------------------------------------------------------------------------
    batches = []

    def add_batch(name, seed, total, offs, lens, inits=None, flags=0):
        data = oracle.splitmix_bytes(total, seed)
        blk = np.zeros(len(offs), dtype=oracle.BLK_DTYPE)
        blk["off"] = offs
        blk["len"] = lens
        blk["init"] = 0 if inits is None else inits
        f = 2 if inits is not None else 0
        crc = ref.batch(data, blk, flags=f)
        masked = ref.batch(data, blk, flags=f | 1)
        batches.append(
            {
                "name": name,
                "seed": seed,
                "total_bytes": int(total),
                "use_init": inits is not None,
                "off": [int(x) for x in offs],
                "len": [int(x) for x in lens],
                "init": [int(x) for x in (blk["init"])],
                "crc": [int(x) for x in crc],
                "masked": [int(x) for x in masked],
            }
        )

    # (1) fixed stride 4 KiB, like config 2 (scaled down)
    nb = 512
    add_batch("fixed4k", 301, nb * 4096, np.arange(nb) * 4096, np.full(nb, 4096))
    # (2) sstable layout: contents n (+1 type byte under the CRC) packed at stride n+5
    rs = np.random.Generator(np.random.PCG64(302))
    ns = rs.integers(4090, 4200, size=300)
    offs = np.concatenate([[0], np.cumsum(ns + 5)[:-1]])
    add_batch("sstable_layout", 302, int(offs[-1] + ns[-1] + 5), offs, ns + 1)
    # (3) Zipf 1..64 KiB, packed back-to-back
    zs = zipf_kib_sizes(120, 303)
    offs = np.concatenate([[0], np.cumsum(zs)[:-1]])
    add_batch("zipf_1_64k", 303, int(zs.sum()), offs, zs)
    # (4) ragged: tiny and odd lengths at random byte offsets (incl. 0-length)
    rr = np.random.Generator(np.random.PCG64(304))
    lens = np.concatenate([np.arange(0, 80), rr.integers(0, 20000, size=120)])
    offs = rr.integers(0, 1 << 20, size=len(lens))
    add_batch("ragged", 304, (1 << 20) + 20000, offs, lens)
    # (5) Extend semantics per block (random init) over ragged blocks
    inits = rr.integers(0, 2**32, size=len(lens), dtype=np.uint64)
    add_batch("ragged_init", 305, (1 << 20) + 20000, offs, lens, inits=inits)
    # (6) large single blocks (>= several rounds of any GPU chunking)
    lens = np.array([1 << 20, 3 * (1 << 20) + 7, 213 * 1024 + 13, 65536, 65537])
    offs = np.array([0, (1 << 20) + 3, 5 * (1 << 20) + 1, 6 * (1 << 20), 6 * (1 << 20) + 65536 + 9])
    add_batch("large", 306, 7 * (1 << 20), offs, lens)
    out["batches"] = batches

    # ---- sstable trailers -----------------------------------------------------------------
    trailers = []
    for i, (n, t) in enumerate([(4091, 0), (4171, 0), (51, 0), (0, 0), (4096, 1), (213 * 1024, 0), (17, 1)]):
        spec = {"kind": "splitmix", "seed": 400 + i, "len": n}
        contents = materialize(spec)
        crc = ref.extend(ref.value(contents), np.array([t], dtype=np.uint8))
        trailer = bytes([t]) + int(ref.mask(crc)).to_bytes(4, "little")
        trailers.append({"input": spec, "type": t, "trailer_hex": trailer.hex(), "crc": crc})
    out["trailers"] = trailers

    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {OUT} ({os.path.getsize(OUT)} bytes)")
    gen_sstables()
    gen_logs()


SST_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sst")
WRITER = os.path.join(ROOT, "oracle", "_ref", "ref_sstwriter")
# (name, nkeys, value_size, seed, block_size, bloom_bits): written by the reference's TableBuilder
SST_SPECS = [
    ("small_bloom", 1000, 100, 7, 4096, 10),   # ~4.1 KiB data blocks + bloom filter block
    ("bigvals", 40, 3000, 8, 4096, 0),         # values near the block size
    ("tinyblocks", 500, 20, 9, 256, 0),        # table_test's block_size 256 (table_test.cc:452-478)
    ("empty", 0, 0, 10, 4096, 0),              # no data block: metaindex + index + footer only
]


def gen_sstables() -> None:
    """sstables written AND re-read with verify_checksums by the reference itself
    (oracle/_ref/ref_sstwriter: the reference's table/*.cc compiled in place)."""
    import subprocess

    os.makedirs(SST_DIR, exist_ok=True)
    manifest = []
    for name, n, vs, seed, bs, bloom in SST_SPECS:
        line = subprocess.check_output([WRITER, SST_DIR, name, str(n), str(vs), str(seed), str(bs), str(bloom)],
                                       text=True)
        rec = json.loads(line)
        assert rec["reference_verify_ok"], rec
        rec.update({"nkeys": n, "value_size": vs, "seed": seed})
        manifest.append(rec)
    with open(os.path.join(SST_DIR, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_golden.py -> oracle/_ref/ref_sstwriter (reference "
                                "TableBuilder + Table::Open/iterator with verify_checksums)",
                   "tables": manifest}, f, indent=1)
    print(f"wrote {len(manifest)} sstables to {SST_DIR}")



LOG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "log")
LOG_WRITER = os.path.join(ROOT, "oracle", "_ref", "ref_logwriter")
# (name, seed, record lengths): written by the reference's log::Writer, re-read by log::Reader
LOG_SPECS = [
    # empty + tiny records, a record that leaves a 4-byte block tail (zero trailer), records that
    # fill a block exactly, and records fragmented First/Middle/Last across 2-3 blocks
    ("wal_mixed", 11, [0, 1, 7, 100, 32757, 10, 32761 - 17, 40000, 70000, 5, 6, 13, 200, 3000, 0]),
    ("manifest_small", 12, [int(x) for x in np.random.Generator(np.random.PCG64(12)).integers(0, 400, 300)]),
]


def gen_logs() -> None:
    import subprocess

    os.makedirs(LOG_DIR, exist_ok=True)
    manifest = []
    for name, seed, lens in LOG_SPECS:
        path = os.path.join(LOG_DIR, name + ".log")
        rec = json.loads(subprocess.check_output([LOG_WRITER, path, str(seed)] + [str(x) for x in lens],
                                                 text=True))
        assert rec["reference_verify_ok"], rec
        rec.update({"name": name, "file": name + ".log", "seed": seed, "lengths": lens,
                    "payload": "record k: byte j = byte (j%8) of splitmix64(seed + k + 3, j//8)"})
        manifest.append(rec)
    with open(os.path.join(LOG_DIR, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_golden.py -> oracle/_ref/ref_logwriter (reference "
                                "log::Writer + log::Reader with checksums)", "logs": manifest}, f, indent=1)
    print(f"wrote {len(manifest)} logs to {LOG_DIR}")


LOG_READER = os.path.join(ROOT, "oracle", "_ref", "ref_logreader")
BS, HDR = 32768, 7


def _walk_clean(img: bytes):
    """(header offset, length, type) of every physical record of a CLEAN log (generation helper)."""
    out, pos, n = [], 0, len(img)
    while pos + HDR <= n:
        if BS - pos % BS < HDR:
            pos += BS - pos % BS
            continue
        length, typ = img[pos + 4] | (img[pos + 5] << 8), img[pos + 6]
        if typ == 0 and length == 0:
            pos += BS - pos % BS
            continue
        out.append((pos, length, typ))
        pos += HDR + length
    return out


def _corruption_recipes(img: bytes, ref):
    """Deterministic corruptions of one clean log: (name, ops), ops = ("xor", off, byte) |
    ("set", off, hex) | ("truncate", nbytes).  "fixcrc" recipes store the re-masked CRC the
    reference computes for the edited record, so the record passes the check with its new type."""
    recs = _walk_clean(img)
    n = len(img)
    last_block = (n - 1) // BS
    short_last = n % BS != 0

    def not_last_in_block(i):
        return i + 1 < len(recs) and recs[i + 1][0] // BS == recs[i][0] // BS

    def fixcrc(off, length, typ):
        body = bytes([typ]) + img[off + HDR : off + HDR + length]
        c = ref.mask(ref.value(np.frombuffer(body, dtype=np.uint8)))
        return ("set", off, int(c).to_bytes(4, "little").hex())

    mid = [i for i in range(len(recs)) if not_last_in_block(i) and recs[i][1] > 1]
    early = [i for i in mid if recs[i][0] // BS < last_block]
    r = []
    i = mid[len(mid) // 2]
    r.append(("payload_flip_mid_block", [("xor", recs[i][0] + HDR + recs[i][1] // 2, 0x01)]))
    i = mid[len(mid) // 3]
    r.append(("crc_byte_flip", [("xor", recs[i][0] + 2, 0x80)]))
    if early:
        i = early[len(early) // 2]
        r.append(("length_overrun_mid_file", [("set", recs[i][0] + 4, "ffff")]))
    i = mid[len(mid) // 4]
    L = recs[i][1] - 1
    r.append(("length_shrink", [("set", recs[i][0] + 4, bytes([L & 0xFF, L >> 8]).hex())]))
    i = mid[(2 * len(mid)) // 3]
    r.append(("unknown_type_valid_crc", [("set", recs[i][0] + 6, "09"), fixcrc(recs[i][0], recs[i][1], 9)]))
    # type bytes that collide with log::Reader's own return values kEof (5) / kBadRecord (6), and
    # type bytes >= 0x80 (a signed char read into an unsigned int), each with a valid CRC
    i = mid[(3 * len(mid)) // 4]
    r.append(("type_keof_valid_crc", [("set", recs[i][0] + 6, "05"), fixcrc(recs[i][0], recs[i][1], 5)]))
    i = mid[(3 * len(mid)) // 5]
    r.append(("type_kbadrecord_valid_crc", [("set", recs[i][0] + 6, "06"), fixcrc(recs[i][0], recs[i][1], 6)]))
    i = mid[(4 * len(mid)) // 5]
    r.append(("type_0x80_valid_crc", [("set", recs[i][0] + 6, "80"), fixcrc(recs[i][0], recs[i][1], 0x80)]))
    r.append(("type_0xff_valid_crc", [("set", recs[i][0] + 6, "ff"), fixcrc(recs[i][0], recs[i][1], 0xFF)]))
    i = mid[len(mid) // 5]
    r.append(("zero_header_mid_block", [("set", recs[i][0], "00" * HDR)]))
    firsts = [k for k in range(len(recs)) if recs[k][2] == 2 and recs[k][1] > 0]
    if firsts:
        k = firsts[len(firsts) // 2]
        r.append(("first_fragment_flip", [("xor", recs[k][0] + HDR + recs[k][1] - 1, 0x40)]))
    tails = [k for k in range(len(recs)) if recs[k][2] in (3, 4)]
    if tails:
        k = tails[len(tails) // 2]
        r.append(("fragment_as_full_valid_crc", [("set", recs[k][0] + 6, "01"), fixcrc(recs[k][0], recs[k][1], 1)]))
        r.append(("fragment_as_first_valid_crc", [("set", recs[k][0] + 6, "02"), fixcrc(recs[k][0], recs[k][1], 2)]))
        # mid-fragment: kBadRecord reports 'error in middle of record'; kEof ends the read silently
        r.append(("fragment_as_kbadrecord_valid_crc", [("set", recs[k][0] + 6, "06"), fixcrc(recs[k][0], recs[k][1], 6)]))
        r.append(("fragment_as_keof_valid_crc", [("set", recs[k][0] + 6, "05"), fixcrc(recs[k][0], recs[k][1], 5)]))
    fulls = [k for k in mid if recs[k][2] == 1]
    if len(fulls) > 2:
        k = fulls[len(fulls) // 2]
        r.append(("full_as_middle_valid_crc", [("set", recs[k][0] + 6, "03"), fixcrc(recs[k][0], recs[k][1], 3)]))
        k2 = fulls[len(fulls) // 2 + 1]
        r.append(("full_as_first_then_full", [("set", recs[k2][0] + 6, "02"), fixcrc(recs[k2][0], recs[k2][1], 2)]))
    lastrec = recs[-1]
    if lastrec[1] > 2:
        r.append(("truncate_inside_last_record", [("truncate", lastrec[0] + HDR + lastrec[1] // 2)]))
    r.append(("truncate_inside_last_header", [("truncate", lastrec[0] + 3)]))
    if short_last:
        lr = [k for k in range(len(recs)) if recs[k][0] // BS == last_block and k + 1 < len(recs)]
        if lr:
            k = lr[len(lr) // 2]
            r.append(("length_overrun_last_block", [("set", recs[k][0] + 4, "ffff")]))
    r.append(("two_bad_records_same_block", [("xor", recs[mid[1]][0] + HDR, 0x01),
                                             ("xor", recs[mid[1] + 1][0] + HDR + recs[mid[1] + 1][1] - 1, 0x01)]
              if recs[mid[1] + 1][1] > 0 else [("xor", recs[mid[1]][0] + HDR, 0x01)]))
    return r


def apply_ops(img: bytes, ops) -> bytes:
    b = bytearray(img)
    for op in ops:
        if op[0] == "xor":
            b[op[1]] ^= op[2]
        elif op[0] == "set":
            v = bytes.fromhex(op[2])
            b[op[1] : op[1] + len(v)] = v
        elif op[0] == "truncate":
            del b[op[1] :]
    return bytes(b)


def gen_log_corruptions() -> None:
    """tests/golden/log/corruptions.json: what the REFERENCE's log::Reader (checksums on) delivers
    from corrupted copies of the golden logs -- logical records (LastRecordOffset, length, FNV-1a-64)
    and corruption reports (bytes, reason) -- pinning the batched verifier's replay of
    log_reader.cc:59-263 (bad CRC drops the rest of the block, bad lengths, zero regions, unknown
    types, fragment assembly, truncated tails)."""
    import subprocess
    import tempfile

    ref = oracle.Reference()
    with open(os.path.join(LOG_DIR, "manifest.json")) as f:
        logs = json.load(f)["logs"]
    cases = []
    for lg in logs:
        with open(os.path.join(LOG_DIR, lg["file"]), "rb") as f:
            img = f.read()
        for name, ops in [("clean", [])] + _corruption_recipes(img, ref):
            bad = apply_ops(img, ops)
            with tempfile.NamedTemporaryFile(suffix=".log") as t:
                t.write(bad)
                t.flush()
                res = json.loads(subprocess.check_output([LOG_READER, t.name], text=True))
            cases.append({"log": lg["name"], "name": name, "ops": [list(o) for o in ops], "records": res["records"],
                          "reports": res["reports"]})
    with open(os.path.join(LOG_DIR, "corruptions.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_golden.py -> oracle/_ref/ref_logreader (reference log::Reader, "
                                "checksums on)",
                   "record": "[LastRecordOffset, length, fnv1a64 hex]", "report": "[bytes, Status::ToString()]",
                   "cases": cases}, f, indent=0)
    print(f"wrote {len(cases)} log corruption cases")


if __name__ == "__main__":
    if "--log-corruptions" in sys.argv:
        gen_log_corruptions()
    else:
        main()
        gen_log_corruptions()
