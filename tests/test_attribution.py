"""CPU: the attribution harness (integration/_build/pdb_dbbench_buffered_cpu: the GPU build's
buffered emission and read-ahead windows, every checksum on the CPU through the reference's own
crc32c, integration/pdb_crc_route.h) writes databases the reference engine reads back with
verify_checksums, and whose every block trailer and log record the oracle accepts -- so the
four-column runs of DESIGN.md §6.1d compare like with like.  No GPU: the binary links no GPU
library."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = os.path.join(ROOT, "integration", "_build")


def _exe(name):
    p = os.path.join(B, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (integration/build.sh needs the reference sources)")
    return p


def _run(args, timeout=300):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout, r.stderr


def test_buffered_cpu_build_links_no_gpu_library():
    exe = _exe("pdb_dbbench_buffered_cpu")
    r = subprocess.run(["ldd", exe], capture_output=True, text=True)
    assert r.returncode == 0 and "pdb_crc32c" not in r.stdout and "amdhip" not in r.stdout, r.stdout


def test_buffered_cpu_database_is_the_reference_format(tmp_path, oracle_lib):
    mine, cpu = _exe("pdb_dbbench_buffered_cpu"), _exe("pdb_dbbench_cpu")
    db = str(tmp_path / "db")
    num = 20000
    rc, out, err = _run([mine, "--benchmarks=fillrandom,readseq,readrandom", f"--num={num}", "--value_size=1024",
                         "--verify_checksums=1", f"--db={db}"])
    assert rc == 0, out + err
    res = {d["bench"]: d for d in (json.loads(l) for l in out.splitlines() if l.startswith('{"bench"'))}
    assert res["fillrandom"]["hook"]["seal_blocks"] > 0  # the batched (buffered) seals ran
    h = res["fillrandom"]["hook"]  # the union of the seal calls' intervals is within their sum
    assert 0 < h["seal_busy_s"] <= h["seal_s"] + 1e-3 and h["seal_overlap_max"] >= 1
    assert res["readseq"]["hook"]["scan_batches"] > 0 and res["readseq"]["hook"]["verify_failed"] == 0
    assert f"({num} of {num} found)" in out
    v = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "verify_db_dir.py"), db],
                       capture_output=True, text=True, timeout=300)
    assert v.returncode == 0, v.stdout + v.stderr
    chk = json.loads(v.stdout.strip().splitlines()[-1])
    assert chk["blocks"] > 0 and chk["blocks_bad_oracle"] == 0 and chk["records_bad_oracle"] == 0
    # the reference engine reopens it (WAL recovery with checksums on) and reads every key verified
    rc, out, err = _run([cpu, "--use_existing_db=1", "--benchmarks=readseq,readrandom", f"--num={num}",
                         "--verify_checksums=1", f"--db={db}"])
    assert rc == 0 and f"({num} of {num} found)" in out, out + err


def test_fillrandom_only_run_exits_cleanly(tmp_path):
    """The teardown path of the harness: a fill-only run whose compactions are
    still backed up when the benchmark ends exits 0 on both the CPU build and the buffered build,
    with the database closed (`--close_db=1`: `delete db` waits for the background threads) and left
    open (the default)."""
    for name in ("pdb_dbbench_cpu", "pdb_dbbench_buffered_cpu"):
        exe = _exe(name)
        db = str(tmp_path / name)
        for close in (1, 0):
            rc, out, err = _run([exe, "--benchmarks=fillrandom", "--num=60000", "--value_size=1024",
                                 f"--close_db={close}", f"--db={db}_{close}"])
            assert rc == 0, (name, close, out[-500:], err[-500:])


def test_backed_up_fill_quiesces_before_delete(tmp_path):
    """The teardown fault: the reference engine's destructor can free the table
    cache while a flush or compaction still runs (the engine's own CPU build faults the same way,
    profiles/r04/teardown/).  The harness waits until the database directory has stopped changing
    (--quiesce_ms) and then, by default, exits with the database left open (crash-consistent): a
    fill large enough to leave compactions backed up at the end exits 0 on both CPU builds, reports
    the wait, and the engine as shipped reopens it (WAL replay) and finds every key."""
    for name in ("pdb_dbbench_cpu", "pdb_dbbench_buffered_cpu"):
        exe = _exe(name)
        db = str(tmp_path / name)
        rc, out, err = _run([exe, "--benchmarks=fillrandom", "--num=300000", "--value_size=1024",
                             "--quiesce_ms=500", f"--db={db}"], timeout=600)
        assert rc == 0, (name, out[-500:], err[-800:])
        q = [l for l in err.splitlines() if l.startswith("quiesce: ")]
        assert len(q) == 1 and float(q[0].split()[1]) >= 0.5, err[-800:]
        assert "teardown: skipped" in err, err[-800:]
    cpu = _exe("pdb_dbbench_cpu")
    rc, out, err = _run([cpu, "--use_existing_db=1", "--benchmarks=readrandom", "--num=300000", "--reads=20000",
                         "--verify_checksums=1", f"--db={tmp_path / 'pdb_dbbench_buffered_cpu'}"],
                        timeout=600)
    assert rc == 0 and "(20000 of 20000 found)" in out, out[-500:] + err[-800:]


def _damaged_db(tmp_path, cpu):
    """A database the reference engine wrote, with one byte flipped in the middle data block of its
    largest table; returns (path, table name)."""
    import shutil  # noqa: F401

    sys.path.insert(0, ROOT)
    from pebblesdb_amd import table as T

    db = str(tmp_path / "src")
    rc, out, err = _run([cpu, "--benchmarks=fillrandom", "--num=20000", "--value_size=1024", f"--db={db}"])
    assert rc == 0, out + err
    tables = [f for f in os.listdir(db) if f.endswith((".sst", ".ldb"))]
    big = max(tables, key=lambda f: os.path.getsize(os.path.join(db, f)))
    p = os.path.join(db, big)
    img = bytearray(open(p, "rb").read())
    h = T.table_layout(bytes(img), verify_checksums=False).data
    h = h[len(h) // 2]
    img[h.offset + h.size // 2] ^= 0x10
    open(p, "wb").write(bytes(img))
    return db, big


def repair_and_scan(exe, src, dst):
    """RepairDB with paranoid_checks (every table scanned verified, a failing one rewritten), then a
    verified readseq with a hash of every key and value.  Returns (repair log lines, readseq line,
    hook counters of the repair)."""
    import shutil

    shutil.copytree(src, dst)
    rc, out, err = _run([exe, "--benchmarks=repair,readseq", "--paranoid_checks=1", "--verify_checksums=1", "--hash=1",
                         "--num=20000", f"--db={dst}"])
    assert rc == 0, out + err
    lines = {d["bench"]: d for d in (json.loads(l) for l in out.splitlines() if l.startswith('{"bench"'))}
    seq = next(l for l in out.splitlines() if l.startswith("readseq"))
    log = open(os.path.join(dst, "LOG.old"), errors="replace").read().splitlines()
    rep = sorted(l.split(" ", 2)[2] for l in log if " Table #" in l or " Log #" in l)
    return rep, (lines["readseq"]["ops"], seq.split("(hash")[1]), lines["repair"].get("hook")


def test_repair_paranoid_buffered_matches_reference(tmp_path):
    """SURVEY §8(f) row 1's RepairDB consumer (db/repair.cc:262-267, 339-391) on the batched hooks:
    the buffered build (read-ahead windows + batched TableBuilder, CPU CRC) repairs a damaged
    database exactly as the reference engine does -- same per-table / per-log report lines, same
    recovered entries (count and hash)."""
    cpu, mine = _exe("pdb_dbbench_cpu"), _exe("pdb_dbbench_buffered_cpu")
    src, big = _damaged_db(tmp_path, cpu)
    ref_log, ref_seq, _ = repair_and_scan(cpu, src, str(tmp_path / "ref"))
    my_log, my_seq, hook = repair_and_scan(mine, src, str(tmp_path / "mine"))
    assert any("Corruption: block checksum mismatch" in l for l in ref_log), ref_log
    assert any("entries repaired" in l for l in ref_log), ref_log
    assert my_log == ref_log and my_seq == ref_seq
    assert hook["scan_batches"] > 0 and hook["seal_blocks"] > 0
