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
    still backed up when the benchmark ends -- `delete db` waits for the background threads --
    exits 0 on both the CPU build and the buffered build."""
    for name in ("pdb_dbbench_cpu", "pdb_dbbench_buffered_cpu"):
        exe = _exe(name)
        db = str(tmp_path / name)
        rc, out, err = _run([exe, "--benchmarks=fillrandom", "--num=60000", "--value_size=1024", f"--db={db}"])
        assert rc == 0, (name, out[-500:], err[-500:])
