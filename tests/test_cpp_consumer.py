"""The C++ drop-in headers (include/pebblesdb_amd/{crc32c,table_blocks,log_records}.h) compile and link
against the library with plain g++ (CPU), and the consumer test passes on the GPU."""
import os
import subprocess

import pytest

from pebblesdb_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "table_blocks_test.cc")
EXE = os.path.join(ROOT, "tests", "cpp", "table_blocks_test")


def _compile():
    build.build(verbose=False)
    libdir = os.path.dirname(build.LIB)
    subprocess.check_call(["g++", "-O2", "-std=c++11", "-Wall", "-Werror", f"-I{ROOT}/include", SRC,
                           "-o", EXE, f"-L{libdir}", "-lpdb_crc32c", f"-Wl,-rpath,{libdir}"])
    return EXE


def test_cpp_consumer_builds_and_links():
    exe = _compile()
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_cpp_consumer_runs_on_gpu():
    exe = _compile()
    r = subprocess.run([exe, os.path.join(ROOT, "tests", "golden", "sst"), os.path.join(ROOT, "tests", "golden", "log")],
                       capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


@pytest.mark.gpu
def test_cpp_log_replay_matches_reference_reader(tmp_path):
    """pdb::log::ReplayLog (one GPU verify batch + the log::Reader replay) on every corrupted log of
    tests/golden/log/corruptions.json: records and corruption reports identical to what the
    reference's own log::Reader delivered from the same bytes."""
    import json

    from test_log import CORR, _corrupted

    exe = _compile()
    paths = []
    for i, case in enumerate(CORR):
        p = tmp_path / f"case{i}.log"
        p.write_bytes(_corrupted(case))
        paths.append(str(p))
    r = subprocess.run([exe, "--replay"] + paths, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(CORR)
    for case, line in zip(CORR, lines):
        got = json.loads(line)
        assert got["records"] == case["records"], (case["log"], case["name"])
        assert got["reports"] == case["reports"], (case["log"], case["name"])
