"""Per-call latency of the scalar drop-in pdb_crc32c_extend (leveldb::crc32c::Extend) on host
data: the path every unmodified reference call site takes (log_writer.cc:121,
table_builder.cc:197-199, format.cc:97).  Prints one JSON line: µs/call and GiB/s per size."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import _native  # noqa: E402


def main():
    lib = _native.lib()
    fn = lib.pdb_crc32c_extend
    out = {"metric": "pdb_crc32c_extend latency (host bytes -> CRC)", "sizes": {}}
    for n in (16, 1024, 4096, 4101, 32768, 65536, 1 << 20, 4 << 20, 16 << 20):
        buf = np.frombuffer(os.urandom(n), dtype=np.uint8)
        p = ctypes.c_void_p(buf.ctypes.data)
        for _ in range(20):
            fn(0, p, n)
        reps = max(20, min(5000, int(2e8 // max(n, 4096) // 10)))
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(0, p, n)
        dt = (time.perf_counter() - t0) / reps
        out["sizes"][str(n)] = {"us_per_call": round(dt * 1e6, 2), "GiB_s": round(n / dt / 2**30, 3),
                                "reps": reps}
        print(f"n={n}: {dt*1e6:.2f} us/call", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
