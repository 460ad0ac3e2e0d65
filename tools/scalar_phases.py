#!/usr/bin/env python3
"""tools/scalar_phases.py [out.json] -- where a scalar Extend call's time goes.

Runs itself in a child process with PDB_SERVER_STAMPS set, so the library records, per call,
host CLOCK_MONOTONIC at entry (h0), after the bytes and the request word went out through the BAR
(h1) and on seeing the answer (h2), and the server's s_memrealtime ticks (100 MHz) when the poll that
found the request returned (g_seen) and after the hash (g_done).  Phases of a call:

    bar        h1 - h0                     memcpy of the bytes + request word into the mailbox
    to_gpu     g_seen - h1 - theta         until the server's poll returns with it (visibility + poll)
    hash       g_done - g_seen             the server wave's loads of the bytes + the hash
    to_host    h2 - g_done + theta         response store across PCIe + the host's spin seeing it

theta (GPU clock - host clock) is unknown; as in NTP it is estimated from the fastest calls, assuming
the minimum one-way delays of the two legs are equal: theta = (min(g_seen - h1) - min(h2 - g_done)) / 2.
The two legs' split therefore rests on that assumption; bar, hash and the total do not.
One thread, `calls` calls per size after a warm-up (the server stays up between them)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

SIZES = (1, 1024, 4172, 16384)


def child(path_csv: str, calls: int) -> None:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pebblesdb_amd import crc32c

    crc32c.init_device(0)
    rng = np.random.default_rng(1)
    buf = rng.integers(0, 256, size=max(SIZES), dtype=np.uint8).tobytes()
    for n in SIZES:
        for _ in range(500):
            crc32c.value(buf[:n])
        for _ in range(calls):
            crc32c.value(buf[:n])


def summarize(csv: str) -> dict:
    d = np.loadtxt(csv, delimiter=",", skiprows=1, dtype=np.float64)
    n, h0, h1, h2, gs, gd = (d[:, i] for i in range(6))
    gs, gd = gs * 10.0, gd * 10.0  # ticks of 10 ns
    out = {"method": __doc__.split("\n\n")[1].strip().replace("\n", " "), "sizes": {}}
    for size in SIZES:
        m = n == size
        if not m.any():
            continue
        m_idx = np.nonzero(m)[0][500:]  # drop the warm-up
        leg1 = gs[m_idx] - h1[m_idx]
        leg2 = h2[m_idx] - gd[m_idx]
        theta = (np.min(leg1) - np.min(leg2)) / 2.0
        ph = {"bar": h1[m_idx] - h0[m_idx], "to_gpu": leg1 - theta, "hash": gd[m_idx] - gs[m_idx],
              "to_host": leg2 + theta, "total": h2[m_idx] - h0[m_idx]}
        out["sizes"][str(size)] = {
            "calls": int(len(m_idx)),
            "us": {k: {"median": round(float(np.median(v)) / 1e3, 3), "p10": round(float(np.percentile(v, 10)) / 1e3, 3),
                       "p90": round(float(np.percentile(v, 90)) / 1e3, 3), "min": round(float(np.min(v)) / 1e3, 3)}
                   for k, v in ph.items()},
        }
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
        return
    dest = sys.argv[1] if len(sys.argv) > 1 else None
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    with tempfile.TemporaryDirectory() as td:
        csv = os.path.join(td, "stamps.csv")
        env = dict(os.environ, PDB_SERVER_STAMPS=csv)
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--child", csv, str(calls)], env=env)
        res = summarize(csv)
    text = json.dumps(res, indent=1)
    print(text)
    if dest:
        with open(dest, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
