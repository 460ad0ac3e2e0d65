#!/usr/bin/env python3
"""tools/span_banks.py -- a model of the record kernel's staging-read bank conflicts (DESIGN.md §6.0
item 14; CPU only).

crc_lanespan_kernel hashes k = 4 lanes per record, 16 records per item: lane (record s, part c)
reads, at chain X's step t, the LDS dword (e_s - 4 P c) / 4 + 8 (3 - X) + t, where e_s is the
record's end and P the part size in words (27 for the 257..512-B class).  A ds_read_b32 is serviced
per 32-lane half, bank = dword mod 32, one LDS cycle per half plus one per extra distinct address
on a bank (MI355X_MICROARCH.md §LDS).  For bench.py's log layouts of equal-sized records and for
random sizes, this prints the mean LDS cycles per staging read instruction (ideal 2) when the 16
records are split into halves as records 0-7 | 8-15 (A, round 2), 0-3, 8-11 | 4-7, 12-15 (C), and
with the kernel's per-row choice of the two by distinct-bank count (auto)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import wal_layout  # noqa: E402

K, P = 4, 27


def read_cycles(e, half):
    tot = 0
    for t in range(8):
        for x in range(4):
            cyc = 0
            for h in (0, 1):
                banks = {}
                for s in range(len(e)):
                    if half(s) != h:
                        continue
                    for c in range(K):
                        a = (int(e[s]) - 4 * P * c) // 4 + 8 * (3 - x) + t
                        banks.setdefault(a % 32, set()).add(a)
                cyc += max((len(v) for v in banks.values()), default=1)
            tot += cyc
    return tot / 32


def distinct(e, half):
    n = 0
    for h in (0, 1):
        b = set()
        for s in range(len(e)):
            if half(s) == h:
                for c in range(K):
                    b.add(((int(e[s]) >> 2) - P * c) % 32)
        n += len(b)
    return n


A = lambda s: (s >> 3) & 1  # noqa: E731
C = lambda s: (s >> 2) & 1  # noqa: E731


def row(e):
    a, c = read_cycles(e, A), read_cycles(e, C)
    return a, c, (c if distinct(e, C) > distinct(e, A) else a)


def main():
    rng = np.random.default_rng(1)
    cases = [(f"{n}-B records", *wal_layout(1 << 21, n)) for n in (400, 411, 419, 423, 427, 431, 435, 443, 455)]
    lens = rng.integers(300, 500, size=4000)
    cases.append(("random 300-500 B", np.concatenate([[0], np.cumsum(lens + 7)[:-1]]) + 6, lens))
    for name, offs, lens in cases:
        e = offs + lens
        r = np.array([row(e[i * 48:i * 48 + 16]) for i in range(30)])
        print(f"{name:18s} A {r[:, 0].mean():5.2f}  C {r[:, 1].mean():5.2f}  auto {r[:, 2].mean():5.2f}  (ideal 2)")


if __name__ == "__main__":
    main()
