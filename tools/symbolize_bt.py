#!/usr/bin/env python3
"""tools/symbolize_bt.py <log> -- name the frames of the harness's fault backtraces (lines
`<binary>(+0xOFF)[addr]`, printed by integration/pdb_dbbench.cc's fatal-signal handler) from the
binary's symbol table (`nm -C`: the enclosing function of each offset).  The binary must be the one
that printed the log."""
import bisect
import re
import subprocess
import sys

_cache = {}


def symbols(binary):
    if binary not in _cache:
        out = subprocess.run(["nm", "-C", "--defined-only", "-n", binary], capture_output=True, text=True).stdout
        addrs, names = [], []
        for ln in out.splitlines():
            parts = ln.split(" ", 2)
            if len(parts) == 3 and parts[1] in "tTwW":
                addrs.append(int(parts[0], 16))
                names.append(parts[2])
        _cache[binary] = (addrs, names)
    return _cache[binary]


def main():
    pat = re.compile(r"^(\S+)\(\+0x([0-9a-f]+)\)\[")
    for ln in open(sys.argv[1], errors="replace"):
        m = pat.match(ln.strip())
        if m and "libc" not in m.group(1):
            addrs, names = symbols(m.group(1))
            off = int(m.group(2), 16)
            i = bisect.bisect_right(addrs, off) - 1
            print("  %s+0x%x  %s" % (m.group(1).rsplit("/", 1)[-1], off, names[i] if i >= 0 else "??"))
        else:
            print(ln.rstrip())


if __name__ == "__main__":
    main()
