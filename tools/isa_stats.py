#!/usr/bin/env python3
"""tools/isa_stats.py <file.s> <kernel-substring> [more substrings...] -- per-kernel register use,
scratch, occupancy and instruction mix from hipcc's device assembly (diagnostics only).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -S \\
        pebblesdb_amd/csrc/crc32c_kernels.hip -o /tmp/k.s
    python tools/isa_stats.py /tmp/k.s lanespan_kernelINS0_7DescSrcENS0_7OutSinkELj512ELi0E
"""
import collections
import re
import sys


def kernels(path):
    cur, body = None, []
    with open(path) as f:
        for line in f:
            m = re.match(r"^(_Z\S+):", line)
            if m:
                if cur:
                    yield cur, body
                cur, body = m.group(1), []
            elif cur is not None:
                body.append(line)
                if line.startswith("\t.end_amdhsa_kernel") or line.startswith(".Lfunc_end"):
                    yield cur, body
                    cur, body = None, []


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    meta = {}
    with open(path) as f:
        text = f.read()
    for name, body in kernels(path):
        if not all(s in name for s in subs):
            continue
        mix = collections.Counter()
        for ln in body:
            m = re.match(r"^\s+((?:ds|v|s|buffer|global)_[a-z0-9_]+)", ln)
            if m:
                op = m.group(1)
                mix["ds_read" if op.startswith("ds_read") and "bpermute" not in op else op] += 0
                mix[op] += 1
        # metadata lines follow the kernel body in the .s (NumVgprs etc. as comments)
        i = text.find(name + ":")
        tail = text[i:i + 2_000_000]
        for key in ("NumVgprs", "ScratchSize", "Occupancy", "NumSgprs"):
            m = re.search(r"; %s: (\d+)" % key, tail)
            meta[key] = int(m.group(1)) if m else None
        print(name[:120])
        print("  ", meta)
        tot_ds = sum(v for k, v in mix.items() if k.startswith("ds_read"))
        print("   ds_read total (static):", tot_ds, {k: v for k, v in mix.items() if k.startswith("ds_")})
        print("   top:", ", ".join("%s %d" % kv for kv in mix.most_common(14)))


if __name__ == "__main__":
    main()
