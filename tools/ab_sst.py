#!/usr/bin/env python3
"""Interleaved A/B of the sstable hooks (pdb_sst_seal_device / pdb_sst_verify_device) across
diagnostics-library variants (pdb_diag_sst) on bench.py's sst image (1 M blocks of 4166-4174 B + type + trailer).
argv[1] = variants (e.g. 0,18; "<name>/<id>" = id in pebblesdb_amd/_lib/ab/libpdb_crc32c_diag_<name>.so, an
earlier revision built by tools/ab_base.sh).  Prints one JSON object (GB/s of algorithmic bytes, median)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pebblesdb_amd import crc32c  # noqa: E402
from pebblesdb_amd import table as T  # noqa: E402
from pebblesdb_amd import diag  # noqa: E402
from pebblesdb_amd._native import lib  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else "0,18").split(",")
_libs = {}


def sst_fn(tok):
    """(pdb_diag_sst of the token's library, variant id)"""
    if "/" not in tok:
        return diag.lib().pdb_diag_sst, int(tok)
    name, v = tok.split("/")
    if name not in _libs:
        L = ctypes.CDLL(os.path.join(os.path.dirname(diag.DIAG_LIB), "ab", f"libpdb_crc32c_diag_{name}.so"))
        L.pdb_diag_sst.restype, L.pdb_diag_sst.argtypes = diag.SIGNATURES["pdb_diag_sst"]
        _libs[name] = L
    return _libs[name].pdb_diag_sst, int(v)


def run(tok, seal, ok=None, nbad=None, sp=None):
    f, v = sst_fn(tok)
    diag.check(f(v, data.data_ptr(), total, d_h.data_ptr(), nblk, 1 if seal else 0,
                 ok.data_ptr() if ok is not None else None, nbad.data_ptr() if nbad is not None else None,
                 sp if sp is not None else int(torch.cuda.current_stream().cuda_stream)))
nblk = 1 << 20
crc32c.init_device(0)
rng = np.random.Generator(np.random.PCG64(301))
sizes = rng.integers(4166, 4175, size=nblk).astype(np.int64)
offs = np.concatenate([[0], np.cumsum(sizes + 5)[:-1]])
total = int(offs[-1] + sizes[-1] + 5)
data = torch.empty(total, dtype=torch.uint8, device="cuda")
diag.fill_splitmix(data, 301)
data[torch.from_numpy(offs + sizes).cuda()] = 0
h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
h["offset"], h["size"] = offs, sizes
d_h = T.handles_to_device(h)
T.seal_device(data, d_h)
ref = data.clone()
for _ in range(20):
    diag.batch_fixed(0, data, 4096, 4096, total // 4096 - 1)
res = {"seal": {}, "verify": {}}
times = {(m, v): [] for m in res for v in variants}
for v in variants:  # every variant seals the same bytes and verifies them all
    run(v, True)
    ok = torch.zeros(nblk, dtype=torch.uint8, device="cuda")
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    run(v, False, ok, nbad)
    torch.cuda.synchronize()
    vid = int(v.split("/")[-1])
    assert torch.equal(data, ref) and ((int(nbad.item()) == 0 and bool(ok.all())) or vid >= 90), v  # >= 90: wrong by design
ok = torch.empty(nblk, dtype=torch.uint8, device="cuda")
nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
sp = int(torch.cuda.current_stream().cuda_stream)
# past the power manager's cold transient (~40 launches) before anything is timed
for _ in range(60):
    run(variants[0], False, ok, nbad, sp)
torch.cuda.synchronize()
for _ in range(8):
    for v in variants:
        for m in res:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                if m == "seal":
                    run(v, True, sp=sp)
                else:
                    run(v, False, ok, nbad, sp)
            e1.record()
            torch.cuda.synchronize()
            times[(m, v)].append(e0.elapsed_time(e1) / 3)
hashed = int((sizes + 1).sum())
for (m, v), t in times.items():
    algo = hashed + nblk * (4 + 16 + (1 if m == "verify" else 0))
    res[m][v] = round(algo / (np.median(t) * 1e-3) / 1e9, 1)
print(json.dumps(res))
