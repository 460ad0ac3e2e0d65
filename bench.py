#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC32C over sstable blocks on MI355X.

Metric (BASELINE.json): "GiB/s CRC32C over batched 4 KiB sstable blocks (device-resident);
% HBM peak".  Default workload = BASELINE configs[1]: 1,048,576 x 4 KiB synthetic blocks
(splitmix64 seed 301), one GPU.  One *step* = one batch CRC over every block of the rank's
shard (one kernel launch through the C-ABI, pdb_crc32c_batch_device_fixed).

Multi-GPU (torchrun, one process per GPU): every rank owns an independent shard of the same
per-GPU size (weak scaling).  RCCL is used only to scatter each rank's block-range index from
rank 0 and, outside the timed region, to gather a checksum-of-checksums.  No data-path
collective: blocks are independent.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
C2_BLOCKS = 1 << 20        # BASELINE config 2: 1 M x 4 KiB on one GPU
C4_BLOCKS_PER_GPU = 4194304  # BASELINE config 4: 128 GiB of 4 KiB blocks over 8 GPUs = 16 GiB per GPU
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "GiB/s CRC32C over batched 4 KiB sstable blocks (device-resident); % HBM peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    # default: 40 for c2 (the first ~20-30 launches of a cold GPU run slower: clock / power
    # settling); the other workloads warm up for at least --warmup-s seconds of
    # launches too (their kernels are 0.2-0.8 ms: 40 of them end inside the ~0.15 s power transient).
    # An explicit --warmup W is exactly W launches (the driver's --warmup 5).
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--warmup-s", type=float, default=0.3,
                    help="non-c2 workloads without --warmup: warm up until this many seconds have passed")
    ap.add_argument("--settle", type=int, default=300,
                    help="untimed launches after the timed region before the steady-state re-timing (0: skip)")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "sstable", "sst_verify", "sst_seal", "sst_crc",
                                                        "sst_tables", "wal", "wal100", "wal400", "wal1000"],
                    help="c2 (default, the headline) / c3: BASELINE configs; sstable: the C2 blocks in "
                         "sstable layout; sst_verify / sst_seal: SURVEY §8(f) rows 1-2 on a device sstable "
                         "image of ~4.17-KiB blocks; sst_tables: pdb_sst_verify_device over REAL tables (data, "
                         "filter, metaindex and index blocks) written by the reference TableBuilder; wal: row 3, "
                         "the log record CRC over 32-KiB log blocks")
    ap.add_argument("--tables", type=int, default=4, help="sst_tables: tables per GPU")
    ap.add_argument("--tables-dir", default=None,
                    help="sst_tables: keep the generated tables in this directory and reuse them")
    ap.add_argument("--table-keys", type=int, default=1000000, help="sst_tables: keys per table (1 KiB values)")
    ap.add_argument("--nblk", type=int, default=None,
                    help="blocks per GPU (c2/sstable); default 1M (C2) on one GPU and, for c2 with --gpus N > 1, "
                         "BASELINE config 4's 4 194 304 (16 GiB per GPU: 128 GiB over 8 GPUs)")
    ap.add_argument("--c3-bytes", type=int, default=16 << 30, help="bytes per GPU for c3 (Zipf)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-copy-inclusive", action="store_true")
    ap.add_argument("--no-c4-shard", action="store_true",
                    help="skip the N = 1 line's c4_shard key (one 16 GiB config-4 shard, the 1 -> 8 GPU curve's "
                         "equal-shard anchor)")
    ap.add_argument("--diag", action="store_true", help="also time the read-stream calibration kernels")
    ap.add_argument("--no-ceiling", action="store_true",
                    help="skip the hash-free pattern-ceiling kernels timed after the timed region (pattern_ceiling)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--timing", default="region", choices=["per-launch", "region"],
                    help="HIP events around every launch (per-launch kernel times) or one pair around "
                         "the timed region (no event packets between launches)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL over xGMI; gloo only to rehearse the "
                         "multi-rank flow with ranks sharing one GPU)")
    ap.add_argument("--process-group", action="store_true",
                    help="create the process group and run every collective even at world size 1 (the RCCL "
                         "branch on one GPU: tests/test_shard.py)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rank plumbing only, on the CPU (gloo): no device, no kernel, value null "
                         "(tests/test_shard.py)")
    args = ap.parse_args()
    args.warmup_timed = args.warmup is None and args.workload != "c2"
    if args.warmup is None:
        args.warmup = 40
    return args


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> None:
    """Make `--gpus N` mean N ranks, one process per GPU.

    * Under a launcher (WORLD_SIZE set, e.g. the driver's torch.distributed.run): WORLD_SIZE must
      equal --gpus, or the run exits non-zero instead of silently measuring another world size.
    * Without one and --gpus > 1: this process re-launches itself under torch.distributed.run with
      N ranks (127.0.0.1 rendezvous) as a CHILD process and exits with its return code.  Nothing
      here has touched the GPU (torch.cuda is not initialised before main() runs in a rank), and
      the parent never execs.
    Returns only in a rank process (or for --gpus 1 without a launcher)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to measure a "
                             "different world size than asked\n")
            sys.exit(2)
        return
    if args.gpus < 1:
        sys.stderr.write("bench.py: --gpus must be >= 1\n")
        sys.exit(2)
    if args.gpus == 1:
        return
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    sys.stdout.flush()
    sys.exit(subprocess.call(cmd, env=env))


def resolve_nblk(args, world: int) -> bool:
    """--nblk's default: C2's 1 M blocks on one GPU; with N > 1 ranks and the c2 workload, config 4's
    4 194 304 blocks per rank, so N = 8 hashes exactly BASELINE config 4's 128 GiB (weak scaling:
    N = 2 / 4 keep the same 16 GiB per GPU).  Returns True when the C4 shard size was chosen."""
    if args.nblk is not None:
        return False
    if world > 1 and args.workload == "c2":
        args.nblk = C4_BLOCKS_PER_GPU
        return True
    args.nblk = C2_BLOCKS
    return False


def wants_c4_shard(args, world: int, c4: bool) -> bool:
    """The N = 1 default line (c2, C2 size) carries the c4_shard anchor; N > 1 lines are c4 shards."""
    return world == 1 and args.workload == "c2" and not c4 and not args.no_c4_shard


def dry_run_main(args, world: int, rank: int) -> None:
    """The multi-rank plumbing of main() with no device: gloo process group, rank 0's index
    scatter, barrier-bracketed (empty) timed region with max-over-ranks time, per-rank row
    gather, and rank 0's JSON line (value null).  Lets a CPU test prove that `--gpus N` without a
    launcher really runs N ranks."""
    import torch
    import torch.distributed as dist

    from pebblesdb_amd.shard import scatter_block_ranges

    cpu = torch.device("cpu")
    c4 = resolve_nblk(args, world)
    distributed = world > 1 or args.process_group
    if distributed:
        dist.init_process_group("gloo")
    lo, hi = scatter_block_ranges(args.nblk * world, world, rank, cpu, dist if distributed else None)
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    if distributed:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    rows = gather_rank_rows([rank, -1, -1, (hi - lo) * 4096, 0, 0, -1], world, cpu, dist if distributed else None)
    if rank == 0:
        line = {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "world_size": world,
                "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                "config": {"workload": "dry run (launcher plumbing only, no device)" + (" of the c4 shards" if c4 else ""),
                           "blocks_per_gpu": args.nblk},
                "ranks": [{"rank": r[0], "blocks": r[3] // 4096, "steady_kernel_avg_ms": None} for r in rows],
                "steady_state": ({"over_ranks": {"ranks": len(rows)}} if world > 1 and args.settle > 0 else None),
                "region_s_max": float(t.item())}
        if wants_c4_shard(args, world, c4):
            line["c4_shard"] = {"blocks": C4_BLOCKS_PER_GPU, "bytes": C4_BLOCKS_PER_GPU * 4096, "dry_run": True}
        if not args.no_copy_inclusive and args.workload in ("c2", "sstable"):
            line["copy_inclusive"] = {"GiB/s": None, "dry_run": True, "concurrent_ranks": world,
                                      "ranks_GiB/s": [None] * world, "entry": "pdb_crc32c_batch_host"}
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


def wal_layout(total_bytes: int, payload: int, block: int = 32768):
    """(offsets, lengths) of the CRC'd spans (type byte + fragment) of a log image holding
    `payload`-byte records back to back: a record that does not fit the rest of a 32-KiB block is
    fragmented (FIRST/MIDDLE/LAST), and a block tail < 7 B is zero padding (db/log_writer.cc:39-81)."""
    offs, lens = [], []
    pos, left, end = 0, payload, block
    while pos < total_bytes:
        avail = end - pos
        if avail < 7:
            pos, end = end, end + block
            continue
        frag = min(left, avail - 7)
        offs.append(pos + 6)
        lens.append(frag + 1)
        pos += 7 + frag
        left = left - frag or payload
        if pos == end:
            end += block
    return np.asarray(offs, dtype=np.int64), np.asarray(lens, dtype=np.int64)


def real_tables(ntables: int, nkeys: int, value_size: int, seed: int, keep_dir: str = None):
    """`ntables` real sstables written by the reference engine's TableBuilder as shipped
    (integration/_build/pdb_tablegen, built by integration/build.sh from the reference sources in
    place; CPU CRC trailers), in parallel, into a temporary directory on this host, concatenated.
    Returns (image bytes, handles of every block -- data blocks from each index block, then the
    filter block from the metaindex, the metaindex and the index (table/table.cc:70-170) -- rebased
    on the image, per-table facts).  With `keep_dir` the tables are kept there and reused by the next
    call with the same arguments (tools/profile.sh makes them before the profiled run)."""
    import shutil
    import subprocess
    import tempfile

    from pebblesdb_amd import crc32c
    from pebblesdb_amd import table as T

    exe = os.path.join(ROOT, "integration", "_build", "pdb_tablegen")
    if not os.path.exists(exe):
        raise SystemExit(f"bench.py: {exe} missing (integration/build.sh builds it)")
    tmp = keep_dir or tempfile.mkdtemp(prefix="pdb_tables_")
    os.makedirs(tmp, exist_ok=True)
    try:
        paths = [os.path.join(tmp, f"t{i}_{nkeys}_{value_size}_{seed + i}.sst") for i in range(ntables)]
        procs = [subprocess.Popen([exe, p, str(nkeys), str(value_size), str(seed + i)], stdout=subprocess.PIPE)
                 for i, p in enumerate(paths) if not os.path.exists(p)]
        for pr in procs:
            if pr.wait() != 0:
                raise SystemExit("bench.py: pdb_tablegen failed")
        parts, hs, info, base = [], [], [], 0
        for p in paths:
            im = np.fromfile(p, dtype=np.uint8)
            f = T.Footer.decode(im[-T.K_FOOTER_ENCODED_LENGTH:].tobytes())
            idx = im[f.index.offset: f.index.offset + f.index.size].tobytes()
            data = [T.BlockHandle.decode(v)[0] for _, v in T.block_entries(idx)]
            mi = im[f.metaindex.offset: f.metaindex.offset + f.metaindex.size].tobytes()
            meta = [T.BlockHandle.decode(v)[0] for _, v in T.block_entries(mi)]
            h = np.zeros(len(data) + len(meta) + 2, dtype=crc32c.HANDLE_DTYPE)
            h["offset"] = [x.offset + base for x in data + meta + [f.metaindex, f.index]]
            h["size"] = [x.size for x in data + meta + [f.metaindex, f.index]]
            hs.append(h)
            parts.append(im)
            info.append({"bytes": int(len(im)), "data_blocks": len(data), "filter_bytes": int(meta[0].size) if meta else 0,
                         "index_bytes": int(f.index.size)})
            base += len(im)
        return np.concatenate(parts), np.concatenate(hs), info
    finally:
        if not keep_dir:
            shutil.rmtree(tmp, ignore_errors=True)


def zipf_kib_sizes(n: int, seed: int, kmax: int = 64) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    k = np.arange(1, kmax + 1)
    p = (1.0 / k) / np.sum(1.0 / k)
    return (rng.choice(k, size=n, p=p) * 1024).astype(np.int64)


def sst_layout(nblk: int, seed: int):
    """The sst_* workloads' image: `nblk` blocks whose contents are 4166..4174 B (db_bench's data
    blocks flush just past the 4-KiB block_size), each followed by its 5-byte
    trailer.  Returns (sizes, offsets, image bytes)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = rng.integers(4166, 4175, size=nblk).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes + 5)[:-1]])
    return sizes, offs, int(offs[-1] + sizes[-1] + 5)


def c3_plan(c3_bytes: int, world: int) -> np.ndarray:
    """BASELINE config 3 for `world` ranks: ONE Zipf 1-64 KiB size list (seed 301) of world x
    c3_bytes, which rank 0 splits into contiguous byte-balanced ranges (weak scaling by bytes)."""
    want = c3_bytes * world
    sizes = zipf_kib_sizes(int(want / (13.5 * 1024) * 1.1) + 16, 301)
    return sizes[: int(np.searchsorted(np.cumsum(sizes), want, side="right"))]


def gather_rank_rows(row, world: int, cdev, dist=None) -> list:
    """All ranks' small integer rows on every rank (one all_gather, outside the timed region)."""
    import torch

    mine = torch.tensor([int(x) for x in row], dtype=torch.int64, device=cdev)
    if dist is None:
        return [[int(x) for x in mine.cpu().tolist()]]
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    return [[int(x) for x in v.cpu().tolist()] for v in allr]


def main():
    args = parse()
    launch_ranks(args)  # --gpus N without a launcher: re-run as N ranks (child process), exit with its rc
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dry_run_main(args, world, rank)
        return
    c4 = resolve_nblk(args, world)
    import torch
    import torch.distributed as dist

    from pebblesdb_amd import crc32c, diag
    from pebblesdb_amd.shard import scatter_block_lens, scatter_block_ranges

    ndev = torch.cuda.device_count()  # counting devices does not initialise HIP
    if ndev < 1:
        sys.stderr.write("bench.py: no GPU visible\n")
        sys.exit(3)
    if args.backend == "nccl" and int(os.environ.get("LOCAL_WORLD_SIZE", "1")) > ndev:
        sys.stderr.write(f"bench.py: {os.environ.get('LOCAL_WORLD_SIZE')} ranks on this node but only {ndev} GPUs "
                         "(one process per GPU; --backend gloo to rehearse ranks sharing a GPU)\n")
        sys.exit(2)
    gpu = local % ndev if args.backend == "gloo" else local  # gloo rehearsal may share a GPU
    torch.cuda.set_device(gpu)
    distributed = world > 1 or args.process_group
    if distributed:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    crc32c.init_device(gpu)
    dev = torch.device("cuda", gpu)
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # collective tensors
    stream = torch.cuda.current_stream()

    # ---- the rank's shard index: scattered from rank 0 over RCCL (the only collective) -------
    c3_sizes = None
    if args.workload == "c3":
        # ONE Zipf 1-64 KiB list of world x c3_bytes (seed 301), built by rank 0 alone and split into
        # contiguous ranges of ~equal BYTES (shard.byte_balanced_ranges); each rank receives its range
        # and its own block lengths by scatter: weak scaling by bytes
        lo, hi, c3_sizes = scatter_block_lens(c3_plan(args.c3_bytes, world) if rank == 0 else None, world, rank, cdev,
                                              dist if distributed else None)
    else:
        lo, hi = scatter_block_ranges(args.nblk * world, world, rank, cdev, dist if distributed else None)

    # ---- synthetic, device-resident input ---------------------------------------------------
    if args.workload == "c2":
        L = stride = 4096
        nblk = hi - lo
        data = torch.empty(nblk * stride, dtype=torch.uint8, device=dev)
        diag.fill_splitmix(data, 301, byte_offset=lo * stride)
        algo_bytes_per_blk = L + 4  # L read + 4 B CRC written
        hashed = nblk * L
        out = torch.empty(nblk, dtype=torch.int32, device=dev)

        def step():
            crc32c.batch_fixed(data, stride, L, nblk, out=out)

        workload = {"workload": (f"c4: {world} x 4M x 4 KiB blocks = {world * 16} GiB ({world} x 16 GiB shards; "
                                 "BASELINE config 4 at 8 GPUs), stride 4096, device-resident" if c4 else
                                 "c2: 1M x 4 KiB blocks per GPU, stride 4096, device-resident"),
                    "block_bytes": L, "blocks_per_gpu": nblk, "bytes_per_gpu": hashed}
    elif args.workload == "sstable":
        # sstable layout: contents 4096 B + type byte under the CRC, trailer 5 B -> stride 4101
        L, stride = 4097, 4101
        nblk = hi - lo
        data = torch.empty(nblk * stride, dtype=torch.uint8, device=dev)
        diag.fill_splitmix(data, 301, byte_offset=lo * stride)
        algo_bytes_per_blk = L + 4
        hashed = nblk * L
        out = torch.empty(nblk, dtype=torch.int32, device=dev)

        def step():
            crc32c.batch_fixed(data, stride, L, nblk, out=out)

        workload = {"workload": "sstable layout: 4096 B contents + type byte, stride 4101 (unaligned)",
                    "block_bytes": L, "blocks_per_gpu": nblk, "bytes_per_gpu": hashed}
    elif args.workload in ("sst_verify", "sst_seal", "sst_crc"):
        # sstable image: contents of 4166..4174 B (db_bench data blocks flush just past the 4-KiB
        # block_size: 4171-4175 B with the type byte), type 0, 5-B trailer
        from pebblesdb_amd import table as T
        from pebblesdb_amd._native import check, lib

        nblk = hi - lo
        sizes, offs, total = sst_layout(nblk, 301 + rank)
        data = torch.empty(total, dtype=torch.uint8, device=dev)
        diag.fill_splitmix(data, 301 + rank)
        data[torch.from_numpy(offs + sizes).to(dev)] = 0  # kNoCompression type bytes
        h = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
        h["offset"], h["size"] = offs, sizes
        d_h = T.handles_to_device(h, dev)
        cpu_blk = crc32c.make_blocks(offs, sizes + 1)  # the CPU reference's CRC spans (contents || type)
        T.seal_device(data, d_h)  # untimed: a sealed image, so verification passes
        ok = torch.empty(nblk, dtype=torch.uint8, device=dev)
        nbad = torch.zeros(1, dtype=torch.int32, device=dev)
        L = stride = None
        hashed = int((sizes + 1).sum())  # contents || type under the CRC
        out = torch.zeros(1, dtype=torch.int32, device=dev)
        sp = int(stream.cuda_stream)
        if args.workload == "sst_verify":
            algo_bytes_per_blk = None  # per block: size + 5 read, 16 B handle, 1 B ok

            def step():
                check(lib().pdb_sst_verify_device(data.data_ptr(), total, d_h.data_ptr(), nblk, ok.data_ptr(),
                                                  nbad.data_ptr(), sp))
        elif args.workload == "sst_crc":  # the seal's trailer words into a compact array
            out = torch.zeros(nblk, dtype=torch.int32, device=dev)

            def step():
                check(lib().pdb_sst_crc_device(data.data_ptr(), total, d_h.data_ptr(), nblk, out.data_ptr(), sp))
        else:
            def step():
                check(lib().pdb_sst_seal_device(data.data_ptr(), total, d_h.data_ptr(), nblk, sp))

        workload = {"workload": f"{args.workload}: sstable image in HBM, 1M blocks of 4166-4174 B + type + "
                                "5-B trailer, " + {"sst_verify": "pdb_sst_verify_device", "sst_seal": "pdb_sst_seal_device",
                                                   "sst_crc": "pdb_sst_crc_device"}[args.workload],
                    "blocks_per_gpu": nblk, "bytes_per_gpu": hashed}
    elif args.workload == "sst_tables":
        # real tables: the reference engine's TableBuilder as shipped writes them (CPU CRC trailers),
        # the image goes to HBM, and every block -- ~4.1-KiB data blocks, the MiB-sized filter and
        # index blocks (the long-block lane), the metaindex -- is checked in one device verify
        from pebblesdb_amd import table as T
        from pebblesdb_amd._native import check, lib

        img, hs, tinfo = real_tables(args.tables, args.table_keys, 1024, 401 + 16 * rank, args.tables_dir)
        total = len(img)
        data = torch.from_numpy(img).to(dev)
        nblk = len(hs)
        sizes, offs = hs["size"].astype(np.int64), hs["offset"].astype(np.int64)
        d_h = T.handles_to_device(hs, dev)
        cpu_blk = crc32c.make_blocks(offs, sizes + 1)
        ok = torch.empty(nblk, dtype=torch.uint8, device=dev)
        nbad = torch.zeros(1, dtype=torch.int32, device=dev)
        L = stride = None
        hashed = int((sizes + 1).sum())
        sp = int(stream.cuda_stream)

        def step():
            check(lib().pdb_sst_verify_device(data.data_ptr(), total, d_h.data_ptr(), nblk, ok.data_ptr(),
                                              nbad.data_ptr(), sp))

        # the seal's trailer words, once (untimed), against the reference's own trailers in the files
        out = T.crc_device(data, d_h)
        stored = np.frombuffer(img.tobytes(), dtype=np.uint8)
        t = offs + sizes + 1
        words = (stored[t].astype(np.uint32) | (stored[t + 1].astype(np.uint32) << 8) |
                 (stored[t + 2].astype(np.uint32) << 16) | (stored[t + 3].astype(np.uint32) << 24))
        same = int(np.count_nonzero(out.cpu().numpy().view(np.uint32) == words))
        long_m = sizes + 1 >= 16384
        workload = {"workload": f"sst_tables: {args.tables} real sstables per GPU ({args.table_keys} keys x 1 KiB values, "
                                "bloom 10 bits/key, kNoCompression) written by the reference TableBuilder "
                                "(integration/_build/pdb_tablegen), every block verified by pdb_sst_verify_device",
                    "blocks_per_gpu": nblk, "bytes_per_gpu": hashed, "tables": tinfo,
                    "long_blocks": {"count": int(long_m.sum()), "bytes": int((sizes[long_m] + 1).sum()),
                                    "max_bytes": int(sizes.max() + 1)},
                    "gpu_trailers_equal_reference": f"{same}/{nblk}"}
    elif args.workload in ("wal", "wal100", "wal400", "wal1000"):
        # log file image: 32-KiB log blocks of physical records [crc 4][len 2][type 1][payload]
        # (db/log_format.h:27-30); fillseq-like 1055-B logical records (1 KiB value + key + batch
        # header) fragmented at block ends; the CRC covers type || fragment (log_writer.cc:111-121)
        # wal100: db_bench's default --value_size=100 -> 131-B batches, a 1 GiB log, the <= 256-B class
        # wal400: --value_size=400 -> 431-B batches, a 2 GiB log, the 257..512-B class
        # wal1000: --value_size=969 -> 1000-B batches, a 2 GiB log, the 513..1023-B class
        small = args.workload == "wal100"
        mid = args.workload == "wal400"
        big = args.workload == "wal1000"
        offs, lens = wal_layout(args.nblk * (1024 if small else (2048 if mid or big else 4096)),
                                131 if small else (431 if mid else (1000 if big else 1055)))
        nblk = len(offs)
        total = int(offs[-1] + lens[-1])
        data = torch.empty(total, dtype=torch.uint8, device=dev)
        diag.fill_splitmix(data, 305 + rank)
        d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, lens), dev)
        L = stride = None
        hashed = int(lens.sum())
        out = torch.empty(nblk, dtype=torch.int32, device=dev)
        hint = "256" if small else ("512" if mid else ("1023" if big else "1k"))

        def step():
            crc32c.batch(data, d_blk, out=out, size_hint=hint)

        workload = {"workload": ("wal100: 1 GiB log image, 32-KiB blocks, 131-B records" if small else
                                 "wal400: 2 GiB log image, 32-KiB blocks, 431-B records" if mid else
                                 "wal1000: 2 GiB log image, 32-KiB blocks, 1000-B records" if big else
                                 "wal: 4 GiB log image, 32-KiB blocks, 1055-B records") +
                                " -> type||payload fragments (descriptor list)",
                    "blocks_per_gpu": nblk, "bytes_per_gpu": hashed}
    else:
        # c3: Zipf 1..64 KiB blocks packed back to back, this rank's byte-balanced range of the list
        sizes = c3_sizes
        n = len(sizes)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
        total = int(sizes.sum())
        data = torch.empty(total, dtype=torch.uint8, device=dev)
        diag.fill_splitmix(data, 303 + rank)
        d_blk = crc32c.blocks_to_device(crc32c.make_blocks(offs, sizes), dev)
        nblk = n
        L = stride = None
        algo_bytes_per_blk = None
        hashed = total
        out = torch.empty(nblk, dtype=torch.int32, device=dev)

        def step():
            crc32c.batch(data, d_blk, out=out)

        workload = {"workload": "c3: Zipf 1-64 KiB blocks, packed, descriptor list (byte-balanced rank ranges)",
                    "blocks_per_gpu": nblk, "bytes_per_gpu": hashed}
    algo_bytes = hashed + 4 * nblk + (16 * nblk if args.workload in ("c3", "wal", "wal100", "wal400", "wal1000") else 0)
    if args.workload in ("sst_verify", "sst_tables"):  # + the 4-B stored trailer read, 16-B handle, 1-B ok written
        algo_bytes = hashed + nblk * (4 + 16 + 1)
    elif args.workload in ("sst_seal", "sst_crc"):  # + 4-B trailer / CRC written, 16-B handle
        algo_bytes = hashed + nblk * (4 + 16)

    # ---- warmup + timed region -------------------------------------------------------------
    warm_t0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.warmup_timed:  # (per rank; the barrier below lines the ranks up)
        while time.perf_counter() - warm_t0 < args.warmup_s:
            for _ in range(10):
                step()
            args.warmup += 10
            torch.cuda.synchronize()
    warm_s = time.perf_counter() - warm_t0
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    per_launch = args.timing == "per-launch"
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps if per_launch else 1)]
    t0 = time.perf_counter()
    if per_launch:
        for s, e in ev:
            s.record(stream)
            step()
            e.record(stream)
    else:  # one event pair around all K launches: the average includes the launch gaps
        ev[0][0].record(stream)
        for _ in range(args.steps):
            step()
        ev[0][1].record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = [s.elapsed_time(e) for s, e in ev] if per_launch else [ev[0][0].elapsed_time(ev[0][1]) / args.steps]
    kern_avg_ms = float(np.mean(kern_ms))

    t = torch.tensor([wall], dtype=torch.float64, device=cdev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())

    # Steady state, AFTER the timed region and not part of `value`: the power manager lowers the
    # clock for the first ~100 launches on a cold GPU (sclk 2.41 -> ~2.05 GHz as board power climbs,
    # then recovers), so K launches after W = 5 warmups catch the transient.  This
    # re-times K launches after `--settle` more untimed ones, on this rank alone.
    # Every rank measures its own steady state; the N > 1 line reports the min and max over ranks.
    steady = None
    st_ms = steady_ms(torch, step, stream, args.settle, args.steps) if args.settle > 0 else None

    # per-rank facts (outside the timed region) gathered to rank 0: device, bytes hashed, kernel
    # time, checksum of checksums, steady-state kernel time -- the SCALE record shows which GPUs
    # RCCL actually saw
    props = torch.cuda.get_device_properties(gpu)
    pci = int(getattr(props, "pci_bus_id", -1))
    xor_local = int(np.bitwise_xor.reduce(out.cpu().numpy().view(np.uint32)))
    rows = gather_rank_rows([rank, gpu, pci, hashed, int(kern_avg_ms * 1e6), xor_local,
                             int(st_ms * 1e6) if st_ms is not None else -1], world, cdev,
                            dist if distributed else None)
    xor_all = 0
    for r in rows:
        xor_all ^= r[5]
    ranks = [{"rank": r[0], "device": r[1], "pci_bus_id": r[2], "bytes": r[3], "kernel_avg_ms": round(r[4] / 1e6, 4),
              "steady_kernel_avg_ms": round(r[6] / 1e6, 4) if r[6] >= 0 else None} for r in rows]
    if st_ms is not None:
        steady = {"settle_launches": args.settle, "kernel_avg_ms": round(st_ms, 4),
                  "GiB_s_per_gpu": round(hashed / (st_ms * 1e-3) / GIB, 3),
                  "frac": round(algo_bytes / (st_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if world > 1:  # every rank's steady state: the slowest and fastest GPU of the node
            per = [(r[3], r[6] / 1e6) for r in rows]
            fr = [algo_bytes * (b / hashed) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS for b, ms in per]
            steady["over_ranks"] = {"kernel_avg_ms_min": round(min(ms for _, ms in per), 4),
                                    "kernel_avg_ms_max": round(max(ms for _, ms in per), 4),
                                    "frac_min": round(min(fr), 4), "frac_max": round(max(fr), 4),
                                    "GiB_s_total_at_slowest": round(sum(b for b, _ in per) / (max(ms for _, ms in per) * 1e-3)
                                                                    / GIB, 3)}

    # the copy-inclusive rate (host-resident blocks, H2D + kernel + D2H): at N > 1 every rank runs it on
    # its own host sample at the same time (each GPU has its own PCIe link), outside `value`
    ci = None
    if not args.no_copy_inclusive and args.workload in ("c2", "sstable"):
        ci = copy_inclusive(crc32c, data, L, stride, min(nblk, 1 << 18), world, cdev, dist if distributed else None)

    total_bytes = sum(r[3] for r in rows) * args.steps  # weak scaling: every rank hashes its own shard
    value = total_bytes / wall_max / GIB
    ms_per_step = wall_max / args.steps * 1e3
    achieved_gbs = algo_bytes / (kern_avg_ms * 1e-3) / 1e9

    extra = {}
    if rank == 0:
        if args.diag:
            extra["diag"] = read_ceiling(torch, dev, data, stream)
        if world == 1 and not args.no_ceiling and args.workload != "sst_tables":
            ceil = pattern_ceiling(torch, args.workload, data, stream, algo_bytes, nblk,
                                   d_h=d_h if args.workload.startswith("sst_") else None,
                                   d_blk=d_blk if args.workload.startswith("wal") or args.workload == "c3" else None,
                                   hint=hint if args.workload.startswith("wal") else None, reseal=step)
            if ceil:
                extra["pattern_ceiling"] = ceil
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            if args.workload in ("c2", "sstable", "c3", "wal", "wal100", "wal400", "wal1000"):
                cpu = cpu_baseline(data, L, stride, nblk, args,
                                   d_blk if args.workload in ("c3", "wal", "wal100", "wal400", "wal1000") else None)
            else:  # sst_verify / sst_seal / sst_tables: the reference's CRC over each block's contents || type
                cpu = cpu_baseline(data, L, stride, nblk, args, cpu_blk)
        if wants_c4_shard(args, world, c4):
            extra["c4_shard"] = c4_shard(torch, crc32c, diag, dev, stream, args)
        if ci is not None:
            extra["copy_inclusive"] = ci
        if args.workload == "sst_tables":  # every launch verified every block of the reference's tables
            extra["verify"] = {"nbad_over_all_launches": int(nbad.item()), "ok_all": bool(ok.cpu().numpy().all())}

    if rank == 0:
        traffic = pmc_traffic(args.workload)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "world_size": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_s": round(warm_s, 3),
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 seed 301, generated on device)",
            "config": dict(workload, parallelism=f"block-range shards x{world}",
                           collectives=("index scatter + checksum all-gather + region-time MAX all-reduce (" +
                                        ("RCCL" if args.backend == "nccl" else "gloo") + "), none on the data path")
                           if distributed else "none (one rank, no process group)"),
            "process_group": (args.backend if distributed else None),
            "hbm_frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": "profiles/pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this "
                                  "workload (tools/profile.sh), per launch, FETCH_SIZE x2 (MI355X_MICROARCH.md)",
                "kernel": {"c2": "crc_pack4k_kernel (lane-quarter tables)", "sstable": "crc_sst4k_kernel<FixedSrc,OutSink,nt,QuadTabs>",
                           "c3": "crc_stream16_kernel<DescSrc,OutSink,dyn,nt,pack,QuadTabs,bal>",
                           "wal": "crc_lanespan_kernel<DescSrc,OutSink,1152>",
                           "wal100": "crc_lanespan_kernel<DescSrc,OutSink,256>",
                           "wal400": "crc_lanespan_kernel<DescSrc,OutSink,512>",
                           "wal1000": "crc_lanespan_kernel<DescSrc,OutSink,1023>",
                           "sst_verify": "crc_sst4k_kernel<SstSrc,SstVerifySink,nt,QuadTabs>",
                           "sst_seal": "crc_sst4k_kernel<SstSrc,ParkSealSink<64>,nt,QuadTabs>",
                           "sst_crc": "crc_sst4k_kernel<SstSrc,SstCrcSink,nt,QuadTabs>",
                           "sst_tables": "crc_sst4k_kernel<SstSrc,SstVerifySink,nt,QuadTabs> + the long-block lane "
                                         "(crc_longpiece_kernel, long_combine_kernel)"}[args.workload],
                "algorithmic_bytes_per_launch": algo_bytes,
                "kernel_avg_ms": round(kern_avg_ms, 4),
                "kernel_min_ms": round(float(np.min(kern_ms)), 4),
                "timing": args.timing,
            },
            "cpu_baseline": cpu,
            "steady_state": steady,
            "ranks": ranks,
            "xor_of_crcs": f"{xor_all:08x}",
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


def steady_ms(torch, step, stream, settle: int, steps: int) -> float:
    """Mean per-launch kernel time (HIP events around every launch) of `steps` launches after
    `settle` untimed ones: the rate a sustained stream of batches gets."""
    for _ in range(settle):
        step()
    se = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for s_, e_ in se:
        s_.record(stream)
        step()
        e_.record(stream)
    torch.cuda.synchronize()
    return float(np.mean([s_.elapsed_time(e_) for s_, e_ in se]))


C4_IDLE_S = 3.0


def c4_shard(torch, crc32c, diag, dev, stream, args) -> dict:
    """The equal-shard anchor of the 1 -> 8 GPU curve, at N = 1 and outside `value`: one 16 GiB
    shard of BASELINE config 4 (rank 0's 4 194 304 x 4 KiB blocks of the global splitmix image, what
    every rank of an N > 1 run hashes), timed exactly as the N > 1 runs time theirs -- W warmups,
    then K launches in one event pair -- after C4_IDLE_S s of idle GPU, so it starts from the same
    cold power state as a fresh N > 1 process, then its own steady state."""
    nblk = C4_BLOCKS_PER_GPU
    data = torch.empty(nblk * 4096, dtype=torch.uint8, device=dev)
    diag.fill_splitmix(data, 301, byte_offset=0)
    out = torch.empty(nblk, dtype=torch.int32, device=dev)

    def step():
        crc32c.batch_fixed(data, 4096, 4096, nblk, out=out)

    torch.cuda.synchronize()
    time.sleep(C4_IDLE_S)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern = e0.elapsed_time(e1) / args.steps
    xor = int(np.bitwise_xor.reduce(out.cpu().numpy().view(np.uint32)))
    algo = nblk * 4100
    res = {"workload": "c4 shard: 4M x 4 KiB blocks = 16 GiB (rank 0's shard of BASELINE config 4), stride 4096, "
                       "device-resident, after %.0f s idle" % C4_IDLE_S,
           "blocks": nblk, "bytes": nblk * 4096, "steps": args.steps, "warmup": args.warmup,
           "GiB_s": round(nblk * 4096 * args.steps / wall / GIB, 3), "ms_per_step": round(wall / args.steps * 1e3, 4),
           "kernel_avg_ms": round(kern, 4), "frac": round(algo / (kern * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "xor_of_crcs": f"{xor:08x}"}
    if args.settle > 0:
        st = steady_ms(torch, step, stream, args.settle, args.steps)
        res["steady_state"] = {"settle_launches": args.settle, "kernel_avg_ms": round(st, 4),
                               "frac": round(algo / (st * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    del data, out
    torch.cuda.empty_cache()
    return res


def pattern_ceiling(torch, workload, data, stream, algo_bytes, nblk, d_h=None, d_blk=None, hint=None, reseal=None):
    """The measured kernel's memory pattern with NO hash (diagnostics library, after the timed
    region): the ceiling the kernel's own loads and stores allow on this box, priced against the
    same algorithmic bytes.  c2: read_pattern4k variant 21 (the 4-KiB path's 1-KiB-contiguous nt
    loads, 4 blocks per wave between barriers); sst_*: seal_pattern_kernel (variant 140 loads only,
    141 loads + the 1 M trailer stores -- the in-place seal's pattern; the image is re-sealed after);
    wal*: the record kernel's loads and LDS staging alone (variant 63).  DESIGN.md §6 / §6.0."""
    from pebblesdb_amd import crc32c, diag

    runs = []
    if workload == "c2":
        o = torch.zeros(1, dtype=torch.int32, device=data.device)
        runs.append(("read_pattern4k variant 21 (loads only)", lambda: diag.read_pattern4k(data, nblk, 21, o, stream)))
    elif workload == "c3":
        o = torch.empty(nblk, dtype=torch.int32, device=data.device)
        runs.append(("crc_stream16_kernel kLoadsOnly (variant 161: the C3 routing's loads, scheduling and "
                     "byte-balanced ranges, no hash)", lambda: diag.batch_desc(161, data, d_blk, flags=0, out=o,
                                                                             stream=stream)))
    elif workload == "sstable":
        # the stride-4101 blocks as sstable handles (offset i * 4101, 4096 B contents + type + trailer):
        # seal_pattern_kernel<0> reads each block's 4101 B with the sst kernel's 1-KiB-contiguous nt
        # loads in 4-block groups (the 4 trailer bytes past the 4097 hashed: +0.1 % of the bytes)
        from pebblesdb_amd import table as T

        hs = np.zeros(nblk, dtype=crc32c.HANDLE_DTYPE)
        hs["offset"], hs["size"] = np.arange(nblk, dtype=np.int64) * 4101, 4096
        d_hs = T.handles_to_device(hs, data.device)
        runs.append(("seal_pattern_kernel<0> (variant 140: loads only) over the stride-4101 blocks",
                     lambda: diag.sst(140, data, d_hs, seal=True, stream=stream)))
    elif workload in ("sst_verify", "sst_crc", "sst_seal"):
        runs.append(("seal_pattern_kernel<0> (variant 140: loads only)",
                     lambda: diag.sst(140, data, d_h, seal=True, stream=stream)))
        if workload == "sst_seal":
            runs.append(("seal_pattern_kernel<1> (variant 141: loads + in-place trailer stores)",
                         lambda: diag.sst(141, data, d_h, seal=True, stream=stream)))
    elif workload.startswith("wal"):
        o = torch.empty(nblk, dtype=torch.int32, device=data.device)
        flags = crc32c._SIZE_HINT[hint]
        runs.append(("crc_lanespan_kernel MODE 1 (variant 63: loads + LDS staging, no hash)",
                     lambda: diag.batch_desc(63, data, d_blk, flags=flags, out=o, stream=stream)))
    res = {}
    for name, fn in runs:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(10):
            fn()
        e.record(stream)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        gbs = algo_bytes / (ms * 1e-3) / 1e9
        res[name] = {"ms": round(ms, 4), "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    if workload == "sst_seal" and reseal is not None:  # the calibration wrote wrong trailers
        reseal()
        torch.cuda.synchronize()
    return res


def read_ceiling(torch, dev, data, stream):
    """Achievable read bandwidth on this box: a coalesced 16-B/lane stream and the exact load
    pattern of the 4-KiB fast path with no CRC work (read_pattern4k variant 21: 1-KiB-contiguous
    nt load instructions, 4 blocks per wave between workgroup barriers -- also the FETCH_SIZE
    calibration kernel of tools/pmc_traffic.py)."""
    from pebblesdb_amd import diag

    nbytes = data.numel()
    o = torch.zeros(1, dtype=torch.int32, device=dev)
    res = {}
    for name, fn in (
        ("read_stream", lambda: diag.read_stream(data, nbytes, o, stream)),
        ("read_pattern4k", lambda: diag.read_pattern4k(data, nbytes // 4096, 21, o, stream)),
    ):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(10):
            fn()
        e.record(stream)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        res[name] = {"GB/s": round(nbytes / (ms * 1e-3) / 1e9, 1), "ms": round(ms, 4)}
    return res


def copy_inclusive(crc32c, data, L, stride, nblk, world: int = 1, cdev=None, dist=None):
    """Host-resident blocks -> pdb_crc32c_batch_host (H2D + kernel + D2H), pageable memory: `nblk`
    blocks of this rank's shard copied to host memory, 3 timed calls.  With N ranks every rank runs it
    at once between barriers (each GPU hashes its own host sample over its own PCIe link): the line
    gives each rank's rate and the aggregate, all ranks' bytes / the slowest rank's time."""
    import torch

    host = data[: nblk * stride].cpu().numpy()
    blk = crc32c.make_blocks(np.arange(nblk) * stride, np.full(nblk, L))
    crc32c.batch_host(host, blk)  # warm (workspace growth)
    reps = 3
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        crc32c.batch_host(host, blk)
    dt = (time.perf_counter() - t0) / reps
    rate = nblk * L / dt / GIB
    res = {"GiB/s": round(rate, 3), "blocks": nblk, "host_memory": "pageable", "entry": "pdb_crc32c_batch_host"}
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rows = gather_rank_rows([int(rate * 1000)], world, cdev, dist)
        res.update({"GiB/s": round(world * nblk * L / float(t.item()) / GIB, 3), "blocks_per_rank": nblk,
                    "ranks_GiB/s": [r[0] / 1000 for r in rows], "concurrent_ranks": world,
                    "aggregate": "all ranks' bytes / the slowest rank's time (each rank its own GPU and PCIe link)"})
        del res["blocks"]
    return res


def cpu_baseline(data, L, stride, nblk, args, d_blk):
    """The reference's own CRC32C (oracle/_ref, compiled from src/util/crc32c.cc) on this box's
    host cores over a bounded sample of the same blocks (1 GiB): every logical CPU (the primary
    figure, `cores` = nproc threads), 16 threads, one thread, and each NUMA node's CPUs alone.
    Threads hash disjoint slices, started together, ~1 s per configuration
    (oracle.timed_batch).  Falls back to the C restatement (kind "port") only if the reference
    .so did not travel."""
    import oracle

    try:
        lib, kind = oracle.Reference(), "reference"
    except (FileNotFoundError, OSError):
        if not os.path.exists(oracle.ORACLE_SO):
            oracle.build()
        lib, kind = oracle.Oracle(), "port"
    cpus = oracle.host_cpus()
    threads = args.cpu_threads or cpus["nproc"] or 1
    if d_blk is None:
        ns = min(nblk, 1 << 18)  # 256 Ki blocks = 1 GiB sample of the same workload
        host = data[: ns * stride].cpu().numpy()
        blk = np.zeros(ns, dtype=oracle.BLK_DTYPE)
        blk["off"] = np.arange(ns) * stride
        blk["len"] = L
    else:
        b = d_blk if isinstance(d_blk, np.ndarray) else d_blk.cpu().numpy().view(oracle.BLK_DTYPE)
        end = np.cumsum(b["len"].astype(np.int64))
        ns = int(np.searchsorted(end, 1 << 30, side="right")) or 1
        blk = b[:ns].copy()
        hi = int(blk["off"][-1] + blk["len"][-1])
        host = data[:hi].cpu().numpy()
    sample_bytes = int(blk["len"].astype(np.int64).sum())
    lib.batch(host, blk, nthreads=min(threads, 64))  # touch the sample once (page faults out of the timing)
    quota = cpus["cgroup_cpu_quota"]
    tset = {1, 16, threads}
    if quota:
        tset.add(max(1, int(quota)))
    res = {t: oracle.timed_batch(lib, host, blk, t, seconds=1.0)["GiB/s"] for t in sorted(tset)}
    best_t = max(res, key=lambda t: res[t])  # the primary figure: the best thread count measured
    numa = {}
    for node, node_cpus in cpus["numa"].items():
        if node_cpus and len(cpus["numa"]) > 1:
            numa[node] = {"threads": len(node_cpus), "GiB/s": round(
                oracle.timed_batch(lib, host, blk, len(node_cpus), seconds=1.0, cpus=node_cpus)["GiB/s"], 3)}
    dbb = None
    if kind == "reference":  # db_bench's own `crc32c` microbench loop, 1 thread
        try:
            mib_s, c = lib.dbbench_crc32c(500 << 20)
            dbb = {"MiB/s": round(mib_s, 1), "crc": f"0x{c:08x}", "loop": "4096 x 'x', 500 MiB, 1 thread"}
        except RuntimeError:
            pass
    return {
        "value": round(res[best_t], 3),
        "unit": "GiB/s",
        "cores": best_t,
        "effective_cores": min(best_t, int(quota)) if quota else best_t,
        "kind": kind,
        "sample": f"{ns} blocks ({sample_bytes / GIB:.2f} GiB) of the same workload in host memory, "
                  f"each thread hashing its own slice over and over for ~1 s; value = the best of "
                  f"{sorted(res)} threads",
        "by_threads_GiB/s": {str(t): round(v, 3) for t, v in sorted(res.items())},
        "single_thread_GiB/s": round(res[1], 3),
        "threads16_GiB/s": round(res[16], 3),
        "per_numa_node": numa or None,
        "db_bench_crc32c": dbb,
        "cpu_model": cpus.get("cpu_model", ""),
        "nproc": cpus["nproc"],
        "affinity_cpus": cpus["affinity"],
        "cgroup_cpu_quota": cpus["cgroup_cpu_quota"],
    }


def pmc_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py),
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM; None when not collected."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    main()
