"""CPU: block-range sharding and the multi-rank index scatter, world_size 2 over
gloo (the GPU run uses the same code over RCCL).  The per-rank CRC here is the oracle -- these
tests check the partitioning and the checksum-of-checksums, not the kernel.  The last test (-m gpu)
runs bench.py's own two-rank main() on the GPU box's one GPU and checks its XOR against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pebblesdb_amd.shard import block_range, byte_balanced_ranges, scatter_block_lens, scatter_block_ranges


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (7, 8), (1 << 20, 8), (33554432, 8), (1000, 3)])
def test_block_range_partitions(n, world):
    rs = [block_range(n, world, r) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    for (a, b), (c, d) in zip(rs, rs[1:]):
        assert b == c and a <= b
    sizes = [b - a for a, b in rs]
    assert max(sizes) - min(sizes) <= 1


def test_byte_balanced_ranges():
    rng = np.random.Generator(np.random.PCG64(1))
    lens = (rng.choice(np.arange(1, 65), size=5000, p=(1 / np.arange(1, 65)) / np.sum(1 / np.arange(1, 65))) * 1024)
    for world in (1, 2, 4, 8):
        rs = byte_balanced_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        for (a, b), (c, d) in zip(rs, rs[1:]):
            assert b == c
        tot = [int(lens[a:b].sum()) for a, b in rs]
        assert max(tot) - min(tot) <= 2 * int(lens.max())
    assert byte_balanced_ranges([], 4) == [(0, 0)] * 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle

    lo, hi = scatter_block_ranges(n_total, world, rank, torch.device("cpu"), dist)
    L = 4096
    data = oracle.splitmix_bytes((hi - lo) * L, 301, lo * L)
    blk = np.zeros(hi - lo, dtype=oracle.BLK_DTYPE)
    blk["off"] = np.arange(hi - lo) * L
    blk["len"] = L
    crcs = oracle.Oracle().batch(data, blk)
    x = torch.tensor([int(np.bitwise_xor.reduce(crcs)) if len(crcs) else 0], dtype=torch.int64)
    allx = [torch.zeros_like(x) for _ in range(world)]
    dist.all_gather(allx, x)
    if rank == 0:
        v = 0
        for t in allx:
            v ^= int(t.item())
        q.put(("xor", v))
    q.put(("range", rank, lo, hi))
    dist.destroy_process_group()


def test_gloo_world2_shards_cover_and_checksum_matches(oracle_lib):
    n_total, world = 3000, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=10) for _ in range(world + 1)]
    ranges = sorted((m[1], m[2], m[3]) for m in msgs if m[0] == "range")
    assert ranges == [(0, 0, 1500), (1, 1500, 3000)]
    xor = next(m[1] for m in msgs if m[0] == "xor")
    import oracle

    data = oracle.splitmix_bytes(n_total * 4096, 301)
    blk = np.zeros(n_total, dtype=oracle.BLK_DTYPE)
    blk["off"] = np.arange(n_total) * 4096
    blk["len"] = 4096
    assert xor == int(np.bitwise_xor.reduce(oracle_lib.batch(data, blk, nthreads=4)))


def _bench_worker(rank, world, port, q):
    """bench.py's multi-rank plumbing (no GPU): the C3 plan, the byte-balanced range scatter and
    the per-rank row gather that feeds the JSON line's `ranks`."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    # the plan exists on rank 0 only; every rank receives its range and its own lengths
    sizes = bench.c3_plan(64 << 20, world) if rank == 0 else None  # 64 MiB per rank (bench default 16 GiB)
    lo, hi, lens = scatter_block_lens(sizes, world, rank, torch.device("cpu"), dist)
    mine = int(lens.sum())
    rows = bench.gather_rank_rows([rank, 0, -1, mine, 123456, rank * 7, -1], world, torch.device("cpu"), dist)
    if rank == 0:
        q.put(("rows", rows, len(sizes), int(sizes.sum())))
    full = bench.c3_plan(64 << 20, world)  # (test only: the same list, to check what rank r received)
    q.put(("range", rank, lo, hi, bool(len(lens) == hi - lo and (lens == full[lo:hi]).all())))
    dist.destroy_process_group()


def test_gloo_world2_bench_c3_byte_balanced():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=10) for _ in range(world + 1)]
    rows, n, total = next(m[1:] for m in msgs if m[0] == "rows")
    ranges = sorted((m[1], m[2], m[3]) for m in msgs if m[0] == "range")
    assert all(m[4] for m in msgs if m[0] == "range")  # each rank's lengths are its slice of the plan
    assert ranges[0][1] == 0 and ranges[-1][2] == n and ranges[0][2] == ranges[1][1]
    assert [r[0] for r in rows] == [0, 1] and sum(r[3] for r in rows) == total
    assert abs(rows[0][3] - rows[1][3]) <= 2 * 64 * 1024  # byte-balanced to within a block or two
    assert abs(total - world * (64 << 20)) <= 64 * 1024


def _bench_cmd(*extra):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return [sys.executable, os.path.join(root, "bench.py"), *extra], root


def test_bench_gpus2_without_launcher_runs_two_ranks():
    """The driver's BENCH form `python bench.py --gpus N` (no torchrun): bench.py must re-launch
    itself as N ranks, not silently measure one.  --dry-run keeps it on the CPU (gloo, no kernel)."""
    import json
    import subprocess

    cmd, root = _bench_cmd("--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run", "--nblk", "1000")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["dry_run"] is True
    assert [x["rank"] for x in line["ranks"]] == [0, 1]
    assert [x["blocks"] for x in line["ranks"]] == [1000, 1000]


def test_bench_gpus2_default_is_c4_shards():
    """Without --nblk, `--gpus N > 1` runs BASELINE config 4's shard size: 4 194 304 x 4 KiB = 16 GiB
    per rank (128 GiB at N = 8); one GPU stays C2 (1 M blocks).  --dry-run: no device."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    for gpus, blocks, c4 in ((2, 4194304, True), (1, 1 << 20, False)):
        cmd, root = _bench_cmd("--gpus", str(gpus), "--steps", "2", "--warmup", "1", "--dry-run")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
        assert [x["blocks"] for x in line["ranks"]] == [blocks] * gpus
        assert line["config"]["blocks_per_gpu"] == blocks
        assert ("c4" in line["config"]["workload"]) == c4


def test_bench_dry_run_curve_keys():
    """The 1 -> 8 curve's keys (--dry-run, no device): the N = 1 default line carries the c4_shard
    anchor (one 16 GiB config-4 shard outside `value`); an N > 1 line carries one steady-state row
    per rank and the steady state over ranks, and no c4_shard (its ranks ARE c4 shards)."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    for gpus in (1, 2):
        cmd, root = _bench_cmd("--gpus", str(gpus), "--steps", "2", "--warmup", "1", "--dry-run")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
        assert [set(x) >= {"rank", "blocks", "steady_kernel_avg_ms"} for x in line["ranks"]] == [True] * gpus
        # the copy-inclusive leg runs on every rank at once (its own PCIe link), N = 1 included
        ci = line["copy_inclusive"]
        assert ci["concurrent_ranks"] == gpus and len(ci["ranks_GiB/s"]) == gpus and ci["entry"] == "pdb_crc32c_batch_host"
        if gpus == 1:
            assert line["c4_shard"]["blocks"] == 4194304 and line["c4_shard"]["bytes"] == 16 << 30
            assert line["steady_state"] is None
        else:
            assert "c4_shard" not in line
            assert line["steady_state"]["over_ranks"]["ranks"] == gpus
    cmd, root = _bench_cmd("--gpus", "1", "--steps", "2", "--dry-run", "--no-c4-shard")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert r.returncode == 0 and "c4_shard" not in json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_process_group_world1_dry_run():
    """--process-group at world size 1: the index scatter, the rows all_gather and the MAX
    all_reduce all run through a (gloo) process group of one rank."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "2", "--dry-run", "--process-group", "--nblk", "777"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
    assert line["world_size"] == 1 and [x["blocks"] for x in line["ranks"]] == [777]


@pytest.mark.parametrize("gpus,world", [(1, "2"), (8, "4")])
def test_bench_gpus_world_size_mismatch_fails(gpus, world):
    import subprocess

    cmd, root = _bench_cmd("--gpus", str(gpus), "--dry-run")
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=root, env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["c2", "c3"])
def test_bench_main_two_ranks_on_the_gpu(oracle_lib, workload):
    """bench.py's own multi-rank main() end to end on the GPU: torchrun with 2 ranks sharing the
    box's one GPU (gloo process group: RCCL refuses two ranks on one device), each hashing its shard
    through libpdb_crc32c.so.  The JSON line must carry both ranks, the per-rank byte counts of the
    count (c2) or byte-balanced (c3) split, and an XOR of all CRCs equal to the oracle's over the
    whole two-rank workload."""
    import json
    import subprocess
    import sys

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nblk, c3_bytes = 4096, 48 << 20
    # c2 under the driver's torchrun form, c3 through bench.py's own re-launch (`--gpus 2`, no launcher)
    launcher = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                 "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] if workload == "c2"
                else [sys.executable])
    cmd = launcher + [os.path.join(root, "bench.py"),
                      "--gpus", "2", "--steps", "3", "--warmup", "1", "--settle", "0", "--backend", "gloo",
                      "--workload", workload, "--nblk", str(nblk), "--c3-bytes", str(c3_bytes), "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["steps"] == 3
    assert [x["rank"] for x in line["ranks"]] == [0, 1]
    import oracle

    if workload == "c2":
        assert [x["bytes"] for x in line["ranks"]] == [nblk * 4096] * 2
        data = oracle.splitmix_bytes(2 * nblk * 4096, 301)  # rank r's shard = blocks [r n, (r+1) n)
        blk = np.zeros(2 * nblk, dtype=oracle.BLK_DTYPE)
        blk["off"] = np.arange(2 * nblk) * 4096
        blk["len"] = 4096
        exp = int(np.bitwise_xor.reduce(oracle_lib.batch(data, blk, nthreads=4)))
    else:
        import bench

        sizes = bench.c3_plan(c3_bytes, 2)
        (lo0, hi0), (lo1, hi1) = byte_balanced_ranges(sizes, 2)
        assert [x["bytes"] for x in line["ranks"]] == [int(sizes[lo0:hi0].sum()), int(sizes[lo1:hi1].sum())]
        exp = 0
        for rank, (lo, hi) in enumerate(((lo0, hi0), (lo1, hi1))):  # rank r fills its image with seed 303 + r
            s = sizes[lo:hi]
            data = oracle.splitmix_bytes(int(s.sum()), 303 + rank)
            blk = np.zeros(len(s), dtype=oracle.BLK_DTYPE)
            blk["off"] = np.concatenate([[0], np.cumsum(s)[:-1]])
            blk["len"] = s
            exp ^= int(np.bitwise_xor.reduce(oracle_lib.batch(data, blk, nthreads=4)))
    assert int(line["xor_of_crcs"], 16) == exp


@pytest.mark.gpu
def test_bench_rccl_branch_world1_on_the_gpu(oracle_lib):
    """The RCCL branch of bench.py, which only the driver's 8-GPU run takes otherwise: torchrun with
    one rank and --process-group, so `init_process_group("nccl", device_id=...)`, the index scatter
    (shard.scatter_block_ranges), the per-rank rows all_gather and the MAX all_reduce of the region
    time all run on device tensors over RCCL -- exactly the calls an N-rank run makes.  The JSON line's
    XOR of all CRCs must equal the oracle's."""
    import json
    import subprocess
    import sys

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nblk = 8192
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--settle", "0", "--backend", "nccl",
           "--process-group", "--nblk", str(nblk), "--no-cpu-baseline", "--no-copy-inclusive", "--no-ceiling"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
    assert line["world_size"] == 1 and line["process_group"] == "nccl"
    assert [x["bytes"] for x in line["ranks"]] == [nblk * 4096]
    import oracle

    data = oracle.splitmix_bytes(nblk * 4096, 301)
    blk = np.zeros(nblk, dtype=oracle.BLK_DTYPE)
    blk["off"] = np.arange(nblk) * 4096
    blk["len"] = 4096
    assert int(line["xor_of_crcs"], 16) == int(np.bitwise_xor.reduce(oracle_lib.batch(data, blk, nthreads=4)))
    # the N = 1 line's equal-shard anchor: rank 0's 16 GiB shard of config 4, every CRC folded into
    # one XOR that must equal the oracle's over the same bytes (generated again here on the device)
    c4 = line["c4_shard"]
    assert c4["blocks"] == 4194304 and c4["steps"] == 3 and c4["warmup"] == 1 and c4["GiB_s"] > 0
    from pebblesdb_amd import diag

    d = torch.empty(c4["blocks"] * 4096, dtype=torch.uint8, device="cuda")
    diag.fill_splitmix(d, 301, byte_offset=0)
    host = d.cpu().numpy()
    del d
    torch.cuda.empty_cache()
    blk = np.zeros(c4["blocks"], dtype=oracle.BLK_DTYPE)
    blk["off"] = np.arange(c4["blocks"], dtype=np.int64) * 4096
    blk["len"] = 4096
    assert int(c4["xor_of_crcs"], 16) == int(np.bitwise_xor.reduce(oracle_lib.batch(host, blk, nthreads=16)))
