"""Block-range sharding across ranks.

Blocks are independent, so N GPUs = N disjoint shards and no data-path collective.  Fixed-size
blocks split by count; variable-size blocks split by bytes (prefix sum over lengths) so each
rank hashes about the same number of bytes.
"""
from __future__ import annotations

import numpy as np


def block_range(nblk: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of `nblk` fixed-size blocks owned by `rank` ([r*N/G, (r+1)*N/G))."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return nblk * rank // world, nblk * (rank + 1) // world


def byte_balanced_ranges(lens, world: int) -> list[tuple[int, int]]:
    """Split a descriptor list into `world` contiguous ranges with ~equal byte totals."""
    lens = np.asarray(lens, dtype=np.int64)
    if world < 1:
        raise ValueError("bad world")
    if lens.size == 0:
        return [(0, 0)] * world
    cs = np.cumsum(lens)
    total = int(cs[-1])
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cs, total * r / world, side="left")) + 1)
    cuts.append(lens.size)
    cuts = np.maximum.accumulate(np.minimum(np.array(cuts), lens.size))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def scatter_block_ranges(n_total: int, world: int, rank: int, device, dist=None,
                         lens=None) -> tuple[int, int]:
    """Rank 0 computes every rank's [lo, hi) (by count, or by bytes when `lens` is given) and
    scatters them over the process group: each rank receives its own 16-B range -- the only
    collective on this path (RCCL over xGMI on GPUs, gloo in the CPU tests).  With `dist` given the
    scatter runs at any world size, 1 included (bench.py --process-group exercises the RCCL branch on
    one GPU).  Returns this rank's range."""
    import torch

    mine = torch.zeros(2, dtype=torch.int64, device=device)
    parts = None
    if rank == 0:
        rngs = (byte_balanced_ranges(lens, world) if lens is not None
                else [block_range(n_total, world, r) for r in range(world)])
        parts = [torch.tensor(r, dtype=torch.int64, device=device) for r in rngs]
    if dist is not None:
        dist.scatter(mine, scatter_list=parts, src=0)
    else:
        if world != 1:
            raise ValueError("scatter_block_ranges: world > 1 needs a process group")
        mine.copy_(parts[0])
    return int(mine[0]), int(mine[1])


def scatter_block_lens(lens, world: int, rank: int, device, dist=None) -> tuple[int, int, np.ndarray]:
    """A variable-size plan held by rank 0 only (`lens` is None on every other rank): rank 0 splits
    it into byte-balanced ranges, scatters each rank's [lo, hi) (scatter_block_ranges), then each
    rank's own block lengths (one scatter of equal-width int64 rows, padded to the longest range).
    Returns (lo, hi, this rank's lengths)."""
    import torch

    rngs = byte_balanced_ranges(lens, world) if rank == 0 else None
    width = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == 0:
        width[0] = max((hi - lo for lo, hi in rngs), default=0)
    if dist is not None:
        dist.broadcast(width, src=0)
    w = int(width.item())
    lo, hi = scatter_block_ranges(len(lens) if rank == 0 else 0, world, rank, device, dist,
                                  lens=lens if rank == 0 else None)
    mine = torch.zeros(max(w, 1), dtype=torch.int64, device=device)
    parts = None
    if rank == 0:
        src = torch.from_numpy(np.asarray(lens, dtype=np.int64))
        parts = []
        for a, b in rngs:
            row = torch.zeros(max(w, 1), dtype=torch.int64)
            row[: b - a] = src[a:b]
            parts.append(row.to(device))
    if dist is not None:
        dist.scatter(mine, scatter_list=parts, src=0)
    else:
        if world != 1:
            raise ValueError("scatter_block_lens: world > 1 needs a process group")
        mine.copy_(parts[0])
    return lo, hi, mine[: hi - lo].cpu().numpy()
