"""Wavelength sharding across GPUs of one node (replaces memoryHandler.py's chunker,
reference memoryHandler.py:13-66, for the multi-device case).

R at one wavelength does not depend on any other wavelength, so the spectrum splits into contiguous
wavelength shards with no exchange step: one process (bench.py under torch.distributed.run) or one
host thread (Transit.sumOverChords(devices=...)) per GPU, and a host-side gather.  Shard edges are
multiples of 256 wavelengths, a multiple of the tau kernel's wavelength tile, which
keeps R bitwise identical
for any number of shards.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

WAVE_ALIGN = 256


def split(n: int, parts: int, align: int = WAVE_ALIGN) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) ranges covering [0, n), edges on multiples of ``align`` (the last edge is n);
    empty ranges are dropped."""
    if parts < 1:
        raise ValueError("parts must be >= 1")
    edges = (np.linspace(0, n / align, parts + 1).round() * align).astype(np.int64)
    edges = np.minimum(edges, n)
    edges[-1] = n
    return [(int(a), int(b)) for a, b in zip(edges[:-1], edges[1:]) if b > a]


def shard_for_rank(n: int, world: int, rank: int, align: int = WAVE_ALIGN) -> Tuple[int, int]:
    """This rank's [lo, hi); ranks beyond the number of non-empty shards get an empty range."""
    shards = split(n, world, align)
    return shards[rank] if rank < len(shards) else (n, n)


def reduce_timing(dist, elapsed_s: float, n_points: float) -> Tuple[float, float]:
    """(max over ranks of the elapsed time, sum over ranks of the points), via the process group
    (gloo / RCCL used only for these two scalars -- never for spectrum data)."""
    if dist is None:
        return float(elapsed_s), float(n_points)
    import torch
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    p = torch.tensor([float(n_points)], dtype=torch.float64)
    dist.all_reduce(p, op=dist.ReduceOp.SUM)
    return float(t.item()), float(p.item())
