"""Wavelength (and orbital-phase) sharding across GPUs of one node (replaces memoryHandler.py's chunker,
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


def phase_subset(host: dict, o0: int, o1: int) -> dict:
    """The host inputs (Transit._host_inputs) of orbital phases [o0, o1) only: the second sharding axis.
    Phases are independent too (per phase: columns, ordering, sigma row, tau), so a phase shard's R rows
    are the full run's rows bit for bit; every per-phase array (phase angles, planet and moon positions,
    Doppler factors, scenario body positions) is sliced, the chord and table inputs are shared."""
    n = len(host["orb"])

    def cut(v):
        a = np.asarray(v)
        return a[..., o0:o1] if a.ndim >= 1 and a.shape[-1] == n else v

    out = dict(host)
    out["orb"] = np.asarray(host["orb"])[o0:o1]
    out["planet_y"] = np.asarray(host["planet_y"])[o0:o1]
    out["moon_y"] = np.asarray(host["moon_y"]).reshape(-1, n)[:, o0:o1]
    scen = []
    for e in host["scenarios"]:
        e2 = dict(e)
        for k in ("shift", "body_x", "body_y"):
            if e.get(k) is not None:
                e2[k] = cut(e[k])
        scen.append(e2)
    out["scenarios"] = scen
    return out


def phase_options(host: dict) -> int:
    """Problem options a phase shard of `host` needs: PROM_OPT_DOPPLER_ROWS when the full problem's phases
    have different Doppler factors (a shard of one phase, or of equal factors, must still take the
    per-phase sigma rows the full run takes)."""
    from . import _native
    for e in host["scenarios"]:
        sh = np.asarray(e.get("shift", 1.0), dtype=np.float64).ravel()
        if sh.size > 1 and not np.all(sh == sh[0]):
            return _native.OPT_DOPPLER_ROWS
    return 0


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
