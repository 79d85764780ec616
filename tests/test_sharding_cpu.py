"""Wavelength sharding on the CPU: shard geometry, and the bench's multi-process
path (torch.distributed, world_size 2, gloo on 127.0.0.1) with the oracle standing in for the GPU
integrator of each rank: the gathered shards reproduce the single-process spectrum."""
import os
import socket

import numpy as np
import pytest

from prometheus_amd import sharding


@pytest.mark.parametrize("n", [1, 255, 256, 257, 1000, 190205, 1_000_000])
@pytest.mark.parametrize("parts", [1, 2, 3, 4, 8])
def test_split_covers_contiguously_on_tile_edges(n, parts):
    s = sharding.split(n, parts)
    assert s[0][0] == 0 and s[-1][1] == n
    for (a, b), (c, d) in zip(s[:-1], s[1:]):
        assert b == c and a < b
    for a, b in s[:-1]:
        assert b % sharding.WAVE_ALIGN == 0
    assert len(s) <= parts
    if n >= parts * sharding.WAVE_ALIGN:
        sizes = [b - a for a, b in s]
        assert len(s) == parts and max(sizes) - min(sizes) <= 2 * sharding.WAVE_ALIGN


def test_shard_for_rank_empty_tail():
    assert sharding.shard_for_rank(300, 4, 3) == (300, 300)
    assert sharding.shard_for_rank(300, 4, 0) == (0, 256)


@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_phase_subset_slices_every_per_phase_array(parts):
    """Phase shards (bench.py --shard-axis phase): split over phases with unit alignment covers them once;
    phase_subset slices exactly the per-phase inputs and shares the chord ones."""
    n = 8
    orb = np.linspace(-0.1, 0.1, n)
    host = {"orb": orb, "y": np.arange(5.0), "z": np.arange(5.0), "fout": np.ones(5), "planet_y": orb * 2,
            "moon_y": np.vstack([orb * 3, orb * 4]), "moon_R": np.ones(2),
            "scenarios": [{"shift": 1 + orb * 1e-5, "body_x": orb * 5, "body_y": 0.0, "n_tabulated": np.ones((5, 3))},
                          {"shift": 1 + orb * 2e-5}]}
    s = sharding.split(n, parts, align=1)
    assert s[0][0] == 0 and s[-1][1] == n and len(s) == min(parts, n)
    for o0, o1 in s:
        h = sharding.phase_subset(host, o0, o1)
        assert np.array_equal(h["orb"], orb[o0:o1]) and np.array_equal(h["planet_y"], orb[o0:o1] * 2)
        assert h["moon_y"].shape == (2, o1 - o0) and np.array_equal(h["moon_y"][1], orb[o0:o1] * 4)
        assert np.array_equal(h["scenarios"][0]["shift"], 1 + orb[o0:o1] * 1e-5)
        assert np.array_equal(h["scenarios"][0]["body_x"], orb[o0:o1] * 5) and h["scenarios"][0]["body_y"] == 0.0
        assert h["scenarios"][0]["n_tabulated"] is host["scenarios"][0]["n_tabulated"]
        assert np.array_equal(h["scenarios"][1]["shift"], 1 + orb[o0:o1] * 2e-5)
        assert h["y"] is host["y"] and h["fout"] is host["fout"]
    assert len(host["orb"]) == n   # the input is not modified


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    import torch.distributed as dist
    from oracle import prom_oracle as O
    from prometheus_amd import configs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = configs.reduced(configs.get("C2"), phi_steps=6, rho_steps=8, orbphase_steps=3, lower_w=5886e-8, upper_w=5892e-8)
    scen, dop, grids = O.from_setup(cfg)
    tabs = O.build_tables(scen, grids)
    wav = O.simulation_wavelengths(grids, O.atomic_species(scen))
    lo, hi = sharding.shard_for_rank(len(wav), world, rank)
    R = O.transit_depth(scen, dop, grids, wav[lo:hi], tabs)
    elapsed, pts = sharding.reduce_timing(dist, 0.5 + rank, R.size)
    np.save(os.path.join(out_dir, "R%d.npy" % rank), R)
    np.save(os.path.join(out_dir, "meta%d.npy" % rank), np.array([lo, hi, elapsed, pts]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shards_gather_to_full_spectrum(tmp_path):
    import torch.multiprocessing as mp
    from oracle import prom_oracle as O
    from prometheus_amd import configs
    port = _free_port()
    mp.spawn(_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    cfg = configs.reduced(configs.get("C2"), phi_steps=6, rho_steps=8, orbphase_steps=3, lower_w=5886e-8, upper_w=5892e-8)
    scen, dop, grids = O.from_setup(cfg)
    tabs = O.build_tables(scen, grids)
    wav = O.simulation_wavelengths(grids, O.atomic_species(scen))
    full = O.transit_depth(scen, dop, grids, wav, tabs)
    parts, covered = [], 0
    for r in range(2):
        lo, hi, elapsed, pts = np.load(tmp_path / ("meta%d.npy" % r))
        assert int(lo) == covered
        covered = int(hi)
        parts.append(np.load(tmp_path / ("R%d.npy" % r)))
        assert elapsed == 1.5                      # max over ranks
        assert pts == full.size                    # sum over ranks
    assert covered == len(wav)
    np.testing.assert_allclose(np.concatenate(parts, axis=1), full, rtol=1e-15, atol=0)
