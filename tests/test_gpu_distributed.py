"""bench.py's multi-process path on the GPU: torch.distributed.run with two ranks (both on device 0 of a
one-GPU box), wavelength shards without any collective on the data, gathered on the host and compared
bitwise with a single-rank run of the same (strong-scaling) spectrum.  Reference: the chunker this
replaces, memoryHandler.py:55-66; SURVEY.md 8(e)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(tmp, world, config, axis="wavelength", scaling=("--scaling", "strong")):
    out = os.path.join(tmp, "w%d_%s_%s" % (world, axis, "_".join(scaling) or "default"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", str(world), "--steps", "3", "--warmup", "1", "--config", config, *scaling,
           *(() if "--strong" in scaling else ("--strong", "")),   # (the default strong legs: their own test)
           "--shard-axis", axis, "--no-cpu-baseline", "--no-projection", "--dump-R", out]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    shards = []
    for r in range(world):
        with open(os.path.join(out, "range_rank%d.json" % r)) as fh:
            rg = json.load(fh)
        shards.append((rg["w0"], rg["w1"], np.load(os.path.join(out, "R_rank%d.npy" % r)), rg["o0"], rg["o1"]))
    return json.loads(line), shards


@pytest.mark.parametrize("config", ["C2", "C4"])
def test_two_rank_bench_gathers_bitwise(config, tmp_path):
    res1, (s1,) = _bench(str(tmp_path), 1, config)
    res2, sh = _bench(str(tmp_path), 2, config)
    assert res2["n_gpus"] == 2 and res2["scaling"] == "strong"
    n_wav = s1[2].shape[1]
    assert s1[0] == 0 and s1[1] == n_wav
    R = np.empty_like(s1[2])
    edge = 0
    for w0, w1, part, _, _ in sh:
        assert w0 == edge and part.shape == (R.shape[0], w1 - w0)
        R[:, w0:w1] = part
        edge = w1
    assert edge == n_wav
    assert np.array_equal(R, s1[2])
    # whole-job points / s counts every rank's shard once
    assert res2["config"]["global_wavelengths"] == res1["config"]["global_wavelengths"]


def test_shard_mode_is_one_ranks_work(tmp_path):
    """bench.py --shard r/N times exactly rank r's shard of an N-way strong split on one GPU: its R is the
    matching slice of the two-rank run's gathered spectrum (C2: bitwise)."""
    res1, (s1,) = _bench(str(tmp_path), 1, "C2")
    out = os.path.join(str(tmp_path), "shard")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1", "--config", "C2",
           "--shard", "1/2", "--shard-axis", "wavelength", "--no-cpu-baseline", "--no-projection", "--dump-R", out]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert res["scaling"] == "strong" and "shard 1/2" in res["config"]["workload"]
    with open(os.path.join(out, "range_rank0.json")) as fh:
        rg = json.load(fh)
    part = np.load(os.path.join(out, "R_rank0.npy"))
    assert rg["w0"] > 0 and rg["w1"] == s1[2].shape[1]
    assert np.array_equal(part, s1[2][:, rg["w0"]:rg["w1"]])


@pytest.mark.parametrize("config", ["C2", "C4"])
def test_phase_shard_is_full_runs_rows(config, tmp_path):
    """bench.py --shard r/N --shard-axis phase: rank r's orbital phases over every wavelength; its R is
    the single-rank run's rows [o0, o1) bit for bit (phases are independent: per-phase columns, ordering,
    sigma row and tau)."""
    res1, (s1,) = _bench(str(tmp_path), 1, config)
    out = os.path.join(str(tmp_path), "pshard")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1", "--config", config,
           "--shard", "1/2", "--shard-axis", "phase", "--no-cpu-baseline", "--no-projection", "--dump-R", out]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert res["scaling"] == "strong" and "phases [" in res["config"]["workload"]
    assert res["config"]["parallelism"].startswith("phase shards")
    with open(os.path.join(out, "range_rank0.json")) as fh:
        rg = json.load(fh)
    part = np.load(os.path.join(out, "R_rank0.npy"))
    n_orb = s1[2].shape[0]
    assert rg["w0"] == 0 and rg["w1"] == s1[2].shape[1] and 0 < rg["o0"] < rg["o1"] == n_orb
    assert np.array_equal(part, s1[2][rg["o0"]:rg["o1"]], equal_nan=True)


def test_two_rank_bench_default_phase_axis(tmp_path):
    """--scaling strong --shard-axis auto splits the orbital phases when they divide evenly (C4: 8 phases over 2
    ranks): the gathered rows are the single-rank run's, bit for bit."""
    res1, (s1,) = _bench(str(tmp_path), 1, "C4", axis="auto")
    res2, sh = _bench(str(tmp_path), 2, "C4", axis="auto")
    assert res2["scaling"] == "strong" and res2["config"]["parallelism"].startswith("phase shards")
    R = np.full_like(s1[2], np.nan)
    edge = 0
    for w0, w1, part, o0, o1 in sorted(sh, key=lambda t: t[3]):
        assert w0 == 0 and w1 == s1[2].shape[1] and o0 == edge and part.shape == (o1 - o0, w1)
        R[o0:o1] = part
        edge = o1
    assert edge == s1[2].shape[0]
    assert np.array_equal(R, s1[2], equal_nan=True)


def test_two_rank_weak_default_over_phases(tmp_path):
    """N > 1 defaults to weak scaling over orbital phases: the config with N x its phases over the same phase range,
    rank r integrating a run of the config's phase count at every wavelength.  Two ranks of C4 (2 x 8 phases): the
    gathered rows are bitwise a single-rank run of the 16-phase problem, and value counts both ranks' points."""
    import copy
    res2, sh = _bench(str(tmp_path), 2, "C4", axis="auto", scaling=())
    assert res2["scaling"] == "weak" and res2["config"]["parallelism"].startswith("phase shards")
    assert res2["config"]["orbital_phases"] == 8 and "weak scaling over phases: 16 global phases" in \
        res2["config"]["workload"]
    from prometheus_amd import configs, setupfile
    cfg = configs.get("C4")
    cfg["Grids"]["orbphase_steps"] = 16
    tr = setupfile.build_transit(copy.deepcopy(cfg))
    R1 = tr.sumOverChords(devices=[0], options=0)
    R = np.full_like(R1, np.nan)
    for w0, w1, part, o0, o1 in sh:
        assert w0 == 0 and w1 == R1.shape[1] and o1 - o0 == 8
        R[o0:o1] = part
    assert np.allclose(R, R1, rtol=1e-13, atol=0)
    assert abs(res2["value"] * res2["ms_per_step"] * 1e-3 - 16 * R1.shape[1]) / (16 * R1.shape[1]) < 1e-9


def test_two_rank_line_carries_strong_wavelength_split(tmp_path):
    """Every N > 1 line carries `strong`: configurations split over the ranks in contiguous wavelength shards (the
    north-star axis, BASELINE.json configs[3]), timed in the same process group, with the full grid on rank 0 alone
    for the speedup.  Two ranks, weak main leg (C4 over phases) and a strong C4 leg: the strong shards gathered on
    the host are bitwise a single-rank run of C4."""
    res1, (s1,) = _bench(str(tmp_path), 1, "C4")
    res2, _ = _bench(str(tmp_path), 2, "C4", axis="auto", scaling=("--strong", "C4"))
    st = res2["strong"]["C4"]
    assert res2["scaling"] == "weak" and st["axis"] == "wavelength"
    assert st["value"] > 0 and st["ms_per_step"] > 0 and st["ms_full_grid_one_gpu"] > 0 and st["speedup_vs_one_gpu"] > 0
    assert "2 contiguous wavelength shards" in st["workload"]
    out = os.path.join(str(tmp_path), "w2_auto_--strong_C4", "strong_C4")
    R = np.full_like(s1[2], np.nan)
    edge = 0
    for r in range(2):
        with open(os.path.join(out, "range_rank%d.json" % r)) as fh:
            rg = json.load(fh)
        part = np.load(os.path.join(out, "R_rank%d.npy" % r))
        assert rg["w0"] == edge and part.shape == (R.shape[0], rg["w1"] - rg["w0"])
        R[:, rg["w0"]:rg["w1"]] = part
        edge = rg["w1"]
    assert edge == R.shape[1]
    assert np.array_equal(R, s1[2])
