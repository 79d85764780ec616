#!/usr/bin/env python3
"""Benchmark: spectrum points per second of the fused transit integrator on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-cpu-baseline]

N=1: the largest single-GPU configuration of BASELINE.json, configs[2] (C3: power-law atmosphere
with Na I + Ca II + Mg I, orbital Doppler shift on, 351,222 wavelengths x 16 orbital phases x
2,400 chords x 30 samples, WASP-49b).  One step = one pass of the hot path over the whole spectrum
with all inputs resident in HBM (prom_transit_run): on the default transmission-curve path
k_columns8 (densities, column densities, culling), k_tc_build (every phase's transmission curve
T_o) and k_sigma_tw (sigma of the merged absorber at every phase's Doppler shift over target windows,
R = T_o(Y); k_sigma_tc without orbital Doppler shift between the phases);
several unmerged species take the windowed path (k_order, k_tau_w / k_tau_p), molecules k_tau_mol.
--config C2 gives the configs[1] line.

N>1 (launched by torch.distributed.run, one process per GPU), sharding with no collective on the data
path (torch.distributed carries only the timing barrier and the max-over-ranks time):
  --scaling weak (default; SURVEY.md 8e: the path partitions, every rank integrates its own part): every rank a
      problem the size of the N = 1 workload, so value(N) / value(1) is the scaling the driver computes.
      --weak-axis phase (default): C3 with N x 16 orbital phases over the same phase range; rank r integrates
      phases [16 r, 16 r + 16) at all 351,222 wavelengths.  --weak-axis wavelength: the grid at N x finer
      resolution, contiguous shard r on rank r.
  --scaling strong: the global spectrum is the config's grid as it stands (default config C4x10, the 8-GPU
      workload BASELINE.json names; also C4x10p64, C5), split into N shards along --shard-axis (auto: orbital
      phases when they divide evenly, else contiguous wavelength ranges).
  --shard r/N (one process): only shard r of N of the config's grid, timed alone on one GPU -- one rank's
      work under an N-way strong split.
  --shard-axis phase: strong splits over orbital phases instead (every wavelength, phases [o0, o1)): the
      phases are independent too, and a phase shard does not repeat the per-phase chord work.

The N=1 line also carries, per kernel of the step, its device duration (prom_transit_kernel_ms: one run in
flight, dispatch-packet events) with its algorithmic bytes and roofline fraction, the path-level fraction
(compulsory bytes / ms_per_step), a live HBM read peak, and the strong-scaling projection of the two
8-GPU configurations (C4x10, C5): T(full grid) / T(shard 0 of 8), each timed on this GPU.

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402  (first: one HIP runtime per process, torch's; used for sync + gloo timing only)

FP64_VALU_PEAK_TFLOPS = 78.6     # MI355X FP64 vector peak (AMD spec; the FP64 matrix peak is the same)
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=None,
                    help="C1..C5, C4x10, C4x10p64 (default: C3, for N = 1 and for the weak-scaling default of N > 1; "
                         "C4x10, the 8-GPU configuration BASELINE.json names, with --scaling strong)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="N > 1: weak (default: every rank integrates a problem the size of the config's -- see "
                         "--weak-axis) or strong (the config's grid split into N shards)")
    ap.add_argument("--weak-axis", choices=("phase", "wavelength"), default="phase",
                    help="weak scaling: phase (default; the config with N x its orbital phases over the same "
                         "orbital-phase range, rank r integrates phases [r n, (r + 1) n) at every wavelength -- "
                         "the same wavelength grid and phase count per rank as N = 1) or wavelength (the grid at "
                         "N x finer resolution, contiguous shard r on rank r)")
    ap.add_argument("--shard", default=None, metavar="r/N",
                    help="time only shard r of an N-way split of the config's grid (strong scaling, one process)")
    ap.add_argument("--shard-axis", choices=("wavelength", "phase", "auto"), default="auto",
                    help="strong splits (--shard, --scaling strong): contiguous wavelength ranges, orbital-phase "
                         "ranges (every wavelength, phases [o0, o1)), or auto (default): phases when every rank "
                         "gets the same number of them, else wavelengths")
    ap.add_argument("--strong", default="C4x10,C4x10p256", metavar="CONFIGS",
                    help="N > 1: after the main leg, also time these configurations split over the N ranks in "
                         "contiguous wavelength shards (the north-star strong-scaling axis; the line's `strong` "
                         "object, with each one's full grid timed on rank 0 alone for the speedup); '' to skip")
    ap.add_argument("--no-projection", action="store_true",
                    help="skip the strong-scaling projection (C4x10 and C5, full grid vs shard 0 of 8)")
    ap.add_argument("--kernel-runs", type=int, default=20,
                    help="serialized runs for the per-kernel durations (prom_transit_kernel_ms)")
    ap.add_argument("--cpu-workers", type=int, default=None,
                    help="processes of the multi-core CPU baseline leg (default: this process's CPU share, <= 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dump-R", default=None, metavar="DIR",
                    help="after the timed loop, save this rank's R shard and its wavelength range under DIR "
                         "(tests: the gathered shards against a single-rank run)")
    ap.add_argument("--cpu-sample-wavelengths", type=int, default=None,
                    help="oracle sample size (default: ~10 s of reference-speed CPU work per config)")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", 1))
    if a.scaling is None:
        a.scaling = "weak"
    if a.config is None:
        a.config = "C4x10" if (world > 1 and a.scaling == "strong") else "C3"
    return a


def resolve_axis(axis: str, n_orb: int, parts: int) -> str:
    """auto: orbital phases when the phases split evenly over the parts (no rank repeats another's per-phase
    chord work and the shards are equal), else wavelengths."""
    if axis != "auto":
        return axis
    return "phase" if parts > 1 and n_orb % parts == 0 else "wavelength"


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def global_config(name: str, world: int, scaling: str = "weak", weak_axis: str = "phase") -> dict:
    """The global problem of an N-rank run.  Weak scaling keeps every rank's work the size of the config's: over
    phases, N x the orbital phases over the same range (orbphase_border unchanged: a finer phase sampling of the
    same transit), each rank a contiguous run of the config's phase count; over wavelengths, N x finer
    resolution."""
    from prometheus_amd import configs
    cfg = configs.get(name)
    if world > 1 and scaling == "weak":
        g = cfg["Grids"]
        if weak_axis == "phase":
            g["orbphase_steps"] = int(g["orbphase_steps"]) * world
        else:
            g["resolutionLow"] = g["resolutionLow"] / world
            g["resolutionHigh"] = g["resolutionHigh"] / world
    return cfg


TAU_TIMING_STRIDE = 8


def flops_per_eval(n_atoms: int) -> int:
    """FP64 flops (FMA = 2) of one exact chord-wavelength evaluation in the tau kernel's window
    (DESIGN.md): y = -tau 1024/ln2 = sum_s N_s sy_s -> 2S - 1;  2^(y/1024): rint, d = y - k, 3-FMA
    polynomial, ldexp -> 9;  F * S -> 1;  acc fma -> 2."""
    return 2 * n_atoms - 1 + 12


def tau_bytes_per_launch(n_wav: int, n_orb: int, n_sigma: int, sigma_rows: int = 1) -> int:
    """Algorithmic HBM bytes of one tau-kernel launch (DESIGN.md "Roofline"): R[n_orb][n_wav] written
    and the resampled cross sections read once: n_sigma arrays (one per species, or one for merged
    species) of sigma_rows rows (one per phase with orbital Doppler shift -- each phase sees its own
    shifted sigma -- else one shared row); window records, windows and tail moments (~1 %) are not
    counted."""
    return 8 * n_orb * n_wav + 8 * n_wav * n_sigma * sigma_rows


def latest_profile_traffic(kernel: str, config: str, suffix: str = ""):
    """Measured HBM bytes per launch of ``kernel`` on ``config`` from the newest committed rocprofv3 PMC
    summary (profiles/r*_<config>_traffic.json, written by tools/bench_traffic.sh through
    tools/traffic_summary.py: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md "HBM"), or None."""
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_%s_traffic.json" % config)), reverse=True):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except Exception:
            continue
        for name, v in d.items():
            if name.startswith(kernel) and name.endswith(suffix):
                return v.get("hbm_bytes_per_launch")
    return None


def describe(cfg: dict) -> str:
    return "; ".join("%s: %s" % (k, "+".join(v.keys())) for k, v in cfg["Species"].items())


_CPU = {}


def _cpu_chunk(sel):
    """One worker's share of the multi-core CPU leg (state inherited from the parent at fork)."""
    from oracle import prom_oracle as O
    scen, dop, grids, tabs = _CPU["state"]
    t0 = time.perf_counter()
    O.transit_depth(scen, dop, grids, sel, tabs)
    return time.perf_counter() - t0


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))   # the GPU box grants 16 CPUs per GPU (nproc shows the whole host)


def cpu_baseline(cfg: dict, n_sample: int, workers: int):
    """The oracle (numpy restatement of the reference dataflow, gasProperties.py:1160-1258) on a bounded
    sample of the same workload, two legs:
      single: one process, the first n_sample wavelengths (what the reference itself does: it is
              single-threaded);
      multi:  `workers` forked processes over a wavelength-chunked sample of workers * n_sample
              wavelengths (the reference's CPU multiprocessing plan, SURVEY.md 8d / BASELINE.md).
    Every phase and chord is integrated.  Runs before this process touches the GPU, so the fork is clean.
    Returns the multi-core leg as the baseline, with the single-core leg beside it."""
    import multiprocessing as mp
    from oracle import prom_oracle as O
    mol = {"H2O": O.synthetic_molecular_table()} if "H2O" in str(cfg["Species"]) else None
    scen, dop, grids = O.from_setup(cfg, mol)
    tabs = O.build_tables(scen, grids)
    wav = O.simulation_wavelengths(grids, O.atomic_species(scen))
    n_orb = int(grids["orbphase_steps"])
    n_pr = int(grids["phi_steps"]) * int(grids["rho_steps"])
    sel = wav[:n_sample]
    t0 = time.perf_counter()
    O.transit_depth(scen, dop, grids, sel, tabs)
    dt1 = time.perf_counter() - t0
    single = len(sel) * n_orb / dt1
    _CPU["state"] = (scen, dop, grids, tabs)
    n_mc = min(len(wav), n_sample * workers)
    chunks = [c for c in np.array_split(wav[:n_mc], workers) if len(c)]
    ctx = mp.get_context("fork")
    with ctx.Pool(len(chunks)) as pool:
        pool.map(_cpu_chunk, [c[:1] for c in chunks])          # workers up (imports, first touch)
        t0 = time.perf_counter()
        pool.map(_cpu_chunk, chunks, chunksize=1)
        dtm = time.perf_counter() - t0
    multi = n_mc * n_orb / dtm
    name = cfg.get("_name", "config")
    return {"value": multi, "unit": "spectrum points/s", "cores": len(chunks), "kind": "port",
            "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "single_core_value": single,
            "sample": "%s: all %d phases x %d chords; multi-core leg: first %d of %d wavelengths (%d points) "
                      "chunked over %d forked numpy processes in %.2f s; single-core leg: first %d wavelengths "
                      "in %.2f s (%.3g points/s)" % (name, n_orb, n_pr, n_mc, len(wav), n_mc * n_orb,
                                                     len(chunks), dtm, len(sel), dt1, single)}


CPU_SAMPLE = {"C1": 219, "C2": 12288, "C3": 6144, "C4": 12288, "C4x10": 12288, "C5": 16}


def measured_read_peak():
    """The measured STREAM-like HBM read peak of an MI355X (SURVEY.md 8d rule (i)): the newest committed
    tools/microbench/hbm_peak result (profiles/r*_hbm_peak.json: 4 GiB streamed with 16-byte loads per lane,
    best of 20 launches), as (GB/s, source) or (None, None)."""
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_hbm_peak.json")), reverse=True):
        try:
            with open(path) as fh:
                d = json.load(fh)
            return float(d["read_gbs_best"]), os.path.relpath(path, REPO)
        except Exception:
            continue
    return None, None


def table_nodes_in_range(tr, host, w0: int, w1: int) -> int:
    """Refined-table nodes the shifted targets of wavelengths [w0, w1) can bracket, summed over the atomic
    constituents (each node's x and log10 sigma: 16 algorithmic bytes)."""
    lo, hi = float(tr.wavelength[w0]), float(tr.wavelength[w1 - 1])
    total = 0
    for e in host["scenarios"]:
        sh = np.asarray(e["shift"], dtype=np.float64)
        for con in e["dist"].constituents:
            if con.isMolecule:
                continue
            x = np.asarray(con.lookupFunction.x)
            a = np.searchsorted(x, lo * sh.min(), side="right") - 1
            b = np.searchsorted(x, hi * sh.max(), side="left") + 1
            total += int(max(0, min(len(x), b) - max(0, a)))
    return total


def time_runs(dev, prob, steps: int, warmup: int) -> float:
    """ms per run of a problem in the pipelined loop (inputs resident; set outside the timed region)."""
    dev.transit_set(prob)
    dev.transit_run()
    dev.synchronize()
    for _ in range(warmup):
        dev.transit_run()
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        dev.transit_run()
    dev.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def strong_projection(dev_id: int, names=("C4x10", "C4x10p64", "C5"), parts: int = 8):
    """Strong scaling measured on one GPU: each configuration's full grid, then the largest
    of `parts` wavelength shards (edges on 256 wavelengths) and the largest of `parts` orbital-phase shards,
    all in the pipelined loop.  T(full) / T(shard) is the speedup `parts` GPUs give at best on that axis (no
    collective, host gather only); `axis` names the faster one (bench.py --scaling strong --shard-axis)."""
    from prometheus_amd import _native, configs, setupfile, sharding, gasProperties
    out = {}
    for name in names:
        cfg = configs.get(name)
        if any(sp not in ("NaI", "KI", "CaII", "MgI") for sc in cfg["Species"].values() for sp in sc):
            gasProperties.register_molecular_table("H2O", configs.synthetic_molecular_table())
        tr = setupfile.build_transit(cfg)
        dev = _native.get_device(dev_id)
        host = tr._host_inputs()
        n = len(tr.wavelength)
        steps, warm = (10, 3) if name == "C5" else ((20, 4) if name == "C4x10p64" else (60, 10))
        t_full = time_runs(dev, tr._problem(dev, host, 0, n, 0.0), steps, warm)
        shards = sharding.split(n, parts)
        a, b = max(shards, key=lambda ab: ab[1] - ab[0])
        k_full = dev.transit_kernel_ms(5)
        t_shard = time_runs(dev, tr._problem(dev, host, a, b, 0.0), steps, warm)
        k_shard = dev.transit_kernel_ms(5)
        # the other axis: the largest phase shard (every wavelength): phases are independent as well, and
        # a phase shard does not repeat the per-phase chord work (columns, ordering) that every
        # wavelength shard repeats in full
        n_orb = len(host["orb"])
        pa, pb = max(sharding.split(n_orb, parts, align=1), key=lambda ab: ab[1] - ab[0])
        t_pshard = time_runs(dev, tr._problem(dev, sharding.phase_subset(host, pa, pb), 0, n, 0.0,
                                              sharding.phase_options(host)), steps, warm)
        k_pshard = dev.transit_kernel_ms(5)
        best = "phase" if t_pshard < t_shard else "wavelength"
        t_best = min(t_shard, t_pshard)
        out[name] = {"wavelengths": n, "phases": n_orb, "shards": parts, "ms_full": t_full,
                     "axis": best, "projected_speedup": t_full / t_best,
                     "projected_efficiency": t_full / t_best / parts, "kernel_ms_full": k_full,
                     "wavelength_shard": {"shard": [a, b], "ms_shard": t_shard, "projected_speedup": t_full / t_shard,
                                          "kernel_ms_shard": k_shard},
                     "phase_shard": {"phases": [pa, pb], "ms_shard": t_pshard,
                                     "projected_speedup": t_full / t_pshard, "kernel_ms_shard": k_pshard}}
        del tr
    return out


def strong_leg(name: str, dev_id: int, dist, rank: int, world: int, steps: int, warmup: int, dump_dir=None):
    """Strong scaling on the wavelength axis inside the N-rank process group (BASELINE.json configs[3]:
    the torus exosphere wavelength-sharded across the GPUs; memoryHandler.py:55-66 is the chunker this replaces):
    the configuration's grid in N contiguous 256-aligned wavelength shards, one per rank, barrier + max-over-ranks
    timing as the main leg; then its full grid on rank 0 alone (the others wait at a barrier), the one-GPU time the
    speedup is taken against."""
    from prometheus_amd import _native, configs, setupfile, sharding
    tr = setupfile.build_transit(configs.get(name))
    dev = _native.get_device(dev_id)
    host = tr._host_inputs()
    n = len(tr.wavelength)
    n_orb = len(host["orb"])
    w0, w1 = sharding.shard_for_rank(n, world, rank)
    dev.transit_set(tr._problem(dev, host, w0, w1, 0.0))
    dev.transit_run()
    dev.synchronize()
    for _ in range(warmup):
        dev.transit_run()
    dev.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        dev.transit_run()
    dev.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    elapsed, total_pts = sharding.reduce_timing(dist, t1 - t0, (w1 - w0) * n_orb)
    if dump_dir:
        os.makedirs(dump_dir, exist_ok=True)
        np.save(os.path.join(dump_dir, "R_rank%d.npy" % rank), dev.transit_result())
        with open(os.path.join(dump_dir, "range_rank%d.json" % rank), "w") as fh:
            json.dump({"w0": int(w0), "w1": int(w1), "n_wav": int(n), "o0": 0, "o1": int(n_orb),
                       "n_orb": int(n_orb), "world": world}, fh)
    ms_full = None
    if rank == 0:
        ms_full = time_runs(dev, tr._problem(dev, host, 0, n, 0.0), steps, warmup)
    dist.barrier()
    ms_step = elapsed / steps * 1e3
    out = {"workload": "%s (%s), %d wavelengths x %d phases, %d contiguous wavelength shards (256-aligned), one per "
                       "rank" % (name, describe(configs.get(name)), n, n_orb, world),
           "axis": "wavelength", "value": total_pts * steps / elapsed, "unit": "spectrum points/s",
           "ms_per_step": ms_step, "steps": steps, "warmup": warmup,
           "ms_full_grid_one_gpu": ms_full, "speedup_vs_one_gpu": (ms_full / ms_step) if ms_full else None}
    del tr
    return out


def main():
    args = parse()
    rank, local_rank, world = dist_env()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.shard:
        # before anything touches the GPU: the multi-core leg forks worker processes
        cfgc = global_config(args.config, 1)
        cfgc["_name"] = args.config
        cpu = cpu_baseline(cfgc, args.cpu_sample_wavelengths or CPU_SAMPLE.get(args.config, 4096),
                           args.cpu_workers or cpu_share())
    if args.gpus != world and world > 1:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811  (gloo: barrier + max-reduce of times only)
        dist.init_process_group("gloo")
    from prometheus_amd import _native, setupfile, gasProperties, sharding  # noqa: F401
    # one process per GPU; ranks beyond the visible devices share them round robin (a world-size-2 run on
    # a one-GPU box puts both ranks on device 0)
    dev_id = local_rank % max(1, _native.device_count())
    _native.set_default_device(dev_id)

    scaling = "strong" if args.shard else args.scaling
    cfg = global_config(args.config, world, scaling, args.weak_axis)
    cfg_name = args.config
    if any(sp not in ("NaI", "KI", "CaII", "MgI") for sc in cfg["Species"].values() for sp in sc):
        from prometheus_amd.configs import synthetic_molecular_table
        gasProperties.register_molecular_table("H2O", synthetic_molecular_table())
    t_setup = time.perf_counter()
    tr = setupfile.build_transit(cfg)   # lambda grid + device Voigt tables on this rank's GPU
    dev = _native.get_device(dev_id)
    n_wav_global = len(tr.wavelength)
    host = tr._host_inputs()
    n_orb_global = len(host["orb"])
    if args.shard:
        sr, sn = (int(v) for v in args.shard.split("/"))
        if not (0 <= sr < sn):
            raise SystemExit("--shard r/N needs 0 <= r < N")
    else:
        sr, sn = rank, world
    o0, o1 = 0, n_orb_global
    opts = 0
    args.shard_axis = resolve_axis(args.shard_axis, n_orb_global, sn)
    if scaling == "weak" and world > 1 and not args.shard:
        args.shard_axis = args.weak_axis
    if args.shard_axis == "phase" and (args.shard or scaling == "strong" or (scaling == "weak" and world > 1)):
        w0, w1 = 0, n_wav_global
        o0, o1 = sharding.shard_for_rank(n_orb_global, sn, sr, align=1)
        if o1 <= o0:
            raise SystemExit("phase shard %d/%d is empty (%d phases)" % (sr, sn, n_orb_global))
        opts = sharding.phase_options(host)
        host = sharding.phase_subset(host, o0, o1)
    else:
        w0, w1 = sharding.shard_for_rank(n_wav_global, sn, sr)   # tile-aligned contiguous shards
    prob = tr._problem(dev, host, w0, w1, 0.0, opts)
    dev.transit_set(prob)
    dev.transit_run()   # first launch of every kernel (code-object load) outside the stats run
    dev.synchronize()
    st = dev.transit_run(stats=True)
    setup_s = time.perf_counter() - t_setup
    n_orb = len(host["orb"])
    n_pts_rank = (w1 - w0) * n_orb

    have_torch_gpu = torch.cuda.is_available()

    def sync():
        dev.synchronize()
        if have_torch_gpu:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        dev.transit_run()
    sync()
    if dist:
        dist.barrier()
    sync()
    # the tau kernel's duration is sampled on every TAU_TIMING_STRIDE-th run (events on a dispatch cost
    # the host ~13 us, more than a run's GPU time: timing every run would measure the host)
    dev.timing_begin(stride=TAU_TIMING_STRIDE)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dev.transit_run()
    sync()
    t1 = time.perf_counter()
    ms_runs = dev.timing_end(max_runs=args.steps)
    if args.dump_R:
        os.makedirs(args.dump_R, exist_ok=True)
        np.save(os.path.join(args.dump_R, "R_rank%d.npy" % rank), dev.transit_result())
        with open(os.path.join(args.dump_R, "range_rank%d.json" % rank), "w") as fh:
            json.dump({"w0": int(w0), "w1": int(w1), "n_wav": int(n_wav_global), "o0": int(o0), "o1": int(o1),
                       "n_orb": int(n_orb_global), "world": world}, fh)
    if dist:
        dist.barrier()
    elapsed, total_pts = sharding.reduce_timing(dist, t1 - t0, n_pts_rank)
    ms_step = elapsed / args.steps * 1e3
    value = total_pts * args.steps / elapsed

    # variant // 10: 3 planned tau kernel on sigma rows, 5 / 6 planned with the Doppler sigma fused in (exp10 /
    # polynomial lookups), 7 fused Doppler rows (k_sigma_poly integrates the light windows; k_tau_p takes the
    # heavy half tiles only)
    # 8 transmission curves (prom_tcurve.hip: k_tc_phase, k_tc_table, then k_sigma_tc looks sigma up and
    # evaluates each phase's curve; no tau kernel)
    tv = st.get("tau_kernel_variant", 0) // 10
    fused = tv in (5, 6)
    sig_tau = tv == 7
    tcurve = tv in (8, 9)
    # 9: the same with the Doppler-shifted lookups over target windows (prom_tw.hip: k_sigma_tw)
    sig_name = "k_sigma_tw" if tv == 9 else "k_sigma_tc"
    mol = bool(getattr(prob, "n_molecules", 0))
    tau_kernel = "k_tau_mol" if mol else {2: "k_tau_w", 3: "k_tau_p", 4: "k_tau_rm"}.get(tv, "k_tau")
    # k_tau_p in the pipelined loop: its span on the device clock (first workgroup start -> last workgroup end)
    tau_ms_events = float(np.mean(ms_runs[:, 2])) if len(ms_runs) else st["ms_tau"]
    dev_ms = ms_runs[:, 3][np.isfinite(ms_runs[:, 3])] if len(ms_runs) else np.zeros(0)
    tau_ms_loop = float(np.mean(dev_ms)) if len(dev_ms) else tau_ms_events

    # per-kernel device durations, one run in flight (what rocprofv3 reports at PROM_PIPELINE=1)
    kms = dev.transit_kernel_ms(args.kernel_runs)
    n_atoms = st["tau_kernel_variant"] % 10 or prob.n_atoms
    cle = st["chord_lambda_evals"]
    evals = st["exp_evals"]
    same_shift = all(np.all(np.asarray(e["shift"]) == np.asarray(e["shift"])[0]) for e in host["scenarios"])
    sigma_rows = 1 if same_shift else n_orb
    n_w = w1 - w0
    n_pr = len(host["y"])
    n_x = len(host["x"])
    merged = n_atoms == 1 and prob.n_atoms > 1
    peak_meas, peak_src = measured_read_peak()

    def hbm(nbytes, ms):
        if not ms:
            return None
        a = nbytes / (ms * 1e-3) / 1e9
        return {"bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS,
                "frac_of_measured_read_peak": (a / peak_meas) if peak_meas else None, "algorithmic_bytes": nbytes}

    kernels = {}
    # tau kernel: R written, the resampled cross-section rows read (8 B per species row and wavelength)
    tau_bytes = tau_bytes_per_launch(n_w, n_orb, 0 if fused else n_atoms, sigma_rows) + (8 * n_w if fused else 0)
    flops_unit = flops_per_eval(n_atoms) + (6 * n_x if mol else 0)
    tau_ms_iso = kms.get("tau")
    if tcurve:
        pass
    elif sig_tau:
        # heavy half tiles only (line cores: windows of > 8 records, spread over the chip); their share of R and
        # of the exponentials is not counted on the host, so no byte roofline
        kernels[tau_kernel] = {"bound": "latency", "ms": tau_ms_iso, "role": "heavy half tiles of the fused rows"}
    else:
        kernels[tau_kernel] = dict(hbm(tau_bytes, tau_ms_iso) or {}, ms=tau_ms_iso, ms_pipelined_loop=tau_ms_loop,
                                   exp_evals=evals, exp_per_s=(evals / (tau_ms_iso * 1e-3)) if tau_ms_iso else None,
                                   valu_tflops=(evals * flops_unit / (tau_ms_iso * 1e-3) / 1e12) if tau_ms_iso else None)
    if mol:
        # SURVEY.md 8d rule (ii): per chord-wavelength n_x table lookups (P-lerp + 10^v + FMA) against the
        # measured table-exp rate (profiles/r02u_fp64_exp_peak.json: 2.8e12/s)
        # (the device counts them in stats runs: exp_evals = the 10^v of in-table samples + one e^-tau per
        # record and wavelength; out-of-table samples are skipped, k_mol_prep compacts them away; a mirror-merged
        # chord pair's samples are listed and counted once -- pow10 is the evaluations performed)
        # achieved / peak / frac in one unit (10^v per second); the byte figures move under "hbm"
        pow10 = max(0, int(st["exp_evals"]) - int(st["tau_records"]) * n_w)
        km = kernels[tau_kernel]
        km.pop("valu_tflops", None)   # (flops_unit counts all n_x samples; only the in-table ones are evaluated)
        km["hbm"] = {k: km.pop(k) for k in ("achieved", "peak", "unit", "frac", "frac_of_measured_read_peak",
                                             "algorithmic_bytes") if k in km}
        rate = pow10 / (tau_ms_iso * 1e-3) if tau_ms_iso else None
        km.update(bound="fp64-exp", pow10_evals=pow10, achieved=rate, peak=2.815e12, unit="pow10/s",
                  frac=(rate / 2.815e12) if rate else None, peak_source="profiles/r02u_fp64_exp_peak.json")
    if kms.get("sigma_tc"):
        kms["sigma"] = kms["sigma_tc"]   # (k_sigma_tc reads the tables as the row kernels do)
    if kms.get("tc_build"):
        kms["order"] = kms["tc_build"]
    if kms.get("sigma"):
        # Doppler sigma rows: one row per phase and wavelength (Y for merged species, else sigma per species)
        # and their zero flags written, the wavelengths and the refined tables' nodes (x, log10 sigma) read
        out_rows = 1 if merged else prob.n_atoms
        nodes = table_nodes_in_range(tr, host, w0, w1)
        lookups = sigma_rows * n_w * prob.n_atoms
        if tcurve:
            # transmission curves: R written (every point), the wavelengths and the table nodes read; the
            # per-phase curve tables (kTcD coefficients per octave) are L2-resident and not counted
            sig_bytes = 8 * n_orb * n_w + 8 * n_w + 16 * nodes
            kernels[sig_name] = dict(hbm(sig_bytes, kms["sigma"]), ms=kms["sigma"], lookups=lookups,
                                         table_nodes=nodes, lookups_per_s=lookups / (kms["sigma"] * 1e-3))
        elif sig_tau:
            # fused rows: R written (every point but the heavy half tiles' -- counted whole), the wavelengths and
            # the table nodes read; no Y rows or zero flags
            sig_bytes = 8 * n_orb * n_w + 8 * n_w + 16 * nodes
            kernels["k_sigma_tau"] = dict(hbm(sig_bytes, kms["sigma"]), ms=kms["sigma"], lookups=lookups,
                                          table_nodes=nodes, lookups_per_s=lookups / (kms["sigma"] * 1e-3),
                                          exp_evals_both_kernels=evals)
        else:
            sig_bytes = 8 * sigma_rows * out_rows * n_w + (sigma_rows * n_w if merged else 0) + 8 * n_w + 16 * nodes
            kernels["k_sigma"] = dict(hbm(sig_bytes, kms["sigma"]), ms=kms["sigma"], lookups=lookups, table_nodes=nodes,
                                      lookups_per_s=lookups / (kms["sigma"] * 1e-3))
    if kms.get("columns"):
        dens = n_orb * n_pr * n_x * len(host["scenarios"])
        col_bytes = 8 * n_orb * n_pr * prob.n_atoms + 4 * n_orb * n_pr + 8 * (3 * n_pr + n_x)
        kernels["k_columns"] = dict(hbm(col_bytes, kms["columns"]), bound="latency", ms=kms["columns"],
                                    density_evals=dens, density_evals_per_s=dens / (kms["columns"] * 1e-3))
    order_name = "k_tc_build" if tcurve else ("k_order" if tv in (2, 3) else "k_chords")
    for k, name in (("order", order_name), ("windows", "k_windows")):
        if kms.get(k):
            kernels[name] = {"bound": "latency", "ms": kms[k],
                             "workgroups": n_orb if (k == "order" and not tcurve) else None}
    if tcurve and kms.get("order"):
        # every active chord at 16 Chebyshev nodes of each table octave (one table exp per four octaves)
        kernels["k_tc_build"].update(node_evals=evals, node_evals_per_s=evals / (kms["order"] * 1e-3))
    # path level: what any implementation must move -- R written, wavelengths and table nodes read -- over
    # the measured step
    path_bytes = 8 * n_orb * n_w + 8 * n_w + (16 * table_nodes_in_range(tr, host, w0, w1) if prob.n_atoms else 0)
    path = hbm(path_bytes, ms_step)
    # the dominant kernel of the step (longest device duration) carries the top-level roofline
    # (latency-bound kernels -- one workgroup per phase -- are listed beside it, never the roofline's)
    cand = [k for k in kernels if kernels[k].get("bound") != "latency"] or list(kernels)
    dom = max(cand, key=lambda k: kernels[k].get("ms") or 0.0)
    dk = kernels[dom]
    # rocprofv3 kernel names: the fused rows are k_sigma_poly<..., true>, the row kernels k_sigma_poly<..., false>
    # (or k_sigma_rows)
    sym, suffix = {"k_sigma_tau": ("prom::k_sigma_poly", ", true>"), "k_sigma": ("prom::k_sigma", ""),
                   "k_sigma_tc": ("prom::k_sigma_tc", ""), "k_sigma_tw": ("prom::k_sigma_tw", "")}.get(dom, ("prom::" + dom, ""))
    traffic = latest_profile_traffic(sym, cfg_name, suffix)
    # latency of one run alone on an idle device (host clock: submit, kernels, synchronize; no stats
    # instrumentation), median of 20 -- what one retrieval sample waits for with inputs resident; not `value`
    dev.transit_set(prob)
    dev.transit_run()
    dev.synchronize()
    lat = []
    for _ in range(20):
        t_l = time.perf_counter()
        dev.transit_run()
        dev.synchronize()
        lat.append(time.perf_counter() - t_l)
    single_run_ms = float(np.median(lat)) * 1e3
    # end-to-end (host prep + H2D + run + D2H) for reference: median of 7 sumOverChords calls after one
    # warm-up call (first-call costs: pinned pool, host threads, page faults)
    R, e2e_s = None, None
    if world == 1 and not args.shard:
        R = tr.sumOverChords(devices=[dev_id])
        calls = []
        for _ in range(7):
            del R
            t_e2e = time.perf_counter()
            R = tr.sumOverChords(devices=[dev_id])
            calls.append(time.perf_counter() - t_e2e)
        e2e_s = float(np.median(calls))
    proj = None
    if world == 1 and not args.shard and not args.no_projection:
        del tr
        proj = strong_projection(dev_id)
    workload = "%s (%s), %d wavelengths x %d phases x %d chords x %d samples" % (
        cfg_name, describe(cfg), n_wav_global, n_orb, n_pr, n_x)
    if args.shard:
        workload += (", shard %s: phases [%d, %d)" % (args.shard, o0, o1) if args.shard_axis == "phase"
                     else ", shard %s: wavelengths [%d, %d)" % (args.shard, w0, w1))
    elif world > 1:
        workload += ", %s scaling over %ss: %d global phases x %d global wavelengths, rank 0 %s" % (
            scaling, args.shard_axis, n_orb_global, n_wav_global,
            "phases [%d, %d)" % (o0, o1) if args.shard_axis == "phase" else "wavelengths [%d, %d)" % (w0, w1))
    result = {
        "metric": "spectrum points/sec (phase x wavelength)",
        "value": value,
        "unit": "spectrum points/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (WASP-49b catalogue system, NIST line list bundled from the reference)",
        "config": {"workload": workload,
                   "global_wavelengths": n_wav_global, "orbital_phases": n_orb,
                   "chords_per_phase": n_pr, "los_samples": n_x,
                   "parallelism": "%s shards x%d (no collective)" % (
                       "phase" if (args.shard_axis == "phase" and (args.shard or world > 1)) else "wavelength",
                       world)},
        "roofline": {"bound": dk.get("bound", "hbm"), "kernel": dom, "achieved": dk.get("achieved"),
                     "peak": dk.get("peak", HBM_PEAK_GBS), "unit": dk.get("unit", "GB/s"), "frac": dk.get("frac"),
                     "traffic": traffic, "algorithmic_bytes": dk.get("algorithmic_bytes"),
                     "kernel_ms": dk.get("ms"), "kernel_ms_source": "prom_transit_kernel_ms: one run in flight, "
                     "dispatch-packet events, mean of %d runs" % args.kernel_runs,
                     "measured_read_peak_gbs": peak_meas, "measured_read_peak_source": peak_src,
                     "sigma_rows": sigma_rows,
                     "kernels": kernels, "path": dict(path or {}, ms_per_step=ms_step),
                     "tau_ms_pipelined_loop": tau_ms_loop, "tau_ms_hip_events": tau_ms_events,
                     "chord_lambda_evals": cle, "fused_sigma": fused},
        "stage_ms_single_run": {"columns_order": st["ms_density"], "tau": st["ms_tau"], "total": st["ms_total"],
                                "note": "the first run, instrumented (evaluation counters on: C5's per-sample "
                                        "counters dominate); single_run_ms is the uninstrumented latency"},
        "single_run_ms": single_run_ms,
        "chords": {"active": st["active_chords"], "transparent": st["transparent_chords"],
                   "blocked": st["blocked_chords"], "integrated_records": st["tau_records"]},
        "setup_s": setup_s,
        "end_to_end_s": e2e_s,
        "end_to_end_points_per_s": (n_wav_global * n_orb / e2e_s) if e2e_s else None,
    }
    if proj is not None:
        result["strong_scaling_projection"] = proj
    if dist and args.strong and not args.shard:
        # (after the main leg; its problem is released first)
        del prob
        strong = {}
        for name in [c for c in args.strong.split(",") if c]:
            strong[name] = strong_leg(name, dev_id, dist, rank, world, args.steps, args.warmup,
                                      os.path.join(args.dump_R, "strong_" + name) if args.dump_R else None)
        result["strong"] = strong
    if cpu is not None:
        result["cpu_baseline"] = cpu
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result))


if __name__ == "__main__":
    main()
