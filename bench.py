#!/usr/bin/env python
"""bench.py -- MSM-scored ions/sec of the molecule-annotation hot path on MI355X (BASELINE.json metric).

One step = the metric's timed region (BASELINE.md:38): ``compute_sf_images(sc, ds, sf_peak_df,
ppm)`` + ``sf_image_metrics(sf_images, sc, formulas, ds, ds_config)`` through the drop-in API, result DataFrame
included -- duplicate flags, global m/z sort and prefix sums of the resident peaks, the ion layout of
sf_peak_df, the window search, the fused imaging + MSM scoring of every ion and the [sf_id, adduct] table.
``value`` = rows of that table (scored ions) / step time.  Workload = config 3 of BASELINE.json: 500x500-px
synthetic dataset, Poisson(2000) centroids per spectrum (~5e8 points, generated in HBM: the timed region
starts with the data resident), 20,000 synthetic formulas x (+H, +Na, +K targets + distinct decoys, 20 decoy
draws per target as fdr.py does) ~ 0.98M ions, ppm 2, nlevels 30.

N > 1 (torch.distributed.run, one rank per GPU, RCCL): STRONG scaling of the same config-3 workload.  The
formula table is sharded once by principal m/z with a cost model (distributed.plan_shards); per step every
rank selects the m/z slice its windows touch from the replicated resident dataset, runs the same two API
calls on its shard, and the metric rows are gathered to rank 0 (one RCCL gather over xGMI), which builds the
full table.  ``value`` = rows of rank 0's table / the max-over-ranks step time.

Beside ``value``: ``device_chain`` (the same kernels without the host API layer), per-stage HIP-event times,
``roofline`` of the dominant kernel (ion_pipe_kernel<512>: 12 B per window point per launch, SURVEY §8d, over
its own HIP-event time on its launch stream), and ``cpu_baseline`` (the oracle on host cores, rank 0, N = 1).

Run:  python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MSM-scored ions/sec (HMDB×3 adducts, 250k-px synth) + imaging-kernel HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
ALG_BYTES_PER_POINT = 12.0  # one (mz f32, int f32, pixel u32) read per point per window


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-sf", type=int, default=20000)
    ap.add_argument("--nrows", type=int, default=500)
    ap.add_argument("--ncols", type=int, default=500)
    ap.add_argument("--peaks", type=float, default=2000.0)
    ap.add_argument("--ppm", type=float, default=2.0)
    ap.add_argument("--nlevels", type=int, default=30)
    ap.add_argument("--plant-fraction", type=float, default=0.02)
    ap.add_argument("--chain-steps", type=int, default=5, help="timed steps of the device-chain leg (0: skip)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU (sharded, RCCL) step even at N = 1 (a check of that path on one GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target wall of the CPU baseline sample")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="cap on CPU-baseline workers (a GPU box's CPU share is 16 cores per GPU)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    # the JSON line is the only thing on stdout: libraries that print at start-up (RCCL's version banner at
    # communicator creation) write to fd 1 directly, so fd 1 points at stderr until the line is printed
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    from sm_distributed_amd import _lib
    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    from sm_distributed_amd import synthetic as syn
    from sm_distributed_amd.dataset import ResidentDataset
    from sm_distributed_amd.formula_imager_segm import compute_sf_images
    from sm_distributed_amd.formula_img_validator import sf_image_metrics
    from sm_distributed_amd.formulas import FormulasSegm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    sharded = world > 1 or args.sharded
    if sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", device_id=device, rank=rank, world_size=world)

    t_setup = time.perf_counter()
    ions = syn.make_ion_table(args.n_sf, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(args.nrows, args.ncols, args.peaks, seed=42, device=device,
                                                  ions=ions, plant_fraction=args.plant_fraction, plant_seed=45)
    peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    formulas = FormulasSegm.from_ion_table(ions, args.ppm)
    ds_config = {"image_generation": {"ppm": args.ppm, "nlevels": args.nlevels, "q": 99, "do_preprocessing": False}}
    if sharded:
        plan = D.plan_shards(formulas, peaks, args.ppm, world, rank)
        step_fn = lambda: D.score_sharded(plan, peaks, ds_config)[0]
        my_formulas = plan.formulas
    else:
        plan = None
        dds = ResidentDataset(peaks)
        sf_peak_df = formulas.get_sf_peak_df()  # built by MSMBasicSearch.search before the timed region

        def step_fn():
            ims = compute_sf_images(None, dds, sf_peak_df, args.ppm)
            return sf_image_metrics(ims, None, formulas, dds, ds_config)
        my_formulas = formulas
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s: {info['n_points']:,} points, "
        f"{formulas.n_ions:,} ions ({my_formulas.n_ions:,} on this rank), planted {info['n_planted_ions']} ions")

    # ---- the metric: timed API steps --------------------------------------------------------------------
    L = _lib.lib()
    for _ in range(max(args.warmup, 1)):
        df = step_fn()
    torch.cuda.synchronize()
    L.smg_debug_main_pass_times(None, 0, ctypes.byref(ctypes.c_int32(0)))  # discard
    L.smg_debug_time_main_pass(1)
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    for _ in range(args.steps):
        df = step_fn()  # ends with the table on the host (a synchronisation)
        marks.append(time.perf_counter())
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    L.smg_debug_time_main_pass(0)
    main_ms = _main_pass_times(L)
    n_rows = len(df) if df is not None else 0
    if sharded:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / max(args.steps, 1) * 1e3
    per_step = np.diff([t0] + marks) * 1e3
    if len(per_step):
        log(f"[rank {rank}] step ms: min {per_step.min():.2f} median {np.median(per_step):.2f} "
            f"max {per_step.max():.2f}")

    # ---- device chain (the same kernels without the API layer) and per-stage HIP events ----------------------
    chain = device_chain(args, peaks, my_formulas, plan) if args.chain_steps > 0 else None

    # ---- roofline of the dominant kernel: 12 B per window point over its own launch time --------------------
    sum_hits = chain["sum_window_points"] if chain else None
    kern_ms = float(np.mean(main_ms)) if len(main_ms) else None
    roofline = None
    if sum_hits and kern_ms:
        ach = ALG_BYTES_PER_POINT * sum_hits / (kern_ms * 1e-3) / 1e9
        is_c3 = _is_config3(args) and world == 1
        traffic, src = measured_traffic() if is_c3 else (None, None)
        roofline = {"bound": "hbm", "kernel": "ion_pipe_kernel<512> (main LDS pass)", "achieved": ach,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                    "traffic_source": src, "alg_bytes_per_launch": ALG_BYTES_PER_POINT * sum_hits,
                    "kernel_ms_avg": kern_ms, "kernel_launches_timed": len(main_ms),
                    "alg_bytes_8B_per_point_frac": 8.0 * sum_hits / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, ions, peaks, dims)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": n_rows / (ms_per_step * 1e-3),
            "unit": "ions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (generated in HBM; HMDB/ChEBI and real imzML are not available offline)",
            "config": {
                "workload": (f"{'config3' if _is_config3(args) else 'custom'}: {args.nrows}x{args.ncols} px, "
                             f"Poisson({args.peaks:g}) centroids/spectrum, {args.n_sf} formulas x (+H,+Na,+K + "
                             f"distinct decoys), ppm {args.ppm:g}, nlevels {args.nlevels}"),
                "timed_region": "compute_sf_images + sf_image_metrics through the drop-in API, DataFrame included",
                "n_points": info["n_points"], "n_ions": formulas.n_ions, "n_rows_per_step": n_rows,
                "n_windows": int(formulas.ion_off[-1]), "sum_window_points": sum_hits,
                "parallelism": (f"formula shards by principal m/z x{world}, dataset replicated, per-rank m/z slice, "
                                f"RCCL gather of metric rows" if sharded else "1 GPU"),
                "shard_est_cost_s": plan.est_cost if plan is not None else None,
            },
            "device_chain": chain,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "lib": _lib.version(),
        }
        print(json.dumps(line), file=json_out, flush=True)
    if sharded:
        dist.destroy_process_group()


def _is_config3(args):
    return (args.nrows, args.ncols, args.peaks, args.n_sf, args.ppm, args.nlevels, args.plant_fraction) == \
        (500, 500, 2000.0, 20000, 2.0, 30, 0.02)


def _main_pass_times(L):
    n = ctypes.c_int32(0)
    buf = (ctypes.c_double * 4096)()
    _lib_check(L.smg_debug_main_pass_times(buf, 4096, ctypes.byref(n)))
    return [buf[i] for i in range(min(n.value, 4096))]


def _lib_check(rc):
    from sm_distributed_amd._lib import check
    check(rc, "smg diagnostics")


def device_chain(args, peaks, formulas, plan):
    """The kernels of one step without the host API layer (ion table pre-staged on the device), with
    per-stage HIP events on the launch stream: flag+sort+scan, window search, ion metrics."""
    import torch

    from sm_distributed_amd import distributed as D
    from sm_distributed_amd import engine as E
    pk = peaks if plan is None else D.slice_peaks(peaks, plan)
    dions = E.DeviceIons.from_arrays(formulas.ion_off, formulas.peak_mz, formulas.peak_int, device=peaks.device)
    n = dions.n_ions
    f64 = lambda: torch.empty(n, dtype=torch.float64, device=peaks.device)
    out = E.IonMetrics(f64(), f64(), f64(), f64(), torch.empty(n, dtype=torch.int32, device=peaks.device))
    events = []

    def step(timed):
        p = pk if plan is None else D.slice_peaks(peaks, plan)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        if ev:
            ev[0].record()
        p.flag_duplicates(args.ppm)
        p.sort()
        p.prefix_sums()
        if ev:
            ev[1].record()
        lo, hi = E.window_bounds(p, dions, args.ppm)
        if ev:
            ev[2].record()
        E.ion_metrics(p, dions, lo, hi, nlevels=args.nlevels, out=out)
        if ev:
            ev[3].record()
            events.append(ev)
        return lo, hi

    for _ in range(2):
        lo, hi = step(False)
    torch.cuda.synchronize()
    sum_hits = int((hi - lo).sum().item())
    n_scored = int(((out.flags & 1) != 0).sum().item())
    t0 = time.perf_counter()
    for _ in range(args.chain_steps):
        step(True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.chain_steps * 1e3
    names = ["flag+sort+scan", "window_search", "ion_metrics"]
    stages = {nm: float(np.mean([e[j].elapsed_time(e[j + 1]) for e in events])) for j, nm in enumerate(names)}
    return {"ms_per_step": ms, "ions_per_s": n_scored / (ms * 1e-3), "n_scored": n_scored, "stages_ms": stages,
            "sum_window_points": sum_hits, "n_points": pk.n_points}


def measured_traffic():
    """HBM bytes per launch of the main ion kernel from the newest committed PMC summary (profiles/*/traffic_*.json,
    scripts/gpu_traffic.sh: FETCH_SIZE calibrated for the kernel's access width, + WRITE_SIZE).  The counters
    cannot be read from inside this process; None when no summary exists."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic_*.json")))
    best = None
    for f in files:  # profiles/round<N>/..., newest round last; only summaries of the main ion kernel
        d = json.load(open(f))
        if d.get("kernel") == "ion_pipe_kernel[512]":
            best = (float(d["traffic_bytes_per_launch"]), os.path.relpath(f, ROOT))
    return best if best else (None, None)


def cpu_baseline(args, ions, peaks, dims):
    """The oracle (reference algorithm restated in numpy/scipy, oracle/cpu_baseline.py) on every host core this
    process may use, over a seeded sample of ions drawn uniformly from the whole ion table (so over the whole
    m/z range); each worker sorts the sample's window points by m/z, then images and scores its ions."""
    from oracle import cpu_baseline as CB
    from oracle import msm_oracle as O
    workers = CB.default_workers(cap=args.cpu_workers)
    # ~11 ions/s per worker (r01/r2a measurements): size the sample to about --cpu-seconds of wall
    n_pick = int(min(4096, max(64, workers * 11 * args.cpu_seconds)))
    rng = np.random.default_rng(7)
    pick = np.sort(rng.choice(ions.n_ions, size=min(n_pick, ions.n_ions), replace=False))
    wins = np.concatenate([np.arange(ions.win_off[i], ions.win_off[i + 1]) for i in pick])
    lower, upper = O.window_bounds(ions.peak_mz[wins], args.ppm)
    b_pix, b_mz, b_int = CB.select_window_points(peaks.mz, peaks.hits, lower, upper)
    tasks = [(int(i), ions.peak_mz[ions.win_off[i]:ions.win_off[i + 1]].copy(),
              ions.peak_int[ions.win_off[i]:ions.win_off[i + 1]].copy()) for i in pick]
    rows, wall, per = CB.run_pool_split(b_pix, b_mz, b_int, dims, args.ppm, args.nlevels, tasks, workers)
    return {"value": len(rows) / wall, "unit": "ions/s", "cores": workers, "kind": "port",
            "sample": (f"{len(pick)} ions drawn uniformly from the {ions.n_ions:,}-ion table ({len(rows)} scored), "
                       f"the {b_mz.size:,} data points of their windows; {workers} worker processes (the box's CPU share; "
                       f"Spark local[*]-style), each sorts its ions' window points by m/z and images + scores them "
                       f"(oracle/cpu_baseline.py); wall {wall:.1f}s"),
            "nproc": os.cpu_count(), "cpus_available": CB.available_cpus(), "cpu_model": CB.cpu_model()}


if __name__ == "__main__":
    main()
