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

``python bench.py --gpus N`` without a launcher (WORLD_SIZE unset) starts the N ranks itself: the parent touches
no GPU, spawns N child processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT, relays
rank 0's JSON line and exits non-zero if any rank fails (``--dry-run`` stops every rank before GPU init).

Run:  python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# KFD queue evictions of this process (each stops every running kernel for >= one 10-ms tick) are counted per step
# (sm_distributed_amd/hostmem.py); SMG_NUMA_OPTOUT=1 takes the process out of NUMA-balancing scans, one trigger of
# them.  A thread inherits the policy when it is created, so this runs before numpy (its BLAS pool) and torch start
# any thread: hostmem imports only the standard library (the package's __init__ imports nothing else)
from sm_distributed_amd import hostmem  # noqa: E402

NUMA_OPTOUT = hostmem.numa_balancing_optout() if os.environ.get("SMG_NUMA_OPTOUT") == "1" else False

import numpy as np  # noqa: E402

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
    ap.add_argument("--no-rebalance", action="store_true",
                    help="N > 1: keep the cost model's cut (default: re-cut once from every rank's measured time)")
    ap.add_argument("--rebalance-rounds", type=int, default=3,
                    help="N > 1: at most this many re-cuts, until the ranks' measured times agree within 3 %%")
    ap.add_argument("--no-head-cut", action="store_true",
                    help="N > 1: re-cut without rank 0's assembly time (default: rank 0's shard is cut smaller by "
                         "it, since the other ranks start the next search while rank 0 assembles the table)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target wall of the CPU baseline sample")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="cap on CPU-baseline workers (a GPU box's CPU share is 16 cores per GPU)")
    ap.add_argument("--config", choices=["3", "5"], default="3",
                    help="workload preset: 3 = BASELINE config 3 (default); 5 = one rank's shard of config 5 "
                         "(1000x1000 px, Poisson(5000), 40k formulas x 6 adducts both polarities; use --shard-of)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="score only this rank's shard of an N-way plan on one GPU (N = --shard-of, rank = "
                         "--shard-rank): one rank of a multi-GPU run measured alone")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--dry-run", action="store_true", help="stop every rank before GPU initialisation")
    ap.add_argument("--legacy-main", action="store_true",
                    help="A/B: the main pass on ion_pipe_kernel<512> instead of ion_sparse_kernel (smg_debug_main_kernel(0))")
    args = ap.parse_args()
    if args.config == "5":
        for k, v in CONFIG5.items():
            if getattr(args, k) == ap.get_default(k):
                setattr(args, k, v)
    return args


# BASELINE config 5 (stress): 1000x1000 px, ~5k peaks per spectrum, HMDB+ChEBI-sized table (~40k formulas), 6
# adducts in both polarities (positive +H/+Na/+K, negative -H/+Cl/+Br), decoys as fdr.py draws them
CONFIG5 = {"nrows": 1000, "ncols": 1000, "peaks": 5000.0, "n_sf": 40000}
CONFIG5_ADDUCTS = {"+": ("+H", "+Na", "+K"), "-": ("-H", "+Cl", "+Br")}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args):
    """Start the N ranks of ``--gpus N`` (no launcher in front of this process): one child per GPU with the
    torch.distributed.run environment; rank 0's stdout (the JSON line) is relayed, the others' go to stderr.
    This process never initialises a GPU (no torch import), so it may start the children as it likes."""
    n = args.gpus
    port = _free_port()
    argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    out0 = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0")
        procs.append(subprocess.Popen(argv, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    log(f"[launcher] started {n} ranks: pids {[p.pid for p in procs]} (MASTER_PORT {port})")
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.remove(r)
            if code != 0 and rc == 0:
                rc = code
                log(f"[launcher] rank {r} exited with {code}: stopping the other ranks")
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    reader.join(timeout=30)
    data = out0[0].decode() if out0 and out0[0] else ""
    if data:
        sys.stdout.write(data)
        sys.stdout.flush()
    if rc == 0 and not data.strip():
        log("[launcher] rank 0 printed no result line")
        rc = 1
    return 1 if rc < 0 else rc


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: one rank per GPU")
    if args.dry_run:
        log(f"[rank {rank}/{world}] dry run: local rank {local_rank}, master "
            f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}")
        if os.environ.get("SMG_BENCH_FAIL_RANK") == str(rank):  # launcher test: a rank that fails
            raise SystemExit(3)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "rank": rank, "local_rank": local_rank}), flush=True)
        return
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

    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    sharded = world > 1 or args.sharded
    rccl_world = None
    if sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", device_id=device, rank=rank, world_size=world)
        rccl_world = dist.get_world_size()
        if rccl_world != world:
            raise SystemExit(f"RCCL reports {rccl_world} ranks, expected {world}")

    t_setup = time.perf_counter()
    if args.config == "5":
        ions = syn.make_ion_table_both_polarities(args.n_sf, seed=43, decoy_seed=44)
    else:
        ions = syn.make_ion_table(args.n_sf, seed=43, decoy_seed=44)
    mz, hits, dims, info = syn.make_dataset_torch(args.nrows, args.ncols, args.peaks, seed=42, device=device,
                                                  ions=ions, plant_fraction=args.plant_fraction, plant_seed=45)
    peaks = E.DevicePeaks.from_device(mz, hits, dims, sp_off=info["sp_off"])
    formulas = FormulasSegm.from_ion_table(ions, args.ppm)
    ds_config = {"image_generation": {"ppm": args.ppm, "nlevels": args.nlevels, "q": 99, "do_preprocessing": False}}
    shard_only = args.shard_of > 1 and not sharded
    phases = None
    if sharded:
        plan = D.plan_shards(formulas, peaks, args.ppm, world, rank)
        if not args.no_rebalance:
            # the cut re-made from every rank's measured shard time (one all_gather of 2 floats per rank): the cost
            # model's per-rank residuals would otherwise set the slowest rank's time.  Re-cut until the ranks (rank
            # 0 with its assembly) agree within 3 %, at most --rebalance-rounds times
            for it in range(args.rebalance_rounds):
                t_rank = _rank_seconds(D, plan, peaks, ds_config)
                t_head = 0.0 if args.no_head_cut else _assembly_seconds(D, plan, peaks, ds_config)
                tt = torch.tensor([t_rank, t_head], dtype=torch.float64, device=device)
                ts = [torch.zeros_like(tt) for _ in range(world)]
                dist.all_gather(ts, tt)
                times = [float(x[0].item()) for x in ts]
                head = float(ts[0][1].item())  # rank 0's
                loads = [times[0] + head] + times[1:]
                spread = max(loads) / min(loads) - 1.0
                if spread <= 0.03:
                    log(f"[rank {rank}] shard times (ms) {[round(x * 1e3, 2) for x in times]}, rank-0 assembly "
                        f"{head * 1e3:.2f} ms: within {spread * 100:.1f} %, cut kept after {it} re-cuts")
                    break
                plan = D.rebalance(plan, formulas, peaks, times, head_seconds=head)
                log(f"[rank {rank}] re-cut {it + 1} from measured shard times (ms) {[round(x * 1e3, 2) for x in times]}"
                    f" (spread {spread * 100:.1f} %), rank-0 assembly {head * 1e3:.2f} ms: counts {plan.counts}")
        # per step: timing events of this rank's rows, gather (its wait for the slowest rank included) and assembly,
        # recorded by score_sharded itself on the stream (no synchronisation added), read after the timed steps
        phases = []

        def step_fn():
            return D.score_sharded(plan, peaks, ds_config, phases=phases)[0]
        my_formulas = plan.formulas
    elif shard_only:
        # one rank of an N-way plan measured alone on this GPU: its slice, images, scores and row block (the
        # step every rank runs before the gather); rows = the ions of the shard that get a table row
        if not 0 <= args.shard_rank < args.shard_of:
            raise SystemExit("--shard-rank must be in [0, --shard-of)")
        plan = D.plan_shards(formulas, peaks, args.ppm, args.shard_of, args.shard_rank)

        def step_fn():
            rows, _ = D._device_rows(plan, peaks, ds_config)
            return int((rows[:, 0] >= 0).sum().item())
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
    if args.legacy_main:
        _lib_check(L.smg_debug_main_kernel(0))
    # the pass timers (HIP events around every pass launch) are on from the warm-up: their first event creations,
    # which may reach the device while a persistent pass runs, fall in the warm-up
    timers = not os.environ.get("SMG_BENCH_NO_TIMERS")  # (A/B: the timed steps without pass timers)
    L.smg_debug_time_main_pass(1 if timers else 0)
    t_first = time.perf_counter()
    df = step_fn()  # the process's first search: library load, workspaces, host caches all cold
    first_step_ms = (time.perf_counter() - t_first) * 1e3
    for _ in range(max(args.warmup, 1) - 1):
        df = step_fn()
    torch.cuda.synchronize()
    _pass_times(L)  # discard
    if sharded:
        dist.barrier()
    if os.environ.get("SMG_BENCH_GC_FREEZE"):  # A/B: collector pauses over the setup's objects
        import gc
        gc.collect()
        gc.freeze()
    clock = ClockSampler(torch.cuda.get_device_properties(device))
    evict = hostmem.EvictionCounter(hostmem.kfd_gpu_id(torch.cuda.get_device_properties(device).pci_bus_id))
    ev_marks = [evict.read()]
    clock.start()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks = []
    verbose = bool(os.environ.get("SMG_BENCH_VERBOSE"))
    host_allocs = []
    for _ in range(args.steps):
        df = step_fn()  # ends with the table on the host (a synchronisation)
        marks.append(time.perf_counter())
        ev_marks.append(evict.read())
        if verbose:  # pinned host allocations so far (diagnostic: step-time outliers)
            host_allocs.append(torch.cuda.host_memory_stats().get("num_host_alloc", -1))
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    sclk = clock.stop()
    L.smg_debug_time_main_pass(0)
    pass_ms = _pass_times(L)
    n_rows = df if isinstance(df, int) else (len(df) if df is not None else 0)
    if sharded:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / max(args.steps, 1) * 1e3
    per_step = np.diff([t0] + marks) * 1e3
    # each step's shader clock: the lowest sample the 20-ms sampler took inside the step (so that an outlier step
    # carries its own clock)
    step_clk = [clock.over(a, b) for a, b in zip([t0] + marks[:-1], marks)]
    if len(per_step):
        log(f"[rank {rank}] step ms: min {per_step.min():.2f} median {np.median(per_step):.2f} "
            f"max {per_step.max():.2f}; shader clock MHz {sclk}")
    # every rank's step min / median / max and clock, gathered for the line (one all_gather of 5 floats)
    mine = [float(per_step.min()), float(np.median(per_step)), float(per_step.max())] if len(per_step) else [0.0] * 3
    mine += [float(sclk["median"]) if sclk else -1.0, float(sclk["min"]) if sclk else -1.0]
    timed_phases = (np.asarray([D.phase_ms(e) for e in phases[-len(per_step):]]) if phases and len(per_step)
                    else np.zeros((0, 3)))
    mine += [float(x) for x in np.median(timed_phases, axis=0)] if len(timed_phases) else [-1.0] * 3
    per_rank = [mine]
    if sharded:
        tt = torch.tensor(mine, dtype=torch.float64, device=device)
        ts = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(ts, tt)
        per_rank = [[float(x) for x in t.tolist()] for t in ts]
    # each timed step's device passes (HIP events around every launch): the descriptor pass and the main pass, so
    # that a slow step shows whether the device or the host took the extra time
    step_desc = [round(t, 3) for p_, t in pass_ms if p_ == _lib.SMG_PASS_DESC]
    step_main = [round(t, 3) for p_, t in pass_ms if p_ == _lib.SMG_PASS_MAIN]
    if os.environ.get("SMG_BENCH_VERBOSE"):
        log(f"[rank {rank}] steps: " + " ".join(f"{x:.1f}" for x in per_step))
        log(f"[rank {rank}] pass launches (pass:ms): " + " ".join(f"{p}:{t:.2f}" for p, t in pass_ms))
        log(f"[rank {rank}] pinned host allocations after each step: {host_allocs}")
        log(f"[rank {rank}] host allocator stats: {dict(torch.cuda.host_memory_stats())}")
    # one more search with the host-side caches dropped (the theoretical-intensity alignment and the shard's
    # global row index are reused between steps while the ion keys are unchanged): a cold first search of a
    # new formula table in a warm process
    cold_ms = cold_step_ms(step_fn, formulas, plan, sharded)

    # ---- device chain (the same kernels without the API layer) and per-stage HIP events ----------------------
    chain = device_chain(args, peaks, my_formulas, plan) if args.chain_steps > 0 else None

    # ---- roofline per pass: 12 B per window point of the ions the pass scored over its own launch time --------
    # PMC traffic summaries exist for the config-3 single-GPU step and rank 0's shard of the 8-way config-5 plan
    traffic_ok = world == 1 and ((args.config == "3" and _is_config3(args) and not shard_only) or
                                 (args.config == "5" and shard_only and args.shard_of == 8 and args.shard_rank == 0))
    roofline, passes = pass_roofline(args, pass_ms, chain, traffic_ok)

    cpu = None
    if rank == 0 and world == 1 and not shard_only and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, ions, peaks, dims)

    if rank == 0:
        if args.config == "5":
            wl = (f"config5{' shard %d/%d' % (args.shard_rank, args.shard_of) if shard_only else ''}: "
                  f"{args.nrows}x{args.ncols} px, Poisson({args.peaks:g}) centroids/spectrum, {args.n_sf} formulas x "
                  f"(+H,+Na,+K positive / -H,+Cl,+Br negative + distinct decoys), ppm {args.ppm:g}, "
                  f"nlevels {args.nlevels}")
        else:
            tag = "config3" if _is_config3(args) else "custom"
            if shard_only:
                tag += f" shard {args.shard_rank}/{args.shard_of}"
            wl = (f"{tag}: {args.nrows}x{args.ncols} px, Poisson({args.peaks:g}) centroids/spectrum, {args.n_sf} "
                  f"formulas x (+H,+Na,+K + distinct decoys), ppm {args.ppm:g}, nlevels {args.nlevels}")
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
                "workload": wl,
                "timed_region": ("one rank's step of the sharded search (slice + compute_sf_images + "
                                 "sf_image_metrics' device rows), measured alone" if shard_only else
                                 "compute_sf_images + sf_image_metrics through the drop-in API, DataFrame included"),
                "n_points": info["n_points"], "n_ions": formulas.n_ions, "n_ions_this_rank": my_formulas.n_ions,
                "n_rows_per_step": n_rows, "n_windows": int(formulas.ion_off[-1]),
                "sum_window_points": chain["sum_window_points"] if chain else None,
                "parallelism": (f"formula shards by principal m/z x{world}, dataset replicated, per-rank m/z slice, "
                                f"RCCL gather of metric rows" if sharded else
                                (f"1 GPU, rank {args.shard_rank} of a {args.shard_of}-way plan" if shard_only
                                 else "1 GPU")),
                "rccl_world_size": rccl_world,
                "shard_est_cost_s": plan.est_cost if plan is not None else None,
            },
            "sclk_mhz": sclk,
            "first_step_ms": first_step_ms,
            "cold_cache_step_ms": cold_ms,
            "step_ms_min_median_max": ([float(per_step.min()), float(np.median(per_step)), float(per_step.max())]
                                       if len(per_step) else None),
            "steps_ms": [round(float(x), 3) for x in per_step],
            "steps_sclk_mhz": step_clk,
            # KFD's queue-eviction time of this process per step (ms; None where sysfs does not show it)
            "steps_evicted_ms": ([b - a for a, b in zip(ev_marks[:-1], ev_marks[1:])]
                                 if None not in ev_marks else None),
            "numa_balancing": {"kernel": hostmem.numa_balancing_enabled(), "process_opted_out": NUMA_OPTOUT},
            "steps_desc_pass_ms": step_desc if len(step_desc) == len(per_step) else None,
            "steps_main_pass_ms": step_main if len(step_main) == len(per_step) else None,
            "per_rank": [{"rank": r, "step_ms_min_median_max": v[:3],
                          "sclk_mhz_median_min": None if v[3] < 0 else v[3:5],
                          "median_ms_rows_gather_assembly": None if v[5] < 0 else v[5:8]}
                         for r, v in enumerate(per_rank)],
            "device_chain": chain,
            "roofline": roofline,
            "passes": passes,
            "cpu_baseline": cpu,
            "lib": _lib.version(),
        }
        if _lib.check_build():  # the -DSMG_CHECK diagnostic library (SMG_LIB): its counters over the whole run
            line["check"] = _lib.check_counters()
        print(json.dumps(line), file=json_out, flush=True)
    if sharded:
        dist.destroy_process_group()


def _rank_seconds(D, plan, peaks, ds_config, reps=3):
    """This rank's time for its shard (slice, images, scores; no collective), best of ``reps`` after one warm-up."""
    import torch
    D._device_rows(plan, peaks, ds_config)
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        D._device_rows(plan, peaks, ds_config)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


class ClockSampler:
    """The GPU's shader clock over the timed region (diagnostic: some boxes of the pool cap it, and the
    latency-bound ion kernel's time follows it): the current DPM level of the device's pp_dpm_sclk (sysfs, the
    card whose PCI bus matches; the only readable one otherwise) read every 20 ms by a host thread.  stop() returns
    {"min", "median", "max", "samples"} in MHz, or None where sysfs does not expose it."""

    def __init__(self, props):
        import glob
        self.path = None
        self.samples = []
        self.times = []
        self._stop = threading.Event()
        self._thr = None
        if os.environ.get("SMG_BENCH_NO_CLOCK"):  # A/B: no sysfs polling during the timed steps
            return
        cands = []
        for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
            f = os.path.join(dev, "pp_dpm_sclk")
            try:
                with open(f) as fh:
                    fh.read()
                slot = ""
                with open(os.path.join(dev, "uevent")) as fh:
                    for ln in fh:
                        if ln.startswith("PCI_SLOT_NAME="):
                            slot = ln.strip().split("=", 1)[1]
                cands.append((f, slot))
            except OSError:
                continue
        bus = getattr(props, "pci_bus_id", None)
        match = [f for f, slot in cands if bus is not None and slot.split(":")[1:2] == [f"{bus:02x}"]]
        if len(match) == 1:
            self.path = match[0]
        elif len(cands) == 1:
            self.path = cands[0][0]
        self.samples = []
        self.times = []
        self._stop = threading.Event()
        self._thr = None

    def _read(self):
        with open(self.path) as fh:
            for ln in fh:
                if ln.rstrip().endswith("*"):
                    return float(ln.split(":")[1].strip().split("M")[0])
        return None

    def _run(self):
        while not self._stop.is_set():
            try:
                v = self._read()
            except (OSError, ValueError, IndexError):
                v = None
            if v is not None:
                self.samples.append(v)
                self.times.append(time.perf_counter())
            self._stop.wait(0.02)

    def start(self):
        if self.path:
            self._thr = threading.Thread(target=self._run, daemon=True)
            self._thr.start()

    def stop(self):
        if self._thr is None:
            return None
        self._stop.set()
        self._thr.join()
        if not self.samples:
            return None
        v = np.asarray(self.samples)
        return {"min": float(v.min()), "median": float(np.median(v)), "max": float(v.max()), "samples": int(v.size)}

    def over(self, t0, t1):
        """The clock over [t0, t1] (perf_counter seconds): the lowest sample inside it, else the nearest one; None
        without samples."""
        if not self.samples:
            return None
        t = np.asarray(self.times)
        v = np.asarray(self.samples)
        inside = (t >= t0) & (t <= t1)
        if inside.any():
            return float(v[inside].min())
        return float(v[np.argmin(np.minimum(np.abs(t - t0), np.abs(t - t1)))])


def _assembly_seconds(D, plan, peaks, ds_config, reps=3):
    """Rank 0's assembly of the gathered table (rows_to_frame, its steady-state form: the row placement kept from
    the previous search), best of ``reps``; 0 on the other ranks.  Every rank scores and gathers once (a
    collective)."""
    import torch
    rows, _ = D._device_rows(plan, peaks, ds_config)
    table = D.gather_rows(rows, plan)
    if table is None:
        return 0.0
    D.rows_to_frame(table, plan.global_keys)
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        D.rows_to_frame(table, plan.global_keys)
        best = min(best, time.perf_counter() - t)
    return best


def cold_step_ms(step_fn, formulas, plan, sharded):
    """Wall time of one search after the host-side caches of the previous searches are dropped."""
    import torch
    import torch.distributed as dist
    pk = formulas.get_sf_peak_ints()
    pk.__dict__.pop("_dev_cache", None)
    if plan is not None:
        plan._glob = None
        plan.formulas.get_sf_peak_ints().__dict__.pop("_dev_cache", None)
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    step_fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


def _is_config3(args):
    return (args.nrows, args.ncols, args.peaks, args.n_sf, args.ppm, args.nlevels, args.plant_fraction) == \
        (500, 500, 2000.0, 20000, 2.0, 30, 0.02)


def _pass_times(L):
    """(pass id, ms) of every pass launch recorded since the last call (smg_debug_pass_times)."""
    n = ctypes.c_int32(0)
    cap = 16384
    ms = (ctypes.c_double * cap)()
    ps = (ctypes.c_int32 * cap)()
    _lib_check(L.smg_debug_pass_times(ps, ms, cap, ctypes.byref(n)))
    return [(int(ps[i]), float(ms[i])) for i in range(min(n.value, cap))]


def pass_roofline(args, pass_ms, chain, is_single):
    """Per pass of smg_ion_metrics: its average launch time (HIP events on the launch stream, timed API steps),
    the window points of the ions it scored (SMG_ION_* flags of the device chain, same data and ions) and their
    12-B algorithmic bytes over that time.  ``roofline`` = the scoring pass with the largest time."""
    from sm_distributed_amd import _lib
    if not chain or not pass_ms:
        return None, None
    by = {}
    for p, t in pass_ms:
        by.setdefault(p, []).append(t)
    passes = {}
    for p, ts in sorted(by.items()):
        name = _lib.PASS_NAMES.get(p, str(p))
        d = {"pass": p, "ms_avg": float(np.mean(ts)), "launches_timed": len(ts)}
        if p not in (_lib.SMG_PASS_DESC, _lib.SMG_PASS_FINALIZE):
            pts = chain["pass_window_points"].get(p, 0)
            d.update({"ions": chain["pass_ions"].get(p, 0), "window_points": pts,
                      "alg_bytes_per_launch": ALG_BYTES_PER_POINT * pts})
            if d["ms_avg"] > 0:
                ach = ALG_BYTES_PER_POINT * pts / (d["ms_avg"] * 1e-3) / 1e9
                d.update({"achieved_GBps": ach, "frac": ach / HBM_PEAK_GBS})
        passes[name] = d
    scoring = [d for d in passes.values() if d["pass"] not in (_lib.SMG_PASS_DESC, _lib.SMG_PASS_FINALIZE)
               and d.get("window_points")]
    if not scoring:
        return None, passes
    dom = max(scoring, key=lambda d: d["ms_avg"])
    name = _lib.PASS_NAMES[dom["pass"]]
    legacy_main = not chain.get("main_pass_sparse", True)  # smg_debug_main_kernel(0): ion_pipe_kernel<512> ran
    if legacy_main and dom["pass"] == _lib.SMG_PASS_MAIN:
        name = "ion_pipe_kernel<512> (main LDS pass)"
    # the LDS passes leave their scores' arithmetic to ion_finalize_kernel (a few per cent of their work): its
    # whole time is charged to the dominant LDS pass, so the roofline does not gain from moving work out of it
    fin = passes.get(_lib.PASS_NAMES[_lib.SMG_PASS_FINALIZE])
    fin_ms = fin["ms_avg"] if fin and dom["pass"] in (_lib.SMG_PASS_MAIN, _lib.SMG_PASS_BIG) else 0.0
    ms_charged = dom["ms_avg"] + fin_ms
    ach = ALG_BYTES_PER_POINT * dom["window_points"] / (ms_charged * 1e-3) / 1e9
    key = {1: "ion_pipe_kernel[512]" if legacy_main else "ion_sparse_kernel", 2: "ion_pipe_kernel[1024]",
           3: "ion_wide_join_kernel", 4: "ion_dense_kernel"}  # (no clip here: the wide pass is the join kernel)
    traffic, src = measured_traffic(key[dom["pass"]], "config5" if args.config == "5" else "config3") \
        if is_single else (None, None)
    roofline = {"bound": "hbm", "kernel": name, "achieved": ach, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                "alg_bytes_per_launch": dom["alg_bytes_per_launch"], "kernel_ms_avg": dom["ms_avg"],
                "finalize_ms_avg_charged": fin_ms, "kernel_launches_timed": dom["launches_timed"],
                "ions_scored_by_pass": dom["ions"],
                "alg_bytes_8B_per_point_frac": ach / HBM_PEAK_GBS * 8.0 / ALG_BYTES_PER_POINT}
    return roofline, passes


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
        p.flag_and_sort(args.ppm)
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
    # the window points of each ion, attributed to the pass that scored it (SMG_ION_* flags)
    from sm_distributed_amd import _lib
    cs = torch.zeros(lo.numel() + 1, dtype=torch.int64, device=lo.device)
    torch.cumsum(hi - lo, 0, out=cs[1:])
    pts = (cs[dions.win_off[1:]] - cs[dions.win_off[:-1]]).cpu().numpy()
    fl = out.flags.cpu().numpy().astype(np.int64)
    pas = np.full(n, _lib.SMG_PASS_MAIN)
    pas[(fl & _lib.SMG_ION_BIG) != 0] = _lib.SMG_PASS_BIG
    pas[(fl & _lib.SMG_ION_DENSE) != 0] = _lib.SMG_PASS_DENSE
    pas[(fl & _lib.SMG_ION_WIDE) != 0] = _lib.SMG_PASS_WIDE
    has = (fl & _lib.SMG_ION_HAS_HITS) != 0
    pass_pts = {int(p): int(pts[has & (pas == p)].sum()) for p in np.unique(pas)}
    pass_ions = {int(p): int((has & (pas == p)).sum()) for p in np.unique(pas)}
    t0 = time.perf_counter()
    for _ in range(args.chain_steps):
        step(True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.chain_steps * 1e3
    names = ["flag+sort+scan", "window_search", "ion_metrics"]
    stages = {nm: float(np.mean([e[j].elapsed_time(e[j + 1]) for e in events])) for j, nm in enumerate(names)}
    return {"ms_per_step": ms, "ions_per_s": n_scored / (ms * 1e-3), "n_scored": n_scored, "stages_ms": stages,
            "sum_window_points": sum_hits, "n_points": pk.n_points, "pass_window_points": pass_pts,
            "pass_ions": pass_ions, "main_pass_sparse": bool(((fl & _lib.SMG_ION_SPARSE) != 0).any())}


def measured_traffic(kernel, workload):
    """HBM bytes per launch of ``kernel`` on ``workload`` from the newest committed PMC summary
    (profiles/*/traffic_*.json, scripts/gpu_traffic.sh: FETCH_SIZE calibrated for the kernel's access width, +
    WRITE_SIZE).  The counters cannot be read from inside this process; None when no summary exists.  Summaries
    without a "config" field are config-3 summaries of the main ion kernel (rounds 1-2)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic_*.json")))
    best = None
    for f in files:  # profiles/round<N>/..., newest round last
        d = json.load(open(f))
        cfg = d.get("config", "config3" if d.get("kernel") == "ion_pipe_kernel[512]" else None)
        if d.get("kernel") == kernel and cfg == workload:
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
                       f"(oracle/cpu_baseline.py); wall {wall:.1f}s.  Favourable to the CPU: the selection of the "
                       f"window points from the resident dataset runs before the timed wall, and each worker sorts only "
                       f"its ions' window points, not a whole m/z segment of every spectrum as formula_imager_segm.py:"
                       f"73-74 does -- an upper bound on the reference CPU path's rate"),
            "nproc": os.cpu_count(), "cpus_available": CB.available_cpus(), "cpu_model": CB.cpu_model()}


if __name__ == "__main__":
    main()
