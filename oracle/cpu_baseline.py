"""CPU baseline leg of bench.py: the oracle (reference algorithm restated in numpy/scipy) timed on host cores.

TEST/BENCH INFRASTRUCTURE ONLY (see oracle/msm_oracle.py header).  It mirrors one Spark worker's share of
the reference job (formula_imager_segm.py:66-92 on an m/z segment: sort the segment's points by m/z,
searchsorted every window, build COO images; then formula_img_validator.py:72-84 per ion), run by a pool
of worker processes the way Spark ``local[*]`` runs Python workers.  Workers never import torch.
"""
from __future__ import annotations

import os
import time

import numpy as np

_DATA = {}


def _init(pix, mz, ints, dims, ppm, nlevels):
    _DATA.update(pix=pix, mz=mz, ints=ints, dims=dims, ppm=ppm, nlevels=nlevels)
    os.environ.setdefault("OMP_NUM_THREADS", "1")


def _work(task):
    """task = list of (ion_id, peak_mz[K], theor[K]); returns (ion_id, chaos, spatial, spectral) rows + seconds."""
    from scipy.sparse import coo_matrix

    from oracle import msm_oracle as O
    t0 = time.perf_counter()
    pix, mz, ints = _DATA["pix"], _DATA["mz"], _DATA["ints"]
    nrows, ncols = _DATA["dims"]
    # formula_imager_segm.py:73-74: sort the segment's points by m/z
    order = np.argsort(mz, kind="stable")
    pix_s, mz_s, int_s = pix[order], mz[order], ints[order].astype(np.float64)
    mz64 = mz_s.astype(np.float64)
    rows = []
    for ion_id, pmz, theor in task:
        lower, upper = O.window_bounds(pmz, _DATA["ppm"])
        lo = np.searchsorted(mz64, lower, "left")
        hi = np.searchsorted(mz64, upper, "right")
        imgs = []
        for l, u in zip(lo, hi):
            if u - l >= 1:
                idx = pix_s[l:u]
                imgs.append(coo_matrix((int_s[l:u], (idx // ncols, idx % ncols)), shape=(nrows, ncols)))
            else:
                imgs.append(None)
        if all(m is None for m in imgs):
            continue
        last = max(j for j, m in enumerate(imgs) if m is not None)
        c, s, p = O.compute_img_metrics(imgs[:last + 1], list(theor), nrows, ncols, _DATA["nlevels"])
        rows.append((ion_id, c, s, p))
    return rows, time.perf_counter() - t0


def available_cpus():
    """Cores this process may use: the affinity mask, capped by a cgroup-v2 CPU quota when one is set (on a
    shared GPU box nproc / os.cpu_count() report the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(float(quota) / float(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def default_workers(cap=None):
    n = available_cpus()
    return min(n, cap) if cap else n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def run_pool(pix, mz, ints, dims, ppm, nlevels, ions, workers):
    """ions: list of (ion_id, peak_mz, theor).  Returns (rows, wall_seconds, per_worker_seconds)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    chunks = [ions[i::workers] for i in range(workers)]
    with ctx.Pool(workers, initializer=_init, initargs=(pix, mz, ints, dims, ppm, nlevels)) as pool:
        pool.map(_noop, range(workers))  # make sure every worker is up and initialised before timing
        t0 = time.perf_counter()
        res = pool.map(_work, chunks)
        wall = time.perf_counter() - t0
    rows = [r for rr, _ in res for r in rr]
    return rows, wall, [t for _, t in res]


def _noop(_):
    return 0


def _work_segment(task):
    """One worker's share: (pix, mz, ints, dims, ppm, nlevels, ions); returns (rows, seconds)."""
    pix, mz, ints, dims, ppm, nlevels, ions = task
    _init(pix, mz, ints, dims, ppm, nlevels)
    return _work(ions)


def _merge_intervals(lower, upper, rel=1e-6):
    lo = np.asarray(lower, np.float64) * (1 - rel)
    hi = np.asarray(upper, np.float64) * (1 + rel)
    order = np.argsort(lo)
    lo, hi = lo[order], hi[order]
    ms, me = [lo[0]], [hi[0]]
    for a, b in zip(lo[1:], hi[1:]):
        if a <= me[-1]:
            me[-1] = max(me[-1], b)
        else:
            ms.append(a)
            me.append(b)
    return np.array(ms), np.array(me)


def select_window_points(mz, hits, lower, upper, block=1 << 27):
    """Points of a resident dataset (torch device tensors: mz f32, packed hits) whose m/z lies in the union of
    the windows [lower, upper] (f64, widened by 1e-6 relative so f32 rounding cannot drop a point); returns
    host (pix, mz, int).  Every point of every window is included, so searchsorted over the selection gives the
    windows of the whole dataset."""
    import torch
    ms, me = _merge_intervals(lower, upper)
    A = torch.tensor(ms, dtype=torch.float64, device=mz.device)
    B = torch.tensor(me, dtype=torch.float64, device=mz.device)
    pm, ph = [], []
    for a in range(0, mz.numel(), block):
        x = mz[a:a + block].to(torch.float64)
        j = torch.searchsorted(A, x, right=True) - 1
        inside = (j >= 0) & (x <= B[j.clamp(min=0)])
        pm.append(mz[a:a + block][inside].cpu().numpy())
        ph.append(hits[a:a + block][inside].cpu().numpy())
    b_mz = np.concatenate(pm)
    b_hits = np.concatenate(ph).view(np.uint64)
    b_pix = (b_hits & np.uint64(0x7FFFFFFF)).astype(np.int64)
    b_int = (b_hits >> np.uint64(32)).astype(np.uint32).view(np.float32)
    return b_pix, b_mz, b_int


def run_pool_split(pix, mz, ints, dims, ppm, nlevels, ions, workers):
    """Like run_pool, but each worker receives only the points of its own ions' windows (its m/z segments, the
    way a Spark executor holds only its partition): ions are split into ``workers`` contiguous groups by
    principal m/z.  Returns (rows, wall_seconds, per_worker_seconds)."""
    import multiprocessing as mp

    from oracle import msm_oracle as O
    ions = sorted(ions, key=lambda t: float(t[1][0]))
    chunks = [ions[len(ions) * w // workers: len(ions) * (w + 1) // workers] for w in range(workers)]
    order = np.argsort(mz, kind="stable")
    mz_s = mz[order].astype(np.float64)
    tasks = []
    for ch in chunks:
        if not ch:
            continue
        lower, upper = O.window_bounds(np.concatenate([t[1] for t in ch]), ppm)
        ms, me = _merge_intervals(lower, upper)
        a = np.searchsorted(mz_s, ms, "left")
        b = np.searchsorted(mz_s, me, "right")
        sel = order[np.concatenate([np.arange(x, y) for x, y in zip(a, b)])] if len(a) else np.zeros(0, np.int64)
        tasks.append((pix[sel], mz[sel], ints[sel], dims, ppm, nlevels, ch))
    ctx = mp.get_context("spawn")
    with ctx.Pool(len(tasks)) as pool:
        pool.map(_noop, range(len(tasks)))  # every worker up before timing
        t0 = time.perf_counter()
        res = pool.map(_work_segment, tasks, chunksize=1)
        wall = time.perf_counter() - t0
    rows = [r for rr, _ in res for r in rr]
    return rows, wall, [t for _, t in res]
