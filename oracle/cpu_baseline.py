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
