"""Multi-GPU hot path: the formula list sharded over ranks by m/z, one collective for the metric rows
(BASELINE.json config 4: strong scaling of config 3 over 2/4/8 GPUs).

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI).  Every rank holds the resident
dataset (replicated: each rank loads it, as each Spark executor reads ds.txt).  The reference partitions the
*data* by m/z segment and shuffles every point to its segment (formula_imager_segm.py:45-49, 112-121, 152-155),
then groups images per ion (:134-138) and collects metric tuples to the driver (formula_img_validator.py:
115-118).  Here the *formulas* are partitioned by m/z instead, so no point ever moves between GPUs:

* ``plan_shards`` (once per dataset / formula table / ppm): ions ordered by principal m/z are cut into
  ``world`` contiguous ranges of equal estimated cost.  The cost model is the analogue of
  ``_estimate_mz_workload`` (formula_imager_segm.py:9-14, a product of the data and theoretical-peak m/z
  histograms): per ion, the expected window points from the dataset's m/z histogram (ion kernel, ~6.5 ps per
  window point on MI355X), a fixed per-ion cost, and the data points its m/z range adds to the rank's slice
  (slice copy + sort, ~33 ps per point).  A rank's slice is [min lower bound, max upper bound] of its windows;
* ``score_sharded`` (per search): each rank copies its m/z slice of the resident peaks (smg_slice_mz_*, with the
  duplicate flags fused into the copy), so its sort covers ~1/world of the points; runs compute_sf_images +
  sf_image_metrics' device batch on its shard; packs fixed-size rows (global ion index, chaos, spatial,
  spectral, msm; 40 B) and gathers them to rank 0 (one RCCL gather over xGMI: the other ranks send their ~5 MB
  blocks over their own links to rank 0 at once); rank 0 builds the reference DataFrame from codes;
* ``search``: MSMBasicSearch.search (msm_basic_search.py:13-20) over the ranks: the table of ``score_sharded``,
  then FDR and the filter on rank 0, the images staying on the rank that made them.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import pandas as pd

# cost model constants (MI355X, config 3): least-squares fit (no intercept) of every rank's measured step in an
# 8-way plan scored on one GPU (scripts/time_shards.py, profiles/round2/r2j_time_shards_8.txt): slice copy + flag +
# sort + scan ~54 ps per slice point, ion stage ~6.2 ps per window point and ~2 ns per ion
C_WINDOW_POINT = 6.2e-12
C_ION = 2.0e-9
C_SLICE_POINT = 54e-12
# Rank 0 alone assembles the gathered rows into the DataFrame (rows_to_frame, ~0.8 ms at config 3).  One search
# alone ends with it after the gather, but back to back (the bench, a search per dataset) the other ranks return
# after the gather and start the next search while rank 0 assembles: rank 0's shard is then cut smaller by the
# assembly (rebalance's head_seconds), so that every rank reaches the next gather together.

ROW_FIELDS = ("ion", "chaos", "spatial", "spectral", "msm")


@dataclass
class ShardPlan:
    rank: int
    world: int
    ion_idx: np.ndarray            # this rank's ions (positions in the formula table's (sf_id, adduct) order)
    formulas: object               # FormulasSegm of this rank's ions
    mz_lo: float                   # the m/z slice this rank's windows touch (f64, inclusive)
    mz_hi: float
    ppm: float
    counts: list                   # ions per rank
    bounds: list                   # [(first, last) principal-order positions] per rank
    global_keys: object            # IonKeys of the whole table (rank 0 builds the DataFrame from codes)
    est_cost: list = field(default_factory=list)  # estimated seconds per rank
    costs: np.ndarray = None       # per-ion seconds in principal order that made this cut (rebalance scales them)
    _sf_peak_df: object = None
    _glob: object = None           # (shard ion keys, device f64 global index of each): reused while they match

    @property
    def sf_peak_df(self):
        if self._sf_peak_df is None:
            self._sf_peak_df = self.formulas.get_sf_peak_df()
        return self._sf_peak_df


def ion_costs(win_off, peak_mz, ppm, mz_hist=None, mz_edges=None):
    """Estimated seconds per ion: expected window points (dataset m/z density x window width) x C_WINDOW_POINT +
    C_ION.  Without a histogram the density is taken as uniform (window points ~ window width ~ m/z)."""
    win_off = np.asarray(win_off)
    peak_mz = np.asarray(peak_mz, dtype=np.float64)
    width = 2.0 * ppm * 1e-6 * peak_mz
    if mz_hist is not None:
        idx = np.clip(np.searchsorted(mz_edges, peak_mz, side="right") - 1, 0, len(mz_hist) - 1)
        dens = np.asarray(mz_hist, dtype=np.float64)[idx] / np.diff(mz_edges)[idx]
        inside = (peak_mz >= mz_edges[0]) & (peak_mz <= mz_edges[-1])
        pts = np.where(inside, dens * width, 0.0)
    else:
        pts = width
    pts = np.where(np.isfinite(pts), pts, 0.0)
    cs = np.concatenate([[0.0], np.cumsum(pts)])
    return (cs[win_off[1:]] - cs[win_off[:-1]]) * C_WINDOW_POINT + C_ION


def shard_bounds(costs, world, head=0.0):
    """Contiguous [a, b) ranges with ~equal summed cost (greedy cut on the cost prefix sum); ``head`` is work
    rank 0 does besides its shard (the assembly), so its range is cut that much smaller."""
    costs = np.asarray(costs, dtype=np.float64)
    n = len(costs)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    pref = np.concatenate([[0.0], np.cumsum(costs)])
    total = pref[-1]
    # rank 0's shard a0 and every other rank's share f: a0 + head = f when the head fits one share, else a0 = 0
    f = (total + head) / world
    a0 = f - head
    if a0 < 0.0:
        a0, f = 0.0, total / (world - 1)
    cuts = [0] + [int(np.searchsorted(pref, a0 + (r - 1) * f)) for r in range(1, world)] + [n]
    cuts = np.maximum.accumulate(np.array(cuts))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def mz_histogram(mz, bins=8192):
    """(counts, edges) of the resident m/z values (a torch tensor, device or host): one pass over the data."""
    import torch
    lo, hi = (float(v) for v in torch.aminmax(mz))
    hi = hi if hi > lo else lo + 1.0
    h = torch.histc(mz.to(torch.float32), bins=bins, min=lo, max=hi).double().cpu().numpy()
    return h, np.linspace(lo, hi, bins + 1)


def _principal_costs(formulas, peaks_or_mz, ppm, bins):
    """(ions in principal m/z order, their estimated seconds in that order)."""
    mz = getattr(peaks_or_mz, "mz", peaks_or_mz)
    hist, edges = mz_histogram(mz, bins)
    off, pmz = formulas.ion_off, formulas.peak_mz
    first = pmz[off[:-1]]
    order = np.argsort(first, kind="stable")           # principal m/z order
    cost = ion_costs(off, pmz, ppm, hist, edges)[order]
    # slice growth: the data points between consecutive principal m/z values enter the slice of whichever rank
    # holds the ion before them
    cum_pts = np.concatenate([[0.0], np.cumsum(hist)])
    pos = np.interp(first[order], edges, cum_pts)
    grow = np.diff(np.concatenate([pos, [cum_pts[-1]]]))
    return order, cost + np.maximum(grow, 0.0) * C_SLICE_POINT


def plan_shards(formulas, peaks_or_mz, ppm, world, rank, bins=8192):
    """Shard ``formulas`` (FormulasSegm) over ``world`` ranks by principal m/z; returns this rank's ShardPlan.
    ``peaks_or_mz``: the resident DevicePeaks (or an m/z tensor) whose histogram drives the cost model."""
    order, cost = _principal_costs(formulas, peaks_or_mz, ppm, bins)
    return _plan_from_costs(formulas, order, cost, ppm, world, rank)


def rebalance(plan, formulas, peaks_or_mz, rank_seconds, bins=8192, head_seconds=0.0):
    """The plan re-cut from measured per-rank step times (one value per rank, e.g. all_gathered after a first
    search): every rank's ions get its measured/estimated ratio as a cost factor, and the shards are cut again on
    the corrected costs (the linear model of ion_costs leaves +-5 % per-rank residuals that no refit removes).
    ``head_seconds``: rank 0's assembly of the gathered table (rows_to_frame), which the other ranks do not wait
    for -- they return after the gather and start the next search -- so rank 0's shard is cut that much smaller
    (shard_bounds' head) and every rank reaches the next gather together.
    Deterministic: every rank computes the same cut from the same times.  Returns this rank's new ShardPlan.

    Repeated calls refine the cut: the costs of a rebalanced plan (``plan.costs``) are scaled again, so each
    call multiplies every ion's cost by its current rank's measured/estimated ratio (bench.py re-cuts until the
    ranks' times agree within a few per cent)."""
    order, cost = _principal_costs(formulas, peaks_or_mz, plan.ppm, bins)
    if plan.costs is not None and len(plan.costs) == len(cost):
        cost = plan.costs
    t = np.asarray(rank_seconds, dtype=np.float64)
    if len(t) != plan.world or not np.all(np.isfinite(t)) or not np.all(t > 0):
        raise ValueError("rank_seconds: one positive time per rank")
    scaled = cost.copy()
    for r, (a, b) in enumerate(plan.bounds):
        est = float(cost[a:b].sum())
        if b > a and est > 0:
            scaled[a:b] *= t[r] / est
    if not np.isfinite(head_seconds) or head_seconds < 0.0:
        raise ValueError("head_seconds: a time >= 0")
    return _plan_from_costs(formulas, order, scaled, plan.ppm, plan.world, plan.rank, head=float(head_seconds))


def _plan_from_costs(formulas, order, cost, ppm, world, rank, head=0.0):
    from .formula_imager_segm import IonKeys
    bounds = shard_bounds(cost, world, head)
    a, b = bounds[rank]
    mine = np.sort(order[a:b])                        # back to (sf_id, adduct) order
    shard = formulas.subset(mine)
    if len(mine) and len(shard.peak_mz):
        lower = shard.peak_mz - shard.peak_mz * ppm * 1e-6   # formula_imager_segm.py:79-80, left to right
        upper = shard.peak_mz + shard.peak_mz * ppm * 1e-6
        mz_lo, mz_hi = float(lower.min()), float(upper.max())
    else:
        mz_lo, mz_hi = 1.0, 0.0  # empty slice
    keys = formulas.ion_sf.astype(np.int64) * max(len(formulas.adducts), 1) + formulas.ion_adduct_code
    return ShardPlan(rank=rank, world=world, ion_idx=mine, formulas=shard, mz_lo=mz_lo, mz_hi=mz_hi, ppm=ppm,
                     counts=[int(y - x) for x, y in bounds], bounds=bounds,
                     global_keys=IonKeys(keys, formulas.adducts), est_cost=[float(cost[x:y].sum()) for x, y in bounds],
                     costs=np.asarray(cost, dtype=np.float64))


def slice_peaks(peaks, plan, cache=True):
    """This rank's m/z slice of the resident dataset, duplicate flags set for plan.ppm (smg_slice_mz_*).

    The slice is a function of the resident dataset and the plan only, so it is made once per (plan bounds, ppm)
    and kept on the DevicePeaks, the way the single-GPU search keeps the whole dataset resident: every search still
    flags (the copy did), sorts and prefix-sums it (compute_sf_images), as the single-GPU search does the whole
    dataset.  ``cache=False`` copies it anew.

    The key names the data as well as the plan: the resident arrays (their device addresses and length) and
    ``peaks.version`` (bumped by every flag pass or sort of them), so that replaced or re-flagged resident data
    is sliced again.  One slice is kept per rank (a new key drops the old one); it holds ~1/N of the dataset."""
    key = (float(plan.mz_lo), float(plan.mz_hi), float(plan.ppm), int(peaks.n_points), int(peaks.version),
           int(peaks.mz.data_ptr()), int(peaks.hits.data_ptr()))
    store = peaks.__dict__.setdefault("_slices", {})
    if cache and key in store:
        return store[key]
    sl = peaks.slice_mz(plan.mz_lo, plan.mz_hi, plan.ppm)
    if cache:
        store.clear()  # one plan per rank at a time: a re-cut plan replaces the old slice
        store[key] = sl
    return sl


def _device_rows(plan, peaks, ds_config):
    """Score this rank's shard on its GPU: [n_shard, 5] float64 rows (global ion index or -1, chaos, spatial,
    spectral, msm) and this rank's IonImageSet."""
    import torch

    from .dataset import ResidentDataset
    from .formula_imager_segm import compute_sf_images
    from .formula_img_validator import _metrics_device_rows
    dev = peaks.device
    n = len(plan.ion_idx)
    rows = torch.full((n, len(ROW_FIELDS)), -1.0, dtype=torch.float64, device=dev)
    if n == 0:
        return rows, None
    sl = slice_peaks(peaks, plan)
    dds = ResidentDataset(sl)
    ims = compute_sf_images(None, dds, plan.sf_peak_df, plan.ppm)
    keep, m = _metrics_device_rows(ims, plan.formulas.get_sf_peak_ints(), ds_config["image_generation"])
    # global ion index of each image-set ion: re-encode its (sf_id, adduct) with the whole table's adduct codes
    # (the shard's sf_peak_df may lack some adducts, so its own codes differ)
    ik = ims.ion_keys
    cached = plan._glob
    if cached is not None and cached[0] is not ik.keys and np.array_equal(cached[0], ik.keys):
        cached = (ik.keys, cached[1])  # the same shard layout as the previous step
    if cached is None or cached[0] is not ik.keys:
        gk, ok = plan.global_keys.encode_codes(ik.sf_values(), ik.adduct_code, ik.adducts)
        pos = np.searchsorted(plan.global_keys.keys, gk)
        if not ok.all() or not (plan.global_keys.keys[np.minimum(pos, len(plan.global_keys.keys) - 1)] == gk).all():
            raise AssertionError("shard ion missing from the formula table")
        cached = (ik.keys, torch.from_numpy(pos.astype(np.float64)).to(dev))
    plan._glob = cached
    glob = cached[1]
    k = glob.numel()
    rows[:k, 0] = torch.where(keep, glob, torch.full_like(glob, -1.0))
    rows[:k, 1] = m.chaos
    rows[:k, 2] = m.spatial
    rows[:k, 3] = m.spectral
    rows[:k, 4] = m.msm
    ims.score_flags = m.flags  # SMG_ION_* per image-set ion (which pass scored it): diagnostics and tests
    return rows, ims


def gather_rows(rows, plan, group=None):
    """Gather every rank's row block, padded to the largest shard, to rank 0 of ``group`` (one RCCL gather);
    returns the [world * n_max, 5] table on that rank, None elsewhere."""
    import torch
    import torch.distributed as dist
    n_max = max(plan.counts) if plan.counts else 0
    send = torch.full((n_max, rows.shape[1]), -1.0, dtype=rows.dtype, device=rows.device)
    send[:rows.shape[0]] = rows
    dst = 0 if group is None else dist.get_global_rank(group, 0)
    if dist.get_rank(group) != 0:
        dist.gather(send, None, dst=dst, group=group)
        return None
    recv = torch.empty(plan.world * n_max, rows.shape[1], dtype=rows.dtype, device=rows.device)
    dist.gather(send, list(recv.view(plan.world, n_max, rows.shape[1]).unbind(0)), dst=dst, group=group)
    return recv


def rows_to_frame(table, global_keys):
    """Rank-0 assembly: gathered rows -> the reference DataFrame (index [sf_id, adduct] in table order,
    columns chaos, spatial, spectral, msm), one row per ion with images.  The rows are put in table order by a
    scatter on the device holding them (no sort; padding rows go to a dummy slot), the metric columns and the
    index codes are gathered there and copied to pinned host memory together (formula_imager_segm.device_frame):
    two host synchronisations.

    The row placement and the MultiIndex depend only on the gathered ion indices (column 0): they are kept on
    ``global_keys`` and reused while the next gathered table carries the same indices (a search per step over
    the same plan), so such a step only gathers and copies the metric columns."""
    import torch

    from .formula_imager_segm import METRIC_COLUMNS, device_frame
    t = table if hasattr(table, "device") else torch.as_tensor(np.asarray(table))
    n = len(global_keys)
    gi = t[:, 0].long()
    gi = torch.where(gi >= 0, gi, torch.full_like(gi, n))
    cache = global_keys.__dict__.get("_frame_cache")
    if cache is not None and t.device.type == "cuda" and cache[0].device == t.device and cache[0].shape == gi.shape:
        # the cached placement, checked on the device and copied back with the columns: one synchronisation
        rows_sel, mi = cache[1], cache[2]
        differs = torch.ne(cache[0], gi).any().reshape(1)
        cols = t[rows_sel, 1:5].T.contiguous()  # [4, rows] in table order
        host = torch.empty(cols.shape, dtype=torch.float64, pin_memory=True)
        flag = torch.empty(1, dtype=torch.bool, pin_memory=True)
        flag.copy_(differs, non_blocking=True)
        host.copy_(cols, non_blocking=True)
        torch.cuda.current_stream(t.device).synchronize()
        if not bool(flag[0]):
            return pd.DataFrame(host.numpy().T, index=mi, columns=METRIC_COLUMNS, copy=False)
    # the gathered row of every ion (-1: none), then the ions with a row in table order and their rows
    row = torch.full((n + 1,), -1, dtype=torch.int64, device=t.device)
    row[gi] = torch.arange(t.shape[0], device=t.device)
    idx = torch.nonzero(row[:n] >= 0).flatten()
    rows_sel = row[idx]
    cols = t[rows_sel, 1:5].T  # [4, rows] in table order
    df = device_frame(global_keys, cols, idx, cols_compact=True)
    if t.device.type == "cuda":
        global_keys._frame_cache = (gi, rows_sel, df.index)
    return df


def score_sharded(plan, peaks, ds_config, group=None, score_local=None, phases=None):
    """compute_sf_images + sf_image_metrics over all ranks: returns (the reference metrics table on rank 0,
    None elsewhere; this rank's IonImageSet).  ``score_local(plan, peaks, ds_config) -> (rows, images)``
    replaces the device scorer (tests on CPU ranks).

    ``phases`` (diagnostics, GPU ranks): a list to which this call appends four timing events recorded on the
    current stream at its start, after the rows, after the gather and after the assembly -- no synchronisation is
    added; ``phase_ms`` turns them into the (rows, gather, assembly) split once they have completed."""
    import torch
    ev = None
    if phases is not None and torch.cuda.is_available() and peaks.device.type == "cuda":
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
    rows, ims = (score_local or _device_rows)(plan, peaks, ds_config)
    if ev:
        ev[1].record()
    table = gather_rows(rows, plan, group)
    if ev:
        ev[2].record()
    df = rows_to_frame(table, plan.global_keys) if table is not None else None
    if ev:
        ev[3].record()
        phases.append(ev)
    return df, ims


def phase_ms(ev):
    """(rows, gather, assembly) milliseconds of one score_sharded call's ``phases`` events (waits for them)."""
    ev[3].synchronize()
    return tuple(ev[j].elapsed_time(ev[j + 1]) for j in range(3))


def search(plan, peaks, formulas, fdr, ds_config, group=None, score_local=None):
    """MSMBasicSearch.search (msm_basic_search.py:13-31) over the ranks: on rank 0 the FDR-annotated, filtered
    metrics table (sf_image_metrics_est_fdr + filter_sf_metrics); on every rank the images of its reported
    ions (filter_sf_images)."""
    import torch.distributed as dist

    from .formula_img_validator import sf_image_metrics_est_fdr
    from .search_algorithm import MSMBasicSearch
    df, ims = score_sharded(plan, peaks, ds_config, group, score_local)
    msm = MSMBasicSearch(None, None, formulas, fdr, ds_config)
    out = None
    if dist.get_rank(group) == 0:
        out = msm.filter_sf_metrics(sf_image_metrics_est_fdr(df, formulas, fdr))
    # every rank filters its own images by the reported keys (broadcast of the reported index)
    obj = [None if out is None else out.index]
    # src is a global rank: group rank 0's (gather_rows sends the table there)
    dist.broadcast_object_list(obj, src=0 if group is None else dist.get_global_rank(group, 0), group=group)
    images = msm.filter_sf_images(ims, obj[0]) if ims is not None else None
    return out, images
